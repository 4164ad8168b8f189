# GRU learner with the XCD-aware GEMM order: parity tests, config-4 bench, GEMM traffic passes
export TMPDIR=/tmp
mkdir -p gpurun_out
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--model gru --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py::test_gemm_xcd_order_bit_identical \
  tests/test_gru_gpu.py "tests/test_parallel_gpu.py" -k "xcd or gru or GRU" > gpurun_out/gx_tests.log 2>&1 || { tail -30 gpurun_out/gx_tests.log; exit 1; }
tail -2 gpurun_out/gx_tests.log
rm -f gpurun_out/abm.txt
bash tools/ab_multi.sh "--model gru" AAC_GRU_XCD=0 AAC_GRU_XCD=1 || exit 1
rm -rf gpurun_out/pmc4f gpurun_out/pmc4w gpurun_out/job.log
bash tools/gpu_job.sh \
  "f4:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pmc4f -o run -- python3 bench.py $SHORT" \
  "w4:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pmc4w -o run -- python3 bench.py $SHORT" > /dev/null
