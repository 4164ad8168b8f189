export TMPDIR=/tmp
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
bash tools/gpu_job.sh \
  "envtests:::400:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_wgru_gpu.py tests/test_multimap_gpu.py" \
  "b3:::200:::python bench.py --no-cpu-baseline --steps 50" \
  "b4:::200:::python bench.py --model gru --no-cpu-baseline --steps 50" \
  "w3:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pmc3w -o run -- python3 bench.py $SHORT" \
  "f3:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pmc3f -o run -- python3 bench.py $SHORT" \
  "gt:::200:::python tools/gemm_table.py --split"
