export TMPDIR=/tmp
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
bash tools/gpu_job.sh \
  "learn:::500:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_learner_gpu.py tests/test_fused_gpu.py tests/test_facade_gpu.py tests/test_gru_gpu.py" \
  "b3:::200:::python bench.py --no-cpu-baseline --steps 50" \
  "prof3:::240:::$T --stats -d gpurun_out/prof3 -o run -- python3 bench.py $SHORT"
