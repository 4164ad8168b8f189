export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::600:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fused_gpu.py tests/test_learner_gpu.py tests/test_config_size_gpu.py tests/test_parallel_gpu.py tests/test_gru_gpu.py" \
  "b4:::200:::python bench.py --model gru --no-cpu-baseline --steps 50 --env-micro 0"
