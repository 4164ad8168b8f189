export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::600:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_config_size_gpu.py -k 'env or Env' tests/test_wgru_gpu.py tests/test_multimap_gpu.py" \
  "b3:::200:::python bench.py --no-cpu-baseline --steps 50"
