export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::500:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_uam_gpu.py tests/test_config_size_gpu.py -k 'uam or UAM'" \
  "b5:::200:::python bench.py --model uam --no-cpu-baseline --steps 50"
