export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::600:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_uam_learner_gpu.py tests/test_parallel_gpu.py tests/test_config_size_gpu.py -k 'uam or head or two_ranks'" \
  "b5:::200:::python bench.py --model uam --no-cpu-baseline --steps 50 --env-micro 0" \
  "b5b:::200:::python bench.py --model uam --no-cpu-baseline --steps 50 --env-micro 0"
