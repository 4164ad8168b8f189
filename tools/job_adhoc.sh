export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::500:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gru_gpu.py tests/test_uam_gpu.py tests/test_uam_learner_gpu.py tests/test_parallel_gpu.py" \
  "b4:::200:::python bench.py --model gru --no-cpu-baseline --steps 50" \
  "b5:::200:::python bench.py --model uam --no-cpu-baseline --steps 50" \
  "b5v:::200:::AAC_LIB=$PWD/tools/variants/lib_uamw1.so python bench.py --model uam --no-cpu-baseline --steps 50" \
  "b5b:::200:::python bench.py --model uam --no-cpu-baseline --steps 50"
