export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::600:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gru_gpu.py tests/test_fused_gpu.py tests/test_config_size_gpu.py -k 'gru or gemm or Gru'" \
  "b4:::200:::python bench.py --model gru --no-cpu-baseline --steps 50" \
  "b4b:::200:::python bench.py --model gru --no-cpu-baseline --steps 50" \
  "b3:::200:::python bench.py --no-cpu-baseline --steps 50"
