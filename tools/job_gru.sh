# config-4 GRU weights-stationary kernel: tests, then the bench with the projection mode off / on,
# then a kernel trace of a short run
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "gt:::300:::python -u -m pytest tests/test_gru_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "b4:::150:::python bench.py --model gru --no-cpu-baseline --env-micro 0" \
  "b4p:::150:::AAC_GRU_WS_PROJ=1 python bench.py --model gru --no-cpu-baseline --env-micro 0" \
  "prof4:::240:::rocprofv3 --kernel-trace --output-format csv --stats -d gpurun_out/prof4 -o run -- python3 bench.py --model gru --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
