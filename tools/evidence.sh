#!/bin/bash
# Round evidence on the GPU box (repo root): full GPU test suite, the three bench lines (config 3
# default, config 4 GRU, config 5 UAM; each with its CPU baseline) and rocprofv3 kernel stats of
# short config-3 and config-5 runs.  Every step runs under its own time limit (tools/gpu_job.sh
# stops at the first crash or timeout).  Copy what is judged from gpurun_out/ into profiles/.
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
bash tools/gpu_job.sh \
  "pytest:::600:::python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
  "bench:::300:::python bench.py" \
  "bench_gru:::300:::python bench.py --model gru" \
  "bench_uam:::300:::python bench.py --model uam" \
  "stats:::300:::$P -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --env-micro 0" \
  "stats_uam:::300:::$P -d gpurun_out/prof_uam -o run -- python3 bench.py --model uam --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
