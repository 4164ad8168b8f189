#!/bin/bash
# Evidence run on the GPU box (from the repo root): the GPU test suite, the default bench line
# (with the CPU baseline), a rocprofv3 kernel-trace/stats pass of a short bench and two separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of the GEMM and env-step kernels.
# Every GPU step runs under its own time limit through tools/gpu_job.sh, which stops at the
# first crash or timeout.  Outputs land in gpurun_out/; copy what is judged into profiles/.
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --output-format csv"
SHORT="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
bash tools/gpu_job.sh \
  "pytest:::900:::python -m pytest tests -m gpu -q" \
  "bench:::600:::python bench.py" \
  "stats:::600:::$P --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --env-micro 0" \
  "fetch:::600:::$P --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- $SHORT" \
  "write:::600:::$P --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- $SHORT"
