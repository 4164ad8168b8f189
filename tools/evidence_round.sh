#!/bin/bash
# Per-round evidence on the GPU box (repo root), in two calls (each fits gpurun's limit):
#   bash tools/evidence_round.sh bench   -> the three bench lines (with CPU baselines) + rocprofv3
#                                         kernel traces / stats of short config 3 / 4 / 5 runs
#   bash tools/evidence_round.sh pmc     -> FETCH_SIZE / WRITE_SIZE passes (config 3 and 4 benches, the
#                                         env at 262 144 envs) and the env's SQ counters at 262 144
# Every step has its own time limit (tools/gpu_job.sh stops at the first crash or timeout); each
# --pmc pass is its own run with no trace domains.  Summaries: tools/evidence_summary.py.
export TMPDIR=/tmp
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--steps 10 --warmup 3 --no-cpu-baseline --env-micro 0 --no-seg-overhead"
if [ "$1" = bench ]; then
  bash tools/gpu_job.sh \
    "bench:::300:::python bench.py" \
    "bench_gru:::300:::python bench.py --model gru" \
    "bench_uam:::300:::python bench.py --model uam" \
    "prof3:::240:::$T --stats -d gpurun_out/prof3 -o run -- python3 bench.py $SHORT" \
    "prof4:::240:::$T --stats -d gpurun_out/prof4 -o run -- python3 bench.py --model gru $SHORT" \
    "prof5:::240:::$T --stats -d gpurun_out/prof5 -o run -- python3 bench.py --model uam $SHORT"
elif [ "$1" = pmc ]; then
  SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
  ENV="python3 tools/env_only.py --envs 262144 --steps 6"
  bash tools/gpu_job.sh \
    "f3:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pmc3f -o run -- python3 bench.py $SHORT" \
    "w3:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pmc3w -o run -- python3 bench.py $SHORT" \
    "f4:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pmc4f -o run -- python3 bench.py --model gru $SHORT" \
    "w4:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pmc4w -o run -- python3 bench.py --model gru $SHORT" \
    "fe:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pmcef -o run -- $ENV" \
    "we:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pmcew -o run -- $ENV" \
    "sq:::90:::timeout -s KILL 80 $T --pmc $SQ -d gpurun_out/pmcsq -o run -- $ENV" \
    "f5:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pmc5f -o run -- python3 bench.py --model uam $SHORT" \
    "w5:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pmc5w -o run -- python3 bench.py --model uam $SHORT" \
    "gt:::200:::python tools/gemm_table.py"
fi
