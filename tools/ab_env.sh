#!/bin/bash
# A/B of one environment knob on the GPU box: bench line + kernel stats with "$1" (a) and "$2" (b)
# exported, e.g. bash tools/ab_env.sh AAC_ATTN_MFMA=0 AAC_ATTN_MFMA=1 [bench args...]
export TMPDIR=/tmp
A=$1; B=$2; shift 2
for tag in a b; do
  kv=$A; [ $tag = b ] && kv=$B
  env "$kv" timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --env-micro 0 "$@" > gpurun_out/ab_$tag.json 2>/dev/null || exit 1
  export "$kv"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_prof_$tag -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0 "$@" > /dev/null 2>&1 || exit 1
done
