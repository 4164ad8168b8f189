#!/bin/bash
# A/B of two builds of libaac_env.so on the GPU box: bench line + kernel stats for each.
# usage: bash tools/ab_lib.sh <lib_a> <lib_b> [bench args...]
export TMPDIR=/tmp
A=$1; B=$2; shift 2
for tag in a b; do
  lib=$A; [ $tag = b ] && lib=$B
  AAC_LIB=$PWD/$lib timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --env-micro 0 "$@" > gpurun_out/ab_$tag.json 2>/dev/null || exit 1
  AAC_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_prof_$tag -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0 "$@" > /dev/null 2>&1 || exit 1
done
