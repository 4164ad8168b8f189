#!/bin/bash
# Interleaved A/B of library builds on one command: bash tools/ab_libs.sh "<python args>" libA.so libB.so ...
# (3 rounds; each line: lib, ms per step / the command's JSON summary)
CMD="$1"; shift
mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in "$@"; do
    AAC_LIB=$PWD/$lib timeout -k 10 200 python $CMD > gpurun_out/abl.log 2>&1 || { tail -5 gpurun_out/abl.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/abl.log | tail -1 | cut -c1-400)" | tee -a gpurun_out/abl.txt
  done
done
