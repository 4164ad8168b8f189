#!/bin/bash
# Interleaved A/B of environment settings on one command: bash tools/ab_env.sh "<python args>" "K=V ..." "K=V ..."
# (3 rounds; each line: the settings, then the command's last JSON line cut to 300 chars)
CMD="$1"; shift
mkdir -p gpurun_out
for i in 1 2 3; do
  for kv in "$@"; do
    env $kv timeout -k 10 200 python $CMD > gpurun_out/abe.log 2>&1 || { tail -5 gpurun_out/abe.log; exit 1; }
    echo "[$kv] $(grep '^{' gpurun_out/abe.log | tail -1 | cut -c1-300)"
  done
done
