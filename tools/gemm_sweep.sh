#!/bin/bash
# GEMM planner knob sweep over the learner's launches (tools/mb_launches.py); one process per
# setting since the knobs are read when libaac_env.so loads.  Run on the GPU box from the repo root.
set -e
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/mb_launches.py 50
done
