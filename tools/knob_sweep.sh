#!/bin/bash
# Bench step time under several environment-knob settings (one bench process each):
# bash tools/knob_sweep.sh "AAC_X=1 AAC_Y=2" "AAC_X=2" ... [-- bench args]
export TMPDIR=/tmp
cfgs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done; [ "$1" = "--" ] && shift
for c in "${cfgs[@]}"; do
  out=$(env $c timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --env-micro 0 "$@" 2>/dev/null | tail -1) || exit 1
  echo "$c :: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["ms_per_step"],4))')"
done
