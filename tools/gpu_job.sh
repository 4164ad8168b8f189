#!/bin/bash
# Runs "label:::timeout:::command" steps in order on the GPU box, each under its own time limit.
# Continues only while every step exits 0 or 1 (pytest test failures); stops on any crash,
# abort, segfault or timeout (rc >= 2), so nothing more touches the GPU after a fault.
mkdir -p gpurun_out
for spec in "$@"; do
  label="${spec%%:::*}"; rest="${spec#*:::}"; tmo="${rest%%:::*}"; cmd="${rest#*:::}"
  echo "=== $label (timeout ${tmo}s): $cmd" >> gpurun_out/job.log
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== $label rc=$rc" >> gpurun_out/job.log
  tail -n 4 "gpurun_out/$label.log" >> gpurun_out/job.log
  if [ $rc -ge 2 ]; then echo "stopping after $label (rc=$rc)" >> gpurun_out/job.log; break; fi
done
cat gpurun_out/job.log
