#!/bin/bash
# Times the env step kernel with the radar phase or the agent (obs + ss_reward) phase compiled
# out, to find the workgroup's critical path.  Run on the GPU box from the repo root.
set -e
mkdir -p gpurun_out/probe
for v in SKIP_RADAR SKIP_AGENT; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 -I include \
    -DAAC_DBG_$v -o gpurun_out/probe/lib_$v.so multi_agent_aac_amd/csrc/aac_env.hip \
    multi_agent_aac_amd/csrc/aac_learn.hip multi_agent_aac_amd/csrc/aac_fused.hip multi_agent_aac_amd/csrc/aac_host.cpp
done
for v in full SKIP_RADAR SKIP_AGENT; do
  if [ $v = full ]; then lib=""; else lib=$PWD/gpurun_out/probe/lib_$v.so; fi
  for r in drones obstacles combined; do
    echo "$v $(AAC_LIB=$lib timeout -k 10 120 python tools/env_only.py --envs 4096 --radar $r --steps 20)"
  done
done
