#!/bin/bash
# probe build with phase stamps -> multi_agent_aac_amd/libaac_probe.so, then tools/attn_stamps.py
cd "$(dirname "$0")/../multi_agent_aac_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DAAC_ATTN_STAMPS --offload-arch=gfx950 \
  -I ../include -o libaac_probe.so csrc/aac_env.hip csrc/aac_learn.hip csrc/aac_fused.hip csrc/aac_gru.hip \
  csrc/aac_mpe.hip csrc/aac_uam.hip csrc/aac_uam_actor.hip csrc/aac_uam_learn.hip csrc/aac_host.cpp
