#!/bin/bash
# Times the learner's GEMM launches (tools/mb_launches.py) with parts of the kernel compiled out
# (epilogue stores, operand loads, both, or the whole body = launch floor), to see what bounds the
# grouped GEMM.  Run on the GPU box from the repo root.
set -e
mkdir -p gpurun_out/probe
for v in "NO_STORE" "NO_LOAD" "NO_LOAD -DAAC_DBG_NO_STORE" "EMPTY"; do
  tag=$(echo $v | tr -d ' -')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 -I include \
    -DAAC_DBG_$v -o gpurun_out/probe/lib_$tag.so multi_agent_aac_amd/csrc/aac_env.hip \
    multi_agent_aac_amd/csrc/aac_learn.hip multi_agent_aac_amd/csrc/aac_fused.hip multi_agent_aac_amd/csrc/aac_host.cpp
done
for v in full NO_STORE NO_LOAD NO_LOADDAAC_DBG_NO_STORE EMPTY; do
  if [ $v = full ]; then lib=""; else lib=$PWD/gpurun_out/probe/lib_$v.so; fi
  echo "== $v"
  AAC_LIB=$lib timeout -k 10 120 python tools/mb_launches.py 50
done
