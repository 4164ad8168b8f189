#!/bin/bash
# A variant of libaac_env.so with one source rebuilt under extra flags, for A/B and stamp runs:
#   bash tools/variant_lib.sh NAME SRC [hipcc flags ...]   ->  tools/vlib/lib_NAME.so
# (e.g. bash tools/variant_lib.sh astamps aac_env.hip -DAAC_ENV_STAMPS -DAAC_ENV_AGENT_STAMPS; then
# AAC_LIB=tools/vlib/lib_astamps.so python tools/agent_stamps.py 4096 8 wgru).  The other objects come
# from build/obj (python -m multi_agent_aac_amd.build first).
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/.."
mkdir -p tools/vlib build/obj/var
objs=""
for o in build/obj/*.o; do
  [ "$(basename "$o" .o)" = "$src" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function --offload-arch=gfx950 "$@" \
  -I include -c -o "build/obj/var/$src.$name.o" "multi_agent_aac_amd/csrc/$src"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "tools/vlib/lib_$name.so" $objs "build/obj/var/$src.$name.o" \
  -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "tools/vlib/lib_$name.so"
