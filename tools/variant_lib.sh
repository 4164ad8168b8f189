#!/bin/bash
# Build a variant of libaac_env.so with extra defines on one source (the others from build/obj):
#   bash tools/variant_lib.sh <tag> <source.hip> [-DFOO ...]   ->  tools/variants/lib_<tag>.so
# (run in this container after python -m multi_agent_aac_amd.build; load on the box with AAC_LIB=...)
set -e
tag=$1; src=$2; shift 2
out=tools/variants
mkdir -p $out
base=$(basename $src)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I include "$@" -c \
  multi_agent_aac_amd/csrc/$base -o $out/$tag.$base.o
objs=""
for o in build/obj/*.o; do
  if [ "$(basename $o)" = "$base.o" ]; then objs="$objs $out/$tag.$base.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/lib_$tag.so $objs -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo $out/lib_$tag.so
