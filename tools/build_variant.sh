#!/bin/bash
# Build tools/ab/lib_<name>.so: the product library with extra compile flags (probe macros).
#   bash tools/build_variant.sh noct -DKVF_PROBE_NOCT
set -eu
name=$1; shift
out=tools/ab/var_$name; mkdir -p $out
objs=""
for s in onepose_amd/csrc/*.hip; do
  o=$out/$(basename $s).o
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function \
    -Wno-unused-variable "$@" -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o tools/ab/lib_$name.so && rm -rf $out
echo tools/ab/lib_$name.so
