#!/bin/bash
# Build tools/ab/lib_<name>.so: the product library with extra compile flags (probe macros).
#   bash tools/build_variant.sh noct -DKVF_PROBE_NOCT
#   EXTRA="tools/experiments/gemm_bal.hip" bash tools/build_variant.sh bal -DONEPOSE_BAL
set -eu
name=$1; shift
out=tools/ab/var_$name; mkdir -p $out
objs=""
for s in onepose_amd/csrc/*.hip ${EXTRA:-}; do
  o=$out/$(basename $s).o
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function \
    -Wno-unused-variable -Ionepose_amd/csrc "$@" -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o tools/ab/lib_$name.so && rm -rf $out
echo tools/ab/lib_$name.so
