#!/bin/bash
# Pose kernels compiled for 2 / 4 waves per SIMD (ONEPOSE_PNP_WPE; fewer registers, more
# spills) vs 1: the pose GPU tests on each variant, then config 2 frames/s alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pnpwpe}
mkdir -p $O
for v in w2 w4; do
  ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 400 python -m pytest tests/test_pnp_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -20 $O/test_$v.log; exit 1; }
  echo "test $v: $(tail -1 $O/test_$v.log)"
done
run() {   # name, lib, args
  if [ $2 = cur ]; then lib=""; else lib=$PWD/tools/ab/lib_$2.so; fi
  ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], k['pnp_ransac'], k['pnp_refit'])"
}
for i in 1 2; do
  for v in cur w2 w4; do run ${v}_$i $v "--steps 300 --warmup 5"; done
done
for i in 1 2 3; do
  for v in cur w2 w4; do run s20_${v}_$i $v "--steps 20 --warmup 5"; done
done
