#!/bin/bash
# What-if map of the frame: bench lines (pose stage off) with one kernel kind's launches
# skipped in a variant library (tools/build_variant.sh with -DONEPOSE_DIAG_SKIP=<kind mask>,
# a temporary, uncommitted OP_LAUNCH guard).  Results are not the metric: the skipped kernels'
# outputs are garbage; the line bounds what removing or fusing that kind could gain.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-diag}
mkdir -p $O
for v in ${VARIANTS:-base kvf l2smx confmut trgat mlp1 qkv mlp2 score base}; do
  ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 5 \
    --no-cpu-baseline --diag-no-pose ${BENCH_ARGS:-} > $O/$v.json 2> $O/$v.err || exit $?
  python -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
