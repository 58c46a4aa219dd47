#!/bin/bash
# A/B/C... frames/s on one box: the current library (cur) and tools/ab/lib_<v>.so for v in
# $VARS, alternating, ROUNDS times.  TEST=1 first runs the matcher GPU tests on each variant.
#   VARS="q128 s128" ROUNDS=3 bash tools/ab_multi.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TEST:-0}" = 1 ]; then
  for v in ${VARS}; do
    ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 600 python -m pytest tests/test_matcher_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abm_test_$v.log 2>&1; rc=$?
    echo "test $v rc=$rc $(tail -1 gpurun_out/abm_test_$v.log)"; [ $rc -eq 0 ] || exit $rc
  done
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in cur ${VARS}; do
    if [ $v = cur ]; then lib=""; else lib=$PWD/tools/ab/lib_$v.so; fi
    ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 10 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abm_$v.json 2> gpurun_out/abm_$v.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/abm_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$v', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], {x: k.get(x) for x in ('qkv_gemm','mlp1_gemm','mlp2_gemm','kv_reduce','score_gemm','conf')})"
  done
done
