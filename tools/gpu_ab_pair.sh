#!/bin/bash
# GPU suite on the in-tree library, then an alternating A/B of two prebuilt libraries
# (tools/ab/lib_$A.so vs lib_$B.so, loaded through ONEPOSE_LIB) on the default line and on the
# harness's 20-step line, ROUNDS rounds each.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-abpair}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-$A $B}; do
    for s in ${STEPLIST:-300 20}; do
      ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --steps $s --warmup 5 \
        --no-cpu-baseline ${BENCH_ARGS:-} > $O/${v}_s${s}_$r.json 2> $O/${v}_s${s}_$r.err || exit $?
      python -c "import json; d=json.loads(open('$O/${v}_s${s}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$v s$s r$r', d['value'], d['ms_per_step'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','kv_reduce')})"
    done
  done
done
