#!/bin/bash
# Balanced fp32 MLP conv 1 (gemm_bal.hip): bit identity against the round-4 build and the same
# tree without it, the GPU suite, then same-box frame rates against lib_nobal.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05bal}
mkdir -p $O
R04=$PWD/tools/ab/lib_r04.so
NOBAL=$PWD/onepose_amd/libonepose_hip.so
BAL=$PWD/tools/ab/lib_bal.so
timeout -k 10 120 ./tools/bal_probe > $O/bal_probe.txt 2>&1 || { cat $O/bal_probe.txt; exit 1; }
tail -1 $O/bal_probe.txt
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; exit 1; }; }
dump r04 $R04
dump nobal $NOBAL
dump new $BAL
[ -n "${MIN2:-}" ] && dump min2 $PWD/tools/ab/lib_balmin2.so
for pair in "r04 nobal" "nobal new" "r04 new" ${MIN2:+"nobal min2"}; do
  set -- $pair
  python tools/bitcmp.py cmp $O/$1.npz $O/$2.npz > $O/cmp_$1_$2.log 2>&1
  echo "$1 vs $2: $(tail -1 $O/cmp_$1_$2.log)"
done
rm -f $O/*.npz
[ -n "${CMP_ONLY:-}" ] && exit 0
if [ -z "${SKIP_TESTS:-}" ]; then
  ONEPOSE_LIB=$BAL timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$1', d['value'], r['kernel'], r['avg_launch_us'], r['frac'], r['alone']['avg_launch_us'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
}
for r in 1 2; do
  line n20_A$r $NOBAL "--steps 20 --warmup 5"
  line n20_B$r $BAL "--steps 20 --warmup 5"
done
for r in 1 2; do
  line n300_A$r $NOBAL "--steps 300 --warmup 5"
  line n300_B$r $BAL "--steps 300 --warmup 5"
done
line f0_B $BAL "--steps 300 --warmup 5 --frames 0"
