#!/bin/bash
# conf_kernel with tile-major column partials: bits against round 4, the GPU suite, conf's
# serial time and the frame rate.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05conf}
mkdir -p $O
R04=$PWD/tools/ab/lib_r04.so
B=$PWD/onepose_amd/libonepose_hip.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump r04 $R04
dump new $B
python tools/bitcmp.py cmp $O/r04.npz $O/new.npz > $O/cmp.log 2>&1
echo "r04 vs new: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['ms_per_step'], {x: k.get(x) for x in ('conf','score_gemm','mutual','kv_reduce','gat')})"
}
line n300_1 "--steps 300 --warmup 5"
line n300_2 "--steps 300 --warmup 5"
line c5 "--steps 100 --warmup 5 --precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
