#!/bin/bash
# The next self layer's 2D QKV forked beside each GAT (a parallel branch of the frame's graph):
# bit comparison against the build without the fork (tools/ab/lib_nofork.so), the GPU suite,
# same-box lines A = no fork, B = fork, and the two-stream kernel trace of B.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05fork}
mkdir -p $O
A=$PWD/tools/ab/lib_nofork.so
B=$PWD/onepose_amd/libonepose_hip.so
dump() { ONEPOSE_LIB=$2 timeout -k 10 300 python tools/bitcmp.py dump $O/$1.npz > $O/dump_$1.log 2>&1 || { tail -20 $O/dump_$1.log; rm -f $O/*.npz; exit 1; }; }
dump nofork $A
dump fork $B
python tools/bitcmp.py cmp $O/nofork.npz $O/fork.npz > $O/cmp.log 2>&1
echo "nofork vs fork: $(tail -1 $O/cmp.log)"
rm -f $O/*.npz
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['ms_per_step'], {x: k.get(x) for x in ('qkv_gemm','gat','kv_reduce')})"
}
for r in 1 2; do
  line n20_A$r $A "--steps 20 --warmup 5"
  line n20_B$r $B "--steps 20 --warmup 5"
  line n300_A$r $A "--steps 300 --warmup 5"
  line n300_B$r $B "--steps 300 --warmup 5"
done
line sp_A $A "--steps 300 --warmup 5 --precision fp32_split"
line sp_B $B "--steps 300 --warmup 5 --precision fp32_split"
line c5_A $A "--steps 100 --warmup 5 --precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
line c5_B $B "--steps 100 --warmup 5 --precision bf16 --desc-dtype fp16 --n1 2048 --n3 8192"
mkdir -p $O/prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err || exit $?
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/timeline.py $f 40 > $O/timeline.txt 2>&1; cat $O/timeline.txt
gzip $f
