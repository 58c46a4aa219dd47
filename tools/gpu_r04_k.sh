#!/bin/bash
# End-of-session check of the committed tree: bit-identity against tools/ab/lib_prev.so, the GPU
# suite, smoke(), and the driver's 20-step bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
PREV=$PWD/tools/ab/lib_prev.so
ONEPOSE_LIB=$PREV timeout -k 10 300 python tools/bitcmp.py dump $O/prev.npz > $O/dump_prev.log 2>&1 || { tail -20 $O/dump_prev.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
rc=$?; tail -2 $O/cmp.log; rm -f $O/*.npz
[ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
