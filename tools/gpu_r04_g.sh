#!/bin/bash
# The DMA loop's MFMAs kept above the stage wait (sched_barrier): bit-identity against the
# previous commit (tools/ab/lib_prev.so), the GPU suite, same-box A/B of the split / bf16 /
# config-5 lines, the phase probe's DMA cases; then the fp32 final-projection A/B (product
# 32 x 256 fused vs lib_fw8 8-wave vs lib_fu unfused).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
PREV=$PWD/tools/ab/lib_prev.so
ONEPOSE_LIB=$PREV timeout -k 10 300 python tools/bitcmp.py dump $O/prev.npz > $O/dump_prev.log 2>&1 || { tail -20 $O/dump_prev.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
rc=$?; tail -2 $O/cmp.log; rm -f $O/*.npz
[ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 ./tools/phase_probe dma > $O/phase_dma.txt 2>&1 || { tail -5 $O/phase_dma.txt; exit 1; }
grep -v "^ *phases" $O/phase_dma.txt | cut -c1-120
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','final_gemm','conf')})"
}
for r in 1 2; do
  line split_A$r $PREV "--precision fp32_split --steps 300 --warmup 5"
  line split_B$r "" "--precision fp32_split --steps 300 --warmup 5"
  line bf16_A$r $PREV "--precision bf16 --steps 300 --warmup 5"
  line bf16_B$r "" "--precision bf16 --steps 300 --warmup 5"
done
line c5_A $PREV "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
line c5_B "" "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
for r in 1 2; do
  line fin_P$r "" "--steps 300 --warmup 5"
  line fin_W$r $PWD/tools/ab/lib_fw8.so "--steps 300 --warmup 5"
  line fin_U$r $PWD/tools/ab/lib_fu.so "--steps 300 --warmup 5"
done
