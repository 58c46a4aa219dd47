#!/bin/bash
# bf16 MLP conv 2 on the DMA-1 loop (W planes by global_load_lds, A through registers with the
# norm + ReLU prologue) instead of the register-staged loop: bit-identity, then same-box A/B of
# the bf16 config-2 and config-5 lines (A = product, B = tools/ab/lib_m2d.so).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
V=$PWD/tools/ab/lib_m2d.so
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
ONEPOSE_LIB=$V timeout -k 10 300 python tools/bitcmp.py dump $O/v.npz > $O/dump_v.log 2>&1 || { tail -20 $O/dump_v.log; exit 1; }
python tools/bitcmp.py cmp $O/new.npz $O/v.npz > $O/cmp.log 2>&1; tail -2 $O/cmp.log; rm -f $O/*.npz
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
}
for r in 1 2; do
  line c2_A$r "" "--precision bf16 --steps 300 --warmup 5"
  line c2_B$r $V "--precision bf16 --steps 300 --warmup 5"
  line c5_A$r "" "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
  line c5_B$r $V "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
done
