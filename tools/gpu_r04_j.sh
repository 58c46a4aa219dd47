#!/bin/bash
# bf16 DMA-2 loop with 4 / 5 LDS buffers (three / four stages of loads in flight) against the
# product's 3: bit-identity of lib_nb4, then same-box A/B of the bf16 config-2 and config-5 lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
ONEPOSE_LIB=$PWD/tools/ab/lib_nb4.so timeout -k 10 300 python tools/bitcmp.py dump $O/nb4.npz > $O/dump_nb4.log 2>&1 || { tail -20 $O/dump_nb4.log; exit 1; }
python tools/bitcmp.py cmp $O/new.npz $O/nb4.npz > $O/cmp_nb4.log 2>&1
rc=$?; tail -2 $O/cmp_nb4.log; rm -f $O/*.npz
[ $rc -ne 0 ] && exit 1
line() {   # tag, lib, args
  ONEPOSE_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['roofline']['avg_launch_us'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
}
for r in 1 2; do
  for v in 3 4 5; do
    if [ $v = 3 ]; then lib=""; else lib=$PWD/tools/ab/lib_nb$v.so; fi
    line c2_nb$v.$r "$lib" "--precision bf16 --steps 300 --warmup 5"
    line c5_nb$v.$r "$lib" "--n1 2048 --n3 8192 --precision bf16 --steps 100 --warmup 3"
  done
done
