#!/bin/bash
# bf16 DMA-2 loop two stages ahead (3 LDS buffers): bit identity against the round-start build,
# then same-box A/B (round-start build A vs this build B) of the bf16 lines (configs 2 and 5).
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-la2}
mkdir -p $O
ONEPOSE_LIB=$PWD/tools/ab/lib_base.so timeout -k 10 300 python tools/bitcmp.py dump $O/base.npz > $O/dump_base.log 2>&1 || { tail -20 $O/dump_base.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/base.npz $O/new.npz > $O/cmp.log 2>&1; tail -3 $O/cmp.log
rm -f $O/base.npz $O/new.npz
ab() {   # name, bench args
  for r in 1 2; do
    for v in A B; do
      if [ $v = A ]; then lib=$PWD/tools/ab/lib_base.so; else lib=""; fi
      ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1_$v$r.json 2> $O/$1_$v$r.err || exit $?
      python -c "import json; d=json.loads(open('$O/$1_$v$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1 $v$r', d['value'], d['roofline']['frac'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
    done
  done
}
ab c2bf16 "--precision bf16 --steps 200 --warmup 5"
ab c5bf16 "--precision bf16 --n1 2048 --n3 8192 --steps 200 --warmup 5"
ab c2split "--precision fp32_split --steps 200 --warmup 5"
