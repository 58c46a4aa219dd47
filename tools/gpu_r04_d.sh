#!/bin/bash
# conf with the softmax statistics fused: bit identity against the round-start build, the GPU
# test suite, same-box fp32 A/B (300 steps) and the driver's 20-step line.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04d}
mkdir -p $O
ONEPOSE_LIB=$PWD/tools/ab/lib_base.so timeout -k 10 300 python tools/bitcmp.py dump $O/base.npz > $O/dump_base.log 2>&1 || { tail -20 $O/dump_base.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/base.npz $O/new.npz > $O/cmp.log 2>&1; tail -3 $O/cmp.log
rm -f $O/base.npz $O/new.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then lib=$PWD/tools/ab/lib_base.so; else lib=""; fi
    ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --warmup 5 > $O/c2_$v$r.json 2> $O/c2_$v$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/c2_$v$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('c2 $v$r', d['value'], d['roofline']['frac'], {x: k.get(x) for x in ('conf','softmax_reduce','mutual','final_gemm','l2norm','mlp1_gemm')})"
  done
done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20.json 2> $O/bench_20.err || exit $?
python -c "import json; d=json.loads(open('$O/bench_20.json').read().strip().splitlines()[-1]); print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
# bf16 MLP conv 1 on 64 x 64 DMA-2 tiles (tools/ab/lib_bf64.so) vs the 64 x 128 default
for r in 1 2; do
  for v in D V; do
    if [ $v = V ]; then lib=$PWD/tools/ab/lib_bf64.so; else lib=""; fi
    for cfg in c2 c5; do
      if [ $cfg = c5 ]; then A="--n1 2048 --n3 8192"; else A=""; fi
      ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 --steps 200 --warmup 5 $A > $O/bf_${cfg}_$v$r.json 2> $O/bf_${cfg}_$v$r.err || exit $?
      python -c "import json; d=json.loads(open('$O/bf_${cfg}_$v$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('bf16 $cfg $v$r', d['value'], d['roofline']['frac'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
    done
  done
done
