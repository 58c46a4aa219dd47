#!/bin/bash
# Split mode on 64 x 128 QKV / MLP conv 1 tiles (tools/ab/lib_sw.so, -DONEPOSE_SPLIT_WIDE):
# the split parity tests on that build, then same-box A/B of the split line (A = the product
# build, B = lib_sw), two rounds, and one config-3 split line each.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04sw
mkdir -p $O
SW=$PWD/tools/ab/lib_sw.so
ONEPOSE_LIB=$SW timeout -k 10 400 python -u -m pytest tests/test_matcher_gpu.py tests/test_configs_gpu.py \
  -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/tests_sw.log 2>&1 \
  || { tail -30 $O/tests_sw.log; exit 1; }
tail -1 $O/tests_sw.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then lib=""; else lib=$SW; fi
    ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --precision fp32_split \
      --steps 300 --warmup 5 > $O/c2s_$v$r.json 2> $O/c2s_$v$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/c2s_$v$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('c2 split $v$r', d['value'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','score_gemm')})"
  done
done
for v in A B; do
  if [ $v = A ]; then lib=""; else lib=$SW; fi
  ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --precision fp32_split \
    --n3 16384 --batch 32 --steps 10 --warmup 2 > $O/c3s_$v.json 2> $O/c3s_$v.err || exit $?
  python -c "import json; d=json.loads(open('$O/c3s_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('c3 split $v', d['value'], {x: k.get(x) for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm')})"
done
timeout -k 10 180 ./tools/phase_probe dma > $O/phase_dma.txt 2>&1 || { tail -5 $O/phase_dma.txt; exit 1; }
grep -v "^ *phases" $O/phase_dma.txt | cut -c1-150
