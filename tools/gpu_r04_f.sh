#!/bin/bash
# (1) the phase probe's wide split / bf16 tiles (8-wave 128 x 128 MLP conv 1, 128 x 128 QKV);
# (2) the fp32 final projection: fused 32 x 256 (product) vs 8-wave 32 x 256 (lib_fw8, must be
#     bit-identical) vs unfused BIAS + l2norm (lib_fu), same-box A/B at config 2, two rounds.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 180 ./tools/phase_probe big > $O/phase_big.txt 2>&1 || { tail -5 $O/phase_big.txt; exit 1; }
grep -v "^ *phases" $O/phase_big.txt | cut -c1-150
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
ONEPOSE_LIB=$PWD/tools/ab/lib_fw8.so timeout -k 10 300 python tools/bitcmp.py dump $O/fw8.npz > $O/dump_fw8.log 2>&1 || { tail -20 $O/dump_fw8.log; exit 1; }
python tools/bitcmp.py cmp $O/new.npz $O/fw8.npz > $O/cmp_fw8.log 2>&1; tail -2 $O/cmp_fw8.log; rm -f $O/*.npz
for r in 1 2; do
  for v in P W U; do
    case $v in P) lib="";; W) lib=$PWD/tools/ab/lib_fw8.so;; U) lib=$PWD/tools/ab/lib_fu.so;; esac
    ONEPOSE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --warmup 5 > $O/c2_$v$r.json 2> $O/c2_$v$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/c2_$v$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('c2 $v$r', d['value'], {x: k.get(x) for x in ('final_gemm','l2norm','score_gemm','conf')})"
  done
done
