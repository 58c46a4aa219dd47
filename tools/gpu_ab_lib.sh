#!/bin/bash
# A/B of two prebuilt libraries on one box: onepose_amd/libonepose_hip_a.so vs _b.so, swapped in
# as libonepose_hip.so between bench processes, alternating, on config 2 fp32 and config 3.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-ablib}
mkdir -p $O
L=onepose_amd/libonepose_hip.so
run() {   # name, lib, args
  cp onepose_amd/libonepose_hip_$2.so $L
  timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], {x: k[x] for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','score_gemm')})"
}
for i in 1 2; do
  run c2_a$i a "--steps 300 --warmup 5"
  run c2_b$i b "--steps 300 --warmup 5"
done
for i in 1 2; do
  run c3_a$i a "--n3 16384 --batch 32 --steps 10 --warmup 2"
  run c3_b$i b "--n3 16384 --batch 32 --steps 10 --warmup 2"
done
cp onepose_amd/libonepose_hip_b.so $L
