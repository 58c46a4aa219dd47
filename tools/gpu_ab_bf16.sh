#!/bin/bash
# bf16 mode on the 64x128 DMA tiles: its matcher tests, then config 5 and config 2 in bf16.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bf16 or cache or prec" > gpurun_out/bf16b_tests.log 2>&1 || { tail -30 gpurun_out/bf16b_tests.log; exit 1; }
tail -1 gpurun_out/bf16b_tests.log
for a in "c5 --n1 2048 --n3 8192" "c2 --n1 1024 --n3 4096"; do
  set -- $a
  n=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --precision bf16 "$@" > gpurun_out/bf16_$n.json 2> gpurun_out/bf16_$n.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bf16_$n.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; r=d['roofline']; print('$n', d['value'], r['kernel'], r['avg_launch_us'], r['frac'], r['alone'], {x: k[x] for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
done
