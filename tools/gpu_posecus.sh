#!/bin/bash
# Pose stage on reserved CUs (the matchers on the rest) vs shared CUs, config 2 fp32,
# alternating: 300 steps, then the driver's 20 steps.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-posecus}
mkdir -p $O
run() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], k['mlp1_gemm'], d.get('pose', d.get('results', ''))) "
}
for i in 1 2; do
  run c0_$i "--steps 300 --warmup 5"
  run c1_$i "--steps 300 --warmup 5 --pose-cus 1"
  run c2_$i "--steps 300 --warmup 5 --pose-cus 2"
  run c8_$i "--steps 300 --warmup 5 --pose-cus 8"
done
for i in 1 2 3; do
  run s20_c0_$i "--steps 20 --warmup 5"
  run s20_c2_$i "--steps 20 --warmup 5 --pose-cus 2"
done
