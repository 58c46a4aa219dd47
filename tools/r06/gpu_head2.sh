#!/bin/bash
# Round 6: staged head 1 vs 3, more repetitions, and the other precisions (same box).
set -o pipefail
O=gpurun_out/r06head2
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['pose']['cmd5'])"
}
for i in 1 2 3 4; do
  for h in 1 3; do
    one s20_h${h}_$i "--steps 20 --warmup 5 --staged-head $h"
  done
done
for i in 1 2; do
  for h in 1 3; do
    one s300_h${h}_$i "--steps 300 --staged-head $h"
    one bf16_h${h}_$i "--precision bf16 --steps 300 --warmup 5 --staged-head $h"
    one split_h${h}_$i "--precision fp32_split --steps 300 --warmup 5 --staged-head $h"
    one c5_h${h}_$i "--n1 2048 --n3 8192 --precision bf16 --desc-dtype fp16 --steps 100 --warmup 3 --staged-head $h"
  done
done
