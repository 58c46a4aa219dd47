#!/bin/bash
# Round 6: the split point again with the staged head 3 (same box).
set -o pipefail
O=gpurun_out/r06head3
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['pose']['cmd5'])"
}
C5="--n1 2048 --n3 8192 --precision bf16 --desc-dtype fp16 --steps 100 --warmup 3 --staged-head 3"
for i in 1 2; do
  for sp in 13 14 15; do
    one c5_s${sp}_$i "$C5 --staged-split $sp"
    one fp32_s${sp}_$i "--steps 300 --staged-head 3 --staged-split $sp"
  done
done
