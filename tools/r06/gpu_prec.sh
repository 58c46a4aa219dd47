#!/bin/bash
# Round 6: the staged split point per precision / config (same box): bf16 attention at config 2,
# config 5 (bf16, fp16 descriptors), fp32_split at config 2.
set -o pipefail
O=gpurun_out/r06prec
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
B16="--precision bf16 --steps 300 --warmup 5"
C5="--n1 2048 --n3 8192 --precision bf16 --desc-dtype fp16 --steps 100 --warmup 3"
SP="--precision fp32_split --steps 300 --warmup 5"
for i in 1 2; do
  for v in "s13:--staged-split 13" "s14:--staged-split 14" "s15:--staged-split 15" "base:--no-staged-inputs"; do
    n=${v%%:*}; a=${v#*:}
    one bf16_${n}_$i "$B16 $a"
    one c5_${n}_$i "$C5 $a"
  done
  one split_s13_$i "$SP"
  one split_base_$i "$SP --no-staged-inputs"
done
