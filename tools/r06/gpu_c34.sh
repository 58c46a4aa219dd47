#!/bin/bash
# Round 6: configs 3 and 4 (batch 32) on the staged schedule's variants (same box).
set -o pipefail
O=gpurun_out/r06c34
mkdir -p $O
one() {   # name, args
  timeout -k 10 300 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['pose']['cmd5'])"
}
C3="--n3 16384 --batch 32 --steps 10 --warmup 2"
C4="--n3 2500 --batch 32 --steps 20 --warmup 2"
for i in 1 2; do
  for v in "def:" "s15h1:--staged-split 15 --staged-head 1" "s13h1:--staged-head 1" "base:--no-staged-inputs"; do
    n=${v%%:*}; a=${v#*:}
    one c3_${n}_$i "$C3 $a"
    one c4_${n}_$i "$C4 $a"
  done
done
