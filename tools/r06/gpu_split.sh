#!/bin/bash
# Round 6: the staged split point for the fp32-accurate split mode (same box, 300 steps).
set -o pipefail
O=gpurun_out/r06split
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
SP="--precision fp32_split --steps 300 --warmup 5"
for i in 1 2; do
  for v in "s13:--staged-split 13" "s14:--staged-split 14" "s15:--staged-split 15" "s12:--staged-split 12" "base:--no-staged-inputs"; do
    n=${v%%:*}; a=${v#*:}
    one split_${n}_$i "$SP $a"
  done
done
