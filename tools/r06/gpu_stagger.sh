#!/bin/bash
# Round 6: the two match streams half a frame apart (--stagger-stage S: a frame's matcher starts
# once the previous frame's has reached stage S) against in step (S = 0), same box.
set -o pipefail
O=gpurun_out/r06stg
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  for st in ${STS:-0 5 7 9}; do
    one s300_st${st}_$i "--steps 300 --stagger-stage $st"
    one s20_st${st}_$i "--steps 20 --warmup 5 --stagger-stage $st"
  done
done
