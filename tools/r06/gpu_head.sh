#!/bin/bash
# Round 6: the staged head -- the forward's first layers run ahead on the pose stream with the
# input stage (--staged-head H: the match streams start at stage H), same box.
set -o pipefail
O=gpurun_out/r06head
mkdir -p $O
one() {   # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['pose']['cmd5'])"
}
for i in 1 2; do
  for h in ${HS:-1 3 4 5}; do
    one s300_h${h}_$i "--steps 300 --staged-head $h $EXTRA"
    one s20_h${h}_$i "--steps 20 --warmup 5 --staged-head $h $EXTRA"
  done
done
