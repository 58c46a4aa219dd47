#!/bin/bash
# fp32 MFMA vs the fp32-accurate split mode on one box, alternated: the driver's 20-step line
# (three each) and the 500-step line (two each).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
line() {   # tag, args
  timeout -k 10 300 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'])"
}
for r in 1 2 3; do
  line f32_20_$r "--gpus 1 --steps 20 --warmup 5"
  line split_20_$r "--gpus 1 --steps 20 --warmup 5 --precision fp32_split"
done
for r in 1 2; do
  line f32_500_$r ""
  line split_500_$r "--precision fp32_split"
done
