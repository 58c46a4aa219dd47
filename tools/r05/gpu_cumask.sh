#!/bin/bash
# Pose streams on their own CUs (hipExtStreamCreateWithCUMask): default against '8' (pose on 8
# CUs spread over the XCDs, matchers on the other 248) and '8p' (pose masked only), alternated.
# (The --diag-cu-mask bench flag this script used was removed after the measurement: DESIGN.md §8b.)
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05cumask}
mkdir -p $O
line() {   # tag, args
  timeout -k 10 200 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'])"
}
line m8_smoke "--steps 20 --warmup 5 --diag-cu-mask 8"
for r in 1 2; do
  line d20_$r "--steps 20 --warmup 5"
  line m8_20_$r "--steps 20 --warmup 5 --diag-cu-mask 8"
  line m8p_20_$r "--steps 20 --warmup 5 --diag-cu-mask 8p"
  line d300_$r "--steps 300 --warmup 5"
  line m8_300_$r "--steps 300 --warmup 5 --diag-cu-mask 8"
  line m8p_300_$r "--steps 300 --warmup 5 --diag-cu-mask 8p"
done
