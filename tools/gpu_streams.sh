#!/bin/bash
# Headline bench at 1..4 concurrent matcher streams (config 2, fp32), no CPU baseline.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in ${STREAMS:-1 2 3 4}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 --match-streams $s \
    > gpurun_out/streams_$s.json 2> gpurun_out/streams_$s.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/streams_$s.json').read().strip().splitlines()[-1]); print($s, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
done
