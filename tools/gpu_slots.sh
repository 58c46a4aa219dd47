#!/bin/bash
# Frame rate against the number of buffer slots (slot reuse waits on the slot's previous pose
# stage), two rounds on one box, with stage marks for the per-stream idle time.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for sl in 3 4 6; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --slots $sl --stage-marks \
      > gpurun_out/slots$sl.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/slots$sl.json').read().strip().splitlines()[-1]); s=d['stage_ms']; print('slots $sl', d['value'], s['stream_gap_mean'], s['stream_gap_max'], s['pose_mean'], s['matcher_mean'])"
  done
done
