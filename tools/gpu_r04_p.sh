#!/bin/bash
# Round-4 final build (two pose streams): the measurement set (tools/gpu_r04_final.sh) into
# gpurun_out/r04p, then three matcher / pose streams as extra lines (not the default).
set -u
export TMPDIR=/tmp
OUT=r04p bash tools/gpu_r04_final.sh || exit $?
O=gpurun_out/r04p
for s in 20 500; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --match-streams 3 --steps $s --warmup 5 > $O/ms3_$s.json 2> $O/ms3_$s.err || exit $?
  python -c "import json; d=json.loads(open('$O/ms3_$s.json').read().strip().splitlines()[-1]); print('3 streams, $s steps', d['value'], d['ms_per_step'])"
done
