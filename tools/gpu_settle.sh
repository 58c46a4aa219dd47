#!/bin/bash
# The harness's 20-step line against the number of untimed settle steps before it (the clock
# leaves its idle state under sustained work), alternating, 3 rounds.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-settle}
mkdir -p $O
for r in 1 2 3; do
  for n in ${SETTLE_LIST:-60 150 400}; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --settle-steps $n > $O/n${n}_$r.json 2> $O/n${n}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/n${n}_$r.json').read().strip().splitlines()[-1]); print('settle $n r$r', d['value'], d['ms_per_step'])"
  done
done
