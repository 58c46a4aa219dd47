#!/bin/bash
# Matcher-stream priority A/B (--match-priority -1: the second matcher stream, i.e. every odd
# frame, at high priority), alternating, on the 20-step and 300-step lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-matchprio}
mkdir -p $O
for r in 1 2 3; do
  for p in 0 -1; do
    for s in 20 300; do
      timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline --match-priority $p > $O/p${p}_s${s}_$r.json 2> $O/p${p}_s${s}_$r.err || exit $?
      python -c "import json; d=json.loads(open('$O/p${p}_s${s}_$r.json').read().strip().splitlines()[-1]); print('prio $p s$s r$r', d['value'], d['ms_per_step'])"
    done
  done
done
