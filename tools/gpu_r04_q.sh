#!/bin/bash
# Last check of the committed tree: smoke() and the driver's default bench command.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_source'], d['cpu_baseline']['value'])"
