#!/bin/bash
# Two pose streams (frame k's pose stage on stream k % 2): the pipeline GPU tests, then the
# driver's 20-step line and the 500-step line with one pose stream (A) and two (B), alternated.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() {   # tag, args
  timeout -k 10 300 python bench.py --no-cpu-baseline $2 > $O/$1.json 2> $O/$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config']['workload'][:0])"
}
for r in 1 2 3; do
  line s20_A$r "--gpus 1 --steps 20 --warmup 5 --pose-streams 1"
  line s20_B$r "--gpus 1 --steps 20 --warmup 5"
done
line s500_A "--pose-streams 1"
line s500_B ""
