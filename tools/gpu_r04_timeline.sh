#!/bin/bash
# Kernel trace of the default two-stream bench: launch gaps per boundary (tools/gaps.py) and
# the concurrency profile (tools/timeline.py).
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-timeline}
mkdir -p $O/prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/gaps.py $f 40 > $O/gaps.txt 2>&1; cat $O/gaps.txt
python tools/timeline.py $f 40 > $O/timeline.txt 2>&1; cat $O/timeline.txt
s=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $s $O/kernel_stats.csv
gzip -c $f > $O/kernel_trace.csv.gz
