#!/bin/bash
# Round 6: staged matcher inputs (the input stage on the pose stream) -- tests, then the same
# box's A/B of the bench line with and without it.
set -o pipefail
O=gpurun_out/r06staged
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pipeline_gpu.py tests/test_matcher_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for i in 1 2 3; do
  for v in staged base; do
    extra=""; [ $v = base ] && extra="--no-staged-inputs"
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $extra > $O/s20_${v}_$i.json 2> $O/s20_${v}_$i.err || exit 1
  done
done
for i in 1 2; do
  for v in staged base; do
    extra=""; [ $v = base ] && extra="--no-staged-inputs"
    timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline $extra > $O/s300_${v}_$i.json 2> $O/s300_${v}_$i.err || exit 1
  done
done
