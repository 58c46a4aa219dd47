#!/bin/bash
# Round 6: staged matcher stages (the input stage and the forward's tail on the pose streams):
# tests, then the same box's A/B of the bench line over the variants in $VARS.
set -o pipefail
O=gpurun_out/r06staged
mkdir -p $O
VARS=${VARS:-"s13 base"}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pipeline_gpu.py tests/test_matcher_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
flags() {   # base: no staging; sN: the pose stream's part of the forward from stage N
  case $1 in
    base) echo "--no-staged-inputs" ;;
    s*) echo "--staged-split ${1#s}" ;;
    *) echo "" ;;
  esac
}
for i in 1 2 3; do
  for v in $VARS; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $(flags $v) > $O/s20_${v}_$i.json 2> $O/s20_${v}_$i.err || exit 1
  done
done
for i in 1 2; do
  for v in $VARS; do
    timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline $(flags $v) > $O/s300_${v}_$i.json 2> $O/s300_${v}_$i.err || exit 1
  done
done
