#!/bin/bash
# Configs 3 and 4 (batched) and config 5, short runs.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-cfg34}
mkdir -p $O
cfg() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err || return $?
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['kernel_ms_per_step'].get('mlp1_gemm'))"
}
cfg config3 --n3 16384 --batch 32 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
cfg config4 --n3 2500 --batch 32 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
cfg config3b --n3 16384 --batch 32 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
