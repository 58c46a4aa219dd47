#!/bin/bash
# BASELINE configs beside the headline: config 3 (1024 x 16384, 32 frames per step) and the
# config-4 per-GPU shard (1024 x 2500, 32 frames per GPU), fp32; config 5 shape in bf16.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/configs
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err
  local rc=$?
  echo "$name rc=$rc"; tail -c 600 gpurun_out/configs/$name.json; echo
  return $rc
}
run config3 --n3 16384 --batch 32 --steps 10 --warmup 2 --no-cpu-baseline &&
run config4 --n3 2500 --batch 32 --steps 10 --warmup 2 --no-cpu-baseline &&
run config5_bf16 --n1 2048 --n3 8192 --precision bf16 --steps 30 --warmup 3 --no-cpu-baseline
