#!/bin/bash
# Lean DMA loop (bf16 / split modes): phase probe, the bf16-mode and split-mode parity tests, then
# config 2 fp32 vs fp32_split (alternating) and config 5 bf16.
set -u
export TMPDIR=/tmp
O=gpurun_out/lean
mkdir -p $O
timeout -k 10 150 ./tools/phase_probe > $O/probe.txt 2>&1 || exit $?
echo probe ok
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or bf16 or fixture or cache or tables or prec or config" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {   # name, args
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline $2 > $O/ab_$1.json 2> $O/ab_$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/ab_$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['roofline']['avg_launch_us'], d['roofline']['alone']['avg_launch_us'], {x: k[x] for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
}
run fp32 "--precision fp32"
run split "--precision fp32_split"
run fp32b "--precision fp32"
run splitb "--precision fp32_split"
run c2_bf16 "--precision bf16"
run c5_bf16 "--precision bf16 --n1 2048 --n3 8192 --steps 100"
