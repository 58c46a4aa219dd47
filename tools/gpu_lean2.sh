#!/bin/bash
# Full GPU suite, then config 2 fp32 (x2), config 2 bf16 and config 5 bf16 benches.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-lean2}
mkdir -p $O
timeout -k 10 150 ./tools/phase_probe > $O/probe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {   # name, args
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline $2 > $O/ab_$1.json 2> $O/ab_$1.err || exit $?
  python -c "import json; d=json.loads(open('$O/ab_$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$1', d['value'], d['roofline']['avg_launch_us'], d['roofline']['alone']['avg_launch_us'], {x: k[x] for x in ('mlp1_gemm','qkv_gemm','mlp2_gemm','kv_reduce')})"
}
run fp32 "--precision fp32"
run c2_bf16 "--precision bf16"
run fp32b "--precision fp32"
run c5_bf16 "--precision bf16 --n1 2048 --n3 8192 --steps 100"
