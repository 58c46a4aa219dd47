#!/bin/bash
# Round 6: the ticketed finalize's partials written by device-scope atomic exchanges (XCHG) and read by atomic RMWs (RMW), and a release placed after the tickets (SLOW, its cost without the ordering)
# instead of write-through stores -- deviation counts under concurrency and the bench lines.
set -o pipefail
O=gpurun_out/r06rmw
mkdir -p $O
for v in base SLOW RMW; do
  echo "== $v"
  ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so RACE_N=50 timeout -k 10 400 python -u tools/r06/race_probe.py stress 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
for i in 1 2; do
  for v in base SLOW RMW; do
    ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline > $O/s300_${v}_$i.json 2>/dev/null || exit 1
    ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --steps 300 --precision fp32_split --no-cpu-baseline > $O/split_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json; a=json.loads(open('$O/s300_${v}_$i.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/split_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', a['value'], a['kernel_ms_per_step']['mlp1_gemm'], b['value'], b['kernel_ms_per_step']['mlp1_gemm'])"
  done
done
