#!/bin/bash
# Round 6: kv_fold with 1 / 2 / 4 quarters of C loaded ahead of the chunk sum (prebuilt in
# tools/ab/) against the committed build: outputs bit for bit, then bench lines.
set -o pipefail
O=gpurun_out/r06kvf
mkdir -p $O
for v in base c1 c2 c4; do
  ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python tools/r06/kvf_dump.py $O/$v.npz 2>&1 | grep -v amdgpu.ids || exit 1
done
python - <<'PY' || exit 1
import numpy as np
O = "gpurun_out/r06kvf"
b = np.load(f"{O}/base.npz")
for v in ("c1", "c2", "c4"):
    x = np.load(f"{O}/{v}.npz")
    bad = [k for k in b.files if not np.array_equal(b[k], x[k])]
    print(v, "differs from base in", bad or "nothing")
PY
for i in 1 2; do
  for v in base c1 c2 c4; do
    ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline > $O/s300_${v}_$i.json 2>/dev/null || exit 1
    ONEPOSE_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --steps 300 --precision fp32_split --no-cpu-baseline > $O/split_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json; a=json.loads(open('$O/s300_${v}_$i.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/split_${v}_$i.json').read().strip().splitlines()[-1]); k=a['kernel_ms_per_step']; print('$v', a['value'], k.get('kv_reduce'), k['mlp1_gemm'], b['value'], b['kernel_ms_per_step'].get('kv_reduce'))"
  done
done
