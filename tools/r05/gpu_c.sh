#!/bin/bash
# The GPU suite on the product build, then the drop-in entry's throughput.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u tools/entry_bench.py --frames 64 --n3 4096 --out $O/entry.json > $O/entry.log 2>&1 || { tail -30 $O/entry.log; exit 1; }
grep -E "^(superpoint|detections)" $O/entry.log
python3 -c "import json; d=json.load(open('$O/entry.json')); print(json.dumps(d['breakdown_ms_per_frame'], indent=1)); print(json.dumps(d['per_call_ms'], indent=1))"
