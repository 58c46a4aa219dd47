#!/bin/bash
# The drop-in entry's throughput: inference(cfg) over a 64-frame on-disk sequence (tools/entry_bench.py).
set -u
O=gpurun_out/r05entry
mkdir -p $O
timeout -k 10 900 python -u tools/entry_bench.py --frames 64 --n3 4096 --out $O/entry.json > $O/entry.log 2>&1 || { tail -30 $O/entry.log; exit 1; }
tail -4 $O/entry.log
