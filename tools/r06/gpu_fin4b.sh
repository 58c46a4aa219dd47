#!/bin/bash
# Round 6: the fp32 final projection + L2 on the 4-wave 32-deep tile (83 KB of LDS) against the
# 8-wave 64-deep tile (156 KB) now that it runs on the pose streams (same box, prebuilt libs).
set -o pipefail
O=gpurun_out/r06fin4b
mkdir -p $O
one() {   # name, lib, args
  ONEPOSE_LIB=$PWD/tools/ab/$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['pose']['cmd5'])"
}
for i in 1 2 3; do
  one s300_base_$i lib_base.so "--steps 300"
  one s300_fin4_$i lib_fin4.so "--steps 300"
  one s20_base_$i lib_base.so "--steps 20 --warmup 5"
  one s20_fin4_$i lib_fin4.so "--steps 20 --warmup 5"
done
