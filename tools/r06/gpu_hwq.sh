#!/bin/bash
# Round 6: the single-process bench with HIP's default 4 hardware queues per process vs 8
# (the staged schedule runs 4 streams: the default stream, a second match stream, 2 pose streams).
set -o pipefail
O=gpurun_out/r06hwq
mkdir -p $O
one() {   # name, env, args
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || exit 1
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  one s20_q4_$i "" "--steps 20 --warmup 5"
  one s20_q8_$i "GPU_MAX_HW_QUEUES=8" "--steps 20 --warmup 5"
  one s300_q4_$i "" "--steps 300"
  one s300_q8_$i "GPU_MAX_HW_QUEUES=8" "--steps 300"
done
one base300_q8 "GPU_MAX_HW_QUEUES=8" "--steps 300 --no-staged-inputs"
one c5_q4 "" "--n1 2048 --n3 8192 --precision bf16 --desc-dtype fp16 --steps 100 --warmup 3"
one c5_q8 "GPU_MAX_HW_QUEUES=8" "--n1 2048 --n3 8192 --precision bf16 --desc-dtype fp16 --steps 100 --warmup 3"
one bf16_q4 "" "--precision bf16 --steps 300 --warmup 5"
one bf16_q8 "GPU_MAX_HW_QUEUES=8" "--precision bf16 --steps 300 --warmup 5"
