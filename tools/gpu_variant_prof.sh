#!/bin/bash
# rocprof kernel stats of the bench with each library variant in tools/ab (VARS="noct nochunk").
set -u
export TMPDIR=/tmp
for v in base ${VARS:-}; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/ab/lib_$v.so; fi
  rm -rf gpurun_out/var_$v; mkdir -p gpurun_out/var_$v
  ONEPOSE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/var_$v -o run -- \
    python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/var_$v/bench.json 2> gpurun_out/var_$v/bench.err || exit $?
  python3 - $v <<'PY'
import csv, sys, glob
v = sys.argv[1]
f = glob.glob(f"gpurun_out/var_{v}/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("kv_fold", "gat_kernel", "gemm_kernel<1", "conf_kernel", "softmax_reduce", "mutual", "l2norm", "pose_error")):
        out.append(f"{n.split('(')[0][-22:]} {float(r['AverageNs'])/1e3:.2f}")
print(v, "|", "; ".join(out))
PY
done
