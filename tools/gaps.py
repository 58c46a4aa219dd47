"""Per-stream launch gaps of a rocprofv3 kernel trace (two-stream bench): for each kernel kind,
the mean time from the previous kernel's end on the same stream to this kernel's start, and its
mean duration, over the trace's last `frames` frames.  Shows what a dependent launch boundary
costs inside the frame (e.g. MLP conv 1 end -> MLP conv 2 start).
    python tools/gaps.py <kernel_trace.csv> [frames]"""
import csv
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    rd = csv.DictReader(f)
    cols = rd.fieldnames
    qcol = next((c for c in ("Stream_Id", "Queue_Id") if c in cols), None)
    for r in rd:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r[qcol] if qcol else "0"))
rows.sort()
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 40


def short(n):
    for k, v in (("gemm_kernel<1,", "qkv"), ("gemm_kernel<2,", "mlp1"), ("gemm_kernel<3,", "mlp2"),
                 ("gemm_kernel<4,", "score"), ("gemm_kernel<0,", "final"), ("gemm_kernel<5,", "acc")):
        if k in n:
            return v
    return n.split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").replace("_kernel", "")


score = [r for r in rows if short(r[2]) == "score"]
t0 = score[-frames - 1][1]
win = [r for r in rows if r[0] > t0]
by_q = defaultdict(list)
for r in win:
    by_q[r[3]].append(r)
gap = defaultdict(list)
dur = defaultdict(list)
pair = defaultdict(list)
for q, rs in by_q.items():
    for a, b in zip(rs, rs[1:]):
        g = b[0] - a[1]
        if g < 50000:   # same-stream dependency (ns); larger gaps are waits on the other streams
            gap[short(b[2])].append(g)
            pair[(short(a[2]), short(b[2]))].append(g)
    for r in rs:
        dur[short(r[2])].append(r[1] - r[0])
print(f"{'kernel':16s} {'n':>5s} {'dur us':>8s} {'gap before us':>14s}")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    g = gap.get(k, [])
    print(f"{k:16s} {len(dur[k]):5d} {sum(dur[k])/len(dur[k])/1e3:8.2f} "
          f"{(sum(g)/len(g)/1e3 if g else float('nan')):14.2f}")
print("\nmost common boundaries (mean gap us):")
for (a, b), g in sorted(pair.items(), key=lambda kv: -len(kv[1]))[:14]:
    print(f"  {a:>14s} -> {b:14s} {len(g):5d} {sum(g)/len(g)/1e3:7.2f}")
