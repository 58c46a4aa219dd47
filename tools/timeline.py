"""Concurrency profile of a rocprofv3 kernel trace (two-stream bench): over the timed tail of
the trace, how much wall time has 0 / 1 / 2+ GEMM launches running, and what runs in the gaps.

    python tools/timeline.py gpurun_out/prof/<...>_kernel_trace.csv [frames]"""
import csv
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
# the tail: last `frames` score GEMM launches (one per frame) bound the window
score = [r for r in rows if "gemm_kernel<4" in r[2]]
t0, t1 = score[-frames - 1][1], score[-1][1]
win = [r for r in rows if r[1] > t0 and r[0] < t1]


def short(n):
    for k in ("gemm_kernel<1,", "gemm_kernel<2,", "gemm_kernel<3,", "gemm_kernel<4,", "gemm_kernel<0,"):
        if k in n:
            return {"gemm_kernel<1,": "qkv", "gemm_kernel<2,": "mlp1", "gemm_kernel<3,": "mlp2",
                    "gemm_kernel<4,": "score", "gemm_kernel<0,": "final"}[k]
    n = n.split("(")[0].split("::")[-1]
    return n.replace("_kernel", "")


ev = []
for s, e, n in win:
    s, e = max(s, t0), min(e, t1)
    g = short(n) in ("qkv", "mlp1", "mlp2", "score", "final")
    ev.append((s, 1, g, short(n)))
    ev.append((e, -1, g, short(n)))
ev.sort(key=lambda x: (x[0], x[1]))
acc = defaultdict(float)        # (ngemm, nother>0) -> ns
alone = defaultdict(float)      # kernel running with no GEMM -> ns
cur_g, cur_o = 0, defaultdict(int)
last = t0
for t, d, g, n in ev:
    dt = t - last
    if dt > 0:
        no = sum(1 for v in cur_o.values() if v > 0)
        acc[(min(cur_g, 2), no > 0)] += dt
        if cur_g == 0:
            for k, v in cur_o.items():
                if v > 0:
                    alone[k] += dt / max(no, 1)
    last = t
    if g:
        cur_g += d
    else:
        cur_o[n] += d
T = t1 - t0
print(f"window {T/1e3:.1f} us over {frames} frames: {T/1e3/frames:.1f} us/frame")
for k in sorted(acc):
    print(f"  gemms={k[0]} others={'y' if k[1] else 'n'}: {acc[k]/T*100:5.1f}%  ({acc[k]/1e3/frames:.1f} us/frame)")
print("non-GEMM kernels running while no GEMM runs (us/frame):")
for k, v in sorted(alone.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {k:20s} {v/1e3/frames:7.1f}")
