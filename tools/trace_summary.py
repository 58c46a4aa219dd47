"""Per-kernel summary of a rocprofv3 kernel-trace CSV, grouped by kernel name and grid.

    python tools/trace_summary.py gpurun_out/spprof/sp_kernel_trace.csv [filter]"""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        if len(sys.argv) > 2 and sys.argv[2] not in name:
            continue
        key = (name, r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", ""))
        rows[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = sorted(rows.items(), key=lambda kv: -sum(kv[1]))
for (name, g, wg), d in out[:40]:
    print(f"{len(d):5d} {sum(d)/len(d)/1000:9.2f}us tot {sum(d)/1e6:8.2f}ms grid {g:>8} wg {wg:>4} {name[:100]}")
