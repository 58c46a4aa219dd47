"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc.sh) into HBM bytes
per launch for each kernel kind.  FETCH_SIZE is doubled (gfx950 tallies 128-B read requests
at 64 B: MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.  Counter values are
KB (rocprofv3 derived-counter unit)."""
import csv
import glob
import json
import os
import re
import sys

# GEMM template instance <EPI, PRO, BN> -> kernel kind (gemm.h enums; one instance per kind)
GEMM_KIND = {(1, 0, 32, 128): "qkv_gemm", (2, 2, 64, 64): "mlp1_gemm",
             (3, 1, 64, 64): "mlp2_gemm", (0, 0, 64, 64): "final_gemm",
             (4, 0, 64, 64): "score_gemm"}


def kind_of(name):
    m = re.search(r"gemm_f32_kernel<(\d+), (\d+), [^<]*Tile<(\d+), (\d+),", name)
    if m:
        return GEMM_KIND.get(tuple(int(x) for x in m.groups()), name)
    m = re.search(r"onepose::(?:\(anonymous namespace\)::)?(\w+?)(?:<|\(|$)", name)
    return m.group(1) if m else name


def load(root, counter):
    files = glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = kind_of(row["Kernel_Name"])
            per.setdefault(k, []).append(float(row["Counter_Value"]))
    return per


def main(root):
    fetch, write = load(root, "FETCH_SIZE"), load(root, "WRITE_SIZE")
    out = {"note": "bytes per launch; fetch = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; "
                   "counter unit KB", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        out["kernels"][k] = {"launches": max(len(f), len(w)), "fetch_bytes": fb,
                             "write_bytes": wb,
                             "hbm_bytes": (fb or 0) + (wb or 0) if fb is not None else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
