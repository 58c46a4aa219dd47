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
GEMM_KIND = {(1, 0): "qkv_gemm", (2, 2): "mlp1_gemm", (3, 1): "mlp2_gemm", (0, 0): "final_gemm",
             (6, 0): "final_gemm", (4, 0): "score_gemm"}


def kind_of(name):
    m = re.search(r"gemm_(?:f32_)?kernel<(\d+), (\d+), [^<]*Tile<[^>]*>(?:, (true|false|\d))?", name)
    if m:   # operand mode: bool (older builds) or GemmPm 0 / 1 (bf16) / 2 (split3)
        k = GEMM_KIND.get((int(m.group(1)), int(m.group(2))), name)
        return k + {"true": "_bf16", "1": "_bf16", "2": "_split3"}.get(m.group(3) or "", "")
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


SQ = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
      "SQ_ACTIVE_INST_ANY", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]


def load_all(root):
    """{kind: {counter: [per-dispatch values]}} plus kernel durations (ns) from the trace."""
    per, dur = {}, {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = kind_of(row["Kernel_Name"])
            d = per.setdefault(k, {}).setdefault(row["Counter_Name"], {})
            d[row.get("Dispatch_Id", len(d))] = d.get(row.get("Dispatch_Id", len(d)), 0.0) + \
                float(row["Counter_Value"])
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = kind_of(row["Kernel_Name"])
            dur.setdefault(k, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}, dur


def main_sq(root, cus=256, simds=4):
    """Wave-state fractions (of SQ_WAVE_CYCLES) and MFMA-busy per SIMD:
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the fraction of the
    dispatch's SIMD-cycles in which a matrix core was busy."""
    per, dur = load_all(root)
    out = {"note": "per kernel kind, averaged over dispatches; wait/active fractions of "
                   "SQ_WAVE_CYCLES; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 "
                   "x 1024 SIMDs); clock_ghz = GRBM_GUI_ACTIVE/8 / kernel-trace duration",
           "kernels": {}}
    for k, cs in sorted(per.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items() if v}
        w = avg.get("SQ_WAVE_CYCLES")
        g = avg.get("GRBM_GUI_ACTIVE")
        e = {"dispatches": max(len(v) for v in cs.values())}
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    e[c.lower()[3:] + "_frac"] = round(avg[c] / w, 4)
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            e["mfma_busy"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * cus * simds), 4)
        if g and k in dur:
            e["avg_us"] = round(sum(dur[k]) / len(dur[k]) / 1e3, 2)
            e["clock_ghz"] = round(g / 8 / (sum(dur[k]) / len(dur[k])), 3)
        e["raw_avg"] = {c: round(v, 1) for c, v in avg.items()}
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


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
    if sys.argv[1] == "--sq":
        main_sq(sys.argv[2])
    else:
        main(sys.argv[1])
