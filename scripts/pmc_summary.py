#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (rocprofv3 kernel trace + PMC passes) for the render
kernel into one JSON (profiles/<name>.json) that DESIGN.md and bench.py cite.

    python scripts/pmc_summary.py gpurun_out/TAG profiles/r01_TAG_pmc.json WORKLOAD_KEY

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB, from separate
passes; FETCH_SIZE under-reports wide coalesced streaming reads by 2x on gfx950 (this kernel
reads only a few KiB of scene tables, so the read side is noted, not corrected); WRITE_SIZE is
exact for 16-B-per-lane stores and uncalibrated for this kernel's 4-12-B stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kernel_filter(name):
    return "k_render" in name and "false>" in name  # the timed render variant (no levels output)


def load_pmc(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_filter(row["Kernel_Name"]):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def load_trace(d):
    f = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
    if not f:
        return None
    with open(f[0]) as fh:
        for row in csv.DictReader(fh):
            if kernel_filter(row["Name"]):
                return {"name": row["Name"], "calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                        "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
    return None


def main():
    src, dst, key = sys.argv[1], sys.argv[2], sys.argv[3]
    pmc, n = load_pmc(src)
    tr = load_trace(src)
    out = {"workload": key, "source": os.path.basename(src.rstrip("/")), "kernel": tr, "counters": pmc,
           "dispatches_per_counter": n}
    d = {}
    if "SQ_INSTS_VALU" in pmc and "SQ_WAVES" in pmc:
        d["valu_insts_per_wave"] = pmc["SQ_INSTS_VALU"] / pmc["SQ_WAVES"]
    if "SQ_THREAD_CYCLES_VALU" in pmc and "SQ_ACTIVE_INST_VALU" in pmc and pmc["SQ_ACTIVE_INST_VALU"]:
        d["valu_lane_utilisation"] = pmc["SQ_THREAD_CYCLES_VALU"] / (64 * pmc["SQ_ACTIVE_INST_VALU"])
    f64 = [pmc.get(c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                "SQ_INSTS_VALU_TRANS_F64")]
    if all(v is not None for v in f64):
        d["f64_wave_insts"] = sum(f64)
        d["f64_share_of_valu"] = sum(f64) / pmc["SQ_INSTS_VALU"] if pmc.get("SQ_INSTS_VALU") else None
        if tr:
            # issue-slot view: every wave64 FP64 instruction occupies 64 lane-slots
            d["f64_lane_slots_per_s"] = sum(f64) * 64 / (tr["avg_ns"] * 1e-9)
            d["f64_issue_frac_of_peak_39.3T"] = d["f64_lane_slots_per_s"] / 39.3e12
    if "SQ_INSTS_VALU_FLOPS_FP64" in pmc and tr:
        d["fp64_flops_per_s"] = pmc["SQ_INSTS_VALU_FLOPS_FP64"] / (tr["avg_ns"] * 1e-9)
    if "GRBM_GUI_ACTIVE" in pmc and tr:
        d["effective_clock_ghz"] = pmc["GRBM_GUI_ACTIVE"] / 8 / tr["avg_ns"]
    if "SQ_WAVE_CYCLES" in pmc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in pmc:
                d[k.lower() + "_share"] = pmc[k] / pmc["SQ_WAVE_CYCLES"]
    fetch = pmc.get("FETCH_SIZE")
    write = pmc.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        d["fetch_bytes"] = fetch * 1024
        d["write_bytes"] = write * 1024
        out["hbm_bytes_per_launch"] = (fetch + write) * 1024
    out["derived"] = d
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({"kernel": tr, "derived": d, "hbm_bytes_per_launch": out.get("hbm_bytes_per_launch")},
                     indent=1))


if __name__ == "__main__":
    main()
