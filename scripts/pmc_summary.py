#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (rocprofv3 kernel trace + separate PMC passes) into one
JSON (profiles/<name>.json) that DESIGN.md and bench.py cite.

    python scripts/pmc_summary.py gpurun_out/TAG profiles/r01_TAG_pmc.json WORKLOAD_KEY [TIMED_FRAMES [ISO_FRAMES]]

The unit is one FRAME LAUNCH (one rt_launch): the dispatch stream is cut into frames at each
timed frame-start kernel (the wavefront engine's k_primary<PREC, false>, or the fused
k_render<ORDER, PREC, false, ...>), and every render kernel up to the next non-render
dispatch belongs to that frame.  The levels pass bench.py runs once (LEVELS=true variants) is
excluded.  Counters are summed over a frame's kernels and averaged over frames; per-kernel
entries are labelled name#i, i = occurrence within the frame (k_reflect#0 makes level 1,
k_shade#0 shades the DEEPEST level).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB and come from
separate passes.  Calibrated here (scripts/hbm_calib.hip, profiles/r04_hbm_calib.txt): a coalesced
16-B-per-lane stream moves 128-B lines and FETCH_SIZE reports half of its bytes; a random gather of
64, 16 or 8 bytes per lane moves one 64-B request per lane and FETCH_SIZE reports exactly that.
The engine's kernels mix both, so a kernel's read bytes lie between the raw FETCH_SIZE (lower
bound, exact for gathers) and twice it (fetch_bytes_corrected, upper bound, exact for streams);
both are reported (hbm_bytes_per_launch = upper, hbm_bytes_per_launch_low = lower).  WRITE_SIZE is
reported raw.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

RENDER = re.compile(r"::(k_\w+)[<(]")


def short(name):
    m = RENDER.search(name)
    return m.group(1) if m else None


def frame_start(name):
    return bool(re.search(r"k_primary<\d+, false>", name) or re.search(r"k_render<\d+, \d+, false", name))


def frames(rows):
    """rows: (dispatch_id, name, payload) in dispatch order -> list of frames, each a list of
    (label, payload)."""
    out, cur, seen = [], None, None
    for _, name, payload in rows:
        s = short(name)
        if s and frame_start(name):
            cur, seen = [], defaultdict(int)
            out.append(cur)
        elif s is None or (s in ("k_primary", "k_render")):
            cur = None  # a non-render dispatch or the levels pass ends the frame
            continue
        if cur is None:
            continue
        cur.append((f"{s}#{seen[s]}", payload))
        seen[s] += 1
    return out


def load_pmc(d):
    per_disp = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (os.path.dirname(f), int(row["Dispatch_Id"]))
                per_disp[key][row["Counter_Name"]] = float(row["Counter_Value"])
                names[key] = row["Kernel_Name"]
    # each pmc pass is its own process: cut frames per pass, then average over all frames
    tot, per_k, nfr = defaultdict(float), defaultdict(lambda: defaultdict(float)), defaultdict(int)
    for pdir in sorted({k[0] for k in per_disp}):
        rows = sorted(((k[1], names[k], per_disp[k]) for k in per_disp if k[0] == pdir))
        fr = frames(rows)
        for f in fr:
            for label, c in f:
                for cn, v in c.items():
                    tot[cn] += v
                    per_k[label][cn] += v
            for cn in {cn for _, c in f for cn in c}:
                nfr[cn] += 1
    frame = {cn: tot[cn] / nfr[cn] for cn in tot if nfr[cn]}
    kern = {lab: {cn: v / nfr[cn] for cn, v in c.items() if nfr[cn]} for lab, c in per_k.items()}
    return frame, kern, dict(nfr)


def load_trace(d, timed=None, iso=0):
    f = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))
    if not f:
        return None, None
    rows = []
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                         (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["VGPR_Count"]))))
    rows.sort()
    fr = frames(rows)
    if not fr:
        return None, None
    busy = [sum(e - s for _, (s, e, _) in f) for f in fr]
    span = [max(e for _, (s, e, _) in f) - min(s for _, (s, e, _) in f) for f in fr]  # streams may overlap
    per = defaultdict(list)
    vg = {}
    for f in fr:
        for lab, (s, e, v) in f:
            per[lab].append(e - s)
            vg[lab] = v
    # frames in flight overlap: the window from the first frame's first kernel to the last
    # frame's last kernel, per frame, is the GPU time per frame the bench's events measure
    # (over the last `timed` frames: the bench's timed region, after its warmup and a sync)
    # bench.py ends with `iso` frames launched back to back on one stream (the dominant kernel
    # timed alone): per-kernel "isolated_avg_ns" over those; the timed frames come before them
    iso_fr = fr[-iso:] if iso else []
    if iso:
        fr = fr[:-iso]
    iso_k = defaultdict(list)
    for f in iso_fr:
        for lab, (s, e, v) in f:
            iso_k[lab].append(e - s)
    tf = fr[-timed:] if timed else fr
    t_first = min(s for f in tf for _, (s, e, _) in f)
    t_last = max(e for f in tf for _, (s, e, _) in f)
    frame = {"frames": len(fr), "kernels_per_frame": len(fr[0]), "avg_busy_ns": sum(busy) / len(busy),
             "avg_span_ns": sum(span) / len(span), "min_busy_ns": min(busy),
             "window_ns_per_frame": (t_last - t_first) / len(tf), "window_frames": len(tf)}
    # rocprofv3's VGPR_Count on gfx950 is half the allocated VGPRs (48 for the compiler's 96-VGPR
    # kernels: checked against -Rpass-analysis=kernel-resource-usage, profiles/*_resource_usage.txt)
    kern = {lab: {"avg_ns": sum(v) / len(v), "rocprof_vgpr_count": vg[lab], "vgpr_alloc": 2 * vg[lab]}
            for lab, v in per.items()}
    for lab, v in iso_k.items():
        kern.setdefault(lab, {})["isolated_avg_ns"] = sum(v) / len(v)
    return frame, kern


def derive(c, ns):
    d = {}
    if c.get("SQ_WAVES"):
        d["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        d["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    f64 = [c.get(k) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                              "SQ_INSTS_VALU_TRANS_F64")]
    if all(v is not None for v in f64):
        d["f64_wave_insts"] = sum(f64)
        if c.get("SQ_INSTS_VALU"):
            d["f64_share_of_valu"] = sum(f64) / c["SQ_INSTS_VALU"]
        if ns:
            # issue-slot view: every wave64 FP64 instruction occupies 64 lane-slots
            d["f64_issue_frac_of_peak_39.3T"] = sum(f64) * 64 / (ns * 1e-9) / 39.3e12
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                d[k.lower() + "_share"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["fetch_bytes"] = c["FETCH_SIZE"] * 1024
        d["fetch_bytes_corrected"] = 2 * c["FETCH_SIZE"] * 1024
        d["write_bytes"] = c["WRITE_SIZE"] * 1024
    return d


def main():
    src, dst, key = sys.argv[1], sys.argv[2], sys.argv[3]
    timed = int(sys.argv[4]) if len(sys.argv) > 4 else None  # the bench's --steps
    spp = int(sys.argv[6]) if len(sys.argv) > 6 else 1       # samples per pixel: spp passes per frame
    iso = (int(sys.argv[5]) if len(sys.argv) > 5 else 0) * spp  # the bench's --iso (in passes)
    timed = timed * spp if timed else timed
    pmc, pmc_k, nfr = load_pmc(src)
    tr, tr_k = load_trace(src, timed, iso)
    out = {"workload": key, "source": os.path.basename(src.rstrip("/")),
           "unit": "one frame launch" if spp == 1 else f"one sample pass ({spp} per frame launch)", "spp": spp,
           "trace": tr, "counters": pmc, "frames_per_counter": nfr,
           # frame-level rates over the GPU time per frame (frames and streams overlap)
           "derived": derive(pmc, tr["window_ns_per_frame"] if tr else None), "kernels": {}}
    for lab in sorted(set(pmc_k) | set(tr_k or {}), key=lambda s: (s.split("#")[0], int(s.split("#")[1]))):
        ent = dict((tr_k or {}).get(lab, {}))
        ent["counters"] = pmc_k.get(lab, {})
        ent["derived"] = derive(ent["counters"], ent.get("avg_ns"))
        out["kernels"][lab] = ent
    dd = out["derived"]
    if "fetch_bytes" in dd:
        out["hbm_bytes_per_launch"] = dd["fetch_bytes_corrected"] + dd["write_bytes"]
        out["hbm_bytes_per_launch_low"] = dd["fetch_bytes"] + dd["write_bytes"]
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({"trace": tr, "derived": dd, "hbm_bytes_per_launch": out.get("hbm_bytes_per_launch"),
                      "hbm_bytes_per_launch_low": out.get("hbm_bytes_per_launch_low")},
                     indent=1))
    for lab, e in out["kernels"].items():
        x = e["derived"]
        print(f"{lab:14s} {e.get('avg_ns', 0) / 1e3:8.1f} us (alone {e.get('isolated_avg_ns', 0) / 1e3:6.1f}) "
              f"vgpr_alloc={e.get('vgpr_alloc', 2 * e.get('vgpr', 0))} "
              f"valu/wave={x.get('valu_insts_per_wave', 0):8.0f} f64frac={x.get('f64_issue_frac_of_peak_39.3T', 0):.3f} "
              f"valu_share={x.get('sq_active_inst_valu_share', 0):.3f} lanes={x.get('valu_lane_utilisation', 0):.2f}")


if __name__ == "__main__":
    main()
