#!/usr/bin/env python3
"""Per-kernel, per-level times of the timed frames in a rocprofv3 kernel trace directory
(frames cut as in pmc_summary.py):  python scripts/klevels.py gpurun_out/kt_TAG"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load_trace  # noqa: E402

d = sys.argv[1]
if not glob.glob(os.path.join(d, "trace")) and glob.glob(os.path.join(d, "*kernel_trace.csv")):
    os.makedirs(os.path.join(d, "trace"), exist_ok=True)
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        os.replace(f, os.path.join(d, "trace", os.path.basename(f)))
fr, k = load_trace(d)
print(f"frames={fr['frames']} kernels/frame={fr['kernels_per_frame']} busy={fr['avg_busy_ns'] / 1e3:.1f} us "
      f"span={fr['avg_span_ns'] / 1e3:.1f} us")
for lab, e in sorted(k.items(), key=lambda kv: (kv[0].split('#')[0], int(kv[0].split('#')[1]))):
    print(f"  {lab:12s} {e['avg_ns'] / 1e3:8.1f} us")

if len(sys.argv) > 2 and sys.argv[2] == "--timeline":
    import csv
    from pmc_summary import frames
    rows = []
    with open(glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))[0]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))))
    rows.sort()
    f = frames(rows)[-1]
    t0 = min(s for _, (s, e) in f)
    for lab, (s, e) in sorted(f, key=lambda x: x[1][0]):
        print(f"  {lab:12s} {(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f} us  ({(e - s) / 1e3:6.1f})")
