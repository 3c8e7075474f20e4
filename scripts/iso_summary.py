#!/usr/bin/env python3
"""Average duration per kernel (name#i = i-th launch within a frame) over the last N frames of a
rocprofv3 kernel trace (bench.py --iso N renders them one at a time), plus the frame span."""
import csv
import glob
import re
import sys
from collections import defaultdict

d, n = sys.argv[1], int(sys.argv[2])
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
frames, cur = [], None
for r in rows:
    m = re.search(r"::(k_\w+)[<(]", r["Kernel_Name"])
    if not m:
        continue
    k = m.group(1)
    if k in ("k_primary", "k_render") and ", true>" not in r["Kernel_Name"].split("(")[0]:
        cur = []
        frames.append(cur)
    if cur is not None:
        cur.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
frames = frames[-n:]
acc, seen_frames = defaultdict(list), 0
spans = []
for fr in frames:
    seen = defaultdict(int)
    for k, s, e in fr:
        acc[f"{k}#{seen[k]}"].append(e - s)
        seen[k] += 1
    spans.append(fr[-1][2] - fr[0][1])
tot = 0.0
for key, v in sorted(acc.items(), key=lambda kv: min(x for x in kv[1])):
    pass
order = []
for k, s, e in frames[-1]:
    pass
seen = defaultdict(int)
for k, s, e in frames[-1]:
    key = f"{k}#{seen[k]}"
    seen[k] += 1
    v = acc[key]
    avg = sum(v) / len(v) / 1e3
    tot += avg
    print(f"{key:22s} {avg:9.1f} us  (n={len(v)})")
print(f"sum of kernels {tot:.1f} us; frame span {sum(spans) / len(spans) / 1e3:.1f} us over {len(spans)} frames")
