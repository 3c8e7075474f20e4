#!/usr/bin/env python3
"""Per-kernel instruction counts of library variants (scripts/gpu_r06.sh TAG pmcv): the average of each
PMC counter over every dispatch of a kernel instantiation, one table per variant, and each variant's
difference from the first.  Counts do not depend on timing, so one short run per variant suffices;
with the ablation builds (RT_ABL_NO_SHADE / RT_ABL_NO_REFLECT / RT_ABL_NO_OCC, results wrong) the
differences attribute a kernel's executed instructions to its parts.

    python3 scripts/pmc_variants.py DIR [KERNEL_SUBSTRING]   # DIR/<variant>/**/run_counter_collection.csv
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(vdir):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for f in glob.glob(os.path.join(vdir, "**", "run_counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if "k_" not in name:
                    continue
                i = name.find("::k_")
                short = (name[i + 2:] if i >= 0 else name).split("(")[0]
                acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_reflect_shade<1, false, 2, false, false, false>"
    variants = sorted(os.listdir(d), key=lambda v: (v != "-", v))
    res = {v: load(os.path.join(d, v)) for v in variants}
    base = res.get("-") or res[variants[0]]
    for v in variants:
        print(f"== {v}")
        for k in sorted(res[v]):
            c = res[v][k]
            cols = " ".join(f"{n.replace('SQ_INSTS_', '')}={c[n] / 1e6:.3f}M" for n in sorted(c) if n.startswith("SQ_"))
            mark = " <-" if sub in k else ""
            print(f"  {k[:70]:70s} n={c['dispatches']:4d} {cols}{mark}")
    print(f"== differences from the first variant, {sub}")
    b = next((c for k, c in base.items() if sub in k), None)
    for v in variants:
        c = next((c for k, c in res[v].items() if sub in k), None)
        if b and c:
            print(f"  {v:14s} " + " ".join(f"{n.replace('SQ_INSTS_', '')}={(c[n] - b[n]) / 1e6:+.3f}M"
                                          for n in sorted(c) if n.startswith("SQ_") and n in b))


if __name__ == "__main__":
    main()
