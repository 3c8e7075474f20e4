"""Table of the compiler's kernel-resource-usage remarks (hipcc -Rpass-analysis=kernel-resource-usage)
read from stdin: one row per kernel instantiation with VGPRs, AGPRs, SGPRs, their spills, scratch
bytes per lane, occupancy (waves per SIMD) and static LDS, plus the configurations (BASELINE.json
configs 2-5, bench.py workloads) whose frames launch that instantiation.

Template arguments are decoded from the Itanium mangling (integer and bool literals only)."""
import re
import sys

# Which instantiations the benchmarked workloads launch (rt_render.hip launch_wavefront / launch_t):
# PREC 1 = RT_OUT_F32, GENPOW false (integer specular powers), SPH 2 = S64 (staged in LDS),
# SPH 1 = S256 (tables in L2), ILP true for levels >= 2, BVH for S256's levels >= 2.
USED = {
    "k_render<0,1,false,false,true>": "c2",
    "k_pmask<false>": "c3 c4",
    "k_pmask<true>": "c5",
    "k_primary<1,false>": "c3 c4 c5",
    "k_items": "c3 c4 c5",
    "k_reflect_shade<1,false,2,false,false,false>": "c3 c4 (level 1)",
    "k_reflect_shade<1,false,2,true,false,false>": "c3 c4 (levels 2-3)",
    "k_reflect_shade<1,false,2,true,false,true>": "c3 c4 (level 4, LAST)",
    "k_reflect_shade<1,false,1,false,false,false>": "c5 (level 1)",
    "k_reflect_shade<1,false,1,true,true,false>": "c5 (levels 2-6, BVH)",
    "k_reflect_shade<1,false,1,true,true,true>": "c5 (level 7, BVH, LAST)",
}


def decode(mangled):
    m = re.search(r"_GLOBAL__N_1(\d+)", mangled)  # the anonymous namespace, then <len><identifier>
    if not m:
        return mangled
    n = int(m.group(1))
    name, tail = mangled[m.end():m.end() + n], mangled[m.end() + n:]
    if not tail.startswith("I"):
        return name
    args = tail[:tail.index("EE") + 1]
    vals = []
    for kind, v in re.findall(r"L(i|b|j|y|m)(\d+)E", args):
        vals.append(("true" if v == "1" else "false") if kind == "b" else v)
    return f"{name}<{','.join(vals)}>"


FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"), ("VGPRs Spill", "vspill"),
          ("SGPRs Spill", "sspill"), (r"ScratchSize \[bytes/lane\]", "scratch"), (r"Occupancy \[waves/SIMD\]", "occ"),
          (r"LDS Size \[bytes/block\]", "lds")]


def main():
    rows, cur = [], None
    for line in sys.stdin:
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": decode(m.group(1))}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, short in FIELDS:
            m = re.search(r"remark:\s+" + key + r": (\d+)", line)
            if m:
                cur[short] = int(m.group(1))
    hdr = ["kernel", "VGPR", "AGPR", "SGPR", "VGPR spill", "SGPR spill", "scratch B/lane", "waves/SIMD", "LDS B",
           "used by"]
    print("# kernel resource usage (hipcc --offload-arch=gfx950, -Rpass-analysis=kernel-resource-usage)")
    print("# " + " | ".join(hdr))
    width = max(len(r["name"]) for r in rows) if rows else 10
    for r in sorted(rows, key=lambda r: (r["name"] not in USED, r["name"])):
        print(f"{r['name']:{width}s} " + " ".join(
            f"{r.get(k, -1):>5d}" for _, k in FIELDS) + "  " + USED.get(r["name"], ""))
    spilled = [r["name"] for r in rows if r["name"] in USED and (r.get("vspill", 0) or r.get("scratch", 0))]
    print(f"# benchmarked instantiations with VGPR spills or scratch: {len(spilled)} of "
          f"{sum(1 for r in rows if r['name'] in USED)}" + (": " + ", ".join(spilled) if spilled else ""))


if __name__ == "__main__":
    main()
