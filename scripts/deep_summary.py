"""Per-kernel latency/cache summary of a scripts/profile_deep.sh run (counters per frame
launch, averaged; labels as scripts/pmc_summary.py)."""
import sys

sys.path.insert(0, "scripts")
from pmc_summary import load_pmc  # noqa: E402

frame, kern, _ = load_pmc(sys.argv[1])


def g(c, k):
    return c.get(k, 0.0)


def row(lab, c):
    out = [f"{lab:20s}"]
    if g(c, "SQ_INSTS_SMEM"):
        out.append(f"smem_lat={g(c, 'SQ_INST_LEVEL_SMEM') / g(c, 'SQ_INSTS_SMEM'):6.0f}")
    nv = g(c, "SQ_INSTS_VMEM_RD") + g(c, "SQ_INSTS_VMEM_WR")
    if nv:
        out.append(f"vmem_lat={g(c, 'SQ_INST_LEVEL_VMEM') / nv:6.0f} vmem/wave={nv / max(g(c, 'SQ_WAVES'), 1):6.1f}")
    if g(c, "SQ_INSTS_LDS"):
        out.append(f"lds_lat={g(c, 'SQ_INST_LEVEL_LDS') / g(c, 'SQ_INSTS_LDS'):5.0f}")
    if g(c, "SQC_DCACHE_REQ"):
        out.append(f"sqc_hit={g(c, 'SQC_DCACHE_HITS') / max(g(c, 'SQC_DCACHE_HITS') + g(c, 'SQC_DCACHE_MISSES'), 1):.3f}")
    if g(c, "TCP_TCC_READ_REQ_sum"):
        out.append(f"l2_lat={g(c, 'TCP_TCC_READ_REQ_LATENCY_sum') / g(c, 'TCP_TCC_READ_REQ_sum'):5.0f}")
    if g(c, "TCC_HIT_sum") + g(c, "TCC_MISS_sum"):
        out.append(f"l2_hit={g(c, 'TCC_HIT_sum') / (g(c, 'TCC_HIT_sum') + g(c, 'TCC_MISS_sum')):.3f}")
    if g(c, "SQ_WAVE_CYCLES") and g(c, "SQ_WAVES"):
        out.append(f"cyc/wave={g(c, 'SQ_WAVE_CYCLES') / g(c, 'SQ_WAVES'):8.0f}")
    if g(c, "SQ_WAVES"):
        out.append(f"valu/wave={g(c, 'SQ_INSTS_VALU') / g(c, 'SQ_WAVES'):6.0f} salu/wave={g(c, 'SQ_INSTS_SALU') / g(c, 'SQ_WAVES'):6.0f}")
    return " ".join(out)


print(row("FRAME", frame))
for lab in sorted(kern, key=lambda s: (s.split("#")[0], int(s.split("#")[1]))):
    print(row(lab, kern[lab]))
