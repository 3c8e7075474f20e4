#!/usr/bin/env python3
"""Static instruction histogram of one kernel in the device assembly (make -C eraytracer_amd/csrc asm
-> /tmp/rt_render.s).  Usage: scripts/isa_hist.py ASM NAME_SUBSTRING [--dump FILE]

Buckets: FP64 VALU, binary32 VALU (beams, cull tests, BVH boxes), integer/address VALU, selects
(v_cndmask), compares, lane moves (v_readlane / v_writelane / v_readfirstlane: SGPR spills,
wave reductions, uniform values), DPP/permutes, conversions, other VALU; SALU, SMEM, VMEM, LDS,
branches.  Counts are static (instructions in the code), not executed."""
import re
import sys
from collections import Counter


def body(lines, name):
    start = None
    for i, ln in enumerate(lines):
        if start is None and ln.startswith("_Z") and name in ln and ln.rstrip().endswith(name.split()[-1] if False else ln.rstrip()) and ":" in ln:
            if ln.split(":")[0].endswith("E") or "k_" in ln:
                start = i
                continue
        if start is not None and (ln.startswith(".Lfunc_end") or ln.strip().startswith(".size")):
            return lines[start:i], lines[i:i + 400]
    raise SystemExit(f"{name}: not found")


def bucket(op):
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane_move"
    if op.startswith("v_cndmask"):
        return "select"
    if op.startswith("v_cmp") or op.startswith("v_cmpx"):
        return "compare_f64" if "_f64" in op else "compare_32"
    if "_dpp" in op or op.startswith(("v_mov_b32_dpp", "ds_bpermute", "ds_swizzle", "v_permlane")):
        return "dpp_permute"
    if op.startswith("v_cvt"):
        return "convert"
    if op.startswith("v_") and ("_f64" in op or op in ("v_rsq_f64", "v_rcp_f64")):
        return "fp64"
    if op.startswith("v_pk_") and "f32" in op:
        return "fp32_packed"
    if op.startswith("v_") and ("_f32" in op or "_f16" in op):
        return "fp32"
    if op.startswith(("v_add", "v_sub", "v_mul_lo", "v_mul_hi", "v_mad", "v_lshl", "v_lshr", "v_ashr", "v_and", "v_or",
                      "v_xor", "v_not", "v_bfe", "v_bfi", "v_alignbit", "v_min_i", "v_max_i", "v_min_u", "v_max_u",
                      "v_mbcnt", "v_bcnt", "v_ffb", "v_lshlrev", "v_lshrrev", "v_ashrrev", "v_perm", "v_sad",
                      "v_med3_i", "v_med3_u", "v_addc", "v_subb", "v_subrev", "v_mul_u32", "v_mul_i32", "v_bfrev")):
        return "int_addr"
    if op.startswith("v_mov"):
        return "v_mov"
    if op.startswith(("v_accvgpr",)):
        return "accvgpr_move"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith(("s_load", "s_buffer", "s_store", "s_dcache")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_endpgm", "s_setprio", "s_sendmsg", "s_trap")):
        return "sync"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem_" + ("st" if "store" in op or "atomic" in op else "ld") + ("_scratch" if op.startswith("scratch_") or "buffer_" in op and "off" in op else "")
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    asm, name = sys.argv[1], sys.argv[2]
    lines = open(asm).read().splitlines()
    code, meta = body(lines, name)
    ops = []
    for ln in code:
        t = ln.strip()
        if not t or t.startswith((";", ".", "_Z")) or t.endswith(":"):
            continue
        ops.append(t.split()[0])
    cb = Counter(bucket(o) for o in ops)
    co = Counter(ops)
    valu = sum(v for k, v in cb.items() if k in ("lane_move", "select", "compare_f64", "compare_32", "dpp_permute", "convert",
                                                 "fp64", "fp32", "fp32_packed", "int_addr", "v_mov", "valu_other",
                                                 "accvgpr_move"))
    print(f"kernel: {code[0].split(':')[0][:160]}")
    for ln in meta:
        m = re.search(r"\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|agpr_count):\s*(\d+)", ln)
        if m:
            print(f"  {m.group(1)} {m.group(2)}")
    print(f"instructions {len(ops)}, VALU {valu}")
    for k, v in cb.most_common():
        print(f"  {k:14s} {v:6d}  {100 * v / max(1, valu if k not in ('salu', 'smem', 'branch', 'sync', 'lds', 'other') and not k.startswith('vmem') else len(ops)):5.1f}%")
    print("top opcodes:")
    for k, v in co.most_common(45):
        print(f"  {k:28s} {v:6d}  ({bucket(k)})")
    if "--dump" in sys.argv:
        open(sys.argv[sys.argv.index("--dump") + 1], "w").write("\n".join(code))


if __name__ == "__main__":
    main()
