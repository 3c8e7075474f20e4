#!/usr/bin/env python3
"""Benchmark of the MI355X render path (BASELINE.json metric: Mpixels/s at 4096x4096,
recursion depth 5, on 1/2/4/8 MI355X).

One step = one frame of the workload (default: synthetic scene S64 — 64 spheres, 4 point
lights — at 4096x4096, depth 5, BASELINE.json configs[2]) rendered by the HIP kernel
into HBM; with N ranks the frame's rows are split over the ranks (strong scaling) and
gathered to rank 0 over RCCL, then put back in row order.  Inputs (the compiled scene)
are resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene s64] [--size 4096] [--depth 5]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Extra keys: "roofline" (the binding FP64-VALU roofline of
the render kernel), "roofline_hbm" (the memory roofline the north star asks for),
"cpu_baseline" (the C oracle running the reference's literal recursion on the host's
cores over a bounded sample of the same frame — the BEAM is not installed on the box),
"kernel_mpx_s" and "boundary_mpx_s" (host-buffer rt_render, PCIe included).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (HIP's default, and the GPU box's setting, is 4): frames in
# flight each use a stream of their own, and with RCCL's streams beside them 4 queues would be
# shared behind event waits (measured: S64 4096^2 d5, 4 frames in flight, 0.68 ms per frame
# with 4 queues, 0.61 with 8).  Set before the HIP runtime initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

PEAK_FP64_VALU_TOPS = 39.3   # MI355X FP64 vector 78.6 TFLOP/s counting an FMA as 2 (spec); this path has no FMA
PEAK_HBM_GBS = 8000.0        # MI355X HBM3E (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50, help="untimed frames (the GPU's clocks settle over ~50)")
    ap.add_argument("--scene", default="s64")
    ap.add_argument("--size", type=int, default=4096, help="square frame side (see --width/--height)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--order", default="exact", choices=["exact", "fast"])
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--row-block", type=int, default=16)
    ap.add_argument("--spp", type=int, default=1, help="samples per pixel (RT_SUPERSAMPLING; BASELINE config 5: 16)")
    ap.add_argument("--seed", type=int, default=0x5EED0005)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-boundary", action="store_true")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight per rank (default 4 at N=1, 3 at N>1; 1 for --gather dense)")
    ap.add_argument("--gather", default="compact", choices=["compact", "dense"],
                    help="N > 1: compact = background pixels not sent (rt_slab_pack, default); dense = whole slabs")
    return ap.parse_args()


def cpu_baseline(scene, W, H, depth, target_s, spp=1, seed=0):
    """The C oracle in the reference's literal recursion (lighting_function recomputes the
    reflection per light, raytracer.erl:211-224), threaded over the box's CPU share, on a
    bounded sample of rows spread over the same frame.  The literal recursion is exponential
    in depth (L^(depth-1) re-evaluations), so deeper or supersampled configs use the
    memoised oracle (same results) and say so."""
    from eraytracer_amd import _native as N
    from oracle import oracle as O
    O.build()
    el = N.marshal(scene)
    threads = min(16, os.cpu_count() or 1)
    literal = spp == 1 and depth <= 5
    mode = O.LITERAL if literal else O.MEMO
    # calibrate on one row, then take evenly spaced rows to fill ~target_s seconds
    t0 = time.perf_counter()
    O.render(el, W, H, depth, mode=mode, threads=threads, row0=H // 2, nrows=1, spp=spp, seed=seed)
    per_row = max(time.perf_counter() - t0, 1e-4)
    nrows = int(max(1, min(H, target_s / per_row)))
    rows = sorted(set(int(r) for r in [(i * H) // nrows + (H // nrows) // 2 for i in range(nrows)]))
    t0 = time.perf_counter()
    for r in rows:
        O.render(el, W, H, depth, mode=mode, threads=threads, row0=r, nrows=1, spp=spp, seed=seed)
    dt = time.perf_counter() - t0
    px = len(rows) * W
    how = ("ORC_LITERAL (the reference's per-light reflection recursion)" if literal else
           "ORC_MEMO (reflection once per hit; the literal recursion is exponential in depth)")
    return {"value": px / dt / 1e6, "unit": "Mpixels/s", "cores": threads, "kind": "port",
            "sample": f"{len(rows)} evenly spaced rows x {W} px of the same {W}x{H} depth-{depth}"
                      + (f" x{spp} spp" if spp > 1 else "") + f" frame ({px} px, {dt:.1f} s), oracle/rt_oracle.c "
                      f"{how}, {threads} threads; BEAM (erl) is not installed on the box"}


def profile_for(workload_key):
    """The committed rocprofv3 summary of the same workload (profiles/*pmc*.json, written by
    scripts/pmc_summary.py from scripts/profile.sh passes; the newest by name wins), or None.
    Supplies the measured HBM bytes per frame launch and the executed FP64 issue fraction."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload_key and d.get("hbm_bytes_per_launch") is not None:
            best = (d, os.path.relpath(p, ROOT))
    return best


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from eraytracer_amd import scenes, workload
    from eraytracer_amd.dist import FrameRenderer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("bench.py: --gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local)
    if world > 1:
        # RCCL brings its own stream(s); with torch's and the library's two shading side streams
        # a rank would exceed the 4 hardware queues a process gets, and streams sharing a queue
        # stall behind each other's event waits.  The gather dominates at N > 1 anyway.
        os.environ.setdefault("RT_LIT_STREAM", "0")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W = args.width or args.size
    H = args.height or args.size
    scene = scenes.named(args.scene)
    counts = workload.scene_counts(scene)
    inflight = args.inflight or (1 if args.gather == "dense" and world > 1 else 4 if world == 1 else 3)
    fr = FrameRenderer(scene, W, H, args.depth, rank=rank, world=world, device=local, row_block=args.row_block,
                       precision=args.precision, order=args.order, spp=args.spp, seed=args.seed, inflight=inflight)

    # untimed: work count of this rank's rows (levels of every pixel's reflection chain)
    lv_fr = FrameRenderer(scene, W, H, args.depth, rank=rank, world=world, device=local, row_block=args.row_block,
                          precision=args.precision, order=args.order, levels=True)
    lv_fr.launch()
    torch.cuda.synchronize()
    from eraytracer_amd.dist import shard_global_rows
    valid = torch.from_numpy(shard_global_rows(H, args.row_block, world, rank) >= 0).to(lv_fr.levels.device)
    hist = torch.bincount(lv_fr.levels[valid].flatten().to(torch.int64), minlength=args.depth + 1).cpu().numpy()
    lv_fr.close()
    del lv_fr
    # with spp > 1 the work is estimated as spp times that of the unjittered frame
    ops_rank = workload.ops_from_levels(hist, args.depth, counts) * args.spp
    px_rank = int(hist.sum())

    # With N > 1 ranks a step is render + gather to rank 0 + reorder; frames are pipelined
    # (frame i+1 renders while frame i's gather is in flight, dist.SlabPipeline) and the
    # timed region ends only when every frame is gathered and reordered.
    # The compact gather (default) sends only the non-background pixels: rank 0's inbound xGMI
    # links, not the render, bound a frame at N = 8 (dist.CompactGather).
    pipe = None
    if world > 1:
        pipe = fr.compact_gather() if args.gather == "compact" else fr.pipeline()

    def one_step():
        if pipe is not None and args.gather == "dense":
            fr.slab = pipe.slab
        fr.launch()  # on the next in-flight slot's stream
        if pipe is None:
            fr.gather()
        elif args.gather == "compact":
            with torch.cuda.stream(fr.stream):
                pipe.submit(fr.slab, rank)
        else:
            pipe.submit()

    for _ in range(args.warmup):
        one_step()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize()

    # GPU time of the timed region: HIP events on the caller's stream, every in-flight slot
    # stream forked from it after the start event and joined into it before the end event
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    fr.fork()
    for i in range(args.steps):
        one_step()
    if pipe is not None:
        pipe.drain()
    fr.join()
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / args.steps

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
        o = torch.tensor([float(ops_rank)], dtype=torch.float64, device="cuda")
        dist.all_reduce(o, op=dist.ReduceOp.SUM)
        ops_total = float(o[0])
    else:
        kern_ms_max = kern_ms
        ops_total = float(ops_rank)

    if rank == 0:
        frame_px = W * H
        ms_step = elapsed / args.steps * 1e3
        value = frame_px * args.steps / elapsed / 1e6
        bytes_px = 12 if args.precision == "f32" else 24
        # roofline of the dominant kernel (this rank's render launch), per launch
        k_s = kern_ms / 1e3
        valu_ach = ops_rank / k_s / 1e12
        hbm_ach = px_rank * bytes_px / k_s / 1e9
        wkey = f"{args.scene}-{W}x{H}-d{args.depth}-{args.order}-{args.precision}-n{world}" + (
            f"-spp{args.spp}" if args.spp > 1 else "")
        prof = profile_for(wkey)
        traffic = prof[0]["hbm_bytes_per_launch"] if prof else None
        # executed work per frame from the profile's counters (counts do not depend on timing),
        # over this run's live GPU time per frame: FP64 issue vs the FP64 peak, and VALU busy
        # (a wave64 FP64 instruction holds a SIMD-32 for 4 cycles, other VALU ops for 2;
        # 256 CUs x 4 SIMDs at 2.4 GHz)
        executed = valu_busy = None
        if prof:
            c = prof[0].get("counters", {})
            f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                              "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
            if f64 and c.get("SQ_INSTS_VALU"):
                executed = f64 * 64 / k_s / (PEAK_FP64_VALU_TOPS * 1e12)
                valu_busy = (4 * f64 + 2 * (c["SQ_INSTS_VALU"] - f64)) / (1024 * 2.4e9 * k_s)
        line = {
            "metric": "Mpixels/sec at 4096x4096, recursion depth 5 (frame rendered into HBM, gathered to rank 0)",
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.scene.upper()} {W}x{H} depth {args.depth}"
                       + (f" x{args.spp} spp" if args.spp > 1 else ""), "scene": args.scene, "spp": args.spp,
                       "width": W, "height": H, "depth": args.depth, "order": args.order,
                       "framebuffer": args.precision, "row_block": args.row_block, "inflight": inflight,
                       "parallelism": f"rows{world}" + (f"+rccl_{args.gather}_gather" if world > 1 else ""),
                       "spheres": counts["spheres"], "triangles": counts["triangles"], "planes": counts["planes"],
                       "lights": counts["lights"]},
            "roofline": {"bound": "valu", "achieved": round(valu_ach, 3), "peak": PEAK_FP64_VALU_TOPS,
                         "unit": "TFLOP/s", "frac": round(valu_ach / PEAK_FP64_VALU_TOPS, 4),
                         "traffic": traffic,
                         "executed_f64_frac": round(executed, 4) if executed is not None else None,
                         "valu_busy_frac": round(valu_busy, 4) if valu_busy is not None else None,
                         "note": "FP64 VALU (binding): algorithmic binary64 ops per frame launch as SURVEY.md 8d "
                                 f"counts them for the reference's brute-force scans ({ops_rank:.4g} ops for "
                                 f"{px_rank} px) / GPU time per frame {kern_ms:.3f} ms (HIP events around the timed "
                                 f"region, {inflight} frames in flight); peak = 78.6 TFLOP/s FP64 vector / 2 (no FMA: contraction off). frac > 1 "
                                 "means the beam/occluder culling skips reference work; executed_f64_frac = the FP64 "
                                 "instructions actually issued per frame (rocprofv3 PMC, x64 lanes) / GPU time per "
                                 "frame / peak; valu_busy_frac = SIMD cycles those VALU instructions occupy per frame "
                                 "(FP64 4, others 2) / (1024 SIMDs x 2.4 GHz x GPU time per frame)"
                                 + (f"; traffic and executed from {prof[1]}" if prof else "")},
            "roofline_hbm": {"bound": "hbm", "achieved": round(hbm_ach, 3), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(hbm_ach / PEAK_HBM_GBS, 6), "traffic": traffic},
            "kernel_ms": round(kern_ms, 4),
            "kernel_ms_max_rank": round(kern_ms_max, 4),
            "kernel_mpx_s": round(px_rank / k_s / 1e6, 3),
            "ops_per_frame": ops_total,
        }
        if world == 1 and not args.no_boundary:
            from eraytracer_amd.raytracer import render
            st = {}
            render(W, H, scene, args.depth, precision=args.precision, order=args.order, stats=st, spp=args.spp,
                   seed=args.seed)
            ts = []
            for _ in range(2):
                st = {}
                render(W, H, scene, args.depth, precision=args.precision, order=args.order, stats=st, spp=args.spp,
                       seed=args.seed)
                ts.append(st["total_ms"])
            line["boundary_mpx_s"] = round(frame_px / (min(ts) / 1e3) / 1e6, 3)
            # raytrace/5 end to end natively: render + P3 text on the GPU + file write
            # (write_pixels_to_ppm/5, byte-exact); the binary64 frame never leaves the GPU
            import tempfile
            from eraytracer_amd.raytracer import render_ppm_file
            with tempfile.TemporaryDirectory() as td:
                path = os.path.join(td, "frame.ppm")
                # one untimed call first: the first rt_render_ppm_file of a process pays ~2 s of
                # one-time set-up (scripts/p3_timing.py), the other legs are timed warm too
                render_ppm_file(W, H, scene, args.depth, path, spp=args.spp, seed=args.seed)
                tp = []
                for _ in range(3):
                    t1 = time.perf_counter()
                    render_ppm_file(W, H, scene, args.depth, path, spp=args.spp, seed=args.seed)
                    tp.append(time.perf_counter() - t1)
                line["p3_file_mpx_s"] = round(frame_px / min(tp) / 1e6, 3)
                line["p3_file_bytes"] = os.path.getsize(path)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene, W, H, args.depth, args.cpu_seconds, args.spp, args.seed)
        print(json.dumps(line), flush=True)
    fr.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
