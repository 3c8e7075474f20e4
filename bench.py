#!/usr/bin/env python3
"""Benchmark of the MI355X render path (BASELINE.json metric: Mpixels/s at 4096x4096,
recursion depth 5, on 1/2/4/8 MI355X).

One step = one frame of the workload (default: synthetic scene S64 — 64 spheres, 4 point
lights — at 4096x4096, depth 5, BASELINE.json configs[2]) rendered by the HIP kernel
into HBM; with N ranks the frame's rows are split over the ranks (strong scaling) and
gathered to rank 0 over RCCL, then put back in row order.  Inputs (the compiled scene)
are resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene s64] [--size 4096] [--depth 5]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 outside torch.distributed.run (no WORLD_SIZE in the environment), bench.py
starts ``python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1
--master-port <free> bench.py <same arguments>`` as a child process, before anything touches
the GPU, and exits with its return code (it does not exec).

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
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (--hw-queues; HIP's default, and the GPU box's setting, is 4).  At
# N = 1 the bench keeps the environment's value, as a library caller (a NIF process) does: 4 and 8
# queues measured the same (profiles/r06c_bench_c3d.json 0.3935 ms at 8, r06c_bench_c3d_q4.json
# 0.3908 at 4).  With N > 1 ranks RCCL's streams and the exchange's side stream join the frames' streams,
# and 4 queues would be shared behind event waits: 8 there.  Set in main() before the HIP runtime
# initialises.
DEFAULT_HW_QUEUES_MULTI = 8

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
    ap.add_argument("--settle", type=float, default=0.3,
                    help="seconds of untimed frames before the warmup steps (clock ramp; 0 = none)")
    ap.add_argument("--iso", type=int, default=20,
                    help="frames launched back to back after the timed region to time the dominant kernel alone")
    ap.add_argument("--span-timing", action="store_true",
                    help="also bracket the dominant kernel with HIP events inside the timed region "
                         "(launch_span_ms_in_flight; off by default: the timed frames run as the product runs them)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-boundary", action="store_true")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight per rank (default 4; 1 for --gather dense at N>1)")
    ap.add_argument("--priorities", default="auto",
                    help="comma-separated stream priority per in-flight slot (torch: lower = higher priority; "
                         "auto: FrameRenderer's default, half the slots high with >= 4 in flight and spp 1; none)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (0 = leave the environment's, HIP's default 4; "
                         "default: 0 at --gpus 1, 8 with more)")
    ap.add_argument("--no-setup", action="store_true",
                    help="skip the setup-cost leg (scene compile, primary masks, new-scene and cold frames)")
    ap.add_argument("--rank0", default="auto", choices=["auto", "render", "assemble"],
                    help="N > 1: rank 0 renders its share of rows (render) or only reassembles the frame while ranks "
                         "1..N-1 render (assemble); auto: assemble from 4 ranks on (compact gather only)")
    ap.add_argument("--gather", default="compact", choices=["compact", "dense"],
                    help="N > 1: compact = background pixels not sent (rt_slab_pack, default); dense = whole slabs")
    return ap.parse_args()


def parse_priorities(text: str):
    """--priorities "0,-1,...": one HIP stream priority (0 or -1) per frame in flight."""
    try:
        pr = [int(x) for x in text.split(",")]
    except ValueError:
        raise SystemExit(f"--priorities: comma-separated 0 / -1 values, 'auto' or 'none'; got {text!r}")
    if any(p not in (0, -1) for p in pr):
        raise SystemExit(f"--priorities: each value must be 0 or -1 (HIP's two stream priorities); got {text!r}")
    return pr


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv, nproc: int, port: int):
    """The torch.distributed.run command that runs this script with one rank per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def self_launch(argv, nproc: int, run=subprocess.run) -> int:
    """Run the N-rank bench as a child process (the caller has not touched the GPU) and
    return its exit code."""
    r = run(launcher_cmd(argv, nproc, free_port()))
    return int(r.returncode)


def cpu_baseline(scene, W, H, depth, target_s, spp=1, seed=0):
    """The C oracle in the reference's literal recursion (lighting_function recomputes the
    reflection per light, raytracer.erl:211-224), threaded over the box's CPU share like the
    `concurrent` strategy's workers (raytracer.erl:101-119), on a bounded sample of rows spread
    over the same frame.  Every call renders a list of rows on all threads (orc_render_rows) and
    `cores` is the number of threads that actually rendered rows.  The literal recursion is
    exponential in depth (L^(depth-1) re-evaluations), so deeper or supersampled configs use the
    memoised oracle (same results) and say so."""
    from eraytracer_amd import _native as N
    from oracle import oracle as O
    O.build()
    el = N.marshal(scene)
    threads = O.host_threads()  # this process's CPU share (OMP_NUM_THREADS, else its CPU affinity)
    literal = spp == 1 and depth <= 5
    mode = O.LITERAL if literal else O.MEMO

    def spread(n):
        return sorted(set(int(r) for r in [(i * H) // n + (H // n) // 2 for i in range(n)]))

    # calibrate on 2 rows per thread spread over the frame, then fill ~target_s seconds
    cal = spread(min(H, 2 * threads))
    t0 = time.perf_counter()
    O.render_rows(el, W, H, cal, depth, mode=mode, threads=threads, spp=spp, seed=seed)
    per_row = max(time.perf_counter() - t0, 1e-4) / len(cal)
    rows = spread(int(max(threads, min(H, target_s / per_row))))
    t0 = time.perf_counter()
    _, workers = O.render_rows(el, W, H, rows, depth, mode=mode, threads=threads, spp=spp, seed=seed)
    dt = time.perf_counter() - t0
    px = len(rows) * W
    how = ("ORC_LITERAL (the reference's per-light reflection recursion)" if literal else
           "ORC_MEMO (reflection once per hit; the literal recursion is exponential in depth)")
    return {"value": px / dt / 1e6, "unit": "Mpixels/s", "cores": workers, "kind": "port",
            "sample": f"{len(rows)} evenly spaced rows x {W} px of the same {W}x{H} depth-{depth}"
                      + (f" x{spp} spp" if spp > 1 else "") + f" frame ({px} px, {dt:.1f} s) in one call, "
                      f"oracle/rt_oracle.c {how}, {workers} of {threads} threads rendering rows; "
                      "BEAM (erl) is not installed on the box",
            "threads_requested": threads, "host": host_cpu_info()}


def host_cpu_info():
    """What the CPU baseline ran on: the machine's CPU count (nproc), the CPUs this process may
    use (affinity), the cgroup CPU quota, OMP_NUM_THREADS and the CPU model."""
    info = {"nproc": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity_cpus"] = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        info["cgroup_cpu_quota"] = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                info["cpu_model"] = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return info


def profile_for(workload_key):
    """The committed rocprofv3 summary of the same workload (profiles/*pmc*.json, written by
    scripts/pmc_summary.py from scripts/profile.sh passes; the newest by name wins), or None.
    Supplies the measured HBM bytes per frame launch and the executed FP64 issue fraction."""
    def tag_order(p):
        # r05ac is newer than r05z: the round, then the tag's length, then the tag
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(p))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, os.path.basename(p))

    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), key=tag_order):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload_key and d.get("hbm_bytes_per_launch") is not None:
            best = (d, os.path.relpath(p, ROOT))
    return best


# The dominant kernel of each engine (the roofline's subject) and its label in the profiles
# (scripts/pmc_summary.py: name#i = i-th launch of that kernel within a frame)
DOMINANT = {"wave": ("k_reflect_shade#0", "RT_KT_LEVEL1",
                     "k_reflect_shade(1): level-0 shading + level-1 reflection scan"),
            "fused": ("k_render#0", "RT_KT_RENDER", "k_render: the fused engine's one kernel per frame")}


def engine_of(N, fr, spp):
    """The engine rt_launch runs for this context (rt_engine: the library's own decision — the
    RT_ENGINE environment override, else the compile-time FUSED_MAX_OBJECTS crossover)."""
    e = N.check(N.lib().rt_engine(fr._ps[0], spp), "rt_engine")
    return "fused" if e == N.RT_ENGINE_FUSED else "wave"


def f64_insts(c):
    return sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                       "SQ_INSTS_VALU_TRANS_F64"))


def main():
    args = parse()
    if args.hw_queues is None:
        args.hw_queues = 0 if args.gpus == 1 else DEFAULT_HW_QUEUES_MULTI
    if not 0 <= args.hw_queues <= 32:
        sys.exit("bench.py: --hw-queues must be in 0..32")
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # python3 bench.py --gpus N: start the N ranks ourselves (nothing has touched HIP yet)
        sys.exit(self_launch(sys.argv[1:], args.gpus))
    import numpy as np
    import torch
    import torch.distributed as dist

    from eraytracer_amd import _native as N
    from eraytracer_amd import scenes, workload
    from eraytracer_amd.dist import FrameRenderer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
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
    inflight = args.inflight or (1 if args.gather == "dense" and world > 1 else 4)
    # Rank 0 as assembler (N >= 4 by default): at N = 8 a rank renders its shard in ~0.1 ms, and rank 0
    # rendering one too while it decodes the whole frame was the slowest stage
    assemble = world > 1 and args.gather == "compact" and (args.rank0 == "assemble" or
                                                          (args.rank0 == "auto" and world >= 4))
    fr = FrameRenderer(scene, W, H, args.depth, rank=rank, world=world, device=local, row_block=args.row_block,
                       precision=args.precision, order=args.order, spp=args.spp, seed=args.seed, inflight=inflight,
                       priorities=("auto" if args.priorities == "auto" else None if args.priorities == "none" else
                                   parse_priorities(args.priorities)), assemble=assemble)

    # untimed: work count of this rank's rows (levels of every pixel's reflection chain)
    lv_fr = FrameRenderer(scene, W, H, args.depth, rank=rank, world=world, device=local, row_block=args.row_block,
                          precision=args.precision, order=args.order, levels=True, assemble=assemble)
    from eraytracer_amd.dist import shard_global_rows
    if lv_fr.renders:
        lv_fr.launch()
        torch.cuda.synchronize()
        valid = torch.from_numpy(shard_global_rows(H, args.row_block, lv_fr.nshards, lv_fr.shard) >= 0)
        valid = valid.to(lv_fr.levels.device)
        hist = torch.bincount(lv_fr.levels[valid].flatten().to(torch.int64), minlength=args.depth + 1).cpu().numpy()
    else:  # an assembling rank 0 renders no pixels
        hist = np.zeros(args.depth + 1, dtype=np.int64)
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
    checked = None
    if world > 1:
        pipe = fr.compact_gather() if args.gather == "compact" else fr.pipeline()
        if args.gather == "compact":
            checked = self_check(fr, pipe, scene, args, rank, world, local)

    def one_step():
        if pipe is not None and args.gather == "dense":
            fr.slab = pipe.slab
        fr.launch()  # on the next in-flight slot's stream
        if pipe is None:
            fr.gather()
        elif args.gather == "compact":
            with torch.cuda.stream(fr.stream):
                pipe.submit(fr.slab if fr.renders else None, fr.shard)
        else:
            pipe.submit()

    # Before the W warmup steps: render frames until --settle seconds have passed (the GPU's
    # clocks ramp over the first ~50 frames; with a short --warmup the timed steps would still
    # see them rising).  Frames only, no gather.
    settle_frames = 0
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        for _ in range(8):
            fr.launch()
        settle_frames += 8
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        one_step()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize()

    # GPU time of the timed region: HIP events on the caller's stream, every in-flight slot
    # stream forked from it after the start event and joined into it before the end event;
    # the dominant kernel's launches are bracketed by events on their own streams
    engine = engine_of(N, fr, args.spp)
    dom_label, dom_kt, dom_desc = DOMINANT[engine]
    if args.span_timing:
        fr.time_kernels(getattr(N, dom_kt))
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
    if pipe is not None and getattr(pipe, "xs", None) is not None:
        torch.cuda.current_stream().wait_stream(pipe.xs)  # the last frames' exchange and decode
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / args.steps
    span_ms, span_n = fr.kernel_time(getattr(N, dom_kt)) if args.span_timing else (None, 0)
    fr.time_kernels(0)
    # The dominant kernel alone: with frames in flight a launch's events also span the time it
    # queues behind other frames' kernels, so its duration is timed again over args.iso frames
    # launched back to back on one context and stream (consecutive launches serialise; rocprof's
    # trace of the same run shows these as the last frames: scripts/pmc_summary.py "isolated")
    dom_ms, dom_n = isolated_kernel_time(fr, getattr(N, dom_kt), args.iso) if args.iso > 0 else (None, 0)

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
        k_s = kern_ms / 1e3
        hbm_ach = px_rank * bytes_px / k_s / 1e9
        wkey = f"{args.scene}-{W}x{H}-d{args.depth}-{args.order}-{args.precision}-n{world}" + (
            f"-spp{args.spp}" if args.spp > 1 else "")
        prof = profile_for(wkey)
        # Roofline of the dominant kernel: its executed binary64 work per launch (the FP64
        # wave-instructions the committed rocprofv3 PMC profile of this workload counts for it,
        # x 64 lanes; counts do not depend on timing) over its average launch duration measured
        # live right after the timed region (HIP events on its own stream, --iso frames launched
        # back to back).  Peak: 39.3 T lane-ops/s
        # (78.6 TFLOP/s FP64 vector counting an FMA as 2; a wave64 FP64 op issues over 4 cycles).
        roof = {"bound": "valu", "kernel": dom_label.split("#")[0], "what": dom_desc, "peak": PEAK_FP64_VALU_TOPS,
                "unit": "TFLOP/s", "achieved": None, "frac": None, "traffic": None,
                "launch_ms_live": round(dom_ms, 4) if dom_ms else None, "launches_timed": dom_n,
                "launch_span_ms_in_flight": round(span_ms, 4) if span_ms else None}
        frame_exec = valu_busy = traffic_frame = traffic_frame_low = None
        if prof:
            d, path = prof
            kd = d.get("kernels", {}).get(dom_label, {})
            f64 = f64_insts(kd.get("counters", {}))
            if f64 and dom_ms:
                ach = f64 * 64 / (dom_ms / 1e3) / 1e12
                roof.update(achieved=round(ach, 3), frac=round(ach / PEAK_FP64_VALU_TOPS, 4),
                            f64_wave_insts_per_launch=round(f64))
                # all VALU issue (binary64 4 cycles per wave instruction, binary32 / integer 2) over the
                # 1024 SIMDs' cycles: the binding roofline once the filters run in binary32
                valu = kd.get("counters", {}).get("SQ_INSTS_VALU")
                if valu:
                    roof["valu_issue_frac"] = round((4 * f64 + 2 * (valu - f64)) / (1024 * 2.4e9 * dom_ms / 1e3), 4)
                    roof["valu_wave_insts_per_launch"] = round(valu)
            kc = kd.get("counters", {})
            if "FETCH_SIZE" in kc and "WRITE_SIZE" in kc:  # KiB; reads between FETCH x1 (gathers) and x2 (streams)
                roof["traffic"] = round((2 * kc["FETCH_SIZE"] + kc["WRITE_SIZE"]) * 1024)
                roof["traffic_low"] = round((kc["FETCH_SIZE"] + kc["WRITE_SIZE"]) * 1024)
            if kd.get("isolated_avg_ns"):
                roof["launch_ms_rocprof"] = round(kd["isolated_avg_ns"] / 1e6, 4)
            if kd.get("avg_ns"):
                roof["launch_ms_rocprof_in_flight"] = round(kd["avg_ns"] / 1e6, 4)
            roof["profile"] = path
            c = d.get("counters", {})
            per = d.get("spp", 1)  # a supersampled profile's unit is one sample pass: spp per frame
            f64f = f64_insts(c) * per
            if f64f and c.get("SQ_INSTS_VALU"):
                frame_exec = f64f * 64 / k_s / (PEAK_FP64_VALU_TOPS * 1e12)
                valu_busy = (4 * f64f + 2 * (c["SQ_INSTS_VALU"] * per - f64f)) / (1024 * 2.4e9 * k_s)
            if d.get("hbm_bytes_per_launch") is not None:
                traffic_frame = d["hbm_bytes_per_launch"] * per
            if d.get("hbm_bytes_per_launch_low") is not None:
                traffic_frame_low = d["hbm_bytes_per_launch_low"] * per
        roof["frame_f64_issue_frac"] = round(frame_exec, 4) if frame_exec is not None else None
        roof["frame_valu_busy_frac"] = round(valu_busy, 4) if valu_busy is not None else None
        roof["ref_work_tops"] = round(ops_rank / k_s / 1e12, 3)
        roof["note"] = ("FP64 VALU roofline (binding; MFMA does not apply, HBM does not bind): achieved = "
                        "the dominant kernel's executed FP64 wave-instructions per launch (rocprofv3 PMC, "
                        "profile named) x 64 lanes / its average launch duration measured live with HIP events "
                        f"on its stream over {args.iso} frames launched back to back after the timed region (the "
                        "timed region itself carries no kernel events; with --span-timing, launch_span_ms_in_flight "
                        f"= the same launches timed among {inflight} frames in flight, queueing included); "
                        "launch_ms_rocprof = rocprofv3's average "
                        "duration of the same launches; traffic = that kernel's HBM bytes per launch, reads counted "
                        "as FETCH_SIZE x2 (upper bound: exact for coalesced streams) + WRITE_SIZE, traffic_low with "
                        "FETCH_SIZE x1 (exact for 8-64 B gathers; scripts/hbm_calib.hip). "
                        "valu_issue_frac: the same kernel's VALU issue cycles (FP64 wave-instructions x 4, other VALU x 2) / "
                        "(1024 SIMDs x 2.4 GHz x launch time) - the beam and BVH filters run in binary32, so the FP64 fraction "
                        "alone understates how busy the VALU is. frame_f64_issue_frac / frame_valu_busy_frac: "
                        "all of a frame's kernels over the GPU time per frame. ref_work_tops: the reference's "
                        "brute-force binary64 op count per frame (SURVEY.md 8d) / GPU time per frame, in T op/s "
                        "(culling skips most of it: not a roofline)")
        line = {
            "metric": "Mpixels/sec at 4096x4096, recursion depth 5 (frame rendered into HBM, gathered to rank 0)",
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_frames": settle_frames,
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
                       "engine": engine,
                       "stream_priorities": [st.priority for st in fr.streams] if fr.streams else None,
                       "parallelism": f"rows{world - 1 if assemble else world}" + (f"+rccl_{args.gather}_gather" if world > 1 else "")
                       + ("+rank0_assembles" if assemble else ""),
                       "world_size": world, "rccl_ranks": dist.get_world_size() if world > 1 else 1,
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4),
                       "spheres": counts["spheres"], "triangles": counts["triangles"], "planes": counts["planes"],
                       "lights": counts["lights"]},
            "roofline": roof,
            "roofline_hbm": {"bound": "hbm", "achieved": round(hbm_ach, 3), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(hbm_ach / PEAK_HBM_GBS, 6), "traffic": traffic_frame,
                             "traffic_low": traffic_frame_low,
                             "note": "algorithmic bytes: the framebuffer store (12 B/px f32, 24 f64) per GPU time per "
                                     "frame; traffic = measured HBM bytes per frame launch (PMC; reads as FETCH_SIZE x2, the "
                                     "upper bound), traffic_low = the same with FETCH_SIZE x1 (lower bound; "
                                     "profiles/r04_hbm_calib.txt)"},
            "kernel_ms": round(kern_ms, 4),
            "kernel_ms_max_rank": round(kern_ms_max, 4),
            "kernel_mpx_s": round(px_rank / k_s / 1e6, 3),
            "ops_per_frame": ops_total,
        }
        if checked is not None:
            line["self_check"] = checked
        if world == 1 and not args.no_setup:
            line["setup"] = setup_costs(N, scene, W, H, args, fr)
        if world == 1 and not args.no_boundary:
            line.update(boundary_legs(N, scene, W, H, args))
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene, W, H, args.depth, args.cpu_seconds, args.spp, args.seed)
        print(json.dumps(line), flush=True)
    fr.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def isolated_kernel_time(fr, kernel, frames):
    """Average duration of `kernel` (RT_KT_*) over `frames` frames launched back to back on the
    first slot's context and stream (one frame in flight: each launch runs alone)."""
    import torch
    fr.time_kernels(kernel)
    for _ in range(frames):
        fr.launch_on(0)
    torch.cuda.synchronize()
    ms, n = fr.kernel_time(kernel)
    fr.time_kernels(0)
    return ms, n


def self_check(fr, pipe, scene, args, rank, world, local):
    """Before timing: a small check frame through this rank's render and the same compact gather
    the timed loop uses; rank 0 compares each reassembled frame bit for bit with a one-shard
    render of the frame (dist.verify_compact_gather).  The check frames share the frame size
    (the gather's buffers are sized for it) but run the scene at depth 1 and 2."""
    import ctypes

    import torch

    from eraytracer_amd import _native as N
    from eraytracer_amd.dist import verify_compact_gather
    L = N.lib()
    depths = [1, 2]

    def make_slab(i):
        if not fr.renders:  # an assembling rank 0
            return None
        slab = fr.slabs[0]
        N.check(L.rt_launch_spp(fr._ps[0], fr.w, fr.h, depths[i], fr.rb, fr.shard, fr.nshards, fr.prec, fr.order,
                                fr.spp, fr.seed, slab.data_ptr(), None, torch.cuda.current_stream().cuda_stream))
        return slab

    def reference(i):
        el = N.marshal(scene)
        p = ctypes.c_void_p()
        N.check(L.rt_prepare(el, len(el), local, ctypes.byref(p)))
        try:
            out = torch.empty((fr.h, fr.w, 3), dtype=fr.dtype, device=fr.device)
            N.check(L.rt_launch_spp(p, fr.w, fr.h, depths[i], fr.rb, 0, 1, fr.prec, fr.order, fr.spp, fr.seed,
                                    out.data_ptr(), None, torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            return out
        finally:
            L.rt_release(p)

    n = verify_compact_gather(pipe, make_slab, reference, rank, nframes=len(depths), shard=fr.shard)
    torch.cuda.synchronize()
    return {"frames": n, "equal_bitwise": True, "what": "compact-gathered frames == one-shard rt_launch frames"} \
        if rank == 0 else None


def setup_costs(N, scene, W, H, args, fr):
    """What the headline amortises (it renders one fixed scene and camera, prepared before the timed
    region): the reference's unit of work is one cold raytrace/5 call (raytracer.erl:695-705,
    :723-733).  All figures in milliseconds:
      compile_ms             rt_prepare: host compile_scene (tables, occluder masks, BVH) + upload, a fresh
                             context each time (median of 5, host wall clock)
      pmask_ms               k_pmask, the primary rays' candidate masks of a new (scene, camera, frame
                             geometry) on a fresh context (HIP events on its stream; 0 when the engine has none)
      first_frame_ms         that context's first frame: work-space allocation + k_pmask + the frame (wall)
      single_frame_kernel_ms one frame, nothing else in flight, on a warm context (median of 10, HIP events)
      new_scene_frame_ms     rt_update_scene with one sphere moved + the frame, on a warm context, to the
                             end of the frame (host wall clock, mean of 20 steps; scene_update_ms: the update alone)
      cold_*                 a child process started before any GPU call: hip_init_ms (runtime and device
                             initialisation), cold_boundary_ms (its first rt_render: context, compile, upload,
                             work space, masks, frame, copy to pageable host memory; C-side total_ms) and
                             warm_boundary_ms (its second, identical call)"""
    import ctypes
    import statistics

    import torch
    L = N.lib()
    el = N.marshal(scene)
    dev = torch.cuda.current_device()
    out = {}
    ts, p = [], None
    for i in range(5):
        q = ctypes.c_void_p()
        t0 = time.perf_counter()
        N.check(L.rt_prepare(el, len(el), dev, ctypes.byref(q)), "rt_prepare")
        ts.append((time.perf_counter() - t0) * 1e3)
        if p is not None:
            L.rt_release(p)
        p = q
    out["compile_ms"] = round(statistics.median(ts), 3)
    st = torch.cuda.Stream()
    slab = torch.empty((H, W, 3), dtype=fr.dtype, device="cuda")
    prec, order = fr.prec, fr.order

    def frame(p_):
        N.check(L.rt_launch_spp(p_, W, H, args.depth, args.row_block, 0, 1, prec, order, args.spp, args.seed,
                                slab.data_ptr(), None, st.cuda_stream), "rt_launch_spp")
    try:
        N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, 0), "rt_configure")
        N.check(L.rt_configure(p, N.RT_CFG_KERNEL_TIMING, N.RT_KT_PMASK), "rt_configure")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frame(p)
        st.synchronize()
        out["first_frame_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        ms, n = ctypes.c_double(0), ctypes.c_uint64(0)
        N.check(L.rt_kernel_time(p, N.RT_KT_PMASK, ctypes.byref(ms), ctypes.byref(n), 1), "rt_kernel_time")
        out["pmask_ms"] = round(ms.value / n.value, 4) if n.value else 0.0
        N.check(L.rt_configure(p, N.RT_CFG_KERNEL_TIMING, 0), "rt_configure")
        ks = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            frame(p)
            e1.record(st)
            st.synchronize()
            ks.append(e0.elapsed_time(e1))
        out["single_frame_kernel_ms"] = round(statistics.median(ks), 4)
        sph = [i for i in range(len(el)) if el[i].kind == N.RT_SPHERE]
        if sph:
            k = sph[0]
            x0 = el[k].u.sphere.center.x
            tu, tf = [], []
            for s in range(20):
                el[k].u.sphere.center.x = x0 + (s + 1) * 2.0 ** -10  # one sphere moved per step
                el[k].canon = -1
                st.synchronize()
                t0 = time.perf_counter()
                N.check(L.rt_update_scene(p, el, len(el)), "rt_update_scene")
                t1 = time.perf_counter()
                frame(p)
                st.synchronize()
                t2 = time.perf_counter()
                tu.append((t1 - t0) * 1e3)
                tf.append((t2 - t0) * 1e3)
            out["new_scene_frame_ms"] = round(statistics.mean(tf), 3)
            out["scene_update_ms"] = round(statistics.mean(tu), 3)
    finally:
        L.rt_release(p)
    out.update(cold_boundary(W, H, args))
    out["note"] = ("the headline renders one scene and camera prepared before the timed region: it excludes "
                   "compile_ms and pmask_ms (paid once per scene / frame geometry) and overlaps frames "
                   "(single_frame_kernel_ms is a frame alone); see setup_costs() in bench.py")
    return out


def cold_boundary(W, H, args):
    """The first rt_render of a process (a child started before any GPU call; see setup_costs)."""
    code = (
        "import json, sys, time\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from eraytracer_amd import _native as N, scenes\n"
        "from eraytracer_amd.raytracer import render\n"
        f"sc = scenes.named({args.scene!r})\n"
        "import ctypes\n"
        "t0 = time.perf_counter(); n = ctypes.c_int(0); N.lib().rt_device_count(ctypes.byref(n))\n"
        "hip = (time.perf_counter() - t0) * 1e3\n"
        "r = {'hip_init_ms': round(hip, 3)}\n"
        "for k in ('cold_boundary_ms', 'warm_boundary_ms'):\n"
        "    st = {}\n"
        f"    render({W}, {H}, sc, {args.depth}, precision={args.precision!r}, order={args.order!r}, stats=st, "
        f"spp={args.spp}, seed={args.seed})\n"
        "    r[k] = round(st['total_ms'], 3)\n"
        "print(json.dumps(r))\n")
    try:
        res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        return json.loads(res.stdout.strip().splitlines()[-1]) if res.returncode == 0 else {
            "cold_error": (res.stderr or res.stdout)[-300:]}
    except Exception as e:  # the setup leg is a report: a failure is recorded, not fatal
        return {"cold_error": repr(e)[-300:]}


def boundary_legs(N, scene, W, H, args):
    """The C-ABI boundary the BEAM NIF uses (rt_render: persistent context, row bands whose
    copies overlap the next band's render), timed warm (C-side total_ms, best of 3): into pinned
    memory (rt_host_alloc — what the NIF hands the BEAM as a resource binary) without levels
    (render_binary) and with the primary-hit mask (RT_LEVELS_HIT: render_frame, what the
    strategy funs call), into fresh pageable memory; plus raytrace/5 natively (render + P3 text on
    the GPU + file)."""
    import numpy as np

    from eraytracer_amd.raytracer import render, render_ppm_file
    out = {}
    dt = np.float32 if args.precision == "f32" else np.float64
    frame_px = W * H
    pinned = N.pinned_empty((H, W, 3), dt)
    for name, dst, lv in (("boundary_mpx_s", pinned, False), ("boundary_hit_mask_mpx_s", pinned, "hit"),
                          ("boundary_pageable_mpx_s", None, False)):
        ts = []
        for i in range(4):
            st = {}
            render(W, H, scene, args.depth, precision=args.precision, order=args.order, stats=st, spp=args.spp,
                   seed=args.seed, out=dst, levels=lv)
            if i:
                ts.append(st["total_ms"])
        out[name] = round(frame_px / (min(ts) / 1e3) / 1e6, 3)
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "frame.ppm")
        render_ppm_file(W, H, scene, args.depth, path, spp=args.spp, seed=args.seed)  # warm
        tp = []
        for _ in range(3):
            t1 = time.perf_counter()
            render_ppm_file(W, H, scene, args.depth, path, spp=args.spp, seed=args.seed)
            tp.append(time.perf_counter() - t1)
        out["p3_file_mpx_s"] = round(frame_px / min(tp) / 1e6, 3)
        out["p3_file_bytes"] = os.path.getsize(path)
    return out


if __name__ == "__main__":
    main()
