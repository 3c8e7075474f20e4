"""The N = 8 step's floor, measured on ONE GPU with the current library.

At N = 8 (bench.py --gpus 8: rows dealt in 16-row blocks, 3 frames in flight per rank, the compact
gather to rank 0, dist.CompactGather) a step is bounded by the slowest of:
  * a rank's render of its shard with frames in flight, plus rt_slab_pack of it (every rank);
  * rank 0: its own shard's render + pack with rt_slab_unpack of all 8 shards beside it (the decode
    runs on the exchange's side stream, behind the render);
  * rank 0's inbound transfer: the 7 peers' compact values over their xGMI links (bytes counted from
    the packed headers; the time at the links' peak is a lower bound).
Each is measured here on one device (no RCCL: the transfer is counted, not run) and the projected
step compared with the N = 1 frame (bench.py's configuration: 4 frames in flight) and north_star's
">= 6x further at 8 GPUs".

    python scripts/n8_floor.py [--scene s64] [--size 4096] [--depth 5] [--reps 40]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")  # as bench.py (before the HIP runtime initialises)

XGMI_LINK_GBS = 153.0  # one MI355X xGMI link, one direction (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="s64")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--inflight", type=int, default=3, help="frames in flight per rank (bench.py at N > 1: 3)")
    ap.add_argument("--sweep", default="2,3,4,6,8", help="frames in flight tried for shard 0")
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    import torch

    from eraytracer_amd import scenes
    from eraytracer_amd.dist import FrameRenderer, SlabCodec
    W = H = a.size
    scene = scenes.named(a.scene)
    ns = a.world
    res = {"scene": a.scene, "size": a.size, "depth": a.depth, "world": ns,
           "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}

    def per_frame(fr, extra=None, reps=a.reps):
        """ms per frame with fr's frames in flight (fr.launch cycles its slots); extra(i) runs after
        each frame's launch on that frame's stream (a pack) or elsewhere (a decode)."""
        for i in range(2 * len(fr._ps)):
            fr.launch()
            if extra:
                extra(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fr.fork()
        for i in range(reps):
            fr.launch()
            if extra:
                extra(i)
        fr.join()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    # N = 1 as bench.py runs it (4 in flight, auto priorities), after a second of frames (clock ramp)
    fr1 = FrameRenderer(scene, W, H, a.depth, precision="f32", inflight=4)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for _ in range(8):
            fr1.launch()
        torch.cuda.synchronize()
    res["n1_frame_ms"] = round(per_frame(fr1), 4)
    fr1.close()
    # shard 0 of ns with k frames in flight (more frames hide more of a small shard's latency-bound tail)
    sweep = {}
    for k in [int(x) for x in a.sweep.split(",")]:
        fk = FrameRenderer(scene, W, H, a.depth, rank=0, world=ns, precision="f32", inflight=k)
        sweep[k] = round(per_frame(fk), 4)
        fk.close()
    res["shard0_frame_ms_by_inflight"] = sweep

    codec = SlabCodec(W, H, 16, ns, "f32")
    rows = fr_rows = None
    shard_ms, shard_pack_ms, values_bytes = [], [], []
    headers, values = [], []
    for s in range(ns):
        fr = FrameRenderer(scene, W, H, a.depth, rank=s, world=ns, precision="f32", inflight=a.inflight)
        fr_rows = fr.rows
        shard_ms.append(round(per_frame(fr), 4))
        # one header / values buffer per slot: packs of frames in flight must not share them (a
        # header packed by two streams at once is inconsistent, as dist.CompactGather's ring avoids)
        hdrs = [torch.empty(codec.header_bytes, dtype=torch.uint8, device="cuda") for _ in fr._ps]
        vals = [torch.empty(fr.rows * W * 3, dtype=torch.float32, device="cuda") for _ in fr._ps]

        def pack(i, fr=fr, hdrs=hdrs, vals=vals, s=s):
            j = (fr.n - 1) % len(fr._ps)  # the slot fr.launch() just used
            with torch.cuda.stream(fr.stream):
                codec.pack(fr.slab, s, hdrs[j], vals[j])
        shard_pack_ms.append(round(per_frame(fr, pack), 4))
        torch.cuda.synchronize()
        hdr, val = hdrs[0], vals[0]
        cnt = int(hdr[:8].view(torch.int64).item())
        values_bytes.append(cnt * 3 * 4)
        headers.append(hdr.clone())
        values.append(val.clone())
        if s == 0:
            pack_bufs = (hdrs, vals)
            # the pack alone (HIP events, back to back on one stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                codec.pack(fr.slabs[0], 0, hdr, val)
            e1.record()
            torch.cuda.synchronize()
            res["pack_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
            fr0 = fr
        else:
            fr.close()
    rows = fr_rows
    res["shard_rows"] = rows
    res["shard_frame_ms"] = shard_ms
    res["shard_frame_pack_ms"] = shard_pack_ms
    frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        codec.unpack(headers, values, frame)
    e1.record()
    torch.cuda.synchronize()
    res["unpack8_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
    # rank 0: its shard rendered and packed with frames in flight, all 8 shards decoded beside it
    xs = torch.cuda.Stream()

    def pack_and_decode(i):
        j = (fr0.n - 1) % len(fr0._ps)
        with torch.cuda.stream(fr0.stream):  # (its own slot's buffers; the decode reads the copies)
            codec.pack(fr0.slab, 0, pack_bufs[0][j], pack_bufs[1][j])
        ev = torch.cuda.Event()
        ev.record(fr0.stream)
        xs.wait_event(ev)
        with torch.cuda.stream(xs):
            codec.unpack(headers, values, frame)
    res["rank0_frame_pack_decode_ms"] = round(per_frame(fr0, pack_and_decode), 4)
    fr0.close()
    # rank 0's inbound bytes per frame: the 7 peers' values + headers
    inbound = sum(values_bytes[1:]) + (ns - 1) * codec.header_bytes
    res["values_bytes_per_shard"] = values_bytes
    res["rank0_inbound_bytes"] = inbound
    res["transfer_ms_at_link_peak"] = round(max(values_bytes[1:]) / (XGMI_LINK_GBS * 1e9) * 1e3, 4)
    floor = max(res["rank0_frame_pack_decode_ms"], max(shard_pack_ms), res["transfer_ms_at_link_peak"])
    res["projected_step_ms"] = round(floor, 4)
    res["bound_by"] = ("rank 0 render + pack + decode" if floor == res["rank0_frame_pack_decode_ms"] else
                       "a rank's render + pack" if floor == max(shard_pack_ms) else "rank 0's inbound links")
    res["projected_speedup_vs_n1"] = round(res["n1_frame_ms"] / floor, 2)
    res["north_star_speedup"] = 6.0
    res["inflight"] = a.inflight
    # the same shards with an assembling rank 0 (bench.py --rank0 assemble: world + 1 GPUs, rank 0
    # renders nothing and only decodes): the slowest rendering rank, or rank 0's decode
    asm = max(max(shard_pack_ms), res["unpack8_ms"], res["transfer_ms_at_link_peak"])
    res["assembler_gpus"] = ns + 1
    res["assembler_projected_step_ms"] = round(asm, 4)
    res["assembler_projected_speedup_vs_n1"] = round(res["n1_frame_ms"] / asm, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
