"""Time the compact-gather codec on one GPU (rt_slab_pack per shard, rt_slab_unpack of all
shards) for a frame split N ways, and report the bytes a rank sends compact vs dense.
    python scripts/slab_codec_bench.py [--scene s64] [--size 4096] [--depth 5] [--ns 8]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="s64")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--ns", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    from eraytracer_amd import _native as N
    from eraytracer_amd import scenes
    from eraytracer_amd.dist import SlabCodec
    L = N.lib()
    W = H = a.size
    rb, ns = 16, a.ns
    el = N.marshal(scenes.named(a.scene))
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
    st = torch.cuda.current_stream().cuda_stream
    rows = L.rt_shard_rows(H, rb, ns)
    codec = SlabCodec(W, H, rb, ns, "f32")
    slabs = [torch.empty((rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(ns)]
    hdrs = [torch.empty(codec.header_bytes, dtype=torch.uint8, device="cuda") for _ in range(ns)]
    vals = [torch.empty(rows * W * 3, dtype=torch.float32, device="cuda") for _ in range(ns)]
    for s in range(ns):
        N.check(L.rt_launch(p, W, H, a.depth, rb, s, ns, N.RT_OUT_F32, N.RT_ORDER_EXACT, slabs[s].data_ptr(), None, st))
    frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(3):
        codec.pack(slabs[1], 1, hdrs[1], vals[1])
    ev[0].record()
    for _ in range(a.reps):
        codec.pack(slabs[1], 1, hdrs[1], vals[1])
    ev[1].record()
    for s in range(ns):
        codec.pack(slabs[s], s, hdrs[s], vals[s])
    torch.cuda.synchronize()
    codec.unpack(hdrs, vals, frame)
    ev[1].synchronize()
    t_pack = ev[0].elapsed_time(ev[1]) / a.reps
    ev[0].record()
    for _ in range(a.reps):
        codec.unpack(hdrs, vals, frame)
    ev[2].record()
    torch.cuda.synchronize()
    t_unpack = ev[0].elapsed_time(ev[2]) / a.reps
    counts = [int(h[:8].cpu().view(torch.int64)[0]) for h in hdrs]
    dense = rows * W * 12
    compact = [codec.header_bytes + c * 12 for c in counts]
    print(json.dumps({"scene": a.scene, "size": W, "nshards": ns, "pack_ms": round(t_pack, 4),
                      "unpack_ms": round(t_unpack, 4), "dense_bytes_per_rank": dense,
                      "compact_bytes_per_rank": compact, "ratio": round(sum(compact) / (ns * dense), 4)}))
    L.rt_release(p)


if __name__ == "__main__":
    main()
