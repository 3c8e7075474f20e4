"""The compact gather's codec alone (rt_slab_pack of one rank's shard, rt_slab_unpack of all N shards into
the frame), on real shards of an S64 frame, against the HBM roofline:

    python scripts/slab_codec_bench.py [--size 4096] [--world 8] [--reps 50]

Algorithmic bytes: pack = the shard read once (12 B/px) + the header and the non-background values written;
unpack = every header and value read once + the frame written once (12 B/px).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="s64")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch

    from eraytracer_amd import scenes
    from eraytracer_amd.dist import FrameRenderer, SlabCodec
    W = H = a.size
    codec = SlabCodec(W, H, 16, a.world, "f32")
    slabs, headers, values = [], [], []
    for s in range(a.world):
        fr = FrameRenderer(scenes.named(a.scene), W, H, a.depth, rank=s, world=a.world, precision="f32")
        fr.launch()
        torch.cuda.synchronize()
        slabs.append(fr.slab.clone())
        fr.close()
        headers.append(torch.empty(codec.header_bytes, dtype=torch.uint8, device="cuda"))
        values.append(torch.empty(slabs[-1].numel(), dtype=torch.float32, device="cuda"))
        codec.pack(slabs[s], s, headers[s], values[s])
    torch.cuda.synchronize()
    frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        for _ in range(5):
            fn()
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    pack_ms = timed(lambda: codec.pack(slabs[0], 0, headers[0], values[0]))
    unpack_ms = timed(lambda: codec.unpack(headers, values, frame))
    counts = [int(h[:8].view(torch.int64).item()) for h in headers]
    shard_px = slabs[0].numel() // 3
    pack_bytes = shard_px * 12 + codec.header_bytes + counts[0] * 12
    unpack_bytes = a.world * codec.header_bytes + sum(counts) * 12 + W * H * 12
    print(json.dumps({"size": a.size, "world": a.world, "shard_px": shard_px, "nonzero_px": counts,
                      "header_bytes": codec.header_bytes,
                      "pack_ms": round(pack_ms, 4), "pack_gbs": round(pack_bytes / pack_ms / 1e6, 1),
                      "unpack_ms": round(unpack_ms, 4), "unpack_gbs": round(unpack_bytes / unpack_ms / 1e6, 1),
                      "hbm_peak_gbs": 8000.0}), flush=True)


if __name__ == "__main__":
    main()
