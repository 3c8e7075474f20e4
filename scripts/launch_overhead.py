"""Host time per frame launch against GPU time per frame, for one rank's shard of an N-way split:
is a small shard's frame bound by the host enqueueing its kernels?  

    [RT_GRAPH=1] python scripts/launch_overhead.py [--world 8] [--inflight 4] [--frames 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="s64")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--frames", type=int, default=400)
    a = ap.parse_args()
    import torch

    from eraytracer_amd import scenes
    from eraytracer_amd.dist import FrameRenderer
    fr = FrameRenderer(scenes.named(a.scene), a.size, a.size, a.depth, rank=0, world=a.world, precision="f32",
                       inflight=a.inflight)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:  # clock ramp
        for _ in range(16):
            fr.launch()
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    fr.fork()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        fr.launch()
    t1 = time.perf_counter()
    fr.join()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"world": a.world, "inflight": a.inflight, "graph": os.environ.get("RT_GRAPH", "0"),
                      "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4"),
                      "host_ms_per_launch": round((t1 - t0) / a.frames * 1e3, 4),
                      "ms_per_frame": round((t2 - t0) / a.frames * 1e3, 4)}), flush=True)
    fr.close()


if __name__ == "__main__":
    main()
