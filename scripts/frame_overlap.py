"""Two frames in flight: alternate two rt_prepared contexts (own work spaces) on two streams,
so frame i+1's head overlaps frame i's latency-bound tail.  Per-frame time vs one context.
    RT_LIT_STREAM=0|1 python scripts/frame_overlap.py [--ns 1]"""
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--inflight", type=int, default=2)
    a = ap.parse_args()
    import torch

    from eraytracer_amd import _native as N
    from eraytracer_amd import scenes
    L = N.lib()
    W = H = a.size
    el = N.marshal(scenes.named(a.scene))
    k = a.inflight
    ps = []
    for _ in range(k):
        p = ctypes.c_void_p()
        N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
        ps.append(p)
    streams = [torch.cuda.Stream() for _ in range(k)]
    res = {"lit_stream": os.environ.get("RT_LIT_STREAM", "1"), "queues": os.environ.get("GPU_MAX_HW_QUEUES", "4"),
           "inflight": k}
    for ns in (1, 2, 4, 8):
        rows = L.rt_shard_rows(H, 16, ns)
        slabs = [torch.empty((rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(k)]
        sh = 1 % ns

        def frame(i):
            j = i % k
            N.check(L.rt_launch(ps[j], W, H, a.depth, 16, sh, ns, N.RT_OUT_F32, N.RT_ORDER_EXACT, slabs[j].data_ptr(),
                                None, streams[j].cuda_stream))
        for i in range(2 * k):
            frame(i)
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        for i in range(a.reps):
            frame(i)
        torch.cuda.synchronize()
        res[f"n{ns}_ms"] = round((time.perf_counter() - t0) / a.reps * 1e3, 4)
    print(json.dumps(res))
    for p in ps:
        L.rt_release(p)


if __name__ == "__main__":
    main()
