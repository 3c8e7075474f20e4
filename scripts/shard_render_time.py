"""Per-rank render time of an N-way row split, measured on one GPU: rt_launch of shard 1 of
N (what each rank of `bench.py --gpus N` renders), HIP events on the launch stream.
    RT_LIT_STREAM=0|1 python scripts/shard_render_time.py [--scene s64] [--size 4096] [--depth 5]"""
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
    a = ap.parse_args()
    import torch

    from eraytracer_amd import _native as N
    from eraytracer_amd import scenes
    L = N.lib()
    W = H = a.size
    el = N.marshal(scenes.named(a.scene))
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
    st = torch.cuda.current_stream().cuda_stream
    res = {"scene": a.scene, "size": W, "depth": a.depth, "lit_stream": os.environ.get("RT_LIT_STREAM", "1")}
    for ns in (1, 2, 4, 8):
        rows = L.rt_shard_rows(H, 16, ns)
        slab = torch.empty((rows, W, 3), dtype=torch.float32, device="cuda")
        sh = 1 % ns
        for _ in range(3):
            N.check(L.rt_launch(p, W, H, a.depth, 16, sh, ns, N.RT_OUT_F32, N.RT_ORDER_EXACT, slab.data_ptr(), None, st))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            N.check(L.rt_launch(p, W, H, a.depth, 16, sh, ns, N.RT_OUT_F32, N.RT_ORDER_EXACT, slab.data_ptr(), None, st))
        e1.record()
        torch.cuda.synchronize()
        res[f"n{ns}_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
    print(json.dumps(res))
    L.rt_release(p)


if __name__ == "__main__":
    main()
