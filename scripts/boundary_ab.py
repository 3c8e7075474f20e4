"""A/B of the rt_render boundary (S64 4096^2 d5 f32): pinned and pageable destinations, best of
5 warm calls; plus the raw pinned D2H rate of one 201 MB frame (1 and 2 DMA queues)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from eraytracer_amd import _native as N, scenes  # noqa: E402
from eraytracer_amd.raytracer import render  # noqa: E402

W = H = 4096
sc = scenes.s64()
out = N.pinned_empty((H, W, 3), np.float32)
res = {"band_mb": os.environ.get("RT_BAND_MB", "24"), "copy_streams": os.environ.get("RT_COPY_STREAMS", "2")}
for name, dst in (("pinned", out), ("pageable", None)):
    ts, ks = [], []
    for i in range(6):
        st = {}
        t0 = time.perf_counter()
        render(W, H, sc, 5, precision="f32", out=dst, stats=st)
        if i:
            ts.append(time.perf_counter() - t0)
            ks.append(st["kernel_ms"])
    res[name + "_ms"] = round(min(ts) * 1e3, 3)
    res[name + "_mpx_s"] = round(W * H / min(ts) / 1e6, 1)
    res[name + "_kernel_ms"] = round(min(ks), 3)
if len(sys.argv) > 1 and sys.argv[1] == "raw":
    d = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
    h = torch.from_numpy(out.reshape(-1))
    for nq in (1, 2, 4):
        ss = [torch.cuda.Stream() for _ in range(nq)]
        best = 1e9
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ch = d.numel() // nq
            for q in range(nq):
                with torch.cuda.stream(ss[q]):
                    h[q * ch:(q + 1) * ch].copy_(d[q * ch:(q + 1) * ch], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        res[f"raw_d2h_gbs_{nq}q"] = round(d.numel() * 4 / best / 1e9, 1)
print(json.dumps(res))
