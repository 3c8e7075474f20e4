"""FrameRenderer(inflight=k) timed like scripts/frame_overlap.py (A/B of the two harnesses)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from eraytracer_amd import scenes  # noqa: E402
from eraytracer_amd.dist import FrameRenderer  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
levels_first = len(sys.argv) > 2 and sys.argv[2] == "lv"
if levels_first:
    lv = FrameRenderer(scenes.s64(), 4096, 4096, 5, levels=True)
    lv.launch()
    torch.cuda.synchronize()
    lv.close()
    del lv
fr = FrameRenderer(scenes.s64(), 4096, 4096, 5, inflight=k)
for _ in range(2 * k):
    fr.launch()
torch.cuda.synchronize()
for trial in range(3):
    t0 = time.perf_counter()
    for _ in range(40):
        fr.launch()
    torch.cuda.synchronize()
    print(k, "lv" if levels_first else "", trial, round((time.perf_counter() - t0) / 40 * 1e3, 4), flush=True)
