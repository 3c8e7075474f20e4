"""Where the end-to-end P3 time goes (bench.py's p3_file_mpx_s): rt_render_ppm_file
repeated into a disk-backed temp dir and into /dev/shm, beside a plain write of the
same byte count to each, so the file system's share can be read off directly."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from eraytracer_amd.raytracer import render_ppm_file  # noqa: E402
from eraytracer_amd.scenes import named  # noqa: E402

W = H = 4096
scene = named("s64")
for root in (tempfile.gettempdir(), "/dev/shm"):
    with tempfile.TemporaryDirectory(dir=root) as td:
        path = os.path.join(td, "frame.ppm")
        ts = []
        for _ in range(4):
            t0 = time.perf_counter()
            render_ppm_file(W, H, scene, 5, path)
            ts.append(time.perf_counter() - t0)
        size = os.path.getsize(path)
        blob = os.urandom(1 << 20) * (size >> 20)
        t0 = time.perf_counter()
        with open(os.path.join(td, "plain.bin"), "wb") as f:
            f.write(blob)
        tw = time.perf_counter() - t0
        print(f"{root}: render_ppm_file s = {[round(t, 4) for t in ts]} "
              f"({W * H / min(ts) / 1e6:.1f} Mpx/s best); plain write of {len(blob)} B = {tw:.4f} s", flush=True)
