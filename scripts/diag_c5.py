"""Diagnostic: one config-5 style rt_render call (S256 d8 4096^2) with the options given."""
import sys
import time

sys.path.insert(0, ".")
from eraytracer_amd import scenes  # noqa: E402
from eraytracer_amd.raytracer import render  # noqa: E402

levels, spp = sys.argv[1] == "1", int(sys.argv[2])
t = time.perf_counter()
r = render(4096, 4096, scenes.s256(), 8, levels=levels, spp=spp, seed=0x5EED0005)
print("ok", levels, spp, round(time.perf_counter() - t, 2), flush=True)
