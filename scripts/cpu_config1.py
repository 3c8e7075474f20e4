"""BASELINE config 1' on the host: the C oracle (the reference's literal recursion, one thread
per core given) rendering the default scene at 640x480, depth 3 — the stand-in for the BEAM
`concurrent` strategy, which is not installed anywhere here.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eraytracer_amd import _native as N  # noqa: E402
from eraytracer_amd import records  # noqa: E402
from oracle import oracle as O  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else O.host_threads()  # this process's CPU share
O.build()
el = N.marshal(records.scene())
out = {}
for mode, name in ((O.LITERAL, "literal"), (O.MEMO, "memo")):
    O.render(el, 64, 48, 3, mode=mode, threads=threads)
    t0 = time.perf_counter()
    O.render(el, 640, 480, 3, mode=mode, threads=threads)
    dt = time.perf_counter() - t0
    out[name] = {"mpx_s": round(640 * 480 / dt / 1e6, 3), "seconds": round(dt, 3)}
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import host_cpu_info  # noqa: E402
print(json.dumps({"config": "default scene 640x480 depth 3 (BASELINE configs[0])", "threads": threads,
                  "oracle": out, "host": host_cpu_info()}))
