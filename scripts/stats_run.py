"""Diagnostic: per-frame event counts from an RT_STATS build (RT_LIB_PATH=...variants/librtmi355x_stats.so)."""
import ctypes, json, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eraytracer_amd import _native as N, scenes
from eraytracer_amd.raytracer import render
NAMES = ["waves", "near_pre", "near_pre_cand", "near_gen", "near_gen_cand", "shadow", "shadow_cand", "shadow_iter",
         "shade", "shadow_cone_on", "beam_on", "shadow_lanes", "near_lanes", "bvh_scans", "bvh_iter", "bvh_leaf",
         "bvh_iter_lanes", "bvh_leaf_lanes"]
L = N.lib()
L.rt_debug_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
buf = (ctypes.c_ulonglong * len(NAMES))()
CASES = [("s64", 4096, 5, "exact"), ("default", 1024, 5, "exact"), ("s256", 1024, 8, "exact")]
if len(sys.argv) > 1:  # name:size:depth ...
    CASES = [(a.split(":")[0], int(a.split(":")[1]), int(a.split(":")[2]), "exact") for a in sys.argv[1:]]
for name, size, depth, order in CASES:
    L.rt_debug_stats(buf, len(NAMES), 1)
    render(size, size, scenes.named(name), depth, order=order, precision="f32")
    L.rt_debug_stats(buf, len(NAMES), 1)
    d = dict(zip(NAMES, list(buf)))
    w = d["waves"]
    print(name, size, depth, json.dumps({k: round(v / w, 3) for k, v in d.items()}))
