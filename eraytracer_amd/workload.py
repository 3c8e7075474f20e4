"""Algorithmic work per frame, for the roofline figures.

The path is FP64-VALU bound: it stores 12 B (f32) or 24 B (f64) per pixel and does
~1e3-2e4 binary64 operations per pixel.  Work is counted from the REFERENCE algorithm
(memoised reflection, full nearest scans for shadows), not from what the kernel happens
to execute (it skips work with early-outs and tabled constants), so the same frame
always has the same count.  Weights, each +, -, *, /, sqrt, compare or pow = 1 op:

    per pixel                    31   primary ray (ray_through_pixel/3, raytracer.erl:483-511)
    per object test in a scan    sphere 20, triangle 48, plane 15   (:364-480)
    per nearest hit              27   hit point + normal
    per hit                      18   bounce + reflection scale     (:216-224, :568-573)
    per hit per light            77 + one shadow scan              (:225-247, :256-297)

The per-pixel count depends only on how many levels of its reflection chain hit, which
the kernel reports (rt_launch's d_levels) and the oracle reproduces exactly.
"""
from __future__ import annotations

import numpy as np

from .records import tag

W_PIXEL, W_SPH, W_TRI, W_PL, W_NEAR_HIT, W_HIT, W_HIT_LIGHT = 31, 20, 48, 15, 27, 18, 77


def scene_counts(scene) -> dict:
    c = {"spheres": 0, "triangles": 0, "planes": 0, "lights": 0}
    for t in scene[1:]:
        k = tag(t)
        if k == "sphere":
            c["spheres"] += 1
        elif k == "triangle":
            c["triangles"] += 1
        elif k == "plane":
            c["planes"] += 1
        elif k == "point_light":
            c["lights"] += 1
    return c


def scan_cost(counts: dict) -> int:
    return W_SPH * counts["spheres"] + W_TRI * counts["triangles"] + W_PL * counts["planes"]


def ops_from_levels(levels_hist, depth: int, counts: dict) -> int:
    """Total algorithmic ops for a frame whose per-pixel hit-level counts have histogram
    ``levels_hist`` (levels_hist[h] = number of pixels whose chain hit h times)."""
    L = counts["lights"]
    sc = scan_cost(counts)
    total = 0
    for h, npx in enumerate(np.asarray(levels_hist, dtype=np.int64).tolist()):
        if npx == 0:
            continue
        scans = h + (1 if (h < depth and (h == 0 or L > 0)) else 0)
        per_px = W_PIXEL + scans * sc + h * (W_NEAR_HIT + W_HIT + L * (W_HIT_LIGHT + sc))
        total += npx * per_px
    return total


def levels_histogram(levels, depth: int) -> np.ndarray:
    return np.bincount(np.asarray(levels).ravel().astype(np.int64), minlength=depth + 1)
