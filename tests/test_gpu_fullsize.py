"""Parity at the BASELINE.json configurations' full sizes (configs 1-5), the general
math:pow/2 path, and the fused wavefront kernels on mixed-object scenes.

Every check: identical per-pixel reflection-chain levels (every hit/miss decision of every
pixel's chain), max per-channel |delta| <= 1e-5 (north_star), and the count of pixels that
are not bit-identical reported and bounded.  The oracle is oracle/rt_oracle.c (memoised mode:
the reflection computed once per hit, bit-identical to the literal recursion,
tests/test_oracle.py::test_literal_equals_memo) on this process's CPU share.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from eraytracer_amd import _native as N
from eraytracer_amd import scenes
from eraytracer_amd.raytracer import render

pytestmark = pytest.mark.gpu
TOL = 1e-5
# Pixels not bit-identical: the oracle calls the host libm's pow (glibc 2.35, as BEAM's
# math:pow/2 does), which is not correctly rounded (its error bound is 0.52 ulp: measured
# here on 2e5 random x^4, x^5, x^20 it differs from the correctly rounded value in ~0.08 % of
# calls); the kernels' integer-exponent pow is correctly rounded (double-double binary powering).
# Measured (round 2): config 1 86 of 307200 pixels, config 2 477 of 2073600, config 3 75 of
# 1048576 sampled, config 5 7 of 24576 sampled; all within 1e-15.  Bound: 0.1 % of the pixels.
BOUND_FRAC = 1e-3
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compare(img, lv, ref, rlv, what, max_nonbitwise):
    np.testing.assert_array_equal(lv, rlv, err_msg=what)
    err = np.abs(img.astype(np.float64) - ref)
    assert np.all(np.isfinite(img))
    assert err.max() <= TOL, f"{what}: max |delta| {err.max()}"
    if img.dtype == np.float64:
        diff = ~np.all(img.view(np.int64) == ref.view(np.int64), axis=-1)
        n = int(diff.sum())
        print(f"{what}: max |delta| {err.max():.3g}, {n} of {diff.size} pixels not bit-identical")
        assert n <= max_nonbitwise, f"{what}: {n} pixels not bit-identical (bound {max_nonbitwise})"


def test_config1_default_640x480_d3(oracle):
    """BASELINE config 1's workload (raytracer:go(640,480) default scene, depth 3), whole frame."""
    scene = scenes.named("default")
    img, lv = render(640, 480, scene, 3, levels=True)
    ref, rlv = oracle.render(N.marshal(scene), 640, 480, 3, mode=oracle.MEMO, levels=True)
    _compare(img, lv, ref, rlv, "config 1", 640 * 480 * BOUND_FRAC)


def test_config2_default_1920x1080_d5(oracle):
    """BASELINE config 2 (default scene, 1920x1080, depth 5), whole frame, f64 and f32."""
    scene = scenes.named("default")
    img, lv = render(1920, 1080, scene, 5, levels=True)
    ref, rlv = oracle.render(N.marshal(scene), 1920, 1080, 5, mode=oracle.MEMO, levels=True)
    _compare(img, lv, ref, rlv, "config 2", 1920 * 1080 * BOUND_FRAC)
    f32 = render(1920, 1080, scene, 5, precision="f32")
    assert np.array_equal(f32, img.astype(np.float32))


def _rows(h, n):
    return sorted({(i * h) // n + (h // n) // 2 for i in range(n)})


def test_config3_s64_4096_d5_256_rows(oracle):
    """BASELINE config 3 (S64, 4096x4096, depth 5): 256 evenly spaced rows of the frame (1 M
    pixels) against the oracle, the rest of the frame through its levels histogram and the
    f32 frame being the f64 frame rounded."""
    scene = scenes.s64()
    W = H = 4096
    img, lv = render(W, H, scene, 5, levels=True)
    rows = _rows(H, 256)
    el = N.marshal(scene)
    ref = np.empty((len(rows), W, 3))
    rlv = np.empty((len(rows), W), np.uint8)
    for i, r in enumerate(rows):
        ref[i], rlv[i] = (a[0] for a in oracle.render(el, W, H, 5, mode=oracle.MEMO, row0=r, nrows=1, levels=True))
    _compare(img[rows], lv[rows], ref, rlv, "config 3 (256 rows)", len(rows) * W * BOUND_FRAC)
    f32 = render(W, H, scene, 5, precision="f32")
    assert np.array_equal(f32, img.astype(np.float32))
    hist = np.bincount(lv.ravel(), minlength=6)
    assert hist[6:].sum() == 0 and hist[0] > 0 and hist[5] > 0


def test_config4_s64_8192_d5_shards(oracle):
    """BASELINE config 4 (S64, 8192x8192, depth 5, rows over 8 GPUs): the 8-way interleaved row
    split through rt_render (8 shards on this device) equals the 1-shard frame bit for bit, and
    512 rows (64 bands of 8 rows spread over the frame: 4.2 M pixels, 6 % of it) equal the oracle
    — identical levels, max |delta| <= 1e-5 on the binary32 frame."""
    scene = scenes.s64()
    W = H = 8192
    one, lv = render(W, H, scene, 5, precision="f32", levels=True)
    eight = N.pinned_empty((H, W, 3), np.float32)
    render(W, H, scene, 5, precision="f32", nshards=8, out=eight)
    assert np.array_equal(one.view(np.int32), eight.view(np.int32))
    del eight
    el = N.marshal(scene)
    bands = _rows(H - 8, 64)
    for i, r in enumerate(bands):
        ref, rlv = oracle.render(el, W, H, 5, mode=oracle.MEMO, row0=r, nrows=8, levels=True)
        _compare(one[r:r + 8], lv[r:r + 8], ref, rlv, f"config 4 rows {r}-{r + 7}", 0)
        if i % 16 == 15:
            print(f"  config 4: {i + 1} of {len(bands)} bands checked", flush=True)


def test_config5_s256_4096_d8_spp16_rows(oracle):
    """BASELINE config 5 (S256, 4096x4096, depth 8, 16 samples per pixel): 6 rows sampled
    across the frame against the oracle's restatement of RT_SUPERSAMPLING."""
    scene = scenes.s256()
    W = H = 4096
    seed = 0x5EED0005
    img, lv = render(W, H, scene, 8, levels=True, spp=16, seed=seed)
    el = N.marshal(scene)
    for r in _rows(H, 6):
        ref, rlv = oracle.render(el, W, H, 8, mode=oracle.MEMO, row0=r, nrows=1, levels=True, spp=16, seed=seed)
        _compare(img[r:r + 1], lv[r:r + 1], ref, rlv, f"config 5 row {r}", max(4, W * BOUND_FRAC))


# (scene, w, h, depth, bound on the pixels not bit-identical): measured round 3 on MI355X
# (default_powers 320x240 d5: 1631, 97x61 d1: 185, mixed 256x192 d5: 1374), bound = x1.5
@pytest.mark.parametrize("name,w,h,d,bound", [("default_powers", 320, 240, 5, 2450), ("default_powers", 97, 61, 1, 280),
                                              ("mixed", 256, 192, 5, 2060)])
def test_general_pow_and_mixed_scenes(oracle, name, w, h, d, bound):
    """Specular powers 0, 0.5, 2.5, 1025 (the general math:pow/2 path, :289, and pow(0,0)=1.0)
    on the fused engine (default scene) and a mixed 58-object scene on the wavefront engine.
    Device pow (~1 ulp) vs host libm differ by an ulp on 2-3 % of the pixels (<= 1e-14): the
    bound is the measured count plus half, the 1e-5 bar does not move."""
    scene = scenes.named(name)
    img, lv = render(w, h, scene, d, levels=True)
    ref, rlv = oracle.render(N.marshal(scene), w, h, d, mode=oracle.MEMO, levels=True)
    _compare(img, lv, ref, rlv, name, bound)


def test_fused_wavefront_kernels_all_paths():
    """k_reflect_shade (frames in flight: no side streams, no levels) in a child process with
    the wavefront engine forced (RT_ENGINE is read once per process): spheres-only, mixed
    triangles/planes, general pow and dense deep levels, each against the oracle and bit
    for bit against the side-stream path (k_light + k_reflect)."""
    code = r"""
import ctypes, numpy as np, torch
from eraytracer_amd import _native as N, scenes
from oracle import oracle as O
L = N.lib()
def frame(sc, w, h, d, side):
    el = N.marshal(sc)
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
    try:
        N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, side))
        img = torch.full((h, w, 3), float('nan'), dtype=torch.float64, device='cuda')
        N.check(L.rt_launch(p, w, h, d, 16, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, img.data_ptr(), None,
                            torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        return img.cpu().numpy()
    finally:
        L.rt_release(p)
# depths 2 .. 8: the inline chain walks (k_reflect_shade's iw) start at depth 3 — there the deepest
# level (2) is never queued, k_items and k_walk are not launched — and from depth 4 leave the sparse
# deep levels to k_walk; 40 lights (more than a record's 32 shadow answers) keep k_walk for every chain
cases = [(n, w, h, d) for n, w, h, d in [('default', 96, 72, 5), ('default_powers', 96, 72, 5), ('mixed', 128, 96, 5),
                                          ('mixed', 64, 48, 2), ('mixed', 128, 96, 3), ('s64', 96, 96, 5),
                                          ('s64', 96, 96, 3), ('s64', 96, 96, 4), ('s256', 64, 48, 8),
                                          ('s256', 64, 48, 3)]]
cases += [('lights40', 64, 48, 3), ('lights40', 64, 48, 4)]
for name, w, h, d in cases:
    sc = scenes.synthetic_scene(24, 0x5EED4040, n_lights=40) if name == 'lights40' else scenes.named(name)
    a, b = frame(sc, w, h, d, 1), frame(sc, w, h, d, 0)
    assert np.array_equal(a.view(np.int64), b.view(np.int64)), name
    ref = O.render(N.marshal(sc), w, h, d, mode=O.MEMO)
    err = np.abs(b - ref).max()
    assert err <= 1e-5, (name, d, err)
print('fused ok')
"""
    env = dict(os.environ, RT_ENGINE="wave", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "fused ok" in r.stdout, r.stdout + r.stderr


_FUSED_FRAME = r"""
import ctypes, numpy as np, torch
from eraytracer_amd import _native as N, scenes
from oracle import oracle as O
L = N.lib()
def frame(sc, w, h, d, side, spp=1, seed=0, shard=0, nshards=1):
    el = N.marshal(sc)
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
    try:
        N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, side))
        rows = L.rt_shard_rows(h, 16, nshards)
        img = torch.full((rows, w, 3), float('nan'), dtype=torch.float64, device='cuda')
        N.check(L.rt_launch_spp(p, w, h, d, 16, shard, nshards, N.RT_OUT_F64, N.RT_ORDER_EXACT, spp, seed,
                                img.data_ptr(), None, torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        return img.cpu().numpy()
    finally:
        L.rt_release(p)
"""


def _child(code, **env):
    e = dict(os.environ, PYTHONPATH=ROOT, **env)
    r = subprocess.run([sys.executable, "-c", _FUSED_FRAME + code], cwd=ROOT, env=e, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout.split(), r.stdout + r.stderr


def test_bvh_forced_on_every_level_and_scene():
    """The per-lane sphere BVH (k_reflect_shade<..., BVH>) forced onto every reflection level of
    scenes it is not chosen for (RT_BVH_MIN=2, RT_BVH_LEVEL=1, read once per process: a child):
    spheres-only S16/S64/S256 and the mixed scene (BVH spheres + scanned triangles and planes).
    Each frame equals the side-stream path (beams only) bit for bit and the oracle within 1e-5."""
    _child(r"""
for name, w, h, d in [('s16', 80, 64, 5), ('s64', 96, 96, 5), ('s256', 64, 48, 8), ('mixed', 128, 96, 5)]:
    sc = scenes.named(name)
    a, b = frame(sc, w, h, d, 1), frame(sc, w, h, d, 0)
    assert np.array_equal(a.view(np.int64), b.view(np.int64)), name
    ref = O.render(N.marshal(sc), w, h, d, mode=O.MEMO)
    assert np.abs(b - ref).max() <= 1e-5, name
print('ok')
""", RT_ENGINE="wave", RT_BVH_MIN="2", RT_BVH_LEVEL="1")


def test_inline_walks_dense_deep_levels():
    """The inline chain walks with dense deep levels (more than DEEP_DENSE_RECORDS level-2 records:
    every level shaded by its own launch, the deepest level's hits shaded where they are found, k_walk
    left with nothing): S256 4096x2048 (about 0.7 M level-2 records) at depths 3, 4 and 6, frames in
    flight vs the side-stream path bit for bit, and rows against the oracle."""
    _child(r"""
sc = scenes.s256()
el = N.marshal(sc)
for d in (3, 4, 6):
    a, b = frame(sc, 4096, 2048, d, 1), frame(sc, 4096, 2048, d, 0)
    assert np.array_equal(a.view(np.int64), b.view(np.int64)), d
    for r in (0, 1037, 2047):
        ref = O.render(el, 4096, 2048, d, mode=O.MEMO, row0=r, nrows=1)
        assert np.abs(b[r:r + 1] - ref).max() <= 1e-5, (d, r)
print('ok')
""", RT_ENGINE="wave")


def test_config5_rows_through_the_bvh_path(oracle):
    """Config 5 as the bench renders it (frames in flight: no side streams, so levels >= 2 of
    S256 traverse the BVH): S256 4096x4096 depth 8 x16 spp, 2 of 8 interleaved row shards, bit for
    bit the side-stream path's (beams only) and 3 rows of each against the oracle."""
    _child(r"""
sc = scenes.s256()
W = H = 4096
seed = 0x5EED0005
el = N.marshal(sc)
for shard in (0, 5):
    a = frame(sc, W, H, 8, 1, 16, seed, shard, 8)
    b = frame(sc, W, H, 8, 0, 16, seed, shard, 8)
    assert np.array_equal(a.view(np.int64), b.view(np.int64)), shard
    for lr in (0, 200, 511):
        gy = (lr // 16 * 8 + shard) * 16 + lr % 16
        ref = O.render(el, W, H, 8, mode=O.MEMO, row0=gy, nrows=1, spp=16, seed=seed)
        assert np.abs(b[lr:lr + 1] - ref).max() <= 1e-5, (shard, lr)
print('ok')
""")
