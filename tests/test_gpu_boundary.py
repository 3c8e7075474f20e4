"""The one-shot boundary rt_render (the drop-in for raytraced_pixel_list_*/4,
raytracer.erl:86-178) on the GPU: persistent per-process contexts, row bands with overlapped
copies, pinned and pageable destinations, the distributed strategy's row shards, and the
pixel list's exact term types."""
import ctypes

import numpy as np
import pytest

from eraytracer_amd import _native as N
from eraytracer_amd import raytracer as rt
from eraytracer_amd import records, scenes
from eraytracer_amd.raytracer import render

pytestmark = pytest.mark.gpu


def _device_frame(scene, w, h, d, precision="f64"):
    """The frame rendered by rt_launch into device memory (the reference point for rt_render)."""
    import torch
    L = N.lib()
    el = N.marshal(scene)
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
    try:
        dt = torch.float64 if precision == "f64" else torch.float32
        out = torch.empty((h, w, 3), dtype=dt, device="cuda")
        prec = N.RT_OUT_F64 if precision == "f64" else N.RT_OUT_F32
        N.check(L.rt_launch(p, w, h, d, 16, 0, 1, prec, N.RT_ORDER_EXACT, out.data_ptr(), None,
                            torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        return out.cpu().numpy()
    finally:
        L.rt_release(p)


def test_repeated_render_is_faster_than_the_first():
    """One process-wide context per device: in a fresh process (HIP already
    initialised by a small render of another scene), the first 4096^2 rt_render pays the scene
    compile and upload and the device allocations (frame, GBs of wavefront work space); later
    calls only the render and the copy into the caller's pinned buffer.  Measured (round 2):
    first 10.2 ms, repeated 4.2 ms (4000 Mpx/s) on one box, 5.2 vs 4.3 ms on another (the one-time
    cost depends on how fast the driver hands out the GBs of work space); round 1's rt_render,
    which prepared, allocated and freed everything and copied into pageable memory on every
    call, took ~16 ms.  Asserted: the repeated call is the faster one and stays >= 3000 Mpx/s."""
    import os
    import subprocess
    import sys
    code = r"""
import time, numpy as np
from eraytracer_amd import _native as N, scenes, records
from eraytracer_amd.raytracer import render
W = H = 4096
out = N.pinned_empty((H, W, 3), np.float32)
render(64, 48, records.scene(), 3)          # HIP initialised, a context exists (another scene)
sc = scenes.s64()
t0 = time.perf_counter(); render(W, H, sc, 5, precision='f32', out=out); first = time.perf_counter() - t0
again, c_side = [], []
for _ in range(3):
    st = {}
    t0 = time.perf_counter(); render(W, H, sc, 5, precision='f32', out=out, stats=st)
    again.append(time.perf_counter() - t0)
    c_side.append(st['total_ms'] / 1e3)
    assert st['pinned']
print('TIMES', first, min(again), min(c_side))
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, PYTHONPATH=root),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    first, again, c_side = map(float, r.stdout.split("TIMES")[1].split())
    print(f"first {first * 1e3:.1f} ms, repeated {again * 1e3:.1f} ms (Python calls); rt_render itself "
          f"{c_side * 1e3:.2f} ms = {4096 * 4096 / c_side / 1e6:.0f} Mpx/s into pinned memory")
    assert again < first, (first, again)
    assert c_side <= 0.0056, c_side  # >= 3000 Mpx/s at the boundary (4096^2 f32)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_bands_pinned_and_pageable_equal_the_device_frame(precision):
    """A frame of several row bands (24 MB of output each) delivered into pinned memory (DMA
    per band) and into pageable memory (staging ring + host copies) equals rt_launch's device
    frame bit for bit."""
    scene = scenes.s64()
    w, h, d = 2000, 1600, 5  # f64: 77 MB = 4 bands; f32: 2 bands
    ref = _device_frame(scene, w, h, d, precision)
    dt = np.float64 if precision == "f64" else np.float32
    pin = N.pinned_empty((h, w, 3), dt)
    pin[...] = -1
    st = {}
    render(w, h, scene, d, precision=precision, out=pin, stats=st)
    assert st["pinned"]
    page = render(w, h, scene, d, precision=precision, stats=st)
    assert not st["pinned"]
    assert np.array_equal(pin.view(np.uint8), ref.view(np.uint8))
    assert np.array_equal(page.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("rb", [16, 7])
def test_distributed_shards_on_one_device(oracle, rb):
    """The distributed strategy's row split (raytracer.erl:121-149) through rt_render with more
    shards than devices (shard s on device s % ndev): 2, 3 and 5 interleaved shards, pinned
    and pageable, with levels, equal the single-shard frame bit for bit."""
    scene = scenes.s64()
    w, h, d = 300, 203, 5
    one, lv1 = render(w, h, scene, d, levels=True, row_block=rb)
    for ns in (2, 3, 5):
        img, lv = render(w, h, scene, d, levels=True, row_block=rb, nshards=ns)
        assert np.array_equal(img.view(np.int64), one.view(np.int64)), ns
        assert np.array_equal(lv, lv1), ns
        pin = N.pinned_empty((h, w, 3), np.float64)
        render(w, h, scene, d, row_block=rb, nshards=ns, out=pin)
        assert np.array_equal(pin.view(np.int64), one.view(np.int64)), ns
    ref, rlv = oracle.render(N.marshal(scene), w, h, d, mode=oracle.MEMO, levels=True)
    assert np.array_equal(lv1, rlv)
    assert np.abs(one - ref).max() <= 1e-5


def test_multi_device_path_through_device_aliases():
    """rt_render's multi-device loop (rt_host.hip: one context, work space and band pipeline per
    device, each device's shards scattered into the one frame; raytracer.erl:121-149) on a
    one-GPU machine: RT_DEVICE_ALIAS=N (a test hook read once per process, so in a child process)
    makes the N devices all device 0.  ndev 2 and 3 with 2, 3 and 5 shards, pinned and pageable,
    f64 and f32, with levels and supersampling, equal the one-device frames bit for bit."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r"""
import numpy as np
from eraytracer_amd import _native as N, scenes
from eraytracer_amd.raytracer import render
scene = scenes.s64()
w, h, d = 300, 203, 5
for prec in ("f64", "f32"):
    one, lv1 = render(w, h, scene, d, levels=True, precision=prec)
    iv = np.int64 if prec == "f64" else np.int32
    for nd, ns in ((2, 0), (2, 3), (3, 0), (3, 5)):
        img, lv = render(w, h, scene, d, levels=True, precision=prec, ndev=nd, nshards=ns)
        assert np.array_equal(img.view(iv), one.view(iv)), (prec, nd, ns)
        assert np.array_equal(lv, lv1), (prec, nd, ns)
        pin = N.pinned_empty((h, w, 3), np.float64 if prec == "f64" else np.float32)
        render(w, h, scene, d, precision=prec, ndev=nd, nshards=ns, out=pin)
        assert np.array_equal(pin.view(iv), one.view(iv)), (prec, nd, ns, "pinned")
s1 = render(96, 72, scenes.named("s256"), 8, spp=4)
s3 = render(96, 72, scenes.named("s256"), 8, spp=4, ndev=3)
assert np.array_equal(s1.view(np.int64), s3.view(np.int64))
print("aliases ok")
"""
    env = dict(os.environ, RT_DEVICE_ALIAS="3", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "aliases ok" in r.stdout, r.stdout + r.stderr


def test_distributed_strategy_all_devices():
    """raytraced_pixel_list_distributed/4 (every visible device) returns the concurrent list."""
    a = rt.raytraced_pixel_list_distributed(40, 30, records.scene(), 3)
    b = rt.raytraced_pixel_list_concurrent(40, 30, records.scene(), 3)
    assert a == b and len(a) == 1200


def test_context_scene_cache_follows_the_scene():
    """The context keeps the last scene compiled; a different scene (and back) must be
    recompiled each time: A, B, A renders equal fresh renders."""
    a, b = scenes.s64(), scenes.named("mixed")
    w, h = 128, 96
    L = N.lib()
    fa = render(w, h, a, 5)
    fb = render(w, h, b, 5)
    fa2 = render(w, h, a, 5)
    assert np.array_equal(fa.view(np.int64), fa2.view(np.int64))
    L.rt_reset_contexts()
    assert np.array_equal(render(w, h, b, 5).view(np.int64), fb.view(np.int64))
    assert not np.array_equal(fa, fb)


def test_concurrent_callers():
    """rt_render from several threads at once (separate contexts, up to 4 per device; more wait)."""
    from concurrent.futures import ThreadPoolExecutor
    scene = scenes.s64()
    ref = render(256, 192, scene, 5)
    with ThreadPoolExecutor(6) as ex:
        outs = list(ex.map(lambda _: render(256, 192, scene, 5), range(12)))
    for o in outs:
        assert np.array_equal(o.view(np.int64), ref.view(np.int64))


@pytest.mark.parametrize("mk,d", [(records.scene, 3), (records.scene, 0), (scenes.default_powers, 2),
                                  (lambda: [s for s in records.scene() if s[0] != "point_light"], 3)])
def test_pixel_list_term_types(mk, d):
    """The strategy's list carries the reference's term types: {0,0,0} integers exactly where
    the term-level restatement has them (tests/test_oracle.py::test_term_types_rule), floats
    elsewhere, and the same numbers."""
    from oracle import erl_restatement as E
    scene = mk()
    w, h = 20, 15
    ours = rt.raytraced_pixel_list_simple(w, h, scene, d)
    ref = E.raytraced_pixel_list_simple(w, h, scene, d)
    assert len(ours) == len(ref)
    for (k1, a), (k2, b) in zip(ours, ref):
        assert k1 == k2 == 1
        assert [type(x) for x in a] == [type(x) for x in b], (a, b)
        assert all(abs(x - y) <= 1e-5 for x, y in zip(a, b)), (a, b)
    keyed = rt.raytraced_pixel_list_concurrent(w, h, scene, d)
    assert [k for k, _ in keyed] == list(range(w * h))


@pytest.mark.parametrize("name,w,h,d,spp", [("default", 160, 120, 5, 1), ("default", 97, 61, 0, 1), ("s64", 256, 256, 5, 1),
                                            ("s256", 128, 96, 8, 4), ("mixed", 128, 96, 5, 1)])
def test_levels_hit_mask(name, w, h, d, spp):
    """RT_LEVELS_HIT (rt_opts.flags): out_levels is the primary-hit mask — 1 exactly where the
    level count is positive — and the frame is the same bits as without levels (the fused
    wavefront kernels stay on; a level count turns them off).  The strategy funs and the NIF's
    render_frame use it for the reference's integer {0,0,0} pixels."""
    scene = scenes.named(name)
    plain = render(w, h, scene, d, spp=spp, seed=7)
    img, mask = render(w, h, scene, d, spp=spp, seed=7, levels="hit")
    img2, lv = render(w, h, scene, d, spp=spp, seed=7, levels=True)
    assert np.array_equal(img.view(np.int64), plain.view(np.int64))
    assert np.array_equal(img2.view(np.int64), plain.view(np.int64))
    assert set(np.unique(mask).tolist()) <= {0, 1}
    assert np.array_equal(mask, (lv > 0).astype(np.uint8))
