"""Every environment variable the library reads, in a child process each (they are read once per
process): the frame it gives equals the brute-force frame (rt_configure(RT_CFG_CULL, 0): every
object tested by every ray) bit for bit and the oracle within 1e-5, on S64, S256 and the mixed
scene, through the kernels' entry point (rt_launch, with and without side streams) and through the
boundary (rt_render, f64 and f32, pinned and pageable).

The knobs and what they select (the A/B switches of earlier rounds are gone from the library):
  RT_ENGINE=fused|wave   the engine (also test_gpu_parity.py, test_gpu_fullsize.py)
  RT_LIT_STREAM=0        no shading side streams by default (the multi-rank bench sets it)
  RT_QUEUE_MB            queue budget per row pass (small: several row passes per slab)
  RT_GRAPH=1             frame graphs (also test_gpu_parity.py::test_frame_graphs_*)
  RT_BEAM_MIN            spheres below which scans skip the wave beams
  RT_BVH_MIN, RT_BVH_LEVEL  the sphere BVH's scene-size threshold and first level
  RT_BAND_MB             rt_render's row-band size (copy overlap)
  RT_COPY_STREAMS=2      rt_render's pinned copies over two DMA queues
  RT_CTX_SIDE_STREAMS=1  rt_render's contexts with shading side streams
  RT_DEVICE_ALIAS=N      test hook: N aliased devices (test_gpu_boundary.py)
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import ctypes, numpy as np, torch
from eraytracer_amd import _native as N, scenes
from eraytracer_amd.raytracer import render
from oracle import oracle as O
L = N.lib()
def launch(sc, w, h, d, side, cull):
    el = N.marshal(sc)
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
    try:
        if side is not None:
            N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, side))
        N.check(L.rt_configure(p, N.RT_CFG_CULL, cull))
        img = torch.full((h, w, 3), float('nan'), dtype=torch.float64, device='cuda')
        for _ in range(3):  # repeated frames: frame graphs capture and replay from the third
            N.check(L.rt_launch(p, w, h, d, 16, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, img.data_ptr(), None,
                                torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        return img.cpu().numpy()
    finally:
        L.rt_release(p)
def bits(a):
    return a.view(np.int64) if a.dtype == np.float64 else a.view(np.int32)
for name, w, h, d in [('s64', 96, 80, 5), ('s256', 64, 48, 8), ('mixed', 96, 64, 5)]:
    sc = scenes.named(name)
    brute = launch(sc, w, h, d, None, 0)
    for side in (None, 0, 1):
        a = launch(sc, w, h, d, side, 1)
        assert np.array_equal(bits(a), bits(brute)), (name, side)
    b64 = render(w, h, sc, d)
    assert np.array_equal(bits(b64), bits(brute)), (name, 'rt_render f64')
    b32 = N.pinned_empty((h, w, 3), np.float32)
    render(w, h, sc, d, precision='f32', out=b32)
    assert np.array_equal(bits(b32), bits(brute.astype(np.float32))), (name, 'rt_render f32 pinned')
    ref = O.render(N.marshal(sc), w, h, d, mode=O.MEMO)
    err = np.abs(brute - ref).max()
    assert err <= 1e-5, (name, err)
print('ok')
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"RT_LIT_STREAM": "0"}, {"RT_QUEUE_MB": "64"}, {"RT_GRAPH": "1"},
                                 {"RT_BEAM_MIN": "1"}, {"RT_BEAM_MIN": "100000"},
                                 {"RT_BVH_MIN": "2", "RT_BVH_LEVEL": "1"}, {"RT_BAND_MB": "1"},
                                 {"RT_COPY_STREAMS": "2"}, {"RT_CTX_SIDE_STREAMS": "1"},
                                 {"RT_ENGINE": "fused"}, {"RT_ENGINE": "wave"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_knob_frames_equal_brute_force_and_oracle(env):
    e = dict(os.environ, PYTHONPATH=ROOT, **env)
    r = subprocess.run([sys.executable, "-c", _CHILD], cwd=ROOT, env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout.split(), r.stdout + r.stderr


def test_every_getenv_knob_is_listed():
    """The library reads no environment variable this module does not cover."""
    import re
    names = set()
    for f in os.listdir(os.path.join(ROOT, "eraytracer_amd", "csrc")):
        src = open(os.path.join(ROOT, "eraytracer_amd", "csrc", f), errors="replace").read()
        names |= set(re.findall(r'getenv\("(RT_[A-Z0-9_]+)"\)', src))
    assert names and names <= set(re.findall(r"RT_[A-Z_]+", __doc__)), names - set(re.findall(r"RT_[A-Z_]+", __doc__))
