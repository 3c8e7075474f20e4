"""GPU parity: the HIP kernel (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): max per-channel |delta| <= 1e-5.  The kernel computes in
binary64 in the reference's operation order, so in practice every hit/shadow decision is
identical (checked exactly through the per-pixel level counts) and colours differ only
where device pow() rounds differently from the host libm (~1e-16).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from eraytracer_amd import _native as N
from eraytracer_amd import records, scenes
from eraytracer_amd.raytracer import render

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _oracle(O, scene, w, h, d, **kw):
    return O.render(N.marshal(scene), w, h, d, mode=O.MEMO, levels=True, **kw)


def _check(gpu, ref, tol=TOL):
    assert gpu.shape == ref.shape
    err = np.abs(gpu.astype(np.float64) - ref)
    assert np.all(np.isfinite(gpu))
    assert err.max() <= tol, f"max |delta| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    return err.max()


CASES = [
    ("default", 64, 48, 0), ("default", 64, 48, 1), ("default", 64, 48, 3), ("default", 64, 48, 5),
    ("default", 160, 120, 5), ("default", 33, 17, 4), ("s64", 64, 64, 5), ("s256", 48, 40, 8),
]


@pytest.mark.parametrize("name,w,h,d", CASES)
def test_render_matches_oracle(oracle, name, w, h, d):
    scene = scenes.named(name)
    img, lv = render(w, h, scene, d, levels=True)
    ref, rlv = _oracle(oracle, scene, w, h, d)
    np.testing.assert_array_equal(lv, rlv)  # identical reflection chains, pixel for pixel
    _check(img, ref)


@pytest.mark.parametrize("idx", range(6))
def test_tricky_scenes(oracle, idx):
    """Duplicates (=:= copies light each other, 4 vs 4.0 copies shadow), no lights, stray
    list elements, a triangle behind the camera (negative t wins), negative colours: the
    any-hit shadow restatement and the type-grouped scans must keep the reference's answers."""
    from tests.test_oracle import TRICKY
    scene = TRICKY[idx]()
    for d in (1, 3, 5):
        img, lv = render(48, 36, scene, d, levels=True)
        ref, rlv = _oracle(oracle, scene, 48, 36, d)
        np.testing.assert_array_equal(lv, rlv)
        _check(img, ref)


@pytest.mark.parametrize("name,w,h,d", [("default", 64, 48, 5), ("s64", 48, 48, 5)])
def test_fast_order_and_f32(oracle, name, w, h, d):
    scene = scenes.named(name)
    ref, rlv = _oracle(oracle, scene, w, h, d)
    fast, lv = render(w, h, scene, d, order="fast", levels=True)
    np.testing.assert_array_equal(lv, rlv)
    _check(fast, ref)
    f32 = render(w, h, scene, d, precision="f32")
    assert f32.dtype == np.float32
    _check(f32, ref)


def test_exact_order_is_bitwise_outside_pow(oracle):
    """With ORDER_EXACT the frame is bit-identical to the oracle except where the host libm's pow
    (0.52 ulp, not correctly rounded) differs from the kernels' correctly rounded one: count
    those pixels and bound them (0.1 %; tests/test_gpu_fullsize.py has the full-size counts)."""
    scene = records.scene()
    img = render(96, 72, scene, 5)
    ref, _ = _oracle(oracle, scene, 96, 72, 5)
    diff = ~np.all(img.view(np.int64) == ref.view(np.int64), axis=-1)
    print(f"{int(diff.sum())} of {diff.size} pixels not bit-identical")
    assert diff.sum() <= max(2, diff.size // 1000), f"{int(diff.sum())} pixels not bit-identical"
    assert np.abs(img - ref).max() <= 1e-15


def test_done_and_bad_sizes():
    assert render(0, 0, records.scene(), 3) == "done"
    with pytest.raises(ValueError):
        render(0, 5, records.scene(), 3)


def test_shard_launch_and_unshard(oracle):
    """rt_launch per shard + rt_unshard reassembles the same image (multi-GPU data path on one device)."""
    import torch
    L = N.lib()
    scene = scenes.s64()
    el = N.marshal(scene)
    w, h, d, rb = 80, 70, 5, 16
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
    try:
        full = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        N.check(L.rt_launch(p, w, h, d, rb, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, full.data_ptr(), None, st))
        for ns in (2, 3, 5):
            rows = L.rt_shard_rows(h, rb, ns)
            slabs = torch.full((ns, rows, w, 3), -1.0, dtype=torch.float64, device="cuda")
            for s in range(ns):
                N.check(L.rt_launch(p, w, h, d, rb, s, ns, N.RT_OUT_F64, N.RT_ORDER_EXACT,
                                    slabs[s].data_ptr(), None, st))
            img = torch.empty_like(full)
            N.check(L.rt_unshard(slabs.data_ptr(), w, h, rb, ns, N.RT_OUT_F64, img.data_ptr(), st))
            torch.cuda.synchronize()
            assert torch.equal(img, full), f"nshards={ns}"
        ref, _ = _oracle(oracle, scene, w, h, d)
        _check(full.cpu().numpy(), ref)
    finally:
        L.rt_release(p)


def test_full_size_sampled_rows(oracle):
    """BASELINE config 3 at full size (4096^2, S64, depth 5): rows sampled across the
    frame must match the oracle; the rest is checked by the levels histogram being sane."""
    scene = scenes.s64()
    W = H = 4096
    img, lv = render(W, H, scene, 5, levels=True)
    el = N.marshal(scene)
    for r0 in (0, 1023, 2048, 3071, 4095):
        ref, rlv = oracle.render(el, W, H, 5, mode=oracle.MEMO, row0=r0, nrows=1, levels=True)
        np.testing.assert_array_equal(lv[r0:r0 + 1], rlv)
        _check(img[r0:r0 + 1], ref)
    assert lv.max() <= 5


@pytest.mark.parametrize("engine", ["fused", "wave"])
def test_forced_engine_parity(engine):
    """Each engine forced for every scene (RT_ENGINE, read once per process, so in a child
    process): by default small scenes take the fused kernel and large ones the wavefront
    pipeline, and both must keep the reference's answers on every case."""
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, sys\n"
        "from eraytracer_amd import _native as N, scenes\n"
        "from eraytracer_amd.raytracer import render\n"
        "from oracle import oracle as O\n"
        "from tests.test_oracle import TRICKY\n"
        "cases = [(scenes.named(n), w, h, d) for n, w, h, d in [('default', 64, 48, 5), ('s64', 64, 64, 5),"
        " ('s256', 40, 32, 8)]] + [(mk(), 40, 30, 3) for mk in TRICKY]\n"
        # more lights than the 32 shadow answers a record keeps: the reshading retests shadows
        "cases.append((scenes.synthetic_scene(24, 0x5EED4040, n_lights=40), 48, 40, 4))\n"
        "for order in ('exact', 'fast'):\n"
        "    for sc, w, h, d in cases:\n"
        "        img, lv = render(w, h, sc, d, levels=True, order=order)\n"
        "        ref, rlv = O.render(N.marshal(sc), w, h, d, mode=O.MEMO, levels=True)\n"
        "        assert np.array_equal(lv, rlv)\n"
        "        assert np.abs(img - ref).max() <= 1e-5, (order, w, h, d)\n"
        "print('engine ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RT_ENGINE=engine, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "engine ok" in r.stdout, r.stdout + r.stderr


def test_repeated_launch_graph_replay(oracle):
    """Identical rt_launch calls go direct, then captured, then replayed from a graph; a larger
    frame in between reallocates the work space, which must invalidate the captured graph."""
    import torch
    L = N.lib()
    scene = scenes.s64()
    el = N.marshal(scene)
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
    try:
        st = torch.cuda.current_stream().cuda_stream
        w, h, d = 96, 80, 5
        out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
        big = torch.empty((400, 320, 3), dtype=torch.float64, device="cuda")
        imgs = []
        for i in range(7):
            out.fill_(-1.0)
            if i == 3:  # a bigger frame grows every work buffer
                N.check(L.rt_launch(p, 320, 400, d, 16, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, big.data_ptr(), None, st))
            N.check(L.rt_launch(p, w, h, d, 16, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, out.data_ptr(), None, st))
            torch.cuda.synchronize()
            imgs.append(out.cpu().numpy().copy())
        for i, im in enumerate(imgs[1:], 1):
            assert np.array_equal(im, imgs[0]), f"launch {i} differs"
        ref, _ = _oracle(oracle, scene, w, h, d)
        _check(imgs[-1], ref)
        refb, _ = _oracle(oracle, scene, 320, 400, d)
        _check(big.cpu().numpy(), refb)
    finally:
        L.rt_release(p)


def test_frame_graphs_follow_the_primary_masks():
    """Frame graphs on (RT_GRAPH=1, read once per process: a child).  One context alternates two
    shards of a frame and a second frame geometry, so the primary rays' candidate masks (k_pmask,
    recomputed when the geometry or shard changes) are rewritten between identical launches that
    would otherwise replay a captured graph holding no k_pmask launch: every launch must equal the
    same frame from a fresh context (graphs off there: first launches run directly), bit for bit."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r"""
import ctypes, numpy as np, torch
from eraytracer_amd import _native as N, scenes
L = N.lib()
el = N.marshal(scenes.s64())
st = torch.cuda.current_stream().cuda_stream
def launch(p, w, h, shard, ns):
    rows = L.rt_shard_rows(h, 16, ns)
    out = torch.full((rows, w, 3), float('nan'), dtype=torch.float64, device='cuda')
    N.check(L.rt_launch(p, w, h, 5, 16, shard, ns, N.RT_OUT_F64, N.RT_ORDER_EXACT, out.data_ptr(), None, st))
    torch.cuda.synchronize()
    return np.nan_to_num(out.cpu().numpy(), nan=-7.0)
def fresh(w, h, shard, ns):
    q = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(q)))
    try:
        N.check(L.rt_configure(q, N.RT_CFG_SIDE_STREAMS, 0))
        return launch(q, w, h, shard, ns)
    finally:
        L.rt_release(q)
p = ctypes.c_void_p()
N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, 0))
seq = [(256, 192, 0, 2)] * 3 + [(256, 192, 1, 2)] * 3 + [(256, 192, 0, 2)] * 3 + [(160, 96, 0, 1)] * 3 + \
      [(256, 192, 1, 2), (256, 192, 0, 2), (256, 192, 0, 2), (256, 192, 0, 2)]
ref = {a: fresh(*a) for a in set(seq)}
for i, a in enumerate(seq):
    got = launch(p, *a)
    assert np.array_equal(got.view(np.int64), ref[a].view(np.int64)), (i, a)
L.rt_release(p)
print('ok')
"""
    env = dict(os.environ, RT_GRAPH="1", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout.split(), r.stdout + r.stderr


@pytest.mark.parametrize("name,w,h,d,spp", [("s64", 48, 40, 5, 4), ("default", 40, 32, 5, 3), ("s256", 32, 24, 8, 16)])
def test_supersampling_matches_oracle(oracle, name, w, h, d, spp):
    """BASELINE config 5's stochastic supersampling (RT_SUPERSAMPLING) against the oracle's
    restatement of the same definition; levels are sample 0's."""
    scene = scenes.named(name)
    seed = 0x5EED0005
    img, lv = render(w, h, scene, d, levels=True, spp=spp, seed=seed)
    ref, rlv = oracle.render(N.marshal(scene), w, h, d, mode=oracle.MEMO, levels=True, spp=spp, seed=seed)
    np.testing.assert_array_equal(lv, rlv)
    _check(img, ref)
    f32 = render(w, h, scene, d, precision="f32", spp=spp, seed=seed)
    _check(f32, ref)


def test_supersampling_shards():
    """rt_launch_spp per shard + rt_unshard equals the single-shard supersampled frame."""
    import torch
    L = N.lib()
    el = N.marshal(scenes.s64())
    w, h, d, rb, spp, seed = 64, 50, 5, 16, 4, 77
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
    try:
        st = torch.cuda.current_stream().cuda_stream
        full = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
        N.check(L.rt_launch_spp(p, w, h, d, rb, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, spp, seed, full.data_ptr(),
                                None, st))
        ns = 3
        rows = L.rt_shard_rows(h, rb, ns)
        slabs = torch.zeros((ns, rows, w, 3), dtype=torch.float64, device="cuda")
        for s in range(ns):
            N.check(L.rt_launch_spp(p, w, h, d, rb, s, ns, N.RT_OUT_F64, N.RT_ORDER_EXACT, spp, seed,
                                    slabs[s].data_ptr(), None, st))
        img = torch.empty_like(full)
        N.check(L.rt_unshard(slabs.data_ptr(), w, h, rb, ns, N.RT_OUT_F64, img.data_ptr(), st))
        torch.cuda.synchronize()
        assert torch.equal(img, full)
        assert L.rt_launch_spp(p, w, h, d, rb, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, 0, seed, full.data_ptr(), None,
                               st) == N.RT_EBADARG
    finally:
        L.rt_release(p)


@pytest.mark.parametrize("name,w,h,d,spp", [("s64", 48, 40, 5, 4), ("default", 40, 37, 5, 3), ("s256", 32, 24, 8, 16),
                                            ("mixed", 40, 32, 4, 2), ("s64", 33, 21, 1, 3), ("s64", 24, 16, 0, 2)])
def test_supersampling_single_write_path(name, w, h, d, spp):
    """Without side streams each pass writes every pixel once and folds its sample into the
    running sum where it writes (no sample slab, no k_accum): bit for bit the frame of the
    sample-slab path (side streams on), f64 and f32, and no row past the image written."""
    import torch
    L = N.lib()
    el = N.marshal(scenes.named(name))
    st = torch.cuda.current_stream().cuda_stream
    rb, seed = 16, 0x5EED0005
    frames = {}
    for side in (1, 0):
        p = ctypes.c_void_p()
        N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
        try:
            N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, side))
            for prec, dt in ((N.RT_OUT_F64, torch.float64), (N.RT_OUT_F32, torch.float32)):
                buf = torch.full((h + 16, w, 3), 12345.0, dtype=dt, device="cuda")
                for _ in range(2):  # a second frame reuses the running sum: no state leaks between frames
                    N.check(L.rt_launch_spp(p, w, h, d, rb, 0, 1, prec, N.RT_ORDER_EXACT, spp, seed, buf.data_ptr(),
                                            None, st))
                torch.cuda.synchronize()
                assert bool((buf[h:] == 12345.0).all())
                frames[side, prec] = buf[:h].cpu()
        finally:
            L.rt_release(p)
    for prec in (N.RT_OUT_F64, N.RT_OUT_F32):
        a, b = frames[1, prec], frames[0, prec]
        assert torch.equal(a.view(torch.int64 if a.dtype == torch.float64 else torch.int32),
                           b.view(torch.int64 if b.dtype == torch.float64 else torch.int32)), (name, prec)


# ---- P3 output on the GPU (write_pixels_to_ppm/5, raytracer.erl:667-685) ---------------------

def _py_ppm(tmp_path, img, maxv=255):
    from eraytracer_amd.raytracer import write_pixels_to_ppm
    path = tmp_path / "py.ppm"
    write_pixels_to_ppm(img.shape[1], img.shape[0], maxv, img, str(path))
    return path.read_bytes()


def test_ppm_gpu_bytes_match_python_writer(tmp_path):
    """rt_ppm_format's text equals the Python mirror of write_pixels_to_ppm/5 byte for byte:
    rendered frames (incl. negative colours) and adversarial values (exact k/255 and
    half-step boundaries, clamping, negatives, zero)."""
    from eraytracer_amd.raytracer import ppm_text_gpu
    from tests.test_oracle import TRICKY
    frames = [render(64, 48, records.scene(), 5), render(40, 30, TRICKY[5](), 3),
              render(48, 40, scenes.s64(), 5, spp=3, seed=9)]
    k = np.arange(0, 600, dtype=np.float64)
    vals = np.concatenate([k / 255.0, (k + 0.5) / 255.0, -k / 255.0, np.nextafter(k / 255.0, -1.0),
                           [0.0, -0.0, 1.0, 2.0, 1e30, -1e5, 254.999999999 / 255.0, 1.0 - 1e-17]])
    vals = np.resize(vals, (len(vals) + 2) // 3 * 3).reshape(-1, 3)
    frames.append(vals.reshape(1, -1, 3))
    for img in frames:
        assert ppm_text_gpu(img) == _py_ppm(tmp_path, img)
    for maxv in (1, 7, 65535):
        assert ppm_text_gpu(frames[0], maxv) == _py_ppm(tmp_path, frames[0], maxv)


def test_ppm_gpu_range_error():
    from eraytracer_amd.raytracer import ppm_text_gpu
    img = np.zeros((2, 3, 3))
    img[1, 2, 0] = -1e12  # -2.55e14 after scaling: BEAM prints a bignum
    with pytest.raises(N.RtError):
        ppm_text_gpu(img)


def test_render_ppm_file_matches_golden_and_python(tmp_path, oracle):
    """rt_render_ppm_file (raytrace/5 with the P3 text made on the GPU) reproduces the
    committed run.sh / run-concurrent.sh P3 fixtures and the Python writer on the oracle's
    frame — including a scene whose colours need BEAM bignums (host formatting path)."""
    import os
    from eraytracer_amd.raytracer import render_ppm_file
    gold = os.path.join(os.path.dirname(__file__), "golden")
    for name, w, h in (("run_sh_32x24_d1.ppm", 32, 24), ("run_concurrent_sh_16x12_d1.ppm", 16, 12)):
        out = tmp_path / name
        assert render_ppm_file(w, h, records.scene(), 1, str(out)) == "ok"
        assert out.read_bytes() == open(os.path.join(gold, name), "rb").read()
    sc = scenes.s64()
    out = tmp_path / "s64.ppm"
    render_ppm_file(56, 40, sc, 5, str(out))
    ref = _oracle(oracle, sc, 56, 40, 5)[0]
    got, want = out.read_bytes(), _py_ppm(tmp_path, ref)
    if got != want:
        ta, tb = got.split(b"\n", 3)[3].split(), want.split(b"\n", 3)[3].split()
        diff = [(k // 3 // 56, k // 3 % 56, k % 3, ta[k], tb[k], repr(ref.reshape(-1)[k]))
                for k in range(min(len(ta), len(tb))) if ta[k] != tb[k]]
        raise AssertionError(f"{len(got)} vs {len(want)} bytes; {len(diff)} values differ: {diff[:6]}")
    huge = records.scene()[:2] + [records.sphere(4, records.vector(4, 0, 10),
                                                 records.material(records.colour(-1e12, 0.5, 1), 20, 1, 0.1))]
    out = tmp_path / "huge.ppm"
    render_ppm_file(24, 18, huge, 3, str(out))
    assert out.read_bytes() == _py_ppm(tmp_path, _oracle(oracle, huge, 24, 18, 3)[0])
    assert b"-" in out.read_bytes()


@pytest.mark.parametrize("name,spp", [("s64", 1), ("s64", 3), ("default", 1)])
def test_launch_writes_only_image_rows(name, spp):
    """A single-shard launch touches only the image's rows: H not a multiple of the row
    block, the output followed by guard rows that must keep their sentinel (an earlier
    version wrote the last block's padding rows past the buffer)."""
    import torch
    L = N.lib()
    el = N.marshal(scenes.named(name))
    w, h, rb = 40, 37, 16
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
    try:
        st = torch.cuda.current_stream().cuda_stream
        buf = torch.full((h + 16, w, 3), 12345.0, dtype=torch.float64, device="cuda")
        lv = torch.full((h + 16, w), 77, dtype=torch.uint8, device="cuda")
        N.check(L.rt_launch_spp(p, w, h, 5, rb, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, spp, 5, buf.data_ptr(),
                                lv.data_ptr(), st))
        torch.cuda.synchronize()
        assert bool((buf[h:] == 12345.0).all()) and bool((lv[h:] == 77).all())
        assert not bool((buf[:h] == 12345.0).any())
    finally:
        L.rt_release(p)


# ---- compact slab transfer (rt_slab_pack / rt_slab_unpack; dist.CompactGather) ----------
@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("w,h,rb,ns", [(80, 70, 16, 3), (64, 64, 16, 1), (33, 17, 4, 2), (100, 9, 16, 8),
                                       (257, 31, 5, 4), (2052, 40, 16, 8), (1024, 33, 7, 3)])
def test_slab_codec_matches_reference_format(prec, w, h, rb, ns):
    """HIP pack gives the header and values of the test-side restatement byte for byte, on
    random sparse slabs (-0.0 and NaN payloads count as non-zero; padding rows hold garbage);
    HIP unpack reassembles the frame exactly."""
    import torch

    from eraytracer_amd.dist import SlabCodec, shard_global_rows
    from tests.slab_ref import RefCodec
    dt = torch.float32 if prec == "f32" else torch.float64
    codec, ref = SlabCodec(w, h, rb, ns, prec), RefCodec(w, h, rb, ns)
    assert codec.header_bytes == ref.header_bytes
    rows = N.lib().rt_shard_rows(h, rb, ns)
    gen = torch.Generator().manual_seed(w * 1000 + h * 10 + ns)
    frame = torch.rand((h, w, 3), generator=gen, dtype=torch.float64).to(dt)
    frame[torch.rand((h, w), generator=gen) < 0.7] = 0.0
    frame[0, 0] = torch.tensor([0.0, -0.0, 0.0], dtype=dt)
    frame[h - 1, w - 1, 2] = float("nan")
    hdrs, vals = [], []
    for s in range(ns):
        g = shard_global_rows(h, rb, ns, s)
        slab = torch.full((rows, w, 3), 5.0, dtype=dt)
        slab[torch.from_numpy(g >= 0)] = frame[torch.from_numpy(g[g >= 0])]
        hd = torch.full((codec.header_bytes,), 0xAB, dtype=torch.uint8, device="cuda")
        vd = torch.full((rows * w * 3,), -9.0, dtype=dt, device="cuda")
        codec.pack(slab.cuda(), s, hd, vd)
        hr = torch.empty(ref.header_bytes, dtype=torch.uint8)
        vr = torch.full((rows * w * 3,), -9.0, dtype=dt)
        ref.pack(slab, s, hr, vr)
        torch.cuda.synchronize()
        n = int(hr[:8].view(torch.int64)[0])
        hdc = hd.cpu()
        # count, offsets and mask agree (bytes between the offsets and the mask are padding)
        assert torch.equal(hdc[:8], hr[:8])
        assert torch.equal(hdc[64:64 + 4 * ref.nblk], hr[64:64 + 4 * ref.nblk])
        assert torch.equal(hdc[ref.mask_at:], hr[ref.mask_at:])
        bits = torch.int32 if prec == "f32" else torch.int64
        assert torch.equal(vd.cpu()[: 3 * n].view(bits), vr[: 3 * n].view(bits))
        hdrs.append(hd)
        vals.append(vd)
    img = torch.full((h, w, 3), 3.0, dtype=dt, device="cuda")
    codec.unpack(hdrs, vals, img)
    torch.cuda.synchronize()
    bits = torch.int32 if prec == "f32" else torch.int64
    assert torch.equal(img.cpu().view(bits), frame.view(bits))


def test_compact_gather_of_rendered_shards(oracle):
    """rt_launch per shard -> rt_slab_pack -> rt_slab_unpack equals the single-shard frame bit
    for bit (the multi-GPU compact gather's data path on one device)."""
    import torch

    from eraytracer_amd.dist import SlabCodec
    L = N.lib()
    scene = scenes.s64()
    el = N.marshal(scene)
    w, h, d, rb = 96, 75, 5, 16
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
    try:
        st = torch.cuda.current_stream().cuda_stream
        for prec, dt in ((N.RT_OUT_F32, torch.float32), (N.RT_OUT_F64, torch.float64)):
            full = torch.empty((h, w, 3), dtype=dt, device="cuda")
            N.check(L.rt_launch(p, w, h, d, rb, 0, 1, prec, N.RT_ORDER_EXACT, full.data_ptr(), None, st))
            for ns in (2, 3, 8):
                codec = SlabCodec(w, h, rb, ns, "f32" if prec == N.RT_OUT_F32 else "f64")
                rows = L.rt_shard_rows(h, rb, ns)
                hdrs, vals = [], []
                for s in range(ns):
                    slab = torch.full((rows, w, 3), float("nan"), dtype=dt, device="cuda")
                    N.check(L.rt_launch(p, w, h, d, rb, s, ns, prec, N.RT_ORDER_EXACT, slab.data_ptr(), None, st))
                    hdrs.append(torch.empty(codec.header_bytes, dtype=torch.uint8, device="cuda"))
                    vals.append(torch.empty(rows * w * 3, dtype=dt, device="cuda"))
                    codec.pack(slab, s, hdrs[-1], vals[-1])
                img = torch.full_like(full, -1.0)
                codec.unpack(hdrs, vals, img)
                torch.cuda.synchronize()
                assert torch.equal(img, full), f"nshards={ns}"
                nz = int(sum(int(hd[:8].cpu().view(torch.int64)[0]) for hd in hdrs))
                bits = torch.int32 if dt == torch.float32 else torch.int64
                assert nz == int((full.view(bits) != 0).any(-1).sum())
        ref, _ = _oracle(oracle, scene, w, h, d)
        _check(full.cpu().numpy(), ref)
    finally:
        L.rt_release(p)


def test_frames_in_flight_match_single_frame():
    """FrameRenderer(inflight=3) (bench.py's default mode): frames on three contexts and
    streams at once, side streams off, each bit-identical to the one-context frame."""
    import torch

    from eraytracer_amd.dist import FrameRenderer
    w, h, d = 128, 96, 5
    one = FrameRenderer(scenes.s64(), w, h, d, precision="f64")
    one.launch()
    torch.cuda.synchronize()
    ref = one.slab[:h].clone()
    one.close()
    fr = FrameRenderer(scenes.s64(), w, h, d, precision="f64", inflight=3)
    for s in fr.slabs:
        s.fill_(float("nan"))
    fr.fork()
    for _ in range(7):
        fr.launch()
    fr.join()
    torch.cuda.synchronize()
    for i, s in enumerate(fr.slabs):
        assert torch.equal(s[:h], ref), f"slot {i}"
    fr.close()


def test_fast_sqrt_and_division_are_the_library_bits():
    """sqrt_n / div_n / normalize3 (the kernels' range-guarded fast paths) against the device
    library's sqrt and division on 2^26 random operands each: no bit differs.  The same kernel checks
    pow_libm's scalar-controlled powering (wave-uniform exponents) against the per-lane powering, bit
    for bit, and the binary32 beams' integer-order wave reductions against a lane-by-lane loop."""
    bad = ctypes.c_uint64(123)
    N.check(N.lib().rt_selftest_math(0, 1 << 26, 0x5EED, ctypes.byref(bad)), "rt_selftest_math")
    assert bad.value == 0


def test_compact_gather_pipeline_over_rccl_one_rank():
    """dist.CompactGather end to end over RCCL (a one-rank nccl group: the GPU box has one
    device) with three frames in flight on their own streams: the side stream, the events,
    the pinned count read-back and the decode run as at N > 1, and every frame rank 0 gets
    back equals the single-context frame bit for bit."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from eraytracer_amd.dist import CompactGather, FrameRenderer, SlabCodec
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        w, h, d = 96, 80, 5
        one = FrameRenderer(scenes.s64(), w, h, d, precision="f32")
        one.launch()
        torch.cuda.synchronize()
        ref = one.slab[:h].clone()
        one.close()
        fr = FrameRenderer(scenes.s64(), w, h, d, precision="f32", inflight=3)
        frame = torch.full((h, w, 3), float("nan"), dtype=torch.float32, device="cuda")
        cg = CompactGather(SlabCodec(w, h, 16, 1, "f32"), 1, 0, fr.slab.numel(), torch.float32, fr.device, frame)
        got = []

        def keep(f):
            torch.cuda.current_stream().wait_event(cg.frame_ready)
            got.append(f.clone())
            torch.cuda.synchronize()  # before the next decode overwrites the frame

        fr.fork()
        for _ in range(6):
            fr.launch()
            with torch.cuda.stream(fr.stream):
                out = cg.submit(fr.slab, 0)
            if out is not None:
                keep(out)
        cg.drain(on_frame=keep)
        fr.join()
        torch.cuda.synchronize()
        assert len(got) == 6
        for i, g in enumerate(got):
            assert torch.equal(g, ref), f"frame {i}"
        fr.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,w,h,d", [("default", 64, 48, 5), ("s64", 64, 64, 5), ("s256", 48, 40, 8),
                                        ("default", 40, 30, 2)])
def test_fused_reflect_shade_matches_oracle(oracle, name, w, h, d):
    """Without side streams (frames in flight) each level's shading is fused into the next
    reflection pass (k_reflect_shade): the frame equals the side-stream path's bit for bit
    and the oracle within the bar, on spheres-only, mixed-object and dense-deep-level scenes."""
    import torch
    L = N.lib()
    scene = scenes.named(name)
    el = N.marshal(scene)
    outs = []
    for side in (1, 0):
        p = ctypes.c_void_p()
        N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)), "rt_prepare")
        try:
            N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, side), "rt_configure")
            img = torch.full((h, w, 3), float("nan"), dtype=torch.float64, device="cuda")
            st = torch.cuda.current_stream().cuda_stream
            N.check(L.rt_launch(p, w, h, d, 16, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, img.data_ptr(), None, st))
            torch.cuda.synchronize()
            outs.append(img.cpu().numpy())
        finally:
            L.rt_release(p)
    assert np.array_equal(outs[0].view(np.int64), outs[1].view(np.int64))
    ref, _ = _oracle(oracle, scene, w, h, d)
    _check(outs[1], ref)


@pytest.mark.parametrize("world", [3, 8])
def test_assembling_rank0_shards_reassemble(world):
    """bench.py --rank0 assemble on one device: FrameRenderer(assemble=True) ranks 1 .. world-1
    render shards 0 .. world-2 of world-1 (packed and decoded as rank 0 would), equal to the
    one-shard frame bit for bit; rank 0's launch() renders nothing."""
    import torch

    from eraytracer_amd.dist import FrameRenderer, SlabCodec
    w, h, d = 160, 100, 5
    one = FrameRenderer(scenes.s64(), w, h, d, precision="f32")
    one.launch()
    torch.cuda.synchronize()
    ref = one.slab[:h].clone()
    one.close()
    codec = SlabCodec(w, h, 16, world - 1, "f32")
    hdrs, vals = [], []
    for r in range(world):
        fr = FrameRenderer(scenes.s64(), w, h, d, rank=r, world=world, precision="f32", inflight=2, assemble=True)
        try:
            assert fr.nshards == world - 1 and fr.shard == max(r - 1, 0) and fr.renders == (r > 0)
            for s in fr.slabs:
                s.fill_(float("nan"))
            fr.fork()
            fr.launch()
            fr.join()
            torch.cuda.synchronize()
            if r == 0:
                assert bool(torch.isnan(fr.slabs[0]).all()), "rank 0 rendered rows"
                continue
            hdrs.append(torch.empty(codec.header_bytes, dtype=torch.uint8, device="cuda"))
            vals.append(torch.empty(fr.rows * w * 3, dtype=torch.float32, device="cuda"))
            codec.pack(fr.slabs[0], fr.shard, hdrs[-1], vals[-1])
        finally:
            fr.close()
    img = torch.full((h, w, 3), -1.0, dtype=torch.float32, device="cuda")
    codec.unpack(hdrs, vals, img)
    torch.cuda.synchronize()
    assert torch.equal(img.view(torch.int32), ref.view(torch.int32))
