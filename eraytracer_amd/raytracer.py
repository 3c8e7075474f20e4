"""Host-side mirror of raytracer.erl's strategy interface, backed by the MI355X kernel.

The reference's pixel loop is a strategy fun ``F(Width, Height, Scene, Recursion_depth)``
chosen by ``tracing_function/1`` (raytracer.erl:714-719) and called once by
``raytrace/5`` (raytracer.erl:723-733).  This module provides the same functions with
the same argument meaning and the same results, rendered by ``librtmi355x.so``:

* :func:`raytraced_pixel_list_simple`      — keys all 1, row-major (raytracer.erl:86-99)
* :func:`raytraced_pixel_list_concurrent`  — keys X+Y*Width, sorted (raytracer.erl:101-119, :155)
* :func:`raytraced_pixel_list_distributed` — same pixels and keys, rendered over every
  visible GPU of the process (raytracer.erl:121-149)
* :func:`raytraced_pixel_list_gpu`         — alias of the concurrent form (the new strategy atom ``gpu``)

plus :func:`raytrace`, :func:`go`, :func:`standalone`, :func:`tracing_function` and the
byte-exact ASCII P3 writer :func:`write_pixels_to_ppm` (raytracer.erl:667-685).
:func:`render` returns the framebuffer as a numpy array, for callers that do not want a
W*H-element list.

Error behaviour mirrors the reference: ``(0, 0, ...)`` returns ``'done'``; a width or
height of 0 with the other positive is a ``function_clause`` (ValueError here); a
malformed scene is a ``badarg`` (ValueError) instead of a crash in a worker process.
"""
from __future__ import annotations

import ctypes
import time

import numpy as np

from . import _native as N
from .records import scene as default_scene
from .terms import Atom

DONE = Atom("done")


def _sizes_ok(width, height):
    for v, n in ((width, "Width"), (height, "Height")):
        if isinstance(v, bool) or not isinstance(v, int):
            raise ValueError(f"function_clause: {n} must be an integer, got {v!r}")
    if width == 0 and height == 0:
        return False
    if not (width > 0 and height > 0):
        raise ValueError("function_clause: Width > 0, Height > 0 required (raytracer.erl:88-89)")
    return True


def _depth_ok(depth):
    if isinstance(depth, bool) or not isinstance(depth, int) or depth < 0:
        raise ValueError(f"badarg: Recursion_depth must be a non-negative integer, got {depth!r}")
    if depth >= 1 << 32:  # the C ABI's uint32_t (no other depth limit: RT_ENOMEM when it does not fit)
        raise ValueError(f"badarg: Recursion_depth {depth} does not fit the library's 32-bit depth")


def render(width: int, height: int, scene=None, depth: int = 5, *, precision: str = "f64",
           order: str = "exact", ndev: int = 1, first_dev: int = 0, row_block: int = 16,
           levels: bool = False, stats: dict | None = None, spp: int = 1, seed: int = 0, out=None,
           nshards: int = 0):
    """Render through ``rt_render`` and return a ``(height, width, 3)`` array (float64 or
    float32), plus the per-pixel levels array if ``levels``.  ``'done'`` for 0x0.
    ``out``: an existing C-contiguous array of that shape and dtype to render into (e.g.
    ``_native.pinned_empty``: pinned memory is written by DMA directly).  ``nshards``: row
    shards of the distributed split (default one per device; shard s on device s % ndev).
    ``spp`` > 1: stochastic supersampling as defined at RT_SUPERSAMPLING in
    include/rt_mi355x.h (not in the reference; levels then report sample 0).
    ``levels="hit"``: the levels array is the primary-hit mask (1 where the primary ray hits,
    RT_LEVELS_HIT) instead of the chain's level count — what the strategy funs need for the
    reference's integer pixels, without turning the fused shading kernels off."""
    if not _sizes_ok(width, height):
        return DONE
    _depth_ok(depth)
    if scene is None:
        scene = default_scene()
    elems = N.marshal(scene)
    L = N.lib()
    prec = {"f64": N.RT_OUT_F64, "f32": N.RT_OUT_F32}[precision]
    dt = np.float64 if prec == N.RT_OUT_F64 else np.float32
    if out is None:
        out = np.empty((height, width, 3), dtype=dt)
    elif out.shape != (height, width, 3) or out.dtype != dt or not out.flags.c_contiguous:
        raise ValueError(f"out must be a C-contiguous {(height, width, 3)} {np.dtype(dt).name} array")
    lv = np.empty((height, width), dtype=np.uint8) if levels else None
    opts = N.RtOpts(ctypes.sizeof(N.RtOpts), first_dev, ndev, prec,
                    {"exact": N.RT_ORDER_EXACT, "fast": N.RT_ORDER_FAST}[order], row_block,
                    lv.ctypes.data if levels else None, spp, nshards, seed,
                    N.RT_LEVELS_HIT if levels == "hit" else 0)
    st = N.RtStats()
    rc = L.rt_render(elems, len(elems), width, height, depth, ctypes.byref(opts), out.ctypes.data, ctypes.byref(st))
    if rc == N.RT_DONE:
        return DONE
    N.check(rc, "rt_render")
    if stats is not None:
        stats.update(kernel_ms=st.kernel_ms, total_ms=st.total_ms, pixels=st.pixels, ndev=st.ndev,
                     pinned=bool(st.flags & 1))
    return (out, lv) if levels else out


def _has_lights(scene) -> bool:
    from .records import tag
    return any(tag(t) == "point_light" for t in scene)


def _pixel_list(img, lv, scene, keyed: bool):
    """The strategy's result list with the reference's exact term types: the integer zeros
    #colour{r=0,g=0,b=0} where the reference returns them — no primary hit (?BACKGROUND_COLOUR,
    raytracer.erl:82, :201), depth 0 (:186-187; the hit mask is 0 there) or a scene without point
    lights (lighting_function/6 folds from #vector{0,0,0}, :250) — floats everywhere else
    (specular_term's math:pow/2 always yields a float, :289).  Keys: 1 (simple, :95) or
    X+Y*Width (:112, :173).  lv: the primary-hit mask or the level counts (0 = no hit either way)."""
    flat = img.reshape(-1, 3).tolist()
    zero = (lv.reshape(-1) == 0) if _has_lights(scene) else np.ones(len(flat), dtype=bool)
    ints = (0, 0, 0)
    if keyed:
        return [(i, ints if z else (r, g, b)) for i, ((r, g, b), z) in enumerate(zip(flat, zero.tolist()))]
    return [(1, ints if z else (r, g, b)) for (r, g, b), z in zip(flat, zero.tolist())]


def _strategy(Width, Height, Scene, Recursion_depth, keyed, ndev=1):
    if not _sizes_ok(Width, Height):
        return DONE
    if Scene is None:
        Scene = default_scene()
    img, lv = render(Width, Height, Scene, Recursion_depth, levels="hit", ndev=ndev)
    return _pixel_list(img, lv, Scene, keyed)


def raytraced_pixel_list_simple(Width, Height, Scene, Recursion_depth):
    """raytraced_pixel_list_simple/4 (raytracer.erl:86-99): ``[{1, {R,G,B}}]`` row-major."""
    return _strategy(Width, Height, Scene, Recursion_depth, keyed=False)


def raytraced_pixel_list_concurrent(Width, Height, Scene, Recursion_depth):
    """raytraced_pixel_list_concurrent/4 (raytracer.erl:101-119): ``[{X+Y*W, {R,G,B}}]``
    sorted by key (the master's lists:keysort, :155), i.e. row-major."""
    return _strategy(Width, Height, Scene, Recursion_depth, keyed=True)


def raytraced_pixel_list_distributed(Width, Height, Scene, Recursion_depth):
    """raytraced_pixel_list_distributed/4 (raytracer.erl:121-149): the same pixels and
    keys as concurrent; rows are sharded over every GPU visible to this process."""
    return _strategy(Width, Height, Scene, Recursion_depth, keyed=True, ndev=-1)


raytraced_pixel_list_gpu = raytraced_pixel_list_concurrent


def tracing_function(strategy):
    """tracing_function/1 (raytracer.erl:714-719), plus the ``gpu`` atom."""
    table = {
        "simple": raytraced_pixel_list_simple,
        "concurrent": raytraced_pixel_list_concurrent,
        "distributed": raytraced_pixel_list_distributed,
        "gpu": raytraced_pixel_list_gpu,
    }
    try:
        return table[str(strategy)]
    except KeyError:
        raise ValueError(f"function_clause: unknown strategy {strategy!r}") from None


def _erl_int(x: float) -> int:
    """trunc/1 of a float (toward zero)."""
    return int(x)


def write_pixels_to_ppm(Width, Height, MaxValue, Pixels, Filename):
    """write_pixels_to_ppm/5 (raytracer.erl:667-685): ASCII P3, every channel written as
    ``min(trunc(C*MaxValue), MaxValue)`` followed by one space; keys are ignored.
    Accepts the pixel list or a (H, W, 3) array."""
    with open(Filename, "w", encoding="ascii", newline="\n") as f:
        f.write("P3\n")
        f.write(f"{Width} {Height}\n")
        f.write(f"{MaxValue}\n")
        if isinstance(Pixels, np.ndarray):
            x = np.minimum(np.trunc(Pixels.astype(np.float64).reshape(-1, 3) * MaxValue), MaxValue)
            if np.all(x > -2.0 ** 62):
                rows = x.astype(np.int64).tolist()
            else:  # BEAM integers are unbounded: exact Python ints for huge negative values
                rows = [[int(v) for v in px] for px in x.tolist()]
            f.write("".join(f"{r} {g} {b} " for r, g, b in rows))
        else:
            parts = []
            for _key, (r, g, b) in Pixels:
                parts.append(f"{min(_erl_int(r * MaxValue), MaxValue)} {min(_erl_int(g * MaxValue), MaxValue)} "
                             f"{min(_erl_int(b * MaxValue), MaxValue)} ")
            f.write("".join(parts))


def raytrace(Width=4, Height=3, Filename="/tmp/traced.ppm", Recursion_depth=5, Function=None):
    """raytrace/1,5 (raytracer.erl:721-733): render scene() with Function, write the PPM.
    The GPU strategy goes through rt_render_ppm_file (the P3 text is produced on the GPU,
    byte-identical to write_pixels_to_ppm)."""
    if Function is None:
        Function = raytraced_pixel_list_gpu
    if Function is raytraced_pixel_list_gpu:
        return render_ppm_file(Width, Height, default_scene(), Recursion_depth, Filename)
    pixels = Function(Width, Height, default_scene(), Recursion_depth)
    return write_pixels_to_ppm(Width, Height, 255, pixels, Filename)


def render_ppm_file(width: int, height: int, scene, depth: int, filename: str, *, max_value: int = 255,
                    ndev: int = 1, first_dev: int = 0, spp: int = 1, seed: int = 0):
    """Render and write the P3 file natively (rt_render_ppm_file): raytrace/5 + write_pixels_to_ppm/5."""
    if not _sizes_ok(width, height):
        return DONE
    _depth_ok(depth)
    elems = N.marshal(scene)
    opts = N.RtOpts(ctypes.sizeof(N.RtOpts), first_dev, ndev, N.RT_OUT_F64, N.RT_ORDER_EXACT, 16, None, spp, 0, seed)
    rc = N.lib().rt_render_ppm_file(elems, len(elems), width, height, depth, ctypes.byref(opts), max_value,
                                    str(filename).encode(), None)
    if rc == N.RT_DONE:
        return DONE
    N.check(rc, "rt_render_ppm_file")
    return "ok"


def ppm_text_gpu(img, max_value: int = 255) -> bytes:
    """The P3 bytes of an (H, W, 3) frame formatted on the GPU (rt_ppm_format); RT_ERANGE
    (a channel below -2^31 after scaling) raises."""
    import torch
    L = N.lib()
    h, w, _ = img.shape
    prec = N.RT_OUT_F64 if img.dtype == np.float64 else N.RT_OUT_F32
    d = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    cap = L.rt_ppm_bound(w, h, max_value)
    buf = torch.empty(cap, dtype=torch.uint8, device="cuda")
    n = ctypes.c_size_t(0)
    st = torch.cuda.current_stream().cuda_stream
    N.check(L.rt_ppm_format(d.data_ptr(), prec, w, h, max_value, buf.data_ptr(), cap, ctypes.byref(n), st),
            "rt_ppm_format")
    return bytes(buf[: n.value].cpu().numpy())


def go(Strategy, Width=None, Height=None, Filename=None, Recursion_depth=None):
    """go/1 (4x3, depth 5, /tmp/traced.ppm; raytracer.erl:707-708, :721-722) and go/5 (:710-712)."""
    if Width is None:
        return raytrace(Function=tracing_function(Strategy))
    return raytrace(Width, Height, Filename, Recursion_depth, tracing_function(Strategy))


def standalone(Width, Height, Filename, Recursion_depth, Strategy):
    """standalone/1,5 (raytracer.erl:688-705): time raytrace/5 (PPM write included, as in
    the reference) and print ``Done in ~w seconds``."""
    t0 = time.perf_counter()
    raytrace(int(Width), int(Height), Filename, int(Recursion_depth), tracing_function(Strategy))
    dt = time.perf_counter() - t0
    print(f"Done in {dt!r} seconds")
    return dt


if __name__ == "__main__":  # python -m eraytracer_amd.raytracer W H File Depth Strategy (cf. run*.sh)
    import sys
    if len(sys.argv) != 6:
        sys.exit("usage: python -m eraytracer_amd.raytracer Width Height Filename Depth Strategy")
    standalone(*sys.argv[1:])
