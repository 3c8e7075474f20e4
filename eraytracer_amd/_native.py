"""ctypes binding of the C-ABI library ``librtmi355x.so`` (include/rt_mi355x.h) and the
marshalling of a reference scene list into ``rt_elem`` records.

This is the Python analogue of the erl_nif shim a BEAM host would use:
it walks the scene list in order, maps each record (raytracer.erl:72-81) to an
``rt_elem``, and computes ``canon`` with Erlang's exact equality (=:=), which
shadow_factor/4's match relies on (raytracer.erl:263).

There is no fallback: if the library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os

from .records import tag
from .terms import exact_key

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_LIB_PATH") or os.path.join(HERE, "librtmi355x.so")  # override: A/B builds

RT_OK, RT_DONE, RT_EBADARG, RT_ENODEV, RT_EHIP, RT_ENOMEM, RT_ETOOBIG = 0, 1, -1, -2, -3, -4, -5
RT_ERANGE = -6
RT_CAMERA, RT_POINT_LIGHT, RT_SPHERE, RT_TRIANGLE, RT_PLANE, RT_OTHER = range(6)
RT_OUT_F64, RT_OUT_F32 = 0, 1
RT_ORDER_EXACT, RT_ORDER_FAST = 0, 1
RT_MAX_SHARDS = 64
RT_CFG_SIDE_STREAMS = 1
RT_CFG_KERNEL_TIMING = 2
RT_CFG_CULL = 3
RT_KT_PRIMARY, RT_KT_LEVEL1, RT_KT_RENDER, RT_KT_PMASK = 1, 2, 4, 8
RT_LEVELS_HIT = 1
RT_ENGINE_WAVE, RT_ENGINE_FUSED = 0, 1

# every symbol include/rt_mi355x.h declares (tests/test_boundary.py checks the export list)
EXPORTS = (
    "rt_abi_version", "rt_strerror", "rt_device_count", "rt_scene_check", "rt_scene_canon",
    "rt_render", "rt_prepare", "rt_shard_rows", "rt_launch", "rt_launch_spp", "rt_unshard", "rt_configure", "rt_release",
    "rt_update_scene",
    "rt_ppm_bound", "rt_ppm_format", "rt_render_ppm_file",
    "rt_slab_header_bytes", "rt_slab_pack", "rt_slab_unpack", "rt_selftest_math",
    "rt_host_alloc", "rt_host_free", "rt_reset_contexts", "rt_kernel_time", "rt_engine",
)


class RtVec3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_double), ("y", ctypes.c_double), ("z", ctypes.c_double)]


class RtMaterial(ctypes.Structure):
    _fields_ = [("colour", RtVec3), ("specular_power", ctypes.c_double), ("shininess", ctypes.c_double),
                ("reflectivity", ctypes.c_double)]


class _Camera(ctypes.Structure):
    _fields_ = [("location", RtVec3), ("rotation", RtVec3), ("fov", ctypes.c_double),
                ("screen_width", ctypes.c_double), ("screen_height", ctypes.c_double)]


class _Light(ctypes.Structure):
    _fields_ = [("diffuse_colour", RtVec3), ("location", RtVec3), ("specular_colour", RtVec3)]


class _Sphere(ctypes.Structure):
    _fields_ = [("radius", ctypes.c_double), ("center", RtVec3), ("material", RtMaterial)]


class _Triangle(ctypes.Structure):
    _fields_ = [("v1", RtVec3), ("v2", RtVec3), ("v3", RtVec3), ("material", RtMaterial)]


class _Plane(ctypes.Structure):
    _fields_ = [("normal", RtVec3), ("distance", ctypes.c_double), ("material", RtMaterial)]


class _U(ctypes.Union):
    _fields_ = [("camera", _Camera), ("point_light", _Light), ("sphere", _Sphere), ("triangle", _Triangle),
                ("plane", _Plane), ("raw", ctypes.c_double * 12)]


class RtElem(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("canon", ctypes.c_int32), ("u", _U)]


class RtOpts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("first_dev", ctypes.c_int32), ("ndev", ctypes.c_int32),
                ("precision", ctypes.c_int32), ("order", ctypes.c_int32), ("row_block", ctypes.c_uint32),
                ("out_levels", ctypes.c_void_p), ("spp", ctypes.c_uint32), ("nshards", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("flags", ctypes.c_uint32)]


class RtStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double), ("pixels", ctypes.c_uint64),
                ("ndev", ctypes.c_int32), ("flags", ctypes.c_int32)]


class RtError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = strerror(code) if _LIB is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


_LIB = None


def lib() -> ctypes.CDLL:
    """Load librtmi355x.so (built in-tree by ``__graft_entry__.build()``)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                           "g.build()'` (there is no CPU fallback)")
    # torch bundles its own libamdhip64.so.7; load it first so this library binds to the
    # same HIP runtime instance (same soname) instead of a second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except Exception:  # torch is plumbing only; the library works without it
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.rt_abi_version.restype = i32
    L.rt_strerror.restype = ctypes.c_char_p
    L.rt_strerror.argtypes = [i32]
    L.rt_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.rt_scene_check.argtypes = [ctypes.POINTER(RtElem), u32]
    L.rt_scene_canon.argtypes = [ctypes.POINTER(RtElem), u32]
    L.rt_render.argtypes = [ctypes.POINTER(RtElem), u32, u32, u32, u32, ctypes.POINTER(RtOpts), vp,
                            ctypes.POINTER(RtStats)]
    L.rt_prepare.argtypes = [ctypes.POINTER(RtElem), u32, i32, ctypes.POINTER(vp)]
    L.rt_shard_rows.restype = u32
    L.rt_shard_rows.argtypes = [u32, u32, u32]
    L.rt_launch.argtypes = [vp, u32, u32, u32, u32, u32, u32, i32, i32, vp, vp, vp]
    L.rt_launch_spp.argtypes = [vp, u32, u32, u32, u32, u32, u32, i32, i32, u32, ctypes.c_uint64, vp, vp, vp]
    L.rt_ppm_bound.restype = ctypes.c_size_t
    L.rt_ppm_bound.argtypes = [u32, u32, u32]
    L.rt_ppm_format.argtypes = [vp, i32, u32, u32, u32, vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), vp]
    L.rt_render_ppm_file.argtypes = [vp, u32, u32, u32, u32, vp, u32, ctypes.c_char_p, vp]
    L.rt_unshard.argtypes = [vp, u32, u32, u32, u32, i32, vp, vp]
    L.rt_release.argtypes = [vp]
    L.rt_update_scene.argtypes = [vp, ctypes.POINTER(RtElem), u32]
    L.rt_configure.argtypes = [vp, i32, ctypes.c_int64]
    L.rt_engine.argtypes = [vp, u32]
    L.rt_selftest_math.argtypes = [i32, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.rt_slab_header_bytes.restype = ctypes.c_size_t
    L.rt_slab_header_bytes.argtypes = [u32, u32, u32, u32]
    L.rt_slab_pack.argtypes = [vp, u32, u32, u32, u32, u32, i32, vp, vp, vp]
    L.rt_slab_unpack.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), u32, u32, u32, u32, i32, vp, vp]
    L.rt_host_alloc.restype = vp
    L.rt_host_alloc.argtypes = [ctypes.c_size_t]
    L.rt_host_free.argtypes = [vp]
    L.rt_reset_contexts.restype = i32
    L.rt_kernel_time.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64), i32]
    _LIB = L
    return L


def strerror(code: int) -> str:
    return lib().rt_strerror(code).decode()


def check(code: int, what: str = "") -> int:
    if code < 0:
        raise RtError(code, what)
    return code


class _Pinned:
    """Owner of one rt_host_alloc block (freed when the last array viewing it goes away)."""

    def __init__(self, nbytes: int):
        self.ptr = lib().rt_host_alloc(nbytes)
        if not self.ptr:
            raise MemoryError(f"rt_host_alloc({nbytes}) failed")
        self.nbytes = nbytes

    def __del__(self):
        if getattr(self, "ptr", None) and _LIB is not None:
            _LIB.rt_host_free(self.ptr)
            self.ptr = None


def pinned_empty(shape, dtype):
    """A numpy array in pinned host memory (rt_host_alloc): rt_render writes it by DMA."""
    import numpy as np
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    owner = _Pinned(max(n, 1))
    buf = (ctypes.c_char * max(n, 1)).from_address(owner.ptr)
    buf._owner = owner  # keeps the block alive while the array exists
    return np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)


# ---- marshalling ------------------------------------------------------------------------
def _num(x, what):
    if isinstance(x, bool) or not isinstance(x, (int, float)):
        raise ValueError(f"badarg: {what} is not a number: {x!r}")
    if isinstance(x, int) and abs(x) > (1 << 53):
        raise ValueError(f"badarg: {what} = {x} is not exact in binary64")
    return float(x)


def _vec(t, what, rtag=None):
    if not (isinstance(t, tuple) and len(t) == 4 and tag(t) is not None):
        raise ValueError(f"badarg: {what} is not a 3-field record: {t!r}")
    if rtag is not None and t[0] != rtag:  # Rec#vector.x / #colour{} matches crash otherwise
        raise ValueError(f"badarg: {what} is a {t[0]}, expected {rtag}")
    return RtVec3(_num(t[1], what + ".x"), _num(t[2], what + ".y"), _num(t[3], what + ".z"))


def _mat(t, what):
    if not (isinstance(t, tuple) and len(t) == 5 and t[0] == "material"):
        raise ValueError(f"badarg: {what} is not a #material{{}}: {t!r}")
    return RtMaterial(_vec(t[1], what + ".colour", "colour"), _num(t[2], what + ".specular_power"),
                      _num(t[3], what + ".shininess"), _num(t[4], what + ".reflectivity"))


def marshal(scene) -> "ctypes.Array[RtElem]":
    """Scene list -> rt_elem array, in list order (element 0 must be the camera)."""
    if not isinstance(scene, list) or not scene:
        raise ValueError("badarg: the scene must be a non-empty list whose head is a #camera{}")
    n = len(scene)
    arr = (RtElem * n)()
    first = {}  # exact_key -> index of the first element =:= to it
    for i, t in enumerate(scene):
        e = arr[i]
        k = tag(t)
        w = f"scene element {i}"
        if k == "camera" and len(t) == 5:
            e.kind = RT_CAMERA
            scr = t[4]
            if not (isinstance(scr, tuple) and len(scr) == 3 and scr[0] == "screen"):
                raise ValueError(f"badarg: {w}.screen is not a #screen{{}}")
            rot = t[2]  # never read by the reference (rotation is a TODO, raytracer.erl:487)
            try:
                rot = _vec(rot, w + ".rotation")
            except ValueError:
                rot = RtVec3(0.0, 0.0, 0.0)
            e.u.camera = _Camera(_vec(t[1], w + ".location", "vector"), rot,
                                 _num(t[3], w + ".fov"), _num(scr[1], w + ".screen.width"),
                                 _num(scr[2], w + ".screen.height"))
        elif k == "point_light" and len(t) == 4:
            e.kind = RT_POINT_LIGHT
            e.u.point_light = _Light(_vec(t[1], w + ".diffuse_colour", "colour"),
                                     _vec(t[2], w + ".location", "vector"),
                                     _vec(t[3], w + ".specular_colour", "colour"))
        elif k == "sphere" and len(t) == 4:
            e.kind = RT_SPHERE
            e.u.sphere = _Sphere(_num(t[1], w + ".radius"), _vec(t[2], w + ".center", "vector"),
                                 _mat(t[3], w + ".material"))
        elif k == "triangle" and len(t) == 5:
            e.kind = RT_TRIANGLE
            e.u.triangle = _Triangle(_vec(t[1], w + ".v1", "vector"), _vec(t[2], w + ".v2", "vector"),
                                     _vec(t[3], w + ".v3", "vector"), _mat(t[4], w + ".material"))
        elif k == "plane" and len(t) == 4:
            e.kind = RT_PLANE
            e.u.plane = _Plane(_vec(t[1], w + ".normal", "vector"), _num(t[2], w + ".distance"),
                               _mat(t[3], w + ".material"))
        else:
            if i == 0:
                raise ValueError("badarg: the scene's first element must be a #camera{} (raytracer.erl:180)")
            e.kind = RT_OTHER
        # canon: first element exactly equal (=:=) to this one
        e.canon = first.setdefault(exact_key(t), i)
    if arr[0].kind != RT_CAMERA:
        raise ValueError("badarg: the scene's first element must be a #camera{} (raytracer.erl:180)")
    return arr
