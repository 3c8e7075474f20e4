"""ctypes wrapper of the C oracle (oracle/rt_oracle.c).  TEST INFRASTRUCTURE ONLY:
used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER
(or the timed CPU baseline), never by the product package eraytracer_amd.

Scenes are passed as the same ``rt_elem`` array the product marshals
(eraytracer_amd._native.marshal), so the oracle sees exactly what the library sees;
the independent term-level restatement (oracle/erl_restatement.py) checks the
marshalling itself.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
LITERAL, MEMO = 0, 1

_LIB = None


def build(quiet: bool = True) -> str:
    """Compile the oracle (gcc) into oracle/_build/liboracle.so."""
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        L.orc_render.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_void_p]
        L.orc_render_spp.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_render_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_focal_length.restype = ctypes.c_double
        L.orc_focal_length.argtypes = [ctypes.c_double, ctypes.c_double]
        L.orc_vec_op.argtypes = [ctypes.c_int, dp, dp, ctypes.c_double, dp]
        L.orc_intersect.argtypes = [ctypes.c_void_p, dp, dp, dp]
        L.orc_nearest.argtypes = [ctypes.c_void_p, ctypes.c_uint32, dp, dp, dp]
        L.orc_point_on_screen.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, dp]
        L.orc_shoot_ray.argtypes = [dp, dp, dp]
        L.orc_trace_pixel.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                      ctypes.c_int, dp, ctypes.POINTER(ctypes.c_int)]
        _LIB = L
    return _LIB


def _d3(v):
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def host_threads() -> int:
    """Threads for the oracle: this process's CPU share (OMP_NUM_THREADS when set — the GPU box
    sets it to its 16-CPU share, while os.cpu_count() there reports the whole machine), else
    the CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def render(elems, width, height, depth, mode=MEMO, threads=None, row0=0, nrows=None, levels=False, spp=1, seed=0):
    """Render rows [row0, row0+nrows) of a width x height image of the marshalled scene
    `elems`; returns a (nrows, width, 3) float64 array (and the levels array).  spp > 1:
    stochastic supersampling as defined at RT_SUPERSAMPLING in include/rt_mi355x.h."""
    if nrows is None:
        nrows = height - row0
    if threads is None:
        threads = host_threads()
    out = np.zeros((nrows, width, 3), dtype=np.float64)
    lv = np.zeros((nrows, width), dtype=np.uint8) if levels else None
    rc = lib().orc_render_spp(ctypes.cast(elems, ctypes.c_void_p), len(elems), width, height, row0, nrows, depth,
                              mode, threads, spp, seed, out.ctypes.data, lv.ctypes.data if levels else None)
    if rc != 0:
        raise ValueError(f"oracle render failed: {rc}")
    return (out, lv) if levels else out


def render_rows(elems, width, height, rows, depth, mode=MEMO, threads=None, spp=1, seed=0):
    """Render the listed image rows in one threaded call (the rows shared out over `threads`
    threads through one counter).  Returns ((len(rows), width, 3) float64 array, the number of
    threads that rendered at least one row)."""
    if threads is None:
        threads = host_threads()
    rows = np.ascontiguousarray(np.asarray(rows, dtype=np.uint32))
    out = np.zeros((len(rows), width, 3), dtype=np.float64)
    rc = lib().orc_render_rows(ctypes.cast(elems, ctypes.c_void_p), len(elems), width, height, rows.ctypes.data,
                               len(rows), depth, mode, threads, spp, seed, out.ctypes.data, None)
    if rc < 1:
        raise ValueError(f"oracle render_rows failed: {rc}")
    return out, int(rc)


OPS = {"add": 0, "sub": 1, "square_mag": 2, "mag": 3, "scalar_mult": 4, "component_mult": 5, "dot": 6,
       "cross": 7, "normalize": 8, "neg": 9, "bounce": 10}


def vec_op(op, a, b=(0, 0, 0), s=0.0):
    out = (ctypes.c_double * 3)()
    lib().orc_vec_op(OPS[op], _d3(a), _d3(b), float(s), out)
    return tuple(out)


def focal_length(angle, dimension):
    return lib().orc_focal_length(float(angle), float(dimension))


def intersect(elem, origin, direction):
    out = (ctypes.c_double * 7)()
    hit = lib().orc_intersect(ctypes.byref(elem), _d3(origin), _d3(direction), out)
    return (out[0], tuple(out[1:4]), tuple(out[4:7])) if hit else None


def nearest(elems, origin, direction):
    out = (ctypes.c_double * 7)()
    i = lib().orc_nearest(ctypes.cast(elems, ctypes.c_void_p), len(elems), _d3(origin), _d3(direction), out)
    return (i, out[0], tuple(out[1:4]), tuple(out[4:7])) if i >= 0 else None


def point_on_screen(cam_elem, X, Y):
    out = (ctypes.c_double * 3)()
    lib().orc_point_on_screen(ctypes.byref(cam_elem), float(X), float(Y), out)
    return tuple(out)


def shoot_ray(frm, through):
    out = (ctypes.c_double * 3)()
    lib().orc_shoot_ray(_d3(frm), _d3(through), out)
    return tuple(out)


def trace_pixel(elems, X, Y, depth, mode=MEMO):
    out = (ctypes.c_double * 3)()
    lv = ctypes.c_int(0)
    lib().orc_trace_pixel(ctypes.cast(elems, ctypes.c_void_p), len(elems), float(X), float(Y), depth, mode, out,
                          ctypes.byref(lv))
    return tuple(out), lv.value
