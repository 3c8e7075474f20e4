"""The C-ABI boundary on the CPU: the library loads without a GPU, exports every entry
point include/rt_mi355x.h declares, and its host-only functions (scene validation,
canonical ids, shard arithmetic, error strings) behave as documented.  No render runs."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from eraytracer_amd import _native as N
from eraytracer_amd import records as R
from eraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt_mi355x.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_]+)\s*\(", src)))


def test_header_declares_the_exports():
    assert declared_functions() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol(native):
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True)
    syms = {ln.split()[-1] for ln in out.stdout.splitlines() if ln.strip()}
    missing = [f for f in declared_functions() if f not in syms]
    assert not missing, missing


def test_library_targets_gfx950(tmp_path):
    # --offloading extracts the bundled code objects next to its input: work on a copy
    lib = tmp_path / "lib.so"
    shutil.copyfile(N.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True)
    assert "gfx950" in out.stdout + out.stderr


def test_abi_version_and_errors(native):
    L = native.lib()
    assert L.rt_abi_version() == 5
    for code in (N.RT_OK, N.RT_DONE, N.RT_EBADARG, N.RT_ENODEV, N.RT_EHIP, N.RT_ENOMEM, N.RT_ETOOBIG):
        assert N.strerror(code) and N.strerror(code) != "unknown error"
    assert N.strerror(-99) == "unknown error"


def test_struct_layout_matches_header():
    # sizes the C compiler sees for the boundary structs
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "rt_mi355x.h"
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(rt_elem), sizeof(rt_opts), sizeof(rt_stats),
 offsetof(rt_elem, u), offsetof(rt_opts, out_levels), offsetof(rt_opts, spp), offsetof(rt_opts, seed)); return 0;}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe], check=True)
        got = list(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    assert got == [ctypes.sizeof(N.RtElem), ctypes.sizeof(N.RtOpts), ctypes.sizeof(N.RtStats),
                   N.RtElem.u.offset, N.RtOpts.out_levels.offset, N.RtOpts.spp.offset, N.RtOpts.seed.offset]


def test_scene_check(native):
    L = native.lib()
    el = N.marshal(R.scene())
    assert L.rt_scene_check(el, len(el)) == N.RT_OK
    assert L.rt_scene_check(el, 0) == N.RT_EBADARG            # [] does not match [Camera|Rest]
    bad = N.marshal(R.scene())
    bad[0].kind = N.RT_SPHERE                                 # head is not a camera
    assert L.rt_scene_check(bad, len(bad)) == N.RT_EBADARG
    nan = N.marshal(R.scene())
    nan[3].u.sphere.radius = float("nan")                     # Erlang has no NaN
    assert L.rt_scene_check(nan, len(nan)) == N.RT_EBADARG
    canon = N.marshal(R.scene())
    canon[4].canon = 3                                        # canon must point at an equal-kind element
    canon[4].kind = N.RT_TRIANGLE
    assert L.rt_scene_check(canon, len(canon)) == N.RT_EBADARG
    big = N.marshal(scenes.synthetic_scene(8, 1))
    assert L.rt_scene_check(big, len(big)) == N.RT_OK


def test_scene_canon_bitwise_rule(native):
    L = native.lib()
    s = R.scene() + [R.sphere(4, R.vector(4, 0, 10), R.material(R.colour(0, 0.5, 1), 20, 1, 0.1))]
    el = N.marshal(s)
    assert el[len(s) - 1].canon == 3                           # =:= copy of element 3
    for e in el:
        e.canon = -1
    assert L.rt_scene_canon(el, len(el)) == N.RT_OK
    assert el[len(s) - 1].canon == 3 and el[3].canon == 3 and el[4].canon == 4


def test_no_count_limits(native):
    """Scenes of any size validate (the reference scans any list and folds over every light,
    raytracer.erl:300-346, :209-252): 5,000 spheres, 100 lights."""
    L = native.lib()
    for sc in (scenes.named("s5000"), scenes.named("s64l100"), scenes.synthetic_scene(16, 7, n_lights=300)):
        el = N.marshal(sc)
        assert L.rt_scene_check(el, len(el)) == N.RT_OK


def test_tables_past_32_bit_offsets_are_enomem(native):
    """The only size limit left (include/rt_mi355x.h): a scene whose per-origin tables (about 16
    doubles per origin and object; the origins are the camera and every light) would not fit the
    kernels' 32-bit offsets fails with RT_ENOMEM — from the host compiler, before any device call,
    so this runs on the CPU."""
    import ctypes
    L = native.lib()
    base = scenes.s64()
    light = [t for t in base if t[0] == "point_light"][0]
    spheres = [t for t in base if t[0] == "sphere"]
    scene = base[:1] + [light] * 70000 + spheres * 16  # 70,001 origins x 1,024 spheres (copies: canon)
    el = N.marshal(scene)
    assert L.rt_scene_check(el, len(el)) == N.RT_OK
    p = ctypes.c_void_p()
    assert L.rt_prepare(el, len(el), 0, ctypes.byref(p)) == N.RT_ENOMEM


def test_scene_canon_large_matches_prefix_rule(native):
    """rt_scene_canon (hashed) against the definition — the first earlier self-canonical element of
    the same kind with the same payload bytes — on a 3,000-element list with planted duplicates
    (some with caller-given canon values)."""
    import random
    L = native.lib()
    base = scenes.synthetic_scene(1500, 11, n_lights=8)
    rnd = random.Random(5)
    sc = list(base)
    for _ in range(1500):
        sc.insert(rnd.randrange(1, len(sc) + 1), base[rnd.randrange(1, len(base))])
    el = N.marshal(sc)
    want = []
    for i in range(len(el)):
        el[i].canon = -1 if rnd.random() < 0.9 else i  # a few elements claim to be their own class
    given = [e.canon for e in el]
    nb = {N.RT_CAMERA: 72, N.RT_POINT_LIGHT: 72, N.RT_SPHERE: 80, N.RT_TRIANGLE: 120, N.RT_PLANE: 80}
    raw = [bytes(e.u)[:nb.get(e.kind, 0)] for e in el]
    for i in range(len(el)):
        c = given[i]
        if c < 0:
            c = i
            if nb.get(el[i].kind, 0):
                for j in range(i):
                    if el[j].kind == el[i].kind and want[j] == j and raw[j] == raw[i]:
                        c = j
                        break
        want.append(c)
    assert L.rt_scene_canon(el, len(el)) == N.RT_OK
    assert [e.canon for e in el] == want


def test_marshal_badarg():
    with pytest.raises(ValueError):
        N.marshal([])
    with pytest.raises(ValueError):
        N.marshal([R.sphere(1, R.vector(0, 0, 0), R.material(R.colour(1, 1, 1), 1, 1, 1))])
    with pytest.raises(ValueError):  # the reference's test sphere: material fields undefined
        N.marshal(R.scene() + [R.sphere(3, R.vector(0, 0, 10), R.material(R.colour(0.4, 0.4, 0.4),
                                                                           "undefined", "undefined", "undefined"))])
    with pytest.raises(ValueError):  # a #colour{} where a #vector{} is read
        N.marshal(R.scene()[:1] + [R.point_light(R.colour(1, 1, 1), R.colour(0, 0, 0), R.colour(1, 1, 1))])


def test_shard_rows(native):
    L = native.lib()
    from eraytracer_amd.dist import shard_rows
    for h, rb, ns in [(4096, 16, 1), (4096, 16, 8), (70, 16, 3), (1, 16, 8), (100, 7, 5)]:
        assert L.rt_shard_rows(h, rb, ns) == shard_rows(h, rb, ns)
    assert L.rt_shard_rows(10, 0, 1) == 0


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-device path")
def test_render_without_device_fails_loudly(native):
    from eraytracer_amd.raytracer import render
    with pytest.raises(N.RtError) as ei:
        render(8, 6, R.scene(), 2)
    assert ei.value.code == N.RT_ENODEV
    assert render(0, 0, R.scene(), 2) == "done"
    with pytest.raises(ValueError):
        render(0, 6, R.scene(), 2)
    with pytest.raises(ValueError):
        render(8, 6, R.scene(), -1)


def test_slab_header_size_and_configure_args(native):
    """Host-only parts of the compact-gather codec and the per-context options: the header
    size matches the documented layout (tests/slab_ref.py); bad arguments are refused."""
    from tests.slab_ref import layout
    L = native.lib()
    for w, h, rb, ns in [(4096, 4096, 16, 8), (33, 17, 4, 2), (1, 1, 16, 1), (257, 31, 5, 4), (1920, 1080, 16, 3)]:
        assert L.rt_slab_header_bytes(w, h, rb, ns) == layout(w, h, rb, ns)[3]
    assert L.rt_slab_header_bytes(0, 10, 16, 1) == 0
    assert L.rt_slab_header_bytes(10, 10, 0, 1) == 0
    assert L.rt_configure(None, N.RT_CFG_SIDE_STREAMS, 0) == N.RT_EBADARG
    assert L.rt_slab_pack(None, 8, 8, 16, 0, 1, N.RT_OUT_F32, None, None, None) == N.RT_EBADARG
    bad = (ctypes.c_void_p * 1)(None)
    assert L.rt_slab_unpack(bad, bad, 8, 8, 16, 1, N.RT_OUT_F32, None, None) == N.RT_EBADARG
