"""Host logic on the CPU: Erlang term text, scenes, the P3 writer, the work model."""
import os

import numpy as np
import pytest

from eraytracer_amd import records as R
from eraytracer_amd import scenes, terms, workload
from eraytracer_amd.raytracer import tracing_function, write_pixels_to_ppm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_term_roundtrip():
    cases = [R.scene(), scenes.s64(), [1, -2, 3.5, 1e-5, 1.0e16, terms.Atom("ok"), terms.Atom("Quoted atom"),
                                       (terms.Atom("t"), [], ())]]
    for t in cases:
        txt = terms.format_term(t)
        assert terms.exact_eq(terms.parse_term(txt + "."), t)


def test_term_parser_features():
    t = terms.parse_terms("% comment\n{a, 16#ff, -3, 2.5e-3, 'b c', \"hi\", [1|[2]]}.\n[x].")
    assert len(t) == 2
    a = t[0]
    assert a[1] == 255 and a[2] == -3 and a[3] == 2.5e-3 and a[4] == "b c" and a[5] == [104, 105]
    assert a[6] == [1, 2]
    with pytest.raises(ValueError):
        terms.parse_term("{1,")


def test_exact_eq():
    assert terms.exact_eq((terms.Atom("v"), 4, 0.5), (terms.Atom("v"), 4, 0.5))
    assert not terms.exact_eq(4, 4.0)
    assert not terms.exact_eq([1], (1,))


def test_synthetic_scenes_are_deterministic_and_valid():
    a, b = scenes.s64(), scenes.s64()
    assert terms.exact_eq(a, b)
    c = workload.scene_counts(a)
    assert c == {"spheres": 64, "triangles": 0, "planes": 0, "lights": 4}
    assert workload.scene_counts(scenes.s256())["spheres"] == 256
    lights = [t[2][1:] for t in a if t[0] == "point_light"]
    for t in a:
        if t[0] == "sphere":
            r, c3 = t[1], t[2][1:]
            assert 0.5 <= r <= 2.0 and -12 <= c3[0] <= 12 and -6 <= c3[1] <= 4 and 6 <= c3[2] <= 40
            assert all(sum((lx - cx) ** 2 for lx, cx in zip(L, c3)) > r * r for L in lights)
            for v in (r,) + tuple(c3) + tuple(t[3][1][1:]) + tuple(t[3][2:]):
                assert float(v) * 1024 == int(float(v) * 1024)  # multiples of 2**-10
    assert not terms.exact_eq(scenes.s64(), scenes.synthetic_scene(64, 1))


def test_tracing_function():
    for s in ("simple", "concurrent", "distributed", "gpu"):
        assert callable(tracing_function(s))
    with pytest.raises(ValueError):
        tracing_function("bogus")


def test_ppm_writer_matches_reference_format(tmp_path, oracle):
    """write_pixels_to_ppm/5 (raytracer.erl:667-685), byte for byte against the golden
    files rendered for run.sh and run-concurrent.sh."""
    from eraytracer_amd import _native as N
    for fn, w, h, d in (("run_sh_32x24_d1.ppm", 32, 24, 1), ("run_concurrent_sh_16x12_d1.ppm", 16, 12, 1)):
        img = oracle.render(N.marshal(R.scene()), w, h, d, mode=oracle.MEMO)
        out = tmp_path / fn
        write_pixels_to_ppm(w, h, 255, [(i, tuple(p)) for i, p in enumerate(img.reshape(-1, 3).tolist())], str(out))
        assert out.read_bytes() == open(os.path.join(GOLDEN, fn), "rb").read()
        out2 = tmp_path / ("arr_" + fn)
        write_pixels_to_ppm(w, h, 255, img, str(out2))  # array form, same bytes
        assert out2.read_bytes() == out.read_bytes()


def test_ppm_clamps_only_above(tmp_path):
    p = tmp_path / "x.ppm"
    write_pixels_to_ppm(3, 1, 255, [(1, (2.5, -0.4, 0)), (1, (1.0, 0.999, -0.0)), (1, (0.5, 0, 0))], str(p))
    assert p.read_text() == "P3\n3 1\n255\n255 -102 0 255 254 0 127 0 0 "


def test_work_model():
    c = {"spheres": 2, "triangles": 1, "planes": 1, "lights": 2}
    sc = 2 * 20 + 48 + 15
    # one pixel missing everything (1 scan), one hitting twice at depth 2 (2 scans, 2 hits)
    hist = [1, 0, 1]
    want = (31 + sc) + (31 + 2 * sc + 2 * (27 + 18 + 2 * (77 + sc)))
    assert workload.ops_from_levels(hist, 2, c) == want
    # depth 0: no scans at all
    assert workload.ops_from_levels([5], 0, c) == 5 * 31
    # no lights: a hit ends the chain
    c0 = dict(c, lights=0)
    assert workload.ops_from_levels([0, 1], 5, c0) == 31 + sc + 27 + 18
    assert np.array_equal(workload.levels_histogram(np.array([[0, 2], [2, 1]]), 3), [1, 1, 2, 0])


def test_scene_compiler_under_host_sanitizers(tmp_path):
    """The library's host code that parses caller input (rt_scene.cpp: check, canon, compile)
    built with AddressSanitizer + UBSan (host only; GPU sanitizers are unavailable) and run on
    the default, S64, S256 and adversarial scenes plus a truncated list and a lone camera."""
    import shutil
    import subprocess

    from eraytracer_amd import _native as N
    from tests.test_oracle import TRICKY
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "scene_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", os.path.join(root, "tests", "csrc", "scene_check.cpp"),
                    os.path.join(root, "eraytracer_amd", "csrc", "rt_scene.cpp"), "-o", exe], check=True)
    scenes_ = [R.scene(), scenes.s64(), scenes.s256()] + [mk() for mk in TRICKY]
    files = []
    for i, sc in enumerate(scenes_):
        el = N.marshal(sc)
        p = tmp_path / f"s{i}.bin"
        p.write_bytes(bytes(el))
        files.append(str(p))
    lone = tmp_path / "lone.bin"
    lone.write_bytes(bytes(N.marshal(R.scene()[:1])))
    files.append(str(lone))
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [ln.split() for ln in r.stdout.splitlines()]
    assert len(rows) == len(files)
    for row in rows[:len(scenes_)]:
        assert row[0] == "0" and row[2] == "0", row  # valid scenes compile
