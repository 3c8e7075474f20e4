"""Static checks of the BEAM shim (erlang/): there is no Erlang/OTP install here or on the GPU
box, so the modules and the NIF cannot be compiled; these checks catch the defects a
compiler or the loader would (round-1 defect: a second module loading the NIF, whose
ERL_NIF_INIT names another module, fails its on_load and is unloaded)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ERL = os.path.join(ROOT, "erlang")


def _read(*p):
    with open(os.path.join(ERL, *p)) as f:
        return f.read()


def _strip_comments(src):
    return "\n".join(ln.split("%", 1)[0] for ln in src.splitlines())


def _nif_table():
    c = _read("c_src", "rt_nif.c")
    mod = re.search(r"ERL_NIF_INIT\((\w+),", c).group(1)
    table = c[c.index("static ErlNifFunc funcs[]"):]
    table = table[:table.index("};")]
    funcs = {(n, int(a)) for n, a in re.findall(r'\{"(\w+)",\s*(\d+),', table)}
    return mod, funcs


def _exports(src):
    m = re.search(r"-export\(\[(.*?)\]\)\.", src, re.S)
    return {(n, int(a)) for n, a in re.findall(r"(\w+)/(\d+)", m.group(1))}


def test_only_the_nif_module_loads_the_nif():
    mod, _ = _nif_table()
    for fn in os.listdir(os.path.join(ERL, "src")):
        src = _strip_comments(_read("src", fn))
        name = re.search(r"-module\((\w+)\)\.", src).group(1)
        assert name + ".erl" == fn
        loads = "erlang:load_nif" in src or "-on_load" in src
        assert loads == (name == mod), f"{fn}: only module {mod} may load the NIF (ERL_NIF_INIT({mod}, ...))"


def test_nif_stubs_match_the_nif_table():
    mod, funcs = _nif_table()
    src = _strip_comments(_read("src", mod + ".erl"))
    exported = _exports(src)
    assert funcs <= exported, f"NIFs without an exported stub: {funcs - exported}"
    for name, arity in funcs:
        # a stub clause of that arity raising nif_not_loaded
        m = re.search(rf"^{name}\(([^)]*)\)\s*->\s*\n\s*erlang:nif_error\(nif_not_loaded\)", src, re.M | re.S)
        assert m, f"no stub for {name}/{arity}"
        args = [a for a in m.group(1).split(",") if a.strip()]
        stubs = {len([a for a in x.split(",") if a.strip()])
                 for x in re.findall(rf"^{name}\(([^)]*)\)\s*->\s*\n\s*erlang:nif_error", src, re.M)}
        assert arity in stubs, f"{name}/{arity}: stub arities {stubs}"
        del args


def test_strategy_module_calls_existing_nifs():
    mod, funcs = _nif_table()
    src = _strip_comments(_read("src", "raytracer_gpu.erl"))
    calls = re.findall(rf"{mod}:(\w+)\(", src)
    assert calls
    names = {n for n, _ in funcs}
    for c in calls:
        assert c in names, f"raytracer_gpu calls {mod}:{c}, which the NIF does not provide"
    # every exported function is defined with that arity
    for name, arity in _exports(src):
        heads = re.findall(rf"^{name}\(([^)]*)\)\s*->", src, re.M)
        arities = {0 if not h.strip() else len(_split_args(h)) for h in heads}
        assert arity in arities, f"raytracer_gpu exports {name}/{arity}, defined with {arities}"


def _split_args(s):
    depth, out, cur = 0, [], ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return [a for a in out if a.strip()]


def test_nif_abi_checks_and_term_rule():
    c = _read("c_src", "rt_nif.c")
    assert "rt_abi_version() == RT_ABI_VERSION" in c
    # the integer-zero rule of tests/test_oracle.py::_int_zero_rule (by the primary-hit mask;
    # none at spp > 1: a supersampled frame is an average of jittered samples, always floats)
    assert "if (!floats && (!by_hit || lv.data[i] == 0))" in c
    assert "spp > 1 ? atom_floats : lights ? atom_true : atom_false" in c
    assert "o.flags = RT_LEVELS_HIT" in c
    # the NIF's dirty calls are the ones that block on the GPU
    for fn in ("render_frame", "render_binary", "render_ppm_file"):
        assert re.search(rf'\{{"{fn}", \d, \w+, ERL_NIF_DIRTY_JOB_IO_BOUND\}}', c), fn


def test_pixels_chunk_is_bounded_and_yields():
    """pixels_chunk runs on a normal scheduler: its work per call is bounded (Count <=
    PIXELS_CHUNK_MAX, badarg beyond), it reports its timeslice use, and raytracer_gpu's chunk is
    within that bound (raytracer.erl's master delivers the list, :116-118, :155)."""
    c = _read("c_src", "rt_nif.c")
    m = re.search(r"#define PIXELS_CHUNK_MAX (\d+)", c)
    assert m
    limit = int(m.group(1))
    assert limit <= 4096
    assert "count > PIXELS_CHUNK_MAX" in c
    body = c[c.index("static ERL_NIF_TERM pixels_chunk_nif"):]
    body = body[:body.index("\n}\n")]
    assert "enif_consume_timeslice(env," in body
    assert re.search(r'\{"pixels_chunk", 5, pixels_chunk_nif, 0\}', c)  # normal scheduler, hence the bound
    erl = _strip_comments(_read("src", "raytracer_gpu.erl"))
    chunk = int(re.search(r"-define\(CHUNK, (\d+)\)", erl).group(1))
    assert 0 < chunk <= limit
