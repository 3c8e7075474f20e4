"""Seeded synthetic scenes for the benchmark configurations (BASELINE.json configs 3-5).

The reference hard-codes one scene (raytracer.erl:618-665) and lists a "randomly
generated scene" as not done (raytracer.erl:35).  The benchmark scenes are defined
here:

* **S64**  — the default camera, 4 point lights, 64 spheres; seed ``0x5EED0064``.
* **S256** — the same with 256 spheres; seed ``0x5EED0256``.

Values come from splitmix64 and are quantised to multiples of 2**-10, so every
number is exact in binary64 and in its decimal Erlang text (``terms.format_term``).
Sphere centre x∈[-12,12], y∈[-6,4], z∈[6,40]; radius∈[0.5,2]; colour∈[0,1]³;
specular power ∈ {1,4,20}; shininess∈[0,1]; reflectivity∈[0,0.7].  Lights: location
x∈[-15,15], y∈[-10,-2], z∈[-5,20]; diffuse and specular colours ∈[0.25,1]³.  Rejection
rules: no light inside (or on) a sphere, no two spheres with the same centre and radius.
"""
from __future__ import annotations

from .records import camera, colour, material, plane, point_light, screen, sphere, triangle, vector

MASK64 = (1 << 64) - 1
SEED_S64 = 0x5EED0064
SEED_S256 = 0x5EED0256


class SplitMix64:
    """splitmix64 (Steele, Lea & Flood 2014)."""

    def __init__(self, seed: int):
        self.state = seed & MASK64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def uniform(self, lo: float, hi: float) -> float:
        """lo + (hi-lo)*u, u in [0,1) with 53 bits, quantised down to a multiple of 2**-10."""
        u = (self.next_u64() >> 11) * (1.0 / (1 << 53))
        v = lo + (hi - lo) * u
        q = int((v * 1024.0) // 1) / 1024.0
        return max(lo, q)


def _default_camera():
    return camera(vector(0, 0, -2), vector(0, 0, 0), 90, screen(4, 3))


def synthetic_scene(n_spheres: int, seed: int, n_lights: int = 4):
    """A camera, `n_lights` point lights, then `n_spheres` spheres, as a scene list."""
    rng = SplitMix64(seed)
    lights = []
    for _ in range(n_lights):
        loc = (rng.uniform(-15, 15), rng.uniform(-10, -2), rng.uniform(-5, 20))
        dif = (rng.uniform(0.25, 1), rng.uniform(0.25, 1), rng.uniform(0.25, 1))
        spc = (rng.uniform(0.25, 1), rng.uniform(0.25, 1), rng.uniform(0.25, 1))
        lights.append((loc, dif, spc))
    spheres = []
    seen = set()
    powers = (1, 4, 20)
    while len(spheres) < n_spheres:
        c = (rng.uniform(-12, 12), rng.uniform(-6, 4), rng.uniform(6, 40))
        r = rng.uniform(0.5, 2.0)
        col = (rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(0, 1))
        sp = powers[rng.next_u64() % 3]
        sh = rng.uniform(0, 1)
        refl = rng.uniform(0, 0.7)
        key = (c, r)
        if key in seen:
            continue
        if any((lx - c[0]) ** 2 + (ly - c[1]) ** 2 + (lz - c[2]) ** 2 <= r * r for (lx, ly, lz), _, _ in lights):
            continue
        seen.add(key)
        spheres.append(sphere(r, vector(*c), material(colour(*col), sp, sh, refl)))
    scene = [_default_camera()]
    for loc, dif, spc in lights:
        scene.append(point_light(colour(*dif), vector(*loc), colour(*spc)))
    scene.extend(spheres)
    return scene


def s64():
    """Benchmark scene S64 (BASELINE.json configs 3-4)."""
    return synthetic_scene(64, SEED_S64)


def s256():
    """Benchmark scene S256 (BASELINE.json config 5)."""
    return synthetic_scene(256, SEED_S256)


def default_powers(powers=(0, 0.5, 2.5, 1025)):
    """The default scene (raytracer.erl:618-665) with its four objects' specular powers
    replaced by ``powers`` (cycled): by default 0 (math:pow(0, 0) = 1.0 where the highlight
    term is 0), non-integer and > 1024 exponents — the general math:pow/2 path (:289) that
    the library compiles in only for such scenes."""
    from .records import scene as default_scene
    out = []
    i = 0
    for t in default_scene():
        if t[0] in ("sphere", "triangle", "plane"):
            m = t[-1]
            t = t[:-1] + (material(m[1], powers[i % len(powers)], m[3], m[4]),)
            i += 1
        out.append(t)
    return out


def synthetic_mixed(n_spheres: int = 48, seed: int = 0x5EED0048, powers=(1, 4, 20, 0.5, 2.5, 0)):
    """A scene for the wavefront engine's mixed-object paths (more than the fused engine's 40
    objects): S-style spheres plus the default scene's triangle and plane, two more triangles
    (one facing away: back-face culled, :410) and a second plane, specular powers from
    ``powers`` (non-integer ones select the general math:pow/2 path)."""
    base = synthetic_scene(n_spheres, seed)
    rng = SplitMix64(seed ^ 0xA5A5)
    out = []
    for t in base:
        if t[0] == "sphere":
            m = t[3]
            t = sphere(t[1], t[2], material(m[1], powers[rng.next_u64() % len(powers)], m[3], m[4]))
        out.append(t)
    out.insert(5, triangle(vector(-2, 5, 5), vector(4, 5, 10), vector(4, -5, 10),
                           material(colour(1, 0.5, 0), 4, 0.25, 0.5)))
    out.append(plane(vector(0, -1, 0), 5, material(colour(1, 1, 1), 1, 0, 0.01)))
    out.append(triangle(vector(-8, -4, 20), vector(-3, 2, 22), vector(2, -4, 24),
                        material(colour(0.25, 0.75, 0.5), 2.5, 0.5, 0.25)))
    out.append(triangle(vector(2, -4, 24), vector(-3, 2, 22), vector(-8, -4, 20),
                        material(colour(0.75, 0.25, 0.5), 20, 0.5, 0.25)))
    out.append(plane(vector(1, 0, 0), 14, material(colour(0.5, 0.5, 1), 0.5, 0.25, 0.3)))
    return out


def named(name: str):
    from .records import scene as default_scene
    table = {"default": default_scene, "s64": s64, "s256": s256, "default_powers": default_powers,
             "mixed": synthetic_mixed,
             # the same mix with the reference's own kind of specular powers (integers: no general pow)
             "mixed_int": lambda: synthetic_mixed(powers=(1, 4, 20))}
    key = name.lower()
    if key in table:
        return table[key]()
    if key.startswith("s") and key[1:].isdigit() and 1 <= int(key[1:]) <= 1 << 20:
        n = int(key[1:])  # sN: N spheres, seed 0x5EED<N as (at least) four decimal digits> like S64 / S256
        return synthetic_scene(n, int(f"5EED{n:04d}", 16))
    if key.startswith("s") and "l" in key[1:]:
        a, b = key[1:].split("l", 1)  # sNlM: sN with M lights (seed as sN's)
        if a.isdigit() and b.isdigit() and 1 <= int(a) <= 1 << 20 and 0 <= int(b) <= 1 << 16:
            n = int(a)
            return synthetic_scene(n, int(f"5EED{n:04d}", 16), n_lights=int(b))
    raise ValueError(f"unknown scene {name!r}; expected one of {sorted(table)} or sN")
