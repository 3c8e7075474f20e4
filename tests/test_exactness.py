"""Exactness arguments the kernels rely on, checked on the CPU in binary64 (numpy): the reformulations
hold bit for bit on the operand ranges the kernels meet and on the edge cases around them."""
import numpy as np


def _ref_sphere(B, disc):
    """ray_sphere_intersect/2's root choice (raytracer.erl:378-383): both roots >= 0, lists:min([T0, T1])
    (the first of equal elements), for Disc >= 0.001."""
    sq = np.sqrt(disc)
    t0 = (-B + sq) / 2
    t1 = (-B - sq) / 2
    hit = (t0 >= 0) & (t1 >= 0)
    t = np.where(t1 < t0, t1, t0)
    return hit, t


def _kernel_sphere(B, disc):
    """sph_t / sph_t_wave (eraytracer_amd/csrc/rt_render.hip): the nearer root alone."""
    t = (-B - np.sqrt(disc)) / 2
    return t >= 0, t


def _check(B, disc):
    with np.errstate(invalid="ignore", over="ignore"):
        h_ref, t_ref = _ref_sphere(B, disc)
        h_k, t_k = _kernel_sphere(B, disc)
    assert np.array_equal(h_ref, h_k)
    # where the reference hits, the distance is the same binary64 value, bit for bit (signed zeros included)
    assert np.array_equal(t_ref[h_ref].view(np.uint64), t_k[h_k].view(np.uint64))


def test_nearer_root_equals_both_root_test_random():
    rng = np.random.default_rng(20261018)
    n = 2_000_000
    # distances and discriminants of unit rays against spheres of the synthetic scenes' scales, and wider
    B = rng.standard_normal(n) * 10.0 ** rng.uniform(-3, 6, n)
    disc = 0.001 + np.abs(rng.standard_normal(n)) * 10.0 ** rng.uniform(-6, 12, n)
    _check(B, disc)


def test_nearer_root_equals_both_root_test_edges():
    sq = np.sqrt(np.array([0.001, 0.0010000000000000002, 1.0, 4.0, 1e6, 1e300]))
    disc = sq * sq
    disc = np.maximum(disc, 0.001)
    sq = np.sqrt(disc)
    # B exactly at +-sqrt(disc) (a root at +0.0), one ulp either side, huge |B| (the roots round equal),
    # infinities and NaN
    cands = [sq, -sq, np.nextafter(sq, np.inf), np.nextafter(sq, -np.inf), np.nextafter(-sq, np.inf),
             np.nextafter(-sq, -np.inf), sq * 1e17, -sq * 1e17, np.full_like(sq, np.inf), np.full_like(sq, -np.inf),
             np.full_like(sq, np.nan), np.zeros_like(sq), -np.zeros_like(sq)]
    B = np.concatenate(cands)
    D = np.tile(disc, len(cands))
    _check(B, D)
    # infinite discriminants (B * B overflowing)
    _check(np.array([1e200, -1e200, 0.0, 1.0]), np.array([np.inf] * 4))
