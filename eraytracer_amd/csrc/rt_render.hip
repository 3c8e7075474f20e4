// rt_render.hip — the MI355X (gfx950) render kernel and the C-ABI of include/rt_mi355x.h.
//
// One work-item per pixel; a wave covers an 8x8 pixel tile (coherent rays), a 256-thread
// workgroup a 16x16 tile.  Per pixel the kernel runs trace_ray_through_pixel/3
// (raytracer.erl:180-184) and everything below it, in IEEE binary64 with the
// reference's operation order and no contraction (-ffp-contract=off + the pragma
// below): the geometry (every hit/miss decision, every hit point and normal) is
// bit-identical to the reference; colours differ from libm only where device pow()
// differs from the host's by an ulp.
//
// Work per hit level (the reference's recursion, raytracer.erl:186-252):
//   * one nearest-object scan (nearest_object_intersecting_ray/6, :303-346) — objects are
//     grouped by type, each type a wave-uniform loop reading its records with scalar
//     loads (uniform index -> s_load into SGPRs, the FP64 VALU reads them directly);
//   * per point light, diffuse + specular shading and one shadow test
//     (shadow_factor/4, :256-267).  The reference's test is "the nearest object seen
//     from the light is the hit object"; it is restated exactly as a bounded any-hit
//     test: with t* = the hit object's own distance along the shadow ray, the light is
//     blocked iff some object has a valid hit with t < t*, or t == t* and an earlier list
//     position.  That lets a lane stop at the first blocker and the wave leave the loop
//     as soon as every lane is decided (a wave-wide ballot).
// The reflection the reference recomputes once per light (:216-224) is the same value
// every time; it is computed once (ORDER_EXACT keeps the reference's summation order by
// shading the chain backwards from its deepest hit; ORDER_FAST accumulates forwards).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_layout.h"
#include "rt_internal.h"
#include "rt_scene.h"

using namespace rtl;

namespace {

constexpr int BLOCK = 256; // 4 waves, 16x16 pixels


// Occupancy target (waves per SIMD); the default is chosen by measurement.
#ifndef RT_WAVES_PER_SIMD
#define RT_WAVES_PER_SIMD 4
#endif
#if RT_WAVES_PER_SIMD > 0
#define RT_LAUNCH_BOUNDS __launch_bounds__(256, RT_WAVES_PER_SIMD)
#else
#define RT_LAUNCH_BOUNDS __launch_bounds__(256)
#endif
constexpr int TILE = 16;

struct D3 {
    double x, y, z;
};

__device__ __forceinline__ double dot3(const D3 &a, const D3 &b) { // vector_dot_product/2 (:546-547)
    return a.x * b.x + a.y * b.y + a.z * b.z;
}

// ---- correctly rounded sqrt and division, bit for bit the compiler's, minus range handling --
// The device sqrt(double) is v_rsq_f64 refined by one Goldschmidt and two Newton steps, wrapped
// in a scaling for inputs below 2^-767 and fix-ups for 0 and inf; 1.0/b is v_rcp_f64 refined
// twice, one correction step, wrapped in v_div_scale / v_div_fmas / v_div_fixup, which leave
// operands and results unchanged for normal-range values.  The *_n forms are those refinement
// sequences alone (operand for operand, so the same bits) and are used only where every lane's
// operand is inside the range where the wrappers are the identity; *_x check that for the wave
// (one compare and a ballot) and otherwise take the full device sequence.  About 40 % fewer
// VALU instructions per normalize (S64 4096^2 d5: 25.3 -> 26.4 Gpx/s).  Not used in the beam
// culling: there the extra wave-uniform branches cost more than they saved (measured).
constexpr double SQRT_N_LO = 0x1p-767, SQRT_N_HI = 0x1p1000;
constexpr double RCP_N_LO = 0x1p-400, RCP_N_HI = 0x1p400;

__device__ __forceinline__ double sqrt_n(double x) {
    const double s = __builtin_amdgcn_rsq(x);
    double g = x * s;
    double h = s * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}

// a / b for |b| in [RCP_N_LO, RCP_N_HI] and |a| small enough that a/b is a normal number or 0
__device__ __forceinline__ double div_n(double a, double b) {
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    const double q = a * y;
    const double r = __builtin_fma(-b, q, a);
    return __builtin_fma(r, y, q);
}

// a / n for a frame dimension n (W, H; 1 <= n <= 2^20) and 0 <= a < 2^44 exactly representable:
// for a power of two the quotient is exact, so the correctly rounded division is the exponent
// shift (one v_ldexp_f64 instead of v_rcp_f64 and seven fma / mul) — the same bits.  n (uniform)
// is made opaque where it is used: otherwise the compiler hoists (double) n and its reciprocal out
// of the kernels' record loops into VGPRs that stay live (and spilled) across everything.
// A wave-uniform value made opaque where it is used: a test on it (and what the compiler derives from
// it) is evaluated there, in a few SALU instructions, instead of being hoisted out of the record loops
// as a 64-bit condition mask held in SGPRs — which spilled to VGPR lanes (v_writelane / v_readlane).
template <typename T>
__device__ __forceinline__ T opq(T v) {
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ double div_dim(double a, int n) {
    n = opq(n);
    if ((n & (n - 1)) == 0) return __builtin_amdgcn_ldexp(a, -__builtin_ctz((unsigned)n)); // (wave-uniform)
    return div_n(a, (double)n);
}
// floor(a / n) for 0 <= a < 2^31, 1 <= n <= 2^20: a shift for a power of two; otherwise the
// correctly rounded binary64 quotient, which truncates to the exact integer quotient
__device__ __forceinline__ int idiv_dim(int a, int n) {
    n = opq(n);
    if ((n & (n - 1)) == 0) return a >> __builtin_ctz((unsigned)n); // (wave-uniform)
    return (int)div_n((double)a, (double)n);
}
// The lane's index in its wave, opaque to the optimiser: lane masks derived from it are recomputed
// where they are used (two instructions) instead of being hoisted out of the record loops and kept
// live — or spilled — across the shading.
__device__ __forceinline__ int lane_id() {
    int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(l));
    return l;
}

// FAST: the caller guarantees x is in range (a sphere test's discriminant, >= 0.001 or 1.0 by
// then, in a spheres-only scene within CULL_EXTENT: every ray is a unit vector — primary rays and
// shadow rays are normalised, reflections off spheres keep the length — so disc <= ~1e10, far
// below 2^1000), and the check is skipped.
template <bool FAST = false>
__device__ __forceinline__ double sqrt_x(double x) { // == sqrt(x)
    // (the fast sequence inside the wave-uniform branch: measured 3-6 % faster per frame than
    // computing it unconditionally and redoing out-of-range waves)
    if (FAST || __ballot(!(x >= SQRT_N_LO && x <= SQRT_N_HI)) == 0) return sqrt_n(x);
    return sqrt(x);
}

// fast (wave-uniform): the host proved m2 inside the range (SceneHdr::norm_ok / prim_ok)
__device__ __forceinline__ D3 normalize3(const D3 &v, bool fast = false) { // vector_normalize/1 (:554-560)
    const double m2 = v.x * v.x + v.y * v.y + v.z * v.z;
    if (fast || __ballot(!(m2 >= RCP_N_LO && m2 <= RCP_N_HI)) == 0) { // mag and 1/mag in range, mag != 0
        const double s = div_n(1.0, sqrt_n(m2));
        return D3{v.x * s, v.y * s, v.z * s};
    }
    double mag = sqrt(m2);
    double s = 1.0 / mag;
    D3 r = {v.x * s, v.y * s, v.z * s};
    if (mag == 0) r = D3{0.0, 0.0, 0.0};
    return r;
}

__device__ __forceinline__ D3 bounce3(const D3 &v, const D3 &n) { // vector_bounce_off_plane/2 (:568-573)
    double k = 2 * (n.x * -v.x + n.y * -v.y + n.z * -v.z);
    return D3{n.x * k + v.x, n.y * k + v.y, n.z * k + v.z};
}

__device__ __forceinline__ double max0(double x) { return x > 0 ? x : 0.0; } // lists:max([0, X])

// math:pow/2 (:289) is the host libm's pow, which is correctly rounded for all but
// vanishingly rare arguments.  For the small non-negative integer exponents scenes use
// (specular_power 1, 4, 20) the kernel evaluates x^n by binary powering in double-double
// arithmetic (~2^-100 relative error, then one rounding), which gives the correctly
// rounded result — cheaper than, and closer to libm than, the device's general pow.  The
// pairs hi + lo are kept unnormalised (|lo| stays within ~2 ulp(hi), the product's exact
// low part plus the cross terms), so a step is one product and its fma error terms; the fma
// calls are error-free product transformations, not contractions.
__device__ __forceinline__ void dd_sqr(double &h, double &l) {
    const double p = h * h;
    const double e = __builtin_fma(h + h, l, __builtin_fma(h, h, -p));
    h = p;
    l = e;
}
__device__ __forceinline__ void dd_mul(double &ah, double &al, double bh, double bl) {
    const double p = ah * bh;
    const double e = __builtin_fma(al, bh, __builtin_fma(ah, bl, __builtin_fma(ah, bh, -p)));
    ah = p;
    al = e;
}
// GENPOW: the scene has a specular power outside {0, 1, ..., 1024} (decided on the host, see
// pow_int_ok in rt_scene.cpp), so the general device pow is compiled in; otherwise its large
// register footprint is kept out of the kernel.
// x^n, n >= 1, by binary powering (the operations depend on n alone).  BR (n wave-uniform): the
// multiplications sit under a branch the empty asm keeps one (if-converted, each ran for every step
// behind four v_cndmask per double-double); for a per-lane n the selects measured faster than exec-
// masked branches (config 3's dominant kernel +1.2 %, profiles/r06u_ab_pow.txt).
template <bool BR, typename U>
__device__ __forceinline__ double pow_bin(double x, U n) {
    double bh = x, bl = 0.0;
    while (!(n & 1u)) { // x^(2^k) for the lowest set bit: the result starts there
        dd_sqr(bh, bl);
        n >>= 1;
    }
    double rh = bh, rl = bl;
    while (n >>= 1) {
        dd_sqr(bh, bl);
        if (n & 1u) {
            if (BR) asm volatile("");
            dd_mul(rh, rl, bh, bl);
        }
    }
    return rh + rl;
}
// act: the lanes whose result is used.  A wave's records mostly lie on one object: when all of its
// active lanes share the exponent, the powering runs under scalar control (the exponent read from
// one lane), with no per-lane loop masks; otherwise each lane loops on its own.  The same operations
// either way, so the same bits.
#ifndef RT_POW_UNIFORM
#define RT_POW_UNIFORM 1
#endif
template <bool GENPOW>
__device__ __forceinline__ double pow_libm(double x, double y, bool act = true) {
    if (GENPOW && !(y >= 0.0 && y <= 1024.0 && y == __builtin_floor(y))) return pow(x, y);
    const unsigned n = (unsigned)y;
#if RT_POW_UNIFORM
    const unsigned long long am = __ballot(act);
    const unsigned n0 = (unsigned)__builtin_amdgcn_readlane((int)n, am ? __builtin_ctzll(am) : 0);
    if (__ballot(act && n != n0) == 0) return n0 == 0 ? 1.0 : pow_bin<true>(x, n0); // (wave-uniform)
#endif
    return n == 0 ? 1.0 : pow_bin<false>(x, n);
}

// ---- primitive tests: return true and t on a valid hit --------------------------------------
// ray_sphere_intersect/2 (:364-397), from B and C (A4 = 4*A hoisted per ray)
template <bool FAST = false>
__device__ __forceinline__ bool sph_t(double B, double C, double A4, double &t) {
    double disc = B * B - A4 * C;
    if (!(disc >= 0.001)) return false;
    double sq = sqrt_x<FAST>(disc);
    // T0 = (-B + sq)/2, T1 = (-B - sq)/2 (:379-383) with sq > 0: T1 <= T0 after rounding too (rounding
    // is monotonic), so lists:min([T0, T1]) is T1 (bit for bit where the two are equal) and both are
    // >= 0 iff T1 is (NaN and infinite B or disc fail either way) — T0 is never needed
    t = (-B - sq) / 2;
    return t >= 0;
}

// ray_triangle_intersect/2 (:402-455), with T = O - v1 and Q = T x Edge1 given
__device__ __forceinline__ bool tri_t(const D3 &d, const D3 &e1, const D3 &e2, const D3 &T, const D3 &Q,
                                      double &t) {
    D3 P = {d.y * e2.z - d.z * e2.y, d.z * e2.x - d.x * e2.z, d.x * e2.y - d.y * e2.x};
    double det = dot3(e1, P);
    if (det < 0.000001) return false;
    double U = dot3(T, P);
    if ((U < 0) || (U > det)) return false;
    double V = dot3(d, Q);
    if ((V < 0) || (U + V > det)) return false;
    t = dot3(e2, Q) / det;
    return true;
}

// ray_plane_intersect/2 (:461-480), with V0 = -(N.O + Distance) given
__device__ __forceinline__ bool pl_t(const D3 &n, const D3 &d, double V0, double &t) {
    double Vd = dot3(n, d);
    if (!(Vd < 0)) return false;
    t = V0 / Vd;
    if (t < 0.001) return false;
    return true;
}

// The same decision as sph_t without divergent branches: the root computation runs for the
// whole wave unless no lane can hit (a wave-uniform test), and the outcome is a mask.
template <bool FAST = false>
__device__ __forceinline__ bool sph_t_wave(double B, double C, double A4, double &t) {
    const double disc = B * B - A4 * C;
    const bool ok = disc >= 0.001;
    t = 0.0;
    if (__ballot(ok) == 0) return false;
    // FAST: the failing lanes' roots (NaN for disc < 0) are dropped by `ok` below; only the range-checked
    // form needs them in range, lest they send the wave down the full sqrt
    const double sq = sqrt_x<FAST>(FAST || ok ? disc : 1.0);
    t = (-B - sq) / 2; // the nearer root (sph_t)
    return ok & (t >= 0);
}

// (without the short circuit — no divergent branch per candidate — measured config 3 +0.9 %, config 5
// -0.7 %: profiles/r05af_ab_nearer_no_short_circuit.txt)
__device__ __forceinline__ bool nearer(double t, int id, double bt, int bid) {
    return t < bt || (t == bt && id < bid); // first in list order among equal distances (:319)
}

struct Scene {
    SceneHdr h;
    const double *__restrict__ tab;
    const int *__restrict__ itab;
};

// The scene header re-read from the kernel argument segment (scalar loads; every kernel here takes
// the SceneHdr its Scene holds as its first argument) instead of being held in SGPRs across a
// long loop: the kernels' uniform values exceed the SGPR file, and spilled ones come back through
// v_readlane on every use (measured on k_reflect_shade: SGPR spills 90 -> 21, config 3 +2 %).
#ifndef RT_HDR_RELOAD
#define RT_HDR_RELOAD 1
#endif
__device__ __forceinline__ Scene fresh_scene(const Scene &S) {
#if RT_HDR_RELOAD && defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const SceneHdr KHdr;
    KHdr *hp = (KHdr *)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(hp)); // opaque: the loads stay where the values are used
    return Scene{*hp, S.tab, S.itab};
#else
    return S;
#endif
}

// ---- scene table access; SPH (template argument of the shading code): 0 = any scene, 1 = spheres
// only (occluder masks), 2 = spheres only with the per-lane-gathered tables staged in LDS.
// Lanes of a wave read these rows by their own object / target / candidate (gathers whose L2
// round trips the shading waits on); staged, they are LDS reads.  Wave-uniform reads stay
// scalar loads from the tables in HBM (scalar cache).
extern __shared__ __attribute__((aligned(16))) char g_lds[];

template <int SPH>
__device__ __forceinline__ const double *obj_row(const Scene &S, int id) {
    if (SPH == 2) return reinterpret_cast<const double *>(g_lds + S.h.l_obj) + id * OBJ_W;
    return S.tab + S.h.o_obj + id * OBJ_W;
}
template <int SPH>
__device__ __forceinline__ int4 obj_meta(const Scene &S, int id) {
    if (SPH == 2) return reinterpret_cast<const int4 *>(g_lds + S.h.l_meta)[id];
    return *reinterpret_cast<const int4 *>(S.itab + S.h.i_obj_meta + id * OBJ_META_W);
}
// per-origin sphere row (o - c, C); staged only for the light origins (org >= 1)
template <int SPH>
__device__ __forceinline__ const double *org_row(const Scene &S, int org, int k) {
    if (SPH == 2) return reinterpret_cast<const double *>(g_lds + S.h.l_org) + ((org - 1) * S.h.n_sph + k) * SPH_ORG_W;
    return S.tab + S.h.o_sph_org + (org * S.h.n_sph + k) * SPH_ORG_W;
}
// occluder masks of `light`, chunk `chunk64`: element (t*OCC_CELLS + e)*n_chunk is the mask of
// target sphere t, direction cell e
template <int SPH>
__device__ __forceinline__ const unsigned long long *occ_masks(const Scene &S, int light, int chunk64) {
    const int w = (light * S.h.n_sph * (SPH == 2 ? 1 : S.h.occ_cells)) * S.h.n_chunk + chunk64; // staged: 1 cell
    if (SPH == 2) return reinterpret_cast<const unsigned long long *>(g_lds + S.h.l_occ) + w;
    return reinterpret_cast<const unsigned long long *>(S.itab + S.h.i_occ) + w;
}
template <int SPH>
__device__ __forceinline__ int sph_id(const Scene &S, int k) {
    if (SPH == 2) return reinterpret_cast<const int *>(g_lds + S.h.l_id)[k];
    return S.itab[S.h.i_sph_id + k];
}
// Copy the staged tables into this workgroup's LDS (every thread of the block, before any use).
template <int SPH>
__device__ __forceinline__ void stage_tables(const Scene &S) {
    if (SPH != 2) return;
    const SceneHdr &h = S.h;
    auto copy16 = [&](int dst, const void *src, int bytes) { // src 16-byte aligned
        const int4 *s4 = reinterpret_cast<const int4 *>(src);
        int4 *d4 = reinterpret_cast<int4 *>(g_lds + dst);
        for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) d4[i] = s4[i];
    };
    auto copy4 = [&](int dst, const int *src, int n) {
        int *d = reinterpret_cast<int *>(g_lds + dst);
        for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = src[i];
    };
    copy16(h.l_obj, S.tab + h.o_obj, h.n_obj * OBJ_W * 8);
    copy16(h.l_meta, S.itab + h.i_obj_meta, h.n_obj * OBJ_META_W * 4);
    copy16(h.l_org, S.tab + h.o_sph_org + h.n_sph * SPH_ORG_W, h.n_light * h.n_sph * SPH_ORG_W * 8);
    copy4(h.l_occ, S.itab + h.i_occ, h.n_light * h.n_sph * h.n_chunk * 2); // 1 cell; 8-byte aligned in the int table
    copy4(h.l_id, S.itab + h.i_sph_id, h.n_sph);
    copy16(h.l_sphb, S.tab + h.o_sph_b, h.n_sph * SPH_B_W * 8);
    __syncthreads();
}

// Diagnostic build only (-DRT_STATS): per-wave event counters read back with rt_debug_stats().
#define RT_NSTATS 20
#ifdef RT_STATS
__device__ unsigned long long g_stats[RT_NSTATS];
#define RT_STAT(i, v)                                                                                              \
    do {                                                                                                           \
        const unsigned long long v_ = (v);                                                                         \
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) atomicAdd(&g_stats[i], v_);                          \
    } while (0)
#else
#define RT_STAT(i, v) \
    do {              \
    } while (0)
#endif
enum { ST_WAVES, ST_NEAR_PRE, ST_NEAR_PRE_CAND, ST_NEAR_GEN, ST_NEAR_GEN_CAND, ST_SHADOW, ST_SHADOW_CAND,
       ST_SHADOW_ITER, ST_SHADE, ST_SHADOW_CONE_ON, ST_BEAM_ON, ST_SHADOW_LANES, ST_NEAR_LANES, ST_BVH_SCANS,
       ST_BVH_ITER, ST_BVH_LEAF, ST_BVH_ITER_LANES, ST_BVH_LEAF_LANES };

// ---- Beam culling ----------------------------------------------------------------------------
// A wave's 64 rays are coherent (an 8x8 pixel tile; shadow rays of one light; their
// reflections).  Before a sphere scan the wave bounds its active rays by a cone of
// directions (axis a, half-angle theta given by a lower bound c on cos and an upper bound s
// on sin) around an origin ball (centre m, radius ro; ro = 0 for the camera and the
// lights).  Lane j then tests sphere j of a 64-sphere chunk against that beam and a ballot
// yields the chunk's candidate mask; the scan visits only candidates, with a wave-uniform
// index (scalar loads).  A sphere is dropped only if its angular distance phi from the axis
// exceeds theta + rho, rho = asin((r + ro) / |c - m|): then no ray of the beam comes within
// r of the centre, and the reference's test (disc >= 0.001 and both roots >= 0, :378-381)
// cannot succeed — its rounding error is < 1e-9 of the threshold for scenes within
// CULL_EXTENT, and every bound below carries a CULL_EPS margin in the safe direction.
// Wave reductions of binary64 values without LDS: four DPP steps reduce each 16-lane row
// (quad_perm xor 1, xor 2, row_half_mirror, row_mirror — each an involution, so every lane
// of a row ends with the same value), then the four row results are read into SGPRs.  The
// wave must be converged (all 64 lanes active).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double lane_f64(double v, int lane) { // v of `lane`, in SGPRs
    const long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((int)b, lane);
    const unsigned hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
// Across the four rows (RT_DPP_BCAST, A/B builds): row_bcast:15 (row_mask 0xA: rows 1 and 3 take lane 15 of
// rows 0 and 2) then row_bcast:31 (row_mask 0xC: rows 2 and 3 take lane 31), so lane 63 holds the wave's
// result and one readlane (two for binary64) reads it, instead of four (eight) and three more operations.
// Rows the mask leaves out keep their own value (`old`); only lane 63's chain matters.
#ifndef RT_DPP_BCAST
#define RT_DPP_BCAST 0 // 1: measured within noise on configs 3 and 5 (profiles/r06m_ab_dpp_row_bcast.txt)
#endif
[[maybe_unused]] constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143;
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64_rows(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, ROWS, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <typename Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
    v = op(v, dpp_f64<DPP_XOR1>(v));
    v = op(v, dpp_f64<DPP_XOR2>(v));
    v = op(v, dpp_f64<DPP_HALF_MIRROR>(v));
    v = op(v, dpp_f64<DPP_MIRROR>(v));
#if RT_DPP_BCAST
    v = op(v, dpp_f64_rows<DPP_ROW_BCAST15, 0xA>(v));
    v = op(v, dpp_f64_rows<DPP_ROW_BCAST31, 0xC>(v));
    return lane_f64(v, 63);
#else
    return op(op(lane_f64(v, 0), lane_f64(v, 16)), op(lane_f64(v, 32), lane_f64(v, 48)));
#endif
}
__device__ __forceinline__ double wave_sum(double v) {
    return wave_reduce(v, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ double wave_min(double v) {
    return wave_reduce(v, [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ double wave_max(double v) {
    return wave_reduce(v, [](double a, double b) { return fmax(a, b); });
}
// every lane holds the same v: keep it in SGPRs
__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long b) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double uniform(double v) {
    unsigned long long b = (unsigned long long)__double_as_longlong(v);
    unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

struct Beam {
    double ax, ay, az; // unit axis
    double c, s;       // cos(theta) lower bound, sin(theta) upper bound
    double mx, my, mz; // origin ball centre (unused when the origin is tabled)
    double ro;         // origin ball radius
    bool on;
};

// Must be called with the whole wave converged (it reduces across lanes).
__device__ __forceinline__ Beam make_beam(const SceneHdr &h, bool act, const D3 &o, const D3 &d, bool fixed_origin) {
    Beam b;
    b.on = false;
    b.ax = b.ay = b.az = b.c = b.s = b.mx = b.my = b.mz = b.ro = 0.0;
    const unsigned long long am = __ballot(act);
    if (!h.beam_ok || am == 0) return b;
    // Axis: the (normalised) direction of one active lane — the tile centre when it is active.
    // Any axis inside the bundle gives a valid cone, at most twice as wide as the best one.
    const int al = ((am >> 27) & 1) ? 27 : __builtin_ctzll(am);
    const double rx = lane_f64(d.x, al), ry = lane_f64(d.y, al), rz = lane_f64(d.z, al);
    const double n2 = rx * rx + ry * ry + rz * rz;
    if (!(n2 > 0.0)) return b;
    const double inv = uniform(1.0 / sqrt(n2));
    const double ax = rx * inv, ay = ry * inv, az = rz * inv;
    // The rays traced here are unit vectors to ~1e-15 (normalize/1 and bounces off unit
    // normals).  Lanes are only required to have |d|^2 within DIR_TOL of 1, and the bounds are
    // widened by 2*DIR_TOL instead of dividing by |d| (a plane normal that is not unit makes
    // its reflections fail the check: that wave simply scans every sphere).
    constexpr double DIR_TOL = 1.0e-6;
    const double dd = d.x * d.x + d.y * d.y + d.z * d.z;
    const double cl = ax * d.x + ay * d.y + az * d.z;
    const double qx = ay * d.z - az * d.y, qy = az * d.x - ax * d.z, qz = ax * d.y - ay * d.x;
    const double sl = sqrt(qx * qx + qy * qy + qz * qz);
    const bool bad = act && !(dd > 1.0 - DIR_TOL && dd < 1.0 + DIR_TOL);
    const double c = uniform(wave_min(act ? cl : 2.0)) - CULL_EPS - 2 * DIR_TOL;
    const double s = uniform(wave_max(act ? sl : 0.0)) + CULL_EPS + 2 * DIR_TOL;
    if (__ballot(bad) != 0 || !(c > 0.0)) return b; // cone wider than a hemisphere: scan everything
    b.ax = ax; b.ay = ay; b.az = az; b.c = c; b.s = s;
    if (!fixed_origin) {
        const int first = __builtin_ctzll(am);
        b.mx = lane_f64(o.x, first);
        b.my = lane_f64(o.y, first);
        b.mz = lane_f64(o.z, first);
        const double ex = o.x - b.mx, ey = o.y - b.my, ez = o.z - b.mz;
        const double r2 = wave_max(act ? ex * ex + ey * ey + ez * ez : 0.0);
        const double mo = wave_max(act ? fmax(fabs(o.x), fmax(fabs(o.y), fabs(o.z))) : 0.0);
        if (!(uniform(mo) <= CULL_EXTENT)) return b;
        b.ro = uniform(sqrt(r2)) * (1 + CULL_EPS) + CULL_EPS;
    }
    b.on = true;
    return b;
}

// Candidate mask of spheres [chunk, chunk+64): lane j tests sphere chunk+j against the beam.
// org >= 0: the beam starts at tabled origin `org` (camera / light) and uses its cone table;
// a sphere whose nearest surface point is farther than tmax from the origin is dropped too
// (its hits have t > tmax; shadow scans only care about t <= t*, and t* <= tmax).
template <int SPH = 0>
__device__ __forceinline__ unsigned long long cull_chunk(const Scene &S, const Beam &b, int chunk, int org,
                                                         double tmax = __builtin_inf()) {
    // Branch-free: every load of the record is issued at once and the decision is a mask.
    const SceneHdr &h = S.h;
    const int k = chunk + (int)(threadIdx.x & 63);
    const bool in = k < h.n_sph;
    const int kk = in ? k : 0;
    bool keep;
    if (org >= 0) { // wave-uniform
        const double2 *q = reinterpret_cast<const double2 *>(S.tab + h.o_sph_ob + (org * h.n_sph + kk) * SPH_OB_W);
        const double2 q01 = q[0], q23 = q[1], q45 = q[2], q67 = q[3];
        const double thr = b.c * q45.y - b.s * q45.x;                  // <= cos(theta + rho)
        const double av = b.ax * q01.x + b.ay * q01.y + b.az * q23.x;  // |v| cos(phi)
        keep = ((q67.x != 0.0) | !(av + CULL_EPS * q23.y < thr * q23.y)) & !(q67.y > tmax);
    } else {
        const double2 *g = SPH == 2 ? reinterpret_cast<const double2 *>(g_lds + h.l_sphb) + kk * (SPH_B_W / 2)
                                    : reinterpret_cast<const double2 *>(S.tab + h.o_sph_b + kk * SPH_B_W);
        const double2 g01 = g[0], g23 = g[1];
        const double vx = g01.x - b.mx, vy = g01.y - b.my, vz = g23.x - b.mz;
        const double vl = sqrt(vx * vx + vy * vy + vz * vz);
        const double rp = g23.y + b.ro;
        const double sr = rp / vl * (1 + CULL_EPS) + CULL_EPS;
        const double cr = sqrt(fmax(1.0 - sr * sr, 0.0)) - CULL_EPS;
        const double thr = b.c * cr - b.s * sr;
        const double av = b.ax * vx + b.ay * vy + b.az * vz;
        keep = (vl <= rp * (1 + CULL_EPS) + CULL_EPS) | (sr >= 1.0) | !(av + CULL_EPS * vl < thr * vl);
    }
    return __ballot(in & keep);
}

// ---- Binary32 beams for reflection rays ------------------------------------------------------
// The reflection scans' beams (origin ball + direction cone over a group of lanes) and their
// per-sphere cull tests are filters: they only have to keep every sphere some ray of the group
// can hit.  They run in binary32 (hardware sqrt / reciprocal, half the issue cost of binary64,
// single-register DPP reductions) with margins far above binary32 rounding: BEAM32_EPS (1e-5,
// vs ~1e-6 accumulated relative error in the O(1) cosines and sines), and the positions' rounding
// (|x| * 2^-24 per coordinate) covered by widening the origin ball by (|origins| + extent) * 1e-6.
// Their square roots are the hardware's v_sqrt_f32 (sqrt_f32f: within ~1 ulp, 2^-23 relative, far
// inside those margins) — the correctly rounded sqrtf the compiler emits under IEEE rules is
// that instruction wrapped in a dozen fix-up operations per call.
// The axis need not be a unit vector: the cone bounds and the sphere test scale with |axis| alike.
struct Beam32 {
    float ax, ay, az; // axis (about unit)
    float c, s;       // lower bound of the lanes' a.d, upper bound of |a x d|
    float mx, my, mz; // origin ball centre
    float ro;         // origin ball radius, position rounding included
    bool on;
};
__device__ __forceinline__ float lane_f32(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ float sqrt_f32f(float x) { return __builtin_amdgcn_sqrtf(x); } // the filters' sqrt
// Wave minimum / maximum of binary32 values by their bit patterns as signed integers, which order
// as the values do for every value >= +0 (lengths, radii, extents: the maxima here).  For the
// minima (the beams' cosine bounds) a negative value anywhere gives some negative result, not
// necessarily the least, and a negative bound is all the callers test for (the beam is off): the
// same decisions.  A NaN (positive as an integer) goes into a maximum, where it turns the beam off
// or keeps every sphere.  Integer min/max need no NaN canonicalisation, so each DPP step is one
// v_min/max_i32_dpp (bound_ctrl: these four permutations read no invalid lane), and the four rows'
// results are read and combined — against a v_mov, a v_mov_dpp and a canonicalising v_max around
// every fminf / fmaxf step.  (Combining them with s_min/s_max in inline asm measured slower:
// profiles/r06ab_ab_salu_bvh_knobs.txt.)
template <bool MAX>
__device__ __forceinline__ float wave_ext32(float x) {
    auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
    int v = __float_as_int(x);
    v = op(v, __builtin_amdgcn_mov_dpp(v, DPP_XOR1, 0xF, 0xF, true));
    v = op(v, __builtin_amdgcn_mov_dpp(v, DPP_XOR2, 0xF, 0xF, true));
    v = op(v, __builtin_amdgcn_mov_dpp(v, DPP_HALF_MIRROR, 0xF, 0xF, true));
    v = op(v, __builtin_amdgcn_mov_dpp(v, DPP_MIRROR, 0xF, 0xF, true));
    return __int_as_float(op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                             op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48))));
}
__device__ __forceinline__ float wave_min32(float x) { return wave_ext32<false>(x); }
__device__ __forceinline__ float wave_max32(float x) { return wave_ext32<true>(x); }
// Must be called with the whole wave converged.  o, d: the lanes' ray origins and directions.
// SPHO: a spheres-only scene's reflection rays — every origin is a hit point on a sphere, so its
// coordinates are within 2 h.ext (h.ext bounds |centre| and |radius| alike; the binary64 hit point's
// rounding is ~1e-16 of that), which replaces the wave maximum of |origin|; and every direction is a
// reflection off a normalised sphere normal of a normalised ray, of unit length to ~1e-15 per level,
// so the DIR_TOL check (which catches the reflections off planes with non-unit normals) cannot fail.
template <bool SPHO = false>
__device__ __forceinline__ Beam32 make_beam32(const SceneHdr &h, bool act, const D3 &o, const D3 &d) {
    Beam32 b;
    b.on = false;
    b.ax = b.ay = b.az = b.c = b.s = b.mx = b.my = b.mz = b.ro = 0.0f;
    const unsigned long long am = __ballot(act);
    if (!h.beam_ok || am == 0) return b;
    const int al = ((am >> 27) & 1) ? 27 : __builtin_ctzll(am);
    const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
    const float rx = lane_f32(dx, al), ry = lane_f32(dy, al), rz = lane_f32(dz, al);
    const float n2 = rx * rx + ry * ry + rz * rz;
    if (!(n2 > 1.0e-6f)) return b;
    const float inv = __builtin_amdgcn_rsqf(n2);
    const float ax = rx * inv, ay = ry * inv, az = rz * inv;
    // the lanes' directions are unit vectors to ~1e-15 (make_beam); bounds widened by 2 * DIR_TOL
    constexpr float DIR_TOL = 1.0e-6f;
    const float dd = dx * dx + dy * dy + dz * dz;
    const float cl = ax * dx + ay * dy + az * dz;
    const bool bad = !SPHO && act && !(dd > 1.0f - 0.5f * DIR_TOL && dd < 1.0f + 0.5f * DIR_TOL);
    const float cmin = wave_min32(act ? cl : 2.0f);
    const float c = cmin - BEAM32_EPS - 2 * DIR_TOL;
    if (__ballot(bad) != 0 || !(c > 0.0f)) return b; // cone wider than a hemisphere: scan everything
    // The sine bound from the cosine bound: every lane has cos >= cmin (to f32 rounding, ~1e-6 with
    // the directions' and the axis' deviation from unit length), so sin^2 = |a|^2 |d|^2 - cos^2 <=
    // 1 + 4 DIR_TOL - cmin^2 (0 < cmin <= 1) — no second reduction (nor the lanes' cross products).
    const float s = sqrt_f32f(fmaxf(1.0f + 4 * DIR_TOL - cmin * cmin, 0.0f)) + BEAM32_EPS + 2 * DIR_TOL;
    const int first = __builtin_ctzll(am);
    const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
    b.mx = lane_f32(ox, first);
    b.my = lane_f32(oy, first);
    b.mz = lane_f32(oz, first);
    const float ex = ox - b.mx, ey = oy - b.my, ez = oz - b.mz;
    const float r2 = wave_max32(act ? ex * ex + ey * ey + ez * ez : 0.0f);
    // the origins' extent in binary32 (|o| rounded to nearest: within 2^-24 relative, far inside the
    // 1e-6 margin below; the extent check keeps a 1e-6 relative slack for it)
    const float mo = SPHO ? (float)(2.0 * h.ext) * (1.0f + 1.0e-6f)
                          : wave_max32(act ? fmaxf(fabsf(ox), fmaxf(fabsf(oy), fabsf(oz))) : 0.0f);
    if (!(mo <= (float)(CULL_EXTENT * (1.0 - 1.0e-6)))) return b;
    b.ax = ax; b.ay = ay; b.az = az; b.c = c; b.s = s;
    b.ro = sqrt_f32f(r2) * (1.0f + BEAM32_EPS) + BEAM32_EPS + (mo + (float)h.ext) * 1.0e-6f;
    b.on = true;
    return b;
}
// Candidate mask of spheres [chunk, chunk+64) for a binary32 beam (lane j tests sphere chunk+j).
template <int SPH = 0>
__device__ __forceinline__ unsigned long long cull_chunk32(const Scene &S, const Beam32 &b, int chunk) {
    const SceneHdr &h = S.h;
    const int k = chunk + (int)(threadIdx.x & 63);
    const bool in = k < h.n_sph;
    const int kk = in ? k : 0;
    const double2 *g = SPH == 2 ? reinterpret_cast<const double2 *>(g_lds + h.l_sphb) + kk * (SPH_B_W / 2)
                                : reinterpret_cast<const double2 *>(S.tab + h.o_sph_b + kk * SPH_B_W);
    const double2 g01 = g[0], g23 = g[1];
    const float vx = (float)g01.x - b.mx, vy = (float)g01.y - b.my, vz = (float)g23.x - b.mz;
    const float vl = sqrt_f32f(vx * vx + vy * vy + vz * vz);
    const float rp = (float)g23.y + b.ro;
    const float sr = rp * __builtin_amdgcn_rcpf(vl) * (1.0f + BEAM32_EPS) + BEAM32_EPS;
    const float cr = sqrt_f32f(fmaxf(1.0f - sr * sr, 0.0f)) - BEAM32_EPS;
    const float thr = b.c * cr - b.s * sr;
    const float av = b.ax * vx + b.ay * vy + b.az * vz;
    const bool keep = (vl <= rp * (1.0f + BEAM32_EPS) + BEAM32_EPS) | (sr >= 1.0f) | !(av + BEAM32_EPS * vl < thr * vl);
    return __ballot(in & keep);
}

// Tabled origin `org` (camera, lights): the host's binary32 cone rows (SPH_OB32_W); a sphere whose
// nearest surface point is farther than tmax from the origin is dropped too.
__device__ __forceinline__ unsigned long long cull_chunk32_org(const Scene &S, const Beam32 &b, int chunk, int org,
                                                               float tmax = __builtin_inff()) {
    const SceneHdr &h = S.h;
    const int k = chunk + (int)(threadIdx.x & 63);
    const bool in = k < h.n_sph;
    const int kk = in ? k : 0;
    const float4 *q = reinterpret_cast<const float4 *>(S.tab + h.o_sph_ob32) + (size_t)(org * h.n_sph + kk) * 2;
    const float4 v = q[0], w = q[1]; // (vx vy vz |v|) (sin, cos, near, dlow)
    const float thr = b.c * w.y - b.s * w.x;
    const float av = b.ax * v.x + b.ay * v.y + b.az * v.z;
    const bool keep = ((w.z != 0.0f) | !(av + BEAM32_EPS * v.w < thr * v.w)) & !(w.w > tmax);
    return __ballot(in & keep);
}

// Beam of a wave holding two primary rays per lane (an 8x16 pixel block) from a tabled origin:
// make_beam32's cone over both ray sets (no origin ball).
__device__ __forceinline__ Beam32 make_beam_pair32(const SceneHdr &h, bool a0, const D3 &d0, bool a1, const D3 &d1) {
    Beam32 b;
    b.on = false;
    b.ax = b.ay = b.az = b.c = b.s = b.mx = b.my = b.mz = b.ro = 0.0f;
    const unsigned long long m0 = __ballot(a0), m1 = __ballot(a1);
    if (!h.beam_ok || (m0 | m1) == 0) return b;
    const float x0 = (float)d0.x, y0 = (float)d0.y, z0 = (float)d0.z;
    const float x1 = (float)d1.x, y1 = (float)d1.y, z1 = (float)d1.z;
    // axis: the ray of pixel (3, 7) of the block (set 0, lane 59), else the first active ray
    float rx, ry, rz;
    if ((m0 >> 59) & 1) {
        rx = lane_f32(x0, 59); ry = lane_f32(y0, 59); rz = lane_f32(z0, 59);
    } else if (m0) {
        const int l = __builtin_ctzll(m0);
        rx = lane_f32(x0, l); ry = lane_f32(y0, l); rz = lane_f32(z0, l);
    } else {
        const int l = __builtin_ctzll(m1);
        rx = lane_f32(x1, l); ry = lane_f32(y1, l); rz = lane_f32(z1, l);
    }
    const float n2 = rx * rx + ry * ry + rz * rz;
    if (!(n2 > 1.0e-6f)) return b;
    const float inv = __builtin_amdgcn_rsqf(n2);
    const float ax = rx * inv, ay = ry * inv, az = rz * inv;
    constexpr float DIR_TOL = 1.0e-6f; // as in make_beam32
    auto lane_terms = [&](bool a, float dx, float dy, float dz, float &cl) {
        const float dd = dx * dx + dy * dy + dz * dz;
        cl = ax * dx + ay * dy + az * dz;
        return a && !(dd > 1.0f - 0.5f * DIR_TOL && dd < 1.0f + 0.5f * DIR_TOL);
    };
    float cl0, cl1;
    const bool bad0 = lane_terms(a0, x0, y0, z0, cl0); // both sets evaluated (no short circuit)
    const bool bad1 = lane_terms(a1, x1, y1, z1, cl1);
    const float cmin = wave_min32(fminf(a0 ? cl0 : 2.0f, a1 ? cl1 : 2.0f));
    const float c = cmin - BEAM32_EPS - 2 * DIR_TOL;
    if (__ballot(bad0 || bad1) != 0 || !(c > 0.0f)) return b;
    const float s = sqrt_f32f(fmaxf(1.0f + 4 * DIR_TOL - cmin * cmin, 0.0f)) + BEAM32_EPS + 2 * DIR_TOL; // make_beam32
    b.ax = ax; b.ay = ay; b.az = az; b.c = c; b.s = s;
    b.on = true;
    return b;
}

__device__ __forceinline__ unsigned long long chunk_all(int n_sph, int chunk) {
    const int n = n_sph - chunk;
    return n >= 64 ? ~0ull : ((1ull << n) - 1);
}

// The sphere candidates in mask m of chunk `chunk`, folded into the running nearest (bt, bid).
// Two candidates per step: the (t, list position) minimum does not depend on the order the
// candidates are visited, and the two tests are independent, which gives the wave
// instruction-level parallelism across the scalar loads and the root computations.
template <bool PRE>
__device__ __forceinline__ void sphere_BC(const Scene &S, int org, const D3 &o, const D3 &d, int k, double &B,
                                          double &C) {
    const SceneHdr &h = S.h;
    if (PRE) {
        const double *q = S.tab + h.o_sph_org + (org * h.n_sph + k) * SPH_ORG_W;
        B = 2 * (d.x * q[0] + d.y * q[1] + d.z * q[2]);
        C = q[3];
    } else {
        const double *s = S.tab + h.o_sph + k * SPH_W;
        D3 oc = {o.x - s[0], o.y - s[1], o.z - s[2]};
        B = 2 * (d.x * oc.x + d.y * oc.y + d.z * oc.z);
        C = oc.x * oc.x + oc.y * oc.y + oc.z * oc.z - s[3];
    }
}
// ILP = false: one candidate per step (the least work: dense, throughput-bound waves).
template <bool PRE, bool ILP = false, bool FAST = false>
__device__ __forceinline__ void scan_spheres(const Scene &S, int org, const D3 &o, const D3 &d, double A4, int chunk,
                                             unsigned long long m, double &bt, int &bid) {
    const SceneHdr &h = S.h;
    RT_STAT(PRE ? ST_NEAR_PRE_CAND : ST_NEAR_GEN_CAND, __popcll(m));
    // (the walk's scalar loads one candidate ahead — the next row and list position requested before
    // the current candidate is tested — measured config 3 +0.8 %, config 2 +1.3 %, config 5 neutral:
    // profiles/r05ak_ab_scan_scalar_prefetch.txt)
    while (!ILP && m) {
        const int k = chunk + __builtin_ctzll(m);
        m &= m - 1;
        double B, C;
        sphere_BC<PRE>(S, org, o, d, k, B, C);
        const int id = S.itab[h.i_sph_id + k];
        double t;
        const bool upd = (int)sph_t_wave<FAST>(B, C, A4, t) & (int)nearer(t, id, bt, bid);
        bt = upd ? t : bt;
        bid = upd ? id : bid;
    }
    while (ILP && m) {
        const int k0 = chunk + __builtin_ctzll(m);
        m &= m - 1;
        const bool two = m != 0;
        const int k1 = two ? chunk + __builtin_ctzll(m) : k0;
        if (two) m &= m - 1;
        double B0, C0, B1, C1;
        sphere_BC<PRE>(S, org, o, d, k0, B0, C0);
        sphere_BC<PRE>(S, org, o, d, k1, B1, C1);
        const int id0 = S.itab[h.i_sph_id + k0], id1 = S.itab[h.i_sph_id + k1];
        // sph_t for both, without divergent branches; the roots only if some lane can hit
        const double disc0 = B0 * B0 - A4 * C0, disc1 = B1 * B1 - A4 * C1;
        const bool ok0 = disc0 >= 0.001, ok1 = disc1 >= 0.001;
        if (__ballot(ok0 | ok1) == 0) continue;
        const double sq0 = sqrt_x<FAST>(FAST || ok0 ? disc0 : 1.0), sq1 = sqrt_x<FAST>(FAST || ok1 ? disc1 : 1.0); // (sph_t_wave)
        const double t0 = (-B0 - sq0) / 2, t1 = (-B1 - sq1) / 2; // the nearer roots (sph_t)
        const bool h0 = ok0 & (t0 >= 0), h1 = two & ok1 & (t1 >= 0);
        const bool u0 = h0 & nearer(t0, id0, bt, bid);
        bt = u0 ? t0 : bt;
        bid = u0 ? id0 : bid;
        const bool u1 = h1 & nearer(t1, id1, bt, bid);
        bt = u1 ? t1 : bt;
        bid = u1 ? id1 : bid;
    }
}

// The triangles and planes of the scene, folded into the running nearest (bt, bid).
template <bool PRE>
__device__ __forceinline__ void scan_tri_pl(const Scene &S, int org, const D3 &o, const D3 &d, double &bt, int &bid) {
    const SceneHdr &h = S.h;
    for (int k = 0; k < h.n_tri; ++k) {
        const double *g = S.tab + h.o_tri + k * TRI_W;
        D3 e1 = {g[3], g[4], g[5]}, e2 = {g[6], g[7], g[8]};
        D3 T, Q;
        if (PRE) {
            const double *q = S.tab + h.o_tri_org + (org * h.n_tri + k) * TRI_ORG_W;
            T = D3{q[0], q[1], q[2]};
            Q = D3{q[3], q[4], q[5]};
        } else {
            T = D3{o.x - g[0], o.y - g[1], o.z - g[2]};
            Q = D3{T.y * e1.z - T.z * e1.y, T.z * e1.x - T.x * e1.z, T.x * e1.y - T.y * e1.x};
        }
        double t;
        if (tri_t(d, e1, e2, T, Q, t)) {
            int id = S.itab[h.i_tri_id + k];
            if (nearer(t, id, bt, bid)) { bt = t; bid = id; }
        }
    }
    for (int k = 0; k < h.n_pl; ++k) {
        const double *p = S.tab + h.o_pl + k * PL_W;
        D3 n = {p[0], p[1], p[2]};
        double V0 = PRE ? S.tab[h.o_pl_org + org * h.n_pl + k] : -(n.x * o.x + n.y * o.y + n.z * o.z + p[3]);
        double t;
        if (pl_t(n, d, V0, t)) {
            int id = S.itab[h.i_pl_id + k];
            if (nearer(t, id, bt, bid)) { bt = t; bid = id; }
        }
    }
}

// ---- Per-lane BVH (incoherent reflection rays) ------------------------------------------------
// Deep reflection levels of large scenes leave every wave's rays pointing everywhere: a wave
// beam then keeps most spheres (S256 depth 8: ~200 of 256 candidates per scan).  Those scans
// walk the host-built sphere BVH instead, each lane on its own ray (ordered traversal: both
// children's boxes tested, the nearer visited first, the other pushed with its entry distance).
// The box tests are binary32 slab tests on boxes rounded outwards and inflated (rt_scene.cpp), a
// conservative filter with a relative tolerance of 2^-16 on every distance compared; a sphere
// leaf that passes is tested with the reference's binary64 expressions (sphere_BC + sph_t), and
// the (t, list position) minimum does not depend on the visiting order, so the result is the
// candidate walk's.  Each lane's stack holds (entry distance rounded down to bfloat16, node) in
// one word, in LDS (BVH_STACK words per lane, lane-interleaved: no bank conflicts).
__device__ __forceinline__ float bvh_inv(double d) {
    float f = (float)d;
    f = fabsf(f) < 1.0e-30f ? copysignf(1.0e-30f, f) : f; // no inf * 0 in the slab test
    return __builtin_amdgcn_rcpf(f);                       // ~1 ulp: inside the tolerance
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
struct BvhRay {
    f32x2 ix, iy, iz;    // 1 / d (binary32, both lanes of the pair)
    f32x2 nox, noy, noz; // -(o * (1 / d))
};
__device__ __forceinline__ BvhRay bvh_ray(const D3 &o, const D3 &d) {
    BvhRay r;
    const float ix = bvh_inv(d.x), iy = bvh_inv(d.y), iz = bvh_inv(d.z);
    r.ix = f32x2{ix, ix};
    r.iy = f32x2{iy, iy};
    r.iz = f32x2{iz, iz};
    r.nox = f32x2{-((float)o.x * ix), -((float)o.x * ix)};
    r.noy = f32x2{-((float)o.y * iy), -((float)o.y * iy)};
    r.noz = f32x2{-((float)o.z * iz), -((float)o.z * iz)};
    return r;
}
// Slab tests of both children of a node: [tn, tx] of each box along the ray, clipped to [0, tlim];
// h0/h1 true where they overlap (tolerant).  The distances are b * (1/d) - o * (1/d) (one packed fma
// per axis and bound); its cancellation error, <= 2^-23 * extent * |1/d|, is far inside the boxes'
// inflation (BVH_BOX_REL * (extent + 1) in space, i.e. that times |1/d| in distance).
__device__ __forceinline__ void bvh_slab2(const BvhRay &r, const float4 &a, const float4 &b, const float4 &c, float tlim,
                                          bool &h0, float &tn0, bool &h1, float &tn1) {
    constexpr float LO = 1.0f - 0x1p-16f, HI = 1.0f + 0x1p-16f;
    const f32x2 tlx = __builtin_elementwise_fma(f32x2{a.x, a.y}, r.ix, r.nox);
    const f32x2 tly = __builtin_elementwise_fma(f32x2{a.z, a.w}, r.iy, r.noy);
    const f32x2 tlz = __builtin_elementwise_fma(f32x2{b.x, b.y}, r.iz, r.noz);
    const f32x2 tux = __builtin_elementwise_fma(f32x2{b.z, b.w}, r.ix, r.nox);
    const f32x2 tuy = __builtin_elementwise_fma(f32x2{c.x, c.y}, r.iy, r.noy);
    const f32x2 tuz = __builtin_elementwise_fma(f32x2{c.z, c.w}, r.iz, r.noz);
    tn0 = fmaxf(fmaxf(fminf(tlx.x, tux.x), fminf(tly.x, tuy.x)), fmaxf(fminf(tlz.x, tuz.x), 0.0f));
    tn1 = fmaxf(fmaxf(fminf(tlx.y, tux.y), fminf(tly.y, tuy.y)), fmaxf(fminf(tlz.y, tuz.y), 0.0f));
    const float tx0 = fminf(fminf(fmaxf(tlx.x, tux.x), fmaxf(tly.x, tuy.x)), fminf(fmaxf(tlz.x, tuz.x), tlim));
    const float tx1 = fminf(fminf(fmaxf(tlx.y, tux.y), fmaxf(tly.y, tuy.y)), fminf(fmaxf(tlz.y, tuz.y), tlim));
    const f32x2 n = f32x2{tn0, tn1} * f32x2{LO, LO}, x = f32x2{tx0, tx1} * f32x2{HI, HI};
    h0 = n.x <= x.x;
    h1 = n.y <= x.y;
}
// Stage the BVH nodes and the sphere rows in this workgroup's LDS (every thread of the block,
// before any traversal) when the launch placed them there (l_bvh >= 0).
__device__ __forceinline__ void stage_bvh(const Scene &S) {
    const SceneHdr &h = S.h;
    if (h.l_bvh < 0) return;
    const int4 *sn = reinterpret_cast<const int4 *>(S.tab + h.o_bvh);
    int4 *dn = reinterpret_cast<int4 *>(g_lds + h.l_bvh);
    for (int i = threadIdx.x; i < h.n_bvh * 4; i += blockDim.x) dn[i] = sn[i];
    if (h.l_bsph >= 0) {
        const int4 *ss = reinterpret_cast<const int4 *>(S.tab + h.o_sph);
        int4 *ds = reinterpret_cast<int4 *>(g_lds + h.l_bsph);
        for (int i = threadIdx.x; i < h.n_sph * 2; i += blockDim.x) ds[i] = ss[i];
    }
    __syncthreads();
}
// LDS: the nodes are staged in LDS (h.l_bvh >= 0), ROWS: the sphere rows too (h.l_bsph >= 0);
// else read from HBM (L2)
template <bool LDS, bool ROWS, bool FAST = false>
__device__ __forceinline__ void scan_bvh(const Scene &S, const D3 &o, const D3 &d, double A4, bool act, double &bt,
                                         int &bid) {
    const SceneHdr &h = S.h;
    const float4 *nodes = LDS ? reinterpret_cast<const float4 *>(g_lds + h.l_bvh)
                              : reinterpret_cast<const float4 *>(S.tab + h.o_bvh);
    const double2 *rows = ROWS ? reinterpret_cast<const double2 *>(g_lds + h.l_bsph)
                               : reinterpret_cast<const double2 *>(S.tab + h.o_sph);
    unsigned *stk = reinterpret_cast<unsigned *>(g_lds + h.l_stack) + (threadIdx.x >> 6) * (64 * h.bvh_depth) +
                    (threadIdx.x & 63);
    const BvhRay ray = bvh_ray(o, d);
    constexpr float HI = 1.0f + 0x1p-16f;
    float tlim = __builtin_inff();
    // sphere k (local index, compact id id), as sphere_BC<false> + sph_t (the candidate walk's
    // expressions)
    auto leaf = [&](int k, int id) {
        RT_STAT(ST_BVH_LEAF, 1);
        RT_STAT(ST_BVH_LEAF_LANES, __popcll(__ballot(1)));
        const double2 c01 = rows[k * 2], c2r = rows[k * 2 + 1];
        const D3 oc = {o.x - c01.x, o.y - c01.y, o.z - c2r.x};
        const double B = 2 * (d.x * oc.x + d.y * oc.y + d.z * oc.z);
        const double C = oc.x * oc.x + oc.y * oc.y + oc.z * oc.z - c2r.y;
        double t;
        // (as one divergent block — sph_t_wave and the nearer test as a mask — measured neutral:
        // profiles/r05ag_ab_bvh_leaf_block.txt)
        if (sph_t<FAST>(B, C, A4, t) && nearer(t, id, bt, bid)) {
            bt = t;
            bid = id;
            tlim = (float)t * HI;
        }
    };
    int node = act ? 0 : -1, sp = 0;
    RT_STAT(ST_BVH_SCANS, 1);
    // the next node from the stack: the nearest pushed entry not beyond tlim (-1: traversal done)
    auto pop = [&]() {
        node = -1;
        while (sp > 0) {
            const unsigned en = stk[--sp * 64];
            if (__uint_as_float(en & 0xffff0000u) <= tlim) {
                node = (int)(en & 0xffffu);
                break;
            }
        }
    };
    // one visit of `node`: both children's boxes tested; the leaves among those hit are returned
    // in l0 / l1, the nearer inner child hit becomes `node` (the farther one pushed), else -1
    auto visit = [&](bool &l0, bool &l1, float4 &e) {
        RT_STAT(ST_BVH_ITER, 1);
        RT_STAT(ST_BVH_ITER_LANES, __popcll(__ballot(1)));
        const float4 a = nodes[node * 4], b = nodes[node * 4 + 1], c = nodes[node * 4 + 2];
        e = nodes[node * 4 + 3];
        float tn0, tn1;
        bool h0, h1;
        bvh_slab2(ray, a, b, c, tlim, h0, tn0, h1, tn1);
        const int c0 = __float_as_int(e.x), c1 = __float_as_int(e.y);
        l0 = h0 && c0 < 0;
        l1 = h1 && c1 < 0;
        h0 = h0 && !l0;
        h1 = h1 && !l1;
        if (h0 && h1) {
            const bool f0 = tn0 <= tn1;
            const float tf = f0 ? tn1 : tn0;
            stk[sp * 64] = (__float_as_uint(tf) & 0xffff0000u) | (unsigned)(f0 ? c1 : c0); // tf >= 0: truncation rounds down
            ++sp;
            node = f0 ? c0 : c1;
        } else {
            node = (h0 | h1) ? (h0 ? c0 : c1) : -1;
        }
    };
    // the leaves a visit returned, child 0's first: one divergent leaf test for every lane with a
    // leaf, a second only for the lanes with two.  (Postponing a lane's leaves until half of the
    // wave's unfinished lanes hold some, so that they are tested together, halved the leaf tests
    // per wave but added visits: config 5 +2 % per frame, not kept.)
    auto leaves = [&](bool l0, bool l1, const float4 &e) {
        if (l0 | l1) {
            leaf(~__float_as_int(l0 ? e.x : e.y), __float_as_int(l0 ? e.z : e.w));
            if (l0 & l1) leaf(~__float_as_int(e.y), __float_as_int(e.w));
        }
    };
    while (node >= 0) {
        bool l0, l1;
        float4 e;
        visit(l0, l1, e);
        leaves(l0, l1, e);
        if (node < 0) pop();
    }
}

#ifndef RT_MAX_GROUPS
#define RT_MAX_GROUPS 3 // reflection beams per wave (lanes grouped by the object they leave)
#endif
constexpr int MAX_GROUPS = RT_MAX_GROUPS;
constexpr int UNION_CHUNKS = 4; // reflection scans of scenes up to 256 spheres walk the union of the groups' candidates
// NB: the scene has no wave beams (beam_ok = 0, host-checked): every chunk is scanned whole and
// the beam code is compiled out (registers: the fused engine's occupancy).
template <bool PRE, bool ILP = false, int SPH = 0, bool NB = false>
__device__ __forceinline__ int nearest(const Scene &S, int org, const D3 &o, const D3 &d, double &bt, bool act,
                                       int grp = -1, bool bvh = false) {
    const SceneHdr &h = S.h;
    bt = __builtin_inf();
    int bid = 0x7fffffff;
    if (__ballot(act) == 0) return -1; // nothing to trace in this wave
    const double A4 = 4 * (d.x * d.x + d.y * d.y + d.z * d.z);
    RT_STAT(PRE ? ST_NEAR_PRE : ST_NEAR_GEN, 1);
    RT_STAT(ST_NEAR_LANES, __popcll(__ballot(act)));
    if constexpr (NB) {
        for (int chunk = 0; chunk < h.n_sph; chunk += 64)
            scan_spheres<PRE, ILP, (SPH >= 1)>(S, org, o, d, A4, chunk, chunk_all(h.n_sph, chunk), bt, bid);
        scan_tri_pl<PRE>(S, org, o, d, bt, bid);
        return (act && bid != 0x7fffffff) ? bid : -1;
    }
    if (!PRE && bvh) { // (wave-uniform) per-lane BVH traversal, then the triangles and planes
        if (h.l_bvh >= 0 && h.l_bsph >= 0)
            scan_bvh<true, true, (SPH >= 1)>(S, o, d, A4, act, bt, bid);
        else if (h.l_bvh >= 0)
            scan_bvh<true, false, (SPH >= 1)>(S, o, d, A4, act, bt, bid);
        else
            scan_bvh<false, false, (SPH >= 1)>(S, o, d, A4, act, bt, bid);
        scan_tri_pl<PRE>(S, org, o, d, bt, bid);
        return (act && bid != 0x7fffffff) ? bid : -1;
    }
    unsigned long long rem = __ballot(act);
    // staged (SPH = 2) scans keep the single-chunk form (S64: fewer registers, measured faster)
    constexpr int UCH = SPH == 2 ? 1 : UNION_CHUNKS;
    if (!PRE && h.n_sph <= 64 * UCH) {
        // The union of the groups' candidate masks (per 64-sphere chunk), walked once by the whole
        // wave (a sphere outside a lane's cone cannot be hit by that lane, so testing it is
        // harmless): each candidate is tested once however many groups share it.
        unsigned long long m[UCH] = {};
        const int nch = (h.n_sph + 63) >> 6;
        bool all = false;
        for (int g = 0; g < MAX_GROUPS && rem; ++g) {
            const int gv = __builtin_amdgcn_readlane(grp, __builtin_ctzll(rem));
            const bool sel = (g == MAX_GROUPS - 1) ? ((rem >> (threadIdx.x & 63)) & 1) != 0 : (act && grp == gv);
            rem &= ~__ballot(sel);
            const Beam32 b = make_beam32<(SPH >= 1)>(h, sel, o, d);
            RT_STAT(ST_BEAM_ON, b.on ? 1 : 0);
            if (!b.on) {
                all = true;
                break;
            }
#pragma unroll
            for (int c = 0; c < UCH; ++c)
                if (c < nch) m[c] |= cull_chunk32<SPH>(S, b, c * 64);
        }
#pragma unroll
        for (int c = 0; c < UCH; ++c)
            if (c < nch) scan_spheres<false, ILP, (SPH >= 1)>(S, org, o, d, A4, c * 64, all ? chunk_all(h.n_sph, c * 64) : m[c], bt, bid);
        rem = 0;
    }
    for (int g = 0; g < MAX_GROUPS && rem; ++g) {
        bool sel = act;
        if (!PRE) {
            const int gv = __builtin_amdgcn_readlane(grp, __builtin_ctzll(rem));
            sel = (g == MAX_GROUPS - 1) ? ((rem >> (threadIdx.x & 63)) & 1) != 0 : (act && grp == gv);
        }
        rem = PRE ? 0ull : (rem & ~__ballot(sel));
        bool on;
        if constexpr (PRE) {
            const Beam b = make_beam(h, sel, o, d, true);
            on = b.on;
            RT_STAT(ST_BEAM_ON, b.on ? 1 : 0);
            for (int chunk = 0; chunk < h.n_sph; chunk += 64) {
                const unsigned long long m = b.on ? cull_chunk<SPH>(S, b, chunk, org) : chunk_all(h.n_sph, chunk);
                scan_spheres<PRE, ILP, (SPH >= 1)>(S, org, o, d, A4, chunk, m, bt, bid);
            }
        } else {
            const Beam32 b = make_beam32<(SPH >= 1)>(h, sel, o, d);
            on = b.on;
            RT_STAT(ST_BEAM_ON, b.on ? 1 : 0);
            for (int chunk = 0; chunk < h.n_sph; chunk += 64) {
                const unsigned long long m = b.on ? cull_chunk32<SPH>(S, b, chunk) : chunk_all(h.n_sph, chunk);
                scan_spheres<PRE, ILP, (SPH >= 1)>(S, org, o, d, A4, chunk, m, bt, bid);
            }
        }
        if (!on) break; // everything was scanned
    }
    scan_tri_pl<PRE>(S, org, o, d, bt, bid);
    return (act && bid != 0x7fffffff) ? bid : -1;
}

// nearest_object_intersecting_ray/6 for two rays per lane from tabled origin `org` (primary
// rays): one beam and one candidate walk serve both, and each candidate's two tests are
// independent (instruction-level parallelism for the wave).
// FAST: the scene's spheres and the camera are within CULL_EXTENT (unit primary rays: every
// discriminant in sqrt_x's range, see there).
// pm (wave-uniform, or null): this wave's candidate masks, one per 64-sphere chunk, precomputed
// for its 8x16 pixel block (k_pmask) — then no beam is built here.
template <bool FAST>
__device__ __forceinline__ void nearest_pair(const Scene &S, int org, const D3 &o, const D3 &d0, const D3 &d1, bool a0,
                                             bool a1, int &id0, double &t0, int &id1, double &t1,
                                             const unsigned long long *pm = nullptr) {
    const SceneHdr &h = S.h;
    double bt0 = __builtin_inf(), bt1 = __builtin_inf();
    int bid0 = 0x7fffffff, bid1 = 0x7fffffff;
    id0 = id1 = -1;
    t0 = t1 = 0.0;
    if (__ballot(a0 | a1) == 0) return;
    const double A40 = 4 * (d0.x * d0.x + d0.y * d0.y + d0.z * d0.z);
    const double A41 = 4 * (d1.x * d1.x + d1.y * d1.y + d1.z * d1.z);
    Beam32 b;
    b.on = false;
    if (!pm) b = make_beam_pair32(h, a0, d0, a1, d1);
    RT_STAT(ST_NEAR_PRE, 1);
    for (int chunk = 0; chunk < h.n_sph; chunk += 64) {
        // (the table's entry is the wave's: read as a uniform value, so the candidate walk below is a
        // wave-uniform loop over scalar-loaded rows — read per lane, the compiler made it a per-lane walk
        // over gathered rows: k_primary's frames 1.4-1.7 % slower, profiles/r05al_ab_uniform_primary_masks.txt)
        unsigned long long m = pm ? uniform_u64(pm[chunk >> 6]) : b.on ? cull_chunk32_org(S, b, chunk, org) : chunk_all(h.n_sph, chunk);
        RT_STAT(ST_NEAR_PRE_CAND, __popcll(m));
        while (m) {
            const int k = chunk + __builtin_ctzll(m);
            m &= m - 1;
            const double *q = S.tab + h.o_sph_org + (org * h.n_sph + k) * SPH_ORG_W;
            const double qx = q[0], qy = q[1], qz = q[2], C = q[3];
            const int id = S.itab[h.i_sph_id + k];
            double u0, u1;
            const bool h0 = sph_t_wave<FAST>(2 * (d0.x * qx + d0.y * qy + d0.z * qz), C, A40, u0);
            const bool h1 = sph_t_wave<FAST>(2 * (d1.x * qx + d1.y * qy + d1.z * qz), C, A41, u1);
            const bool up0 = h0 & nearer(u0, id, bt0, bid0), up1 = h1 & nearer(u1, id, bt1, bid1);
            bt0 = up0 ? u0 : bt0; bid0 = up0 ? id : bid0;
            bt1 = up1 ? u1 : bt1; bid1 = up1 ? id : bid1;
        }
    }
    if (h.n_tri | h.n_pl) {
        scan_tri_pl<true>(S, org, o, d0, bt0, bid0);
        scan_tri_pl<true>(S, org, o, d1, bt1, bid1);
    }
    if (a0 && bid0 != 0x7fffffff) { id0 = bid0; t0 = bt0; }
    if (a1 && bid1 != 0x7fffffff) { id1 = bid1; t1 = bt1; }
}

// Hit point and normal of object `id` at distance t (as computed inside the reference's
// intersect functions: Intersection = O + D*t, :384-390, :443-451, :471-476).
__device__ __forceinline__ void hit_geom(const Scene &S, int id, const D3 &o, const D3 &d, double t, D3 &hit,
                                         D3 &N) {
    hit = D3{o.x + d.x * t, o.y + d.y * t, o.z + d.z * t};
    const double *r = S.tab + S.h.o_obj + id * OBJ_W;
    int kind = S.itab[S.h.i_obj_meta + id * OBJ_META_W];
    if (kind == K_SPHERE)
        N = normalize3(D3{hit.x - r[0], hit.y - r[1], hit.z - r[2]});
    else
        N = D3{r[0], r[1], r[2]};
}

// Bounding ball of the active lanes' hit points (centre = their centroid), shared by the
// shadow cones of every light at this level.  Called by the converged wave.
struct HitBall {
    double cx, cy, cz, r;
    bool on;
};
__device__ __forceinline__ HitBall make_hitball(const SceneHdr &h, bool act, const D3 &hit) {
    HitBall hb;
    hb.on = false;
    hb.cx = hb.cy = hb.cz = hb.r = 0.0;
    const unsigned long long am = __ballot(act);
    if (!h.beam_ok || am == 0) return hb;
    const double inv_n = 1.0 / (double)__popcll(am);
    hb.cx = uniform(wave_sum(act ? hit.x : 0.0) * inv_n);
    hb.cy = uniform(wave_sum(act ? hit.y : 0.0) * inv_n);
    hb.cz = uniform(wave_sum(act ? hit.z : 0.0) * inv_n);
    const double ex = hit.x - hb.cx, ey = hit.y - hb.cy, ez = hit.z - hb.cz;
    const double r2 = wave_max(act ? ex * ex + ey * ey + ez * ez : 0.0);
    const double mo = wave_max(act ? fmax(fabs(hit.x), fmax(fabs(hit.y), fabs(hit.z))) : 0.0);
    if (!(mo <= CULL_EXTENT)) return hb;
    hb.r = uniform(sqrt(r2)) * (1 + CULL_EPS) + CULL_EPS;
    hb.on = true;
    return hb;
}

// The cone of shadow-ray directions from light position Lp to the hit ball, and the largest
// shadow-ray distance t* any lane can have (a target is hit no farther than its hit point).
__device__ __forceinline__ Beam shadow_cone(const HitBall &hb, const D3 &Lp, double &tmax) {
    Beam b;
    b.on = false;
    b.ax = b.ay = b.az = b.c = b.s = b.mx = b.my = b.mz = b.ro = 0.0;
    tmax = __builtin_inf();
    if (!hb.on) return b;
    const double wx = hb.cx - Lp.x, wy = hb.cy - Lp.y, wz = hb.cz - Lp.z;
    const double D = sqrt(wx * wx + wy * wy + wz * wz);
    if (!(D > hb.r * (1 + CULL_EPS) + CULL_EPS)) return b; // light inside the ball
    const double sr = hb.r / D * (1 + CULL_EPS) + CULL_EPS;
    if (!(sr < 1.0)) return b;
    const double inv = 1.0 / D;
    b.ax = wx * inv; b.ay = wy * inv; b.az = wz * inv;
    b.s = sr;
    b.c = sqrt(1.0 - sr * sr) - CULL_EPS;
    if (!(b.c > 0.0)) return b;
    tmax = (D + hb.r) * (1 + CULL_EPS) + CULL_EPS;
    b.on = true;
    return b;
}

// shadow_factor/4 (:256-267) as the exact bounded any-hit test described at the top.
// c = canonical compact id of the hit object, sd = normalize(Hit - Light).
// The shadow target of a lane at one level: canonical id, its kind and index within its type,
// and (wave-uniform) the sphere every shading lane shares, if there is one (-1 otherwise).
struct Target {
    int c, kind, loc, skip;
};
template <int SPH = 0>
__device__ __forceinline__ Target make_target(const Scene &S, int obj, bool active) {
    // one row: kind, local, canonical id, the canonical element's local index (same kind)
    const int4 mt = obj_meta<SPH>(S, obj);
    Target T;
    T.c = mt.z;
    T.kind = mt.x;
    T.loc = mt.w;
    T.skip = -1;
    const unsigned long long am = __ballot(active);
    if (am != 0) {
        const int first = __builtin_ctzll(am);
        const int cu = __builtin_amdgcn_readlane(T.c, first);
        if (__ballot(active && T.c != cu) == 0 && __builtin_amdgcn_readlane(T.kind, first) == K_SPHERE)
            T.skip = __builtin_amdgcn_readlane(T.loc, first); // uniform target: a sphere cannot block itself
    }
    return T;
}

// Direction cell of a shadow ray sd from a light towards a target sphere (q = light - centre,
// C: the target's per-origin row): along the two world axes i, j on which a = -q/|q|, the
// cone's axis, is shortest, the signs of (sd - a) and (16 cells) whether |sd - a| exceeds half
// the cone's sine r/(2|q|) (r^2 = |q|^2 - C).  Evaluated in binary32; the host's masks are built
// for the same cells, each widened by OCC_CELL_EPS, far above this evaluation's error, so a ray
// near a cell border is covered by the mask of either side.  Only the axis choice must agree
// exactly, and it is the same binary32 comparison on both sides (rt_scene.cpp).
__device__ __forceinline__ int occ_cell(const double *q, const D3 &sd) {
    const float qx = (float)q[0], qy = (float)q[1], qz = (float)q[2];
    const float D = sqrt_f32f(qx * qx + qy * qy + qz * qz); // (a filter: cells overlap by OCC_CELL_EPS)
    const float ax = __builtin_fabsf(qx), ay = __builtin_fabsf(qy), az = __builtin_fabsf(qz);
    const int drop = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    const float ex = (float)sd.x * D + qx, ey = (float)sd.y * D + qy, ez = (float)sd.z * D + qz;
    const float ei = drop == 0 ? ey : ex, ej = drop == 2 ? ey : ez;
    if (OCC_CELLS == 64) { // per axis: the sign and |e| against r/4, r/2, 3r/4 (8 bins), cell = bi + 8 bj
        const float t2 = (float)(((q[0] * q[0] + q[1] * q[1] + q[2] * q[2]) - q[3]) * 0.25); // (r/2)^2
        auto bin = [&](float e) {
            const float e2 = e * e;
            return (e >= 0.0f ? 4 : 0) + (e2 >= 0.25f * t2 ? 1 : 0) + (e2 >= t2 ? 1 : 0) + (e2 >= 2.25f * t2 ? 1 : 0);
        };
        return bin(ei) + 8 * bin(ej);
    }
    int cell = (ei >= 0.0f ? 1 : 0) + (ej >= 0.0f ? 2 : 0);
    if (OCC_CELLS == 16) {
        const float t2 = (float)(((q[0] * q[0] + q[1] * q[1] + q[2] * q[2]) - q[3]) * 0.25); // (r/2)^2
        cell += (ei * ei >= t2 ? 4 : 0) + (ej * ej >= t2 ? 8 : 0);
    }
    return cell;
}

// SPH: the scene holds only spheres and culling is on (host-checked), so every target is a
// sphere with occluder masks: the cone and triangle/plane paths are compiled out (registers).
template <int SPH = 0, bool NB = false>
__device__ __forceinline__ bool lit_by(const Scene &S, int light, const Target &T, const D3 &sd, bool active,
                                       const HitBall &hb, const D3 &Lp) {
    const SceneHdr &h = S.h;
    const int org = 1 + light;
    const int c = T.c, kind = T.kind, loc = T.loc, skip = T.skip;
    const double A4 = 4 * (sd.x * sd.x + sd.y * sd.y + sd.z * sd.z);
    // t* of the target itself along the shadow ray
    double ts = 0;
    bool valid = false;
    int cell = 0;
    if (active) {
        if (SPH || kind == K_SPHERE) {
            const double *q = org_row<SPH>(S, org, loc);
            double B = 2 * (sd.x * q[0] + sd.y * q[1] + sd.z * q[2]);
            valid = SPH ? sph_t<true>(B, q[3], A4, ts) : sph_t(B, q[3], A4, ts);
            if (SPH != 2 && h.occ_cells > 1) cell = occ_cell(q, sd); // (staged scenes: one cell)
        } else if (kind == K_TRIANGLE) {
            const double *g = S.tab + h.o_tri + loc * TRI_W;
            const double *q = S.tab + h.o_tri_org + (org * h.n_tri + loc) * TRI_ORG_W;
            valid = tri_t(sd, D3{g[3], g[4], g[5]}, D3{g[6], g[7], g[8]}, D3{q[0], q[1], q[2]}, D3{q[3], q[4], q[5]},
                          ts);
        } else {
            const double *p = S.tab + h.o_pl + loc * PL_W;
            valid = pl_t(D3{p[0], p[1], p[2]}, sd, S.tab[h.o_pl_org + org * h.n_pl + loc], ts);
        }
    }
    bool blocked = !valid; // a target the shadow ray misses is never lit
    if (__all(blocked)) return false;
    // Candidate occluders.  Sphere targets: the union of the host-precomputed occluder masks of
    // the wave's distinct targets (no reductions).  Otherwise the cone from the light to the
    // hit ball of the wave, culled lane-parallel.
    const bool sph_targets = SPH || (h.occ_ok && __ballot(!blocked && kind != K_SPHERE) == 0);
    double tmax = __builtin_inf();
    Beam b;
    b.on = false;
    if (!SPH && !NB && !sph_targets) b = shadow_cone(hb, Lp, tmax); // shadow rays all start at the light
    RT_STAT(ST_SHADOW, 1);
    RT_STAT(ST_SHADOW_CONE_ON, (sph_targets || b.on) ? 1 : 0);
    for (int chunk = 0; chunk < h.n_sph; chunk += 64) {
        unsigned long long m;
        if (sph_targets) {
            // Every lane walks its own target's occluder mask: the trip count is the largest
            // per-lane candidate count, not the size of the union over the wave's targets
            // (which grows with every distinct target an incoherent wave holds).
            const unsigned long long *occ = occ_masks<SPH>(S, light, chunk >> 6);
            const int ncell = SPH == 2 ? 1 : h.occ_cells;
            unsigned long long mine = blocked ? 0ull : occ[(loc * ncell + cell) * h.n_chunk]; // never holds the target
#ifdef RT_ABL_NO_OCC // timing ablation builds only (results wrong): no occluder tests
            mine = 0;
#endif
            // (software-pipelined — the next candidate's row loaded while the current one is tested —
            // measured config 5 +4 %, config 3 +1.3 %: profiles/r05ai_ab_occluder_prefetch.txt)
            for (;;) {
                const bool w = !blocked && mine != 0;
                if (__ballot(w) == 0) break;
                // the row from the chunk's (wave-uniform) first row: one address operation per lane
                const int lk = w ? __builtin_ctzll(mine) : 0, k = chunk + lk;
                mine &= mine - 1;
                RT_STAT(ST_SHADOW_ITER, 1);
                const double2 *q = reinterpret_cast<const double2 *>(org_row<SPH>(S, org, chunk)) + 2 * lk;
                const double2 q01 = q[0], q23 = q[1];
                const double B = 2 * (sd.x * q01.x + sd.y * q01.y + sd.z * q23.x);
                double t;
                const bool hit = sph_t_wave<(SPH >= 1)>(B, q23.y, A4, t);
                // the candidate's list position matters only at an exact tie with the target's t*
                // (next to never): it is read for such waves alone.  The branch is taken on the bare
                // compare's ballot (one v_cmp, no mask materialised): a lane off the walk that equals
                // t* by chance only takes it, and the test inside is the exact one.
                bool blk = w & hit & (t < ts);
                if (__ballot(t == ts) != 0) blk = blk | (w & hit & (t == ts) & (sph_id<SPH>(S, k) < c));
                blocked = blocked | blk;
            }
            if (__all(blocked)) return false;
            continue;
        } else if (!SPH) {
            m = (!NB && b.on) ? cull_chunk(S, b, chunk, org, tmax) : chunk_all(h.n_sph, chunk);
            if (skip >= chunk && skip < chunk + 64) m &= ~(1ull << (skip - chunk));
        }
        RT_STAT(ST_SHADOW_CAND, __popcll(m));
        while (!SPH && m) {
            const int k = chunk + __builtin_ctzll(m);
            m &= m - 1;
            RT_STAT(ST_SHADOW_ITER, 1);
            const double *q = S.tab + h.o_sph_org + (org * h.n_sph + k) * SPH_ORG_W;
            const int id = S.itab[h.i_sph_id + k];
            const double B = 2 * (sd.x * q[0] + sd.y * q[1] + sd.z * q[2]);
            double t;
            const bool hit = sph_t_wave(B, q[3], A4, t);
            blocked = blocked | (hit & ((t < ts) | ((t == ts) & (id < c))));
            if (__all(blocked)) return false;
        }
    }
    if (SPH) return !blocked;
    for (int k = 0; k < h.n_tri; ++k) {
        if (!blocked) {
            const double *g = S.tab + h.o_tri + k * TRI_W;
            const double *q = S.tab + h.o_tri_org + (org * h.n_tri + k) * TRI_ORG_W;
            double t;
            if (tri_t(sd, D3{g[3], g[4], g[5]}, D3{g[6], g[7], g[8]}, D3{q[0], q[1], q[2]}, D3{q[3], q[4], q[5]}, t)) {
                int id = S.itab[h.i_tri_id + k];
                blocked = t < ts || (t == ts && id < c);
            }
        }
        if (__all(blocked)) return false;
    }
    for (int k = 0; k < h.n_pl; ++k) {
        if (!blocked) {
            const double *p = S.tab + h.o_pl + k * PL_W;
            double t;
            if (pl_t(D3{p[0], p[1], p[2]}, sd, S.tab[h.o_pl_org + org * h.n_pl + k], t)) {
                int id = S.itab[h.i_pl_id + k];
                blocked = t < ts || (t == ts && id < c);
            }
        }
        if (__all(blocked)) return false;
    }
    return !blocked;
}

// lighting_function/6 (:209-252) for one hit.  The reflection the reference adds for every
// light is R = col * refl (col = colour of the level below); it is formed at each use — the
// same operation on the same operands, so the same bits — which keeps fewer values live
// across the shadow scans (register pressure sets this kernel's occupancy).  The material is
// re-read per light for the same reason.
// bits (optional): bit i set where light i's shadow test passed (lights 0..31; only lanes whose
// light term is not exactly zero are tested, the others' bits are 0 and never matter).
// OPQ (col a live value, not the background's constant): col is made opaque inside the light loop,
// so col * refl is formed per light as written instead of being hoisted out of the loop into three
// more live doubles (the fused kernel spilled them).
template <bool GENPOW, int SPH = 0, bool NB = false, bool OPQ = false>
__device__ __forceinline__ D3 shade(const Scene &S, int id, const D3 &d, const D3 &hit, const D3 &N, const D3 &col,
                                    double refl, bool active, unsigned *bits = nullptr) {
    const SceneHdr &h = S.h;
    if (__ballot(active) == 0) return D3{0.0, 0.0, 0.0}; // no hit to shade in this wave
    const Target T = make_target<SPH>(S, id, active);
    // the hit ball is only needed for non-sphere shadow targets (see lit_by)
    HitBall hb;
    hb.on = false;
    hb.cx = hb.cy = hb.cz = hb.r = 0.0;
    // (and for every target when the scene has no occluder masks: occ_ok = 0)
    if (!SPH && !NB && (!h.occ_ok || __ballot(active && T.kind != K_SPHERE) != 0)) hb = make_hitball(h, active, hit);
    RT_STAT(ST_SHADE, 1);
    D3 F = {0.0, 0.0, 0.0};
    for (int i = 0; i < h.n_light; ++i) {
        const Scene &SL = S; // (re-reading the header per light, fresh_scene: measured neutral)
        const double *L = SL.tab + SL.h.o_light + i * LIGHT_W;
        // the material row's address formed per light from the (opaque) object id: one live
        // register instead of a 64-bit pointer across the loop
        int idl = id;
        asm volatile("" : "+v"(idl));
        const double *m = obj_row<SPH>(S, idl);
        const D3 Lc = {L[0], L[1], L[2]}, Lp = {L[3], L[4], L[5]}, Sc = {L[6], L[7], L[8]};
        const double2 m34 = *reinterpret_cast<const double2 *>(m + 4), m67 = *reinterpret_cast<const double2 *>(m + 6);
        const D3 mc = {m[3], m34.x, m34.y};
        const double spow = m67.x, shin = m67.y;
        // diffuse_term/4 (:272-279)
        const D3 ln = normalize3(D3{Lp.x - hit.x, Lp.y - hit.y, Lp.z - hit.z}, SPH && SL.h.norm_ok);
        const double dd = max0(dot3(N, ln));
        const D3 diff = {mc.x * dd, mc.y * dd, mc.z * dd};
        // specular_term/7 (:285-297)
        const D3 hn = normalize3(D3{ln.x + -d.x, ln.y + -d.y, ln.z + -d.z});
        const double sp = shin * pow_libm<GENPOW>(max0(dot3(hn, N)), spow, active);
        const D3 spec = {Sc.x * sp, Sc.y * sp, Sc.z * sp};
        const D3 con = {diff.x + spec.x, diff.y + spec.y, diff.z + spec.z};
        // A lane whose light term Lc (x) con is exactly zero gets the same bits for lit = 0 and
        // lit = 1 (the factor only multiplies signed zeros by 0 or 1): skip its shadow test.
        const D3 lc = {Lc.x * con.x, Lc.y * con.y, Lc.z * con.z};
        const bool need = active && !(lc.x == 0.0 && lc.y == 0.0 && lc.z == 0.0);
        // shadow ray direction normalize(Hit - Light) == -normalize(Light - Hit), bit for bit
        const bool lb = lit_by<SPH, NB>(SL, i, T, D3{-ln.x, -ln.y, -ln.z}, need, hb, Lp);
        if (bits && lb && i < 32) *bits |= 1u << i;
        const double lit = lb ? 1.0 : 0.0;
        D3 c = col;
        if (OPQ) asm volatile("" : "+v"(c.x), "+v"(c.y), "+v"(c.z));
        F.x = F.x + (c.x * refl + lc.x * lit);
        F.y = F.y + (c.y * refl + lc.y * lit);
        F.z = F.z + (c.z * refl + lc.z * lit);
    }
    return F;
}

// The beam-free build (NB) needs fewer registers: its own occupancy target.
#ifndef RT_FUSED_NB_WAVES
#define RT_FUSED_NB_WAVES 5
#endif
#ifndef RT_FUSED_NB
#define RT_FUSED_NB 1
#endif
template <int ORDER, int PREC, bool LEVELS, bool GENPOW, bool NB>
__global__ __launch_bounds__(256, NB ? RT_FUSED_NB_WAVES : RT_WAVES_PER_SIMD) void k_render(SceneHdr hdr, const double *__restrict__ tab,
                                                  const int *__restrict__ itab, int W, int H, int depth, int rb,
                                                  int shard, int nshards, int row0, int row_end, void *__restrict__ out,
                                                  uint8_t *__restrict__ levels, int levels_hit) {
    // this launch covers slab rows [row0, row_end); out / levels point at slab row 0
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Scene S{hdr, tab, itab};
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x = blockIdx.x * TILE + (wave & 1) * 8 + (lane & 7);
    const int ly = row0 + blockIdx.y * TILE + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = x < W && ly < row_end;
    // slab row -> image row: the tile's first row split once (wave-uniform), the offset (< 16) added
    const int ly_base = row0 + blockIdx.y * TILE, q_base = ly_base / rb;
    int rr = ly_base - q_base * rb + (ly - ly_base), qq = q_base;
    while (rr >= rb) {
        rr -= rb;
        ++qq;
    }
    const int gy = (qq * nshards + shard) * rb + rr;
    const bool active = inside && gy < H;
    RT_STAT(ST_WAVES, 1);

    // primary ray: ray_through_pixel/3 (:510-511) at {X/Width, Y/Height} (:112)
    const double X = div_n((double)x, (double)W), Y = div_n((double)gy, (double)H); // == / (W, H <= 2^20)
    const double px = 0.0 + ((X - 0.5) * hdr.screen_w + hdr.sx);
    const double py = (Y - 0.5) * hdr.screen_h + hdr.sy;
    const D3 cam = {hdr.cam_x, hdr.cam_y, hdr.cam_z};
    const D3 d0 = normalize3(D3{px - hdr.cam_x, py - hdr.cam_y, hdr.dz}, hdr.prim_ok);

    D3 col = {0.0, 0.0, 0.0};
    int nlev = 0;
    if (ORDER == RT_ORDER_EXACT) {
        double *st = reinterpret_cast<double *>(smem);               // [depth][BLOCK] distances
        int *so = reinterpret_cast<int *>(smem + (size_t)depth * BLOCK * 8); // [depth][BLOCK] object ids
        // [3][BLOCK] the primary direction, read back by each level's replay instead of being kept
        // live (spilled) across the chain
        double *sd0 = reinterpret_cast<double *>(smem + (size_t)depth * BLOCK * 12);
        sd0[tid] = d0.x;
        sd0[BLOCK + tid] = d0.y;
        sd0[2 * BLOCK + tid] = d0.z;
        // forward: the reflection chain's nearest-object scans
        D3 o = cam, d = d0;
        bool alive = active;
        int prev = -1;
        for (int k = 0; k < depth; ++k) {
            const Scene SL = fresh_scene(S); // the header re-read per level (fresh_scene)
            double t = 0;
            int id = -1;
            id = (k == 0) ? nearest<true, false, 0, NB>(SL, 0, o, d, t, alive)
                           : nearest<false, false, 0, NB>(SL, 0, o, d, t, alive, prev);
            if (id < 0) alive = false;
            prev = id;
            if (alive) {
                st[k * BLOCK + tid] = t;
                so[k * BLOCK + tid] = id;
                nlev = k + 1;
                if (k == depth - 1 || hdr.n_light == 0) alive = false;
            }
            if (alive) {
                D3 hit, N;
                hit_geom(SL, id, o, d, t, hit, N);
                d = bounce3(d, N);
                o = hit;
            }
            if (__all(!alive)) break;
        }
        // backward: shade each level with the colour of the level below it (:216-247)
        int maxlev = 0;
        while (maxlev < depth && __ballot(nlev > maxlev) != 0) ++maxlev; // wave-wide max level
        for (int m = 0; m < maxlev; ++m) {
            const Scene SL = fresh_scene(S); // the header re-read per level (fresh_scene)
            const int k = nlev - 1 - m;
            const bool on = k >= 0;
            D3 o2 = cam, d2 = D3{sd0[tid], sd0[BLOCK + tid], sd0[2 * BLOCK + tid]}, hit = cam, N = cam;
            int id = 0;
            if (on) {
                for (int j = 0; j < k; ++j) { // replay the chain to level k
                    hit_geom(SL, so[j * BLOCK + tid], o2, d2, st[j * BLOCK + tid], hit, N);
                    d2 = bounce3(d2, N);
                    o2 = hit;
                }
                id = so[k * BLOCK + tid];
                hit_geom(SL, id, o2, d2, st[k * BLOCK + tid], hit, N);
            }
            const double refl = SL.tab[SL.h.o_obj + id * OBJ_W + 8];
            const D3 F = shade<GENPOW, 0, NB, true>(SL, id, d2, hit, N, col, refl, on);
            if (on) col = F;
        }
    } else {
        // ORDER_FAST: colour = sum_k W_k * S_k with W_0 = 1, W_{k+1} = W_k * (L * refl_k)
        D3 o = cam, d = d0;
        double w = 1.0;
        bool alive = active;
        int prev = -1;
        for (int k = 0; k < depth; ++k) {
            double t = 0;
            int id = -1;
            id = (k == 0) ? nearest<true, false, 0, NB>(S, 0, o, d, t, alive)
                           : nearest<false, false, 0, NB>(S, 0, o, d, t, alive, prev);
            if (id < 0) alive = false;
            prev = id;
            D3 hit = cam, N = cam;
            if (alive) {
                nlev = k + 1;
                hit_geom(S, id, o, d, t, hit, N);
            }
            if (__all(!alive)) break;
            const D3 F = shade<GENPOW, 0, NB>(S, alive ? id : 0, d, hit, N, D3{0.0, 0.0, 0.0}, 0.0, alive);
            if (alive) {
                col.x = col.x + w * F.x;
                col.y = col.y + w * F.y;
                col.z = col.z + w * F.z;
                w = w * (hdr.n_light_d * S.tab[hdr.o_obj + id * OBJ_W + 8]);
                if (k == depth - 1 || hdr.n_light == 0) alive = false;
                d = bounce3(d, N);
                o = hit;
            }
        }
    }
    if (!active) return; // slab rows past the image are not written
    // the pixel's address recomputed from an opaque thread index rather than kept live (spilled)
    // across the chain
    int t2 = threadIdx.x;
    asm volatile("" : "+v"(t2));
    const int x2 = blockIdx.x * TILE + ((t2 >> 6) & 1) * 8 + (t2 & 7);
    const int ly2 = row0 + blockIdx.y * TILE + ((t2 >> 6) >> 1) * 8 + ((t2 & 63) >> 3);
    const size_t pix = (size_t)ly2 * W + x2;
    if (PREC == RT_OUT_F64) {
        double *o = reinterpret_cast<double *>(out) + pix * 3;
        o[0] = col.x; o[1] = col.y; o[2] = col.z;
    } else {
        float *o = reinterpret_cast<float *>(out) + pix * 3;
        o[0] = (float)col.x; o[1] = (float)col.y; o[2] = (float)col.z;
    }
    if (LEVELS) levels[pix] = (uint8_t)(levels_hit ? (nlev > 0) : min(nlev, 255)); // (counts saturate at 255)
}

#include "rt_wave.inc" // the wavefront engine (default)

// rt_selftest_math: sqrt_n / div_n against the device library's sqrt and division, bit for bit,
// on operands spread log-uniformly over the ranges where the kernels use them; pow_libm's wave-
// uniform path against the per-lane powering; the binary32 wave reductions against a lane loop.
__global__ __launch_bounds__(256) void k_selftest_math(unsigned long long n, unsigned long long seed,
                                                       unsigned long long *__restrict__ bad) {
    unsigned long long local = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * 256) {
        const unsigned long long r = splitmix64(seed ^ i), r2 = splitmix64(seed ^ ~i);
        // sqrt over [2^-767, 2^1000]: random exponent, random 52-bit mantissa
        const long long e = 1023 - 767 + (long long)((r >> 52) % (767 + 1000));
        const double x = __longlong_as_double((long long)((unsigned long long)e << 52 | (r & 0xFFFFFFFFFFFFFull)));
        if (__double_as_longlong(sqrt_n(x)) != __double_as_longlong(sqrt(x))) ++local;
        // structured operands (scenes are written with small integers and short fractions): the
        // squared length of a vector of integers in [-2^10, 2^10] scaled by 2^-k
        {
            const double sx = (double)((long long)(r & 0x7FF) - 1024), sy = (double)((long long)((r >> 11) & 0x7FF) - 1024),
                         sz = (double)((long long)((r >> 22) & 0x7FF) - 1024);
            const double sc = __builtin_amdgcn_ldexp(1.0, -(int)((r >> 33) & 15));
            const D3 w = {sx * sc, sy * sc, sz * sc};
            const D3 uw = normalize3(w);
            const double mw = sqrt(w.x * w.x + w.y * w.y + w.z * w.z), sw = 1.0 / mw;
            if (mw != 0 && (__double_as_longlong(uw.x) != __double_as_longlong(w.x * sw) ||
                            __double_as_longlong(uw.y) != __double_as_longlong(w.y * sw) ||
                            __double_as_longlong(uw.z) != __double_as_longlong(w.z * sw)))
                ++local;
        }
        // 1/b and a/b: b over [2^-400, 2^400], a an integer below 2^21 (the primary-ray divisions)
        const long long eb = 1023 - 400 + (long long)((r2 >> 52) % 800);
        const double b = __longlong_as_double((long long)((unsigned long long)eb << 52 | (r2 & 0xFFFFFFFFFFFFFull)));
        if (__double_as_longlong(div_n(1.0, b)) != __double_as_longlong(1.0 / b)) ++local;
        const double a = (double)(r >> 43), w = (double)((r2 >> 44) + 1);
        if (__double_as_longlong(div_n(a, w)) != __double_as_longlong(a / w)) ++local;
        // normalize3 on random vectors (both paths)
        const D3 v = {x * (r & 1 ? 1 : -1) * 0x1p-600, b * 1e-3, a - 1e6};
        const D3 u = normalize3(v);
        const double m = sqrt(v.x * v.x + v.y * v.y + v.z * v.z), sc = 1.0 / m;
        if (m != 0 && (__double_as_longlong(u.x) != __double_as_longlong(v.x * sc) ||
                       __double_as_longlong(u.y) != __double_as_longlong(v.y * sc) ||
                       __double_as_longlong(u.z) != __double_as_longlong(v.z * sc)))
            ++local;
        // pow_libm's scalar-controlled powering (a wave-uniform exponent: one per 64 consecutive i,
        // every other group) against the per-lane powering, bit for bit; x over [0, 1 + 2^-20)
        {
            const double px = (double)(r2 & 0xFFFFFFFFFFFull) * 0x1p-44 * (1.0 + 0x1p-20);
            const unsigned pu = (unsigned)(splitmix64(seed ^ (i >> 6)) % 1025u), pl = (unsigned)((r2 >> 44) % 1025u);
            const unsigned pn = ((i >> 6) & 1) ? pu : pl;
            const double want = pn == 0 ? 1.0 : pow_bin<false>(px, pn);
            if (__double_as_longlong(pow_libm<false>(px, (double)pn)) != __double_as_longlong(want)) ++local;
        }
        // the binary32 wave reductions (whole waves only): the maximum of values >= +0 exactly, the
        // minimum exactly when no value is negative and negative when one is
        if (__ballot(true) == ~0ull) {
            const float f0 = (float)((double)(r & 0xFFFFFF) * 0x1p-20);
            const float fv = (r >> 40) % 97 == 0 ? -1.0f - f0 : f0; // (no -0.0: its bits order below +0.0's)
            const float fa = __builtin_fabsf(fv);
            float tmin = 3.0e38f, tmax = 0.0f;
            bool neg = false;
            for (int l = 0; l < 64; ++l) { // (wave-uniform)
                const float a = lane_f32(fv, l), b = lane_f32(fa, l);
                tmin = a < tmin ? a : tmin;
                tmax = b > tmax ? b : tmax;
                neg = neg || a < 0.0f;
            }
            const float gmin = wave_min32(fv), gmax = wave_max32(fa);
            if (__float_as_int(gmax) != __float_as_int(tmax) || (neg ? !(gmin < 0.0f) : __float_as_int(gmin) != __float_as_int(tmin)))
                ++local;
        }
    }
    if (local) atomicAdd(bad, local);
}

} // namespace

// =====================================================================================
// C ABI
// =====================================================================================
struct rt_prepared {
    int device;
    SceneHdr hdr;      // what the kernels get: hdr_full, with the filters off when cull == 0
    SceneHdr hdr_full; // the compiled scene's header
    int cull = 1;      // rt_configure(RT_CFG_CULL)
    double *d_tab;
    int *d_itab;
    // wavefront-engine work space, grown on demand (one rt_launch in flight per rt_prepared)
    void *d_queue = nullptr;  // HitRec[slab pixels * depth]
    size_t queue_bytes = 0;
    double *d_colbuf = nullptr; // colours of levels 1 .. depth-1, COL_W doubles per slot
    uint8_t *d_child = nullptr; // per level and slot: the record's reflection hit something
    size_t child_bytes = 0;
    unsigned *d_lit = nullptr;  // per level and slot: shadow answers of lights 0..31 (k_light)
    size_t lit_bytes = 0;
    double *d_sample = nullptr; // supersampling: one sample's slab and the running sum
    size_t sample_bytes = 0;
    size_t colbuf_bytes = 0;
    int *d_counts = nullptr;  // per level and tile: queue lengths
    size_t counts_bytes = 0;
    int *d_items = nullptr;   // per-level record counts, then per-level dense slot lists
    size_t items_bytes = 0;
    // primary rays' candidate masks per 8x16 pixel block of the slab (k_pmask), kept while the
    // frame geometry and the scene stay the same
    unsigned long long *d_pmask = nullptr;
    size_t pmask_bytes = 0;
    long long pmask_key[8] = {};
    bool pmask_valid = false;
    // the shadow pass runs on a second, low-priority stream beside the reflection chain
    // shading of level 0 and of the deeper levels.  The caller's stream plus these stay
    // within the hardware queues a process gets by default (GPU_MAX_HW_QUEUES=4): streams
    // sharing a queue block each other behind their event waits (measured: 5 streams, S64
    // 11 Gpx/s; 3 side streams were no faster than 2 — the chip is saturated in the overlap)
    hipStream_t side[2] = {};
    int side_mode = -1; // rt_configure(RT_CFG_SIDE_STREAMS): -1 = environment (RT_LIT_STREAM), 0 off, 1 on
    std::vector<hipEvent_t> ev_level; // level k's list is ready (depth + 1 of them, grown with the depth)
    std::vector<hipEvent_t> ev_lit;   // level k is shaded
    // Frames repeat with identical arguments (bench, multi-GPU renderer): the second identical
    // rt_launch captures the frame's launch sequence into a graph, later ones replay it.
    // gen counts changes that invalidate a captured frame: work-space reallocations (captured
    // pointers), new scene tables or header, and recomputed primary candidate masks (a graph
    // captured while they were valid holds no k_pmask launch).
    unsigned gen = 0;
    // scene_gen counts new scene tables and culling changes (the primary masks depend on them)
    unsigned scene_gen = 0;
    // RT_CFG_KERNEL_TIMING: per timed kernel (RT_KT_* bit i), a ring of event pairs; a full ring
    // folds its oldest pair into the sum (waiting for it)
    int timing_mask = 0;
    struct KTimer {
        std::vector<hipEvent_t> a, b;
        size_t head = 0, n = 0;
        double sum_ms = 0;
        unsigned long long count = 0;
    } kt[4];
    hipStream_t cap = nullptr;
    hipGraphExec_t gexec = nullptr;
    long long gkey[12] = {};
    long long last_key[12] = {};
    bool last_valid = false;
};

#define HIPCHK(x)                                                                                                  \
    do {                                                                                                           \
        hipError_t e_ = (x);                                                                                       \
        if (e_ != hipSuccess) {                                                                                    \
            std::fprintf(stderr, "rt_mi355x: %s failed: %s\n", #x, hipGetErrorString(e_));                        \
            return RT_EHIP;                                                                                        \
        }                                                                                                          \
    } while (0)

namespace {

struct DevGuard { // restore the caller's current device on scope exit
    int prev = -1;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// RT_CFG_CULL = 0: every scan tests every object (no wave beams or cones, no occluder masks, no
// BVH, no LDS-staged tables, no host-proven skips of range checks) — the reference's brute-force
// scans, against which the filters' frames are checked bit for bit (tests/test_gpu_frames.py).
void apply_cull(rt_prepared *p) {
    p->hdr = p->hdr_full;
    if (!p->cull) {
        p->hdr.cull_ok = 0;
        p->hdr.occ_ok = 0;
        p->hdr.beam_ok = 0;
        p->hdr.bvh_ok = 0;
        p->hdr.l_bytes = 0;
        p->hdr.norm_ok = 0; // and every range check of normalize3 on
        p->hdr.prim_ok = 0;
    }
}

constexpr size_t KT_RING = 64;
int kt_index(int kernel) {
    return kernel == RT_KT_PRIMARY ? 0 : kernel == RT_KT_LEVEL1 ? 1 : kernel == RT_KT_RENDER ? 2 : kernel == RT_KT_PMASK ? 3 : -1;
}
void kt_fold_oldest(rt_prepared::KTimer &t) {
    const size_t i = (t.head + KT_RING - t.n) % KT_RING;
    float ms = 0;
    if (hipEventSynchronize(t.b[i]) == hipSuccess && hipEventElapsedTime(&ms, t.a[i], t.b[i]) == hipSuccess) {
        t.sum_ms += ms;
        ++t.count;
    }
    --t.n;
}
// bracket one launch of `kernel` (an RT_KT_* bit) on `st` when the context times it
struct KtScope {
    rt_prepared::KTimer *t = nullptr;
    hipStream_t st;
    KtScope(rt_prepared *p, int kernel, hipStream_t s) : st(s) {
        if (!(p->timing_mask & kernel)) return;
        rt_prepared::KTimer &k = p->kt[kt_index(kernel)];
        if (k.a.empty()) {
            k.a.resize(KT_RING);
            k.b.resize(KT_RING);
            for (size_t i = 0; i < KT_RING; ++i)
                if (hipEventCreate(&k.a[i]) != hipSuccess || hipEventCreate(&k.b[i]) != hipSuccess) return;
        }
        if (k.n == KT_RING) kt_fold_oldest(k);
        if (hipEventRecord(k.a[k.head], st) != hipSuccess) return;
        t = &k;
    }
    ~KtScope() {
        if (!t) return;
        (void)hipEventRecord(t->b[t->head], st);
        t->head = (t->head + 1) % KT_RING;
        ++t->n;
    }
};

template <int ORDER, int PREC, bool GENPOW>
int launch_t(rt_prepared *p, int W, int H, int depth, int rb, int shard, int nshards, int row0, int row_end,
             void *out, uint8_t *levels, hipStream_t st, int levels_hit) {
    dim3 grid((W + TILE - 1) / TILE, (row_end - row0 + TILE - 1) / TILE);
    size_t lds = ORDER == RT_ORDER_EXACT ? (size_t)depth * BLOCK * 12 + (size_t)BLOCK * 24 : 0;
    KtScope kt(p, RT_KT_RENDER, st);
    // scenes without wave beams (few spheres, e.g. the reference's own scene) take the beam-free build
#define RT_K_RENDER(LV, NB)                                                                                            \
    hipLaunchKernelGGL((k_render<ORDER, PREC, LV, GENPOW, NB>), grid, dim3(BLOCK), lds, st, p->hdr, p->d_tab,        \
                       p->d_itab, W, H, depth, rb, shard, nshards, row0, row_end, out, levels, levels_hit)
    const bool nb = RT_FUSED_NB && !p->hdr.beam_ok;
    if (levels) {
        if (nb) RT_K_RENDER(true, true);
        else RT_K_RENDER(true, false);
    } else {
        if (nb) RT_K_RENDER(false, true);
        else RT_K_RENDER(false, false);
    }
#undef RT_K_RENDER
    HIPCHK(hipGetLastError());
    return RT_OK;
}

} // namespace

extern "C" {

#ifdef RT_STATS
// diagnostic builds only (not part of include/rt_mi355x.h)
int rt_debug_stats(unsigned long long *out, int n, int reset) {
    if (n > RT_NSTATS) n = RT_NSTATS;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), n * sizeof(unsigned long long)));
    if (reset) {
        unsigned long long z[RT_NSTATS] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof(z)));
    }
    return RT_OK;
}
#endif

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_selftest_math(int device, uint64_t n, uint64_t seed, uint64_t *mismatches) {
    if (!mismatches) return RT_EBADARG;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return RT_ENODEV;
    DevGuard g(device);
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, sizeof(*d)) != hipSuccess) return RT_ENOMEM;
    int rc = RT_OK;
    if (hipMemset(d, 0, sizeof(*d)) != hipSuccess) rc = RT_EHIP;
    if (rc == RT_OK) {
        hipLaunchKernelGGL(k_selftest_math, dim3(4096), dim3(256), 0, nullptr, (unsigned long long)n,
                           (unsigned long long)seed, d);
        unsigned long long h = 0;
        if (hipGetLastError() != hipSuccess || hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
            rc = RT_EHIP;
        *mismatches = h;
    }
    (void)hipFree(d);
    return rc;
}

const char *rt_strerror(int code) {
    switch (code) {
    case RT_OK: return "ok";
    case RT_DONE: return "done (width = height = 0)";
    case RT_EBADARG: return "bad argument (malformed scene or sizes)";
    case RT_ENODEV: return "no HIP device / device index out of range";
    case RT_EHIP: return "HIP runtime error";
    case RT_ENOMEM: return "out of memory";
    case RT_ETOOBIG: return "size exceeds a library limit";
    case RT_ERANGE: return "a colour outside the device P3 formatter's range (below -2^31 after scaling)";
    default: return "unknown error";
    }
}

int rt_device_count(int *count) {
    if (!count) return RT_EBADARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return n > 0 ? RT_OK : RT_ENODEV;
}

int rt_scene_check(const rt_elem *scene, uint32_t n) { return check_scene(scene, n); }

int rt_scene_canon(rt_elem *scene, uint32_t n) { return fill_canon(scene, n); }

uint32_t rt_shard_rows(uint32_t height, uint32_t row_block, uint32_t nshards) {
    if (row_block == 0 || nshards == 0) return 0;
    uint64_t span = (uint64_t)row_block * nshards;
    uint64_t blocks = (height + span - 1) / span;
    return (uint32_t)(blocks * row_block);
}

int rt_prepare(const rt_elem *scene, uint32_t n, int device, rt_prepared **out) {
    if (!out) return RT_EBADARG;
    *out = nullptr;
    Compiled c;
    int rc = compile_scene(scene, n, c);
    if (rc != RT_OK) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RT_ENODEV;
    DevGuard g(device);
    rt_prepared *p = new (std::nothrow) rt_prepared();
    if (!p) return RT_ENOMEM;
    p->device = device;
    p->hdr_full = c.hdr;
    apply_cull(p);
    if (hipMalloc(&p->d_tab, c.tab.size() * sizeof(double)) != hipSuccess) {
        delete p;
        return RT_ENOMEM;
    }
    if (hipMalloc(&p->d_itab, c.itab.size() * sizeof(int)) != hipSuccess) {
        (void)hipFree(p->d_tab);
        delete p;
        return RT_ENOMEM;
    }
    if (hipMemcpy(p->d_tab, c.tab.data(), c.tab.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_itab, c.itab.data(), c.itab.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(p->d_tab);
        (void)hipFree(p->d_itab);
        delete p;
        return RT_EHIP;
    }
    *out = p;
    return RT_OK;
}

} // extern "C"

int rt_prepare_scene(rt_prepared *p, const rt_elem *scene, uint32_t n) {
    if (!p) return RT_EBADARG;
    Compiled c;
    int rc = compile_scene(scene, n, c);
    if (rc != RT_OK) return rc;
    DevGuard g(p->device);
    double *tab = nullptr;
    int *itab = nullptr;
    if (hipMalloc(&tab, c.tab.size() * sizeof(double)) != hipSuccess) return RT_ENOMEM;
    if (hipMalloc(&itab, c.itab.size() * sizeof(int)) != hipSuccess) {
        (void)hipFree(tab);
        return RT_ENOMEM;
    }
    if (hipMemcpy(tab, c.tab.data(), c.tab.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(itab, c.itab.data(), c.itab.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(tab);
        (void)hipFree(itab);
        return RT_EHIP;
    }
    (void)hipFree(p->d_tab);
    (void)hipFree(p->d_itab);
    p->d_tab = tab;
    p->d_itab = itab;
    p->hdr_full = c.hdr;
    apply_cull(p);
    ++p->gen; // captured graphs hold the old tables
    ++p->scene_gen;
    p->last_valid = false;
    return RT_OK;
}

extern "C" {

int rt_update_scene(rt_prepared *p, const rt_elem *scene, uint32_t n_elems) {
    return rt_prepare_scene(p, scene, n_elems);
}

int rt_configure(rt_prepared *p, int option, int64_t value) {
    if (!p) return RT_EBADARG;
    switch (option) {
    case RT_CFG_SIDE_STREAMS:
        if (value < -1 || value > 1) return RT_EBADARG;
        p->side_mode = (int)value;
        return RT_OK;
    case RT_CFG_KERNEL_TIMING:
        if (value < 0 || value > 15) return RT_EBADARG;
        p->timing_mask = (int)value;
        return RT_OK;
    case RT_CFG_CULL:
        if (value < 0 || value > 1) return RT_EBADARG;
        p->cull = (int)value;
        apply_cull(p);
        ++p->gen; // captured graphs hold the old header
        ++p->scene_gen;
        p->last_valid = false;
        return RT_OK;
    default:
        return RT_EBADARG;
    }
}

} // extern "C"


extern "C" {

int rt_kernel_time(rt_prepared *p, int kernel, double *total_ms, uint64_t *launches, int reset) {
    const int i = p ? kt_index(kernel) : -1;
    if (i < 0) return RT_EBADARG;
    DevGuard g(p->device);
    rt_prepared::KTimer &t = p->kt[i];
    while (t.n) kt_fold_oldest(t);
    if (total_ms) *total_ms = t.sum_ms;
    if (launches) *launches = t.count;
    if (reset) {
        t.sum_ms = 0;
        t.count = 0;
    }
    return RT_OK;
}

int rt_release(rt_prepared *p) {
    if (!p) return RT_EBADARG;
    DevGuard g(p->device);
    (void)hipFree(p->d_tab);
    (void)hipFree(p->d_itab);
    if (p->d_queue) (void)hipFree(p->d_queue);
    if (p->d_colbuf) (void)hipFree(p->d_colbuf);
    if (p->d_child) (void)hipFree(p->d_child);
    if (p->d_lit) (void)hipFree(p->d_lit);
    if (p->d_sample) (void)hipFree(p->d_sample);
    if (p->d_counts) (void)hipFree(p->d_counts);
    if (p->d_items) (void)hipFree(p->d_items);
    if (p->d_pmask) (void)hipFree(p->d_pmask);
    for (hipEvent_t &e : p->ev_level)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t &e : p->ev_lit)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t &x : p->side)
        if (x) (void)hipStreamDestroy(x);
    if (p->gexec) (void)hipGraphExecDestroy(p->gexec);
    if (p->cap) (void)hipStreamDestroy(p->cap);
    for (auto &t : p->kt) {
        for (hipEvent_t e : t.a) (void)hipEventDestroy(e);
        for (hipEvent_t e : t.b) (void)hipEventDestroy(e);
    }
    delete p;
    return RT_OK;
}

} // extern "C"

// Free the wavefront work space of an idle context (rt_internal.h); the next launch regrows it.
size_t rt_trim(rt_prepared *p) {
    if (!p) return 0;
    DevGuard g(p->device);
    size_t freed = 0;
    auto drop = [&](void *&b, size_t &n) {
        if (b) (void)hipFree(b);
        b = nullptr;
        freed += n;
        n = 0;
    };
    drop(p->d_queue, p->queue_bytes);
    drop(reinterpret_cast<void *&>(p->d_colbuf), p->colbuf_bytes);
    drop(reinterpret_cast<void *&>(p->d_child), p->child_bytes);
    drop(reinterpret_cast<void *&>(p->d_lit), p->lit_bytes);
    drop(reinterpret_cast<void *&>(p->d_sample), p->sample_bytes);
    drop(reinterpret_cast<void *&>(p->d_counts), p->counts_bytes);
    drop(reinterpret_cast<void *&>(p->d_items), p->items_bytes);
    drop(reinterpret_cast<void *&>(p->d_pmask), p->pmask_bytes);
    p->pmask_valid = false;
    ++p->gen; // captured frame graphs hold the old pointers
    return freed;
}

namespace {

// Queue memory per pass is bounded (RT_QUEUE_MB, default 8 GiB); taller slabs are rendered
// in several row passes.
size_t queue_budget() {
    static size_t b = [] {
        const char *s = std::getenv("RT_QUEUE_MB");
        size_t mb = s ? std::strtoull(s, nullptr, 10) : 8192;
        return (mb < 64 ? 64 : mb) << 20;
    }();
    return b;
}

// Shading beside the reflection chain on the context's two side streams: per context
// (rt_configure RT_CFG_SIDE_STREAMS), else RT_LIT_STREAM=0 turns it off, for A/B runs.
bool lit_overlap(const rt_prepared *p) {
    static bool env_on = [] {
        const char *s = std::getenv("RT_LIT_STREAM");
        return !(s && std::strcmp(s, "0") == 0);
    }();
    return p->side_mode < 0 ? env_on : p->side_mode != 0;
}

// The side streams and one pair of level events per level 0 .. depth (created once, grown with the depth).
int side_stream(rt_prepared *p, int depth) {
    if (!p->side[0]) {
        int least = 0, greatest = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        for (hipStream_t &x : p->side) HIPCHK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, least));
    }
    while (p->ev_level.size() < (size_t)depth + 1) {
        hipEvent_t a = nullptr, b = nullptr;
        HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
        if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) {
            (void)hipEventDestroy(a);
            return RT_EHIP;
        }
        p->ev_level.push_back(a);
        p->ev_lit.push_back(b);
    }
    return RT_OK;
}

int grow(void **buf, size_t *have, size_t need, unsigned *gen) {
    if (*have >= need) return RT_OK;
    ++*gen;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    if (hipMalloc(buf, need) != hipSuccess) {
        *buf = nullptr;
        return RT_ENOMEM;
    }
    *have = need;
    return RT_OK;
}

// The slab rows of shard sh that lie inside the image (a prefix of the slab).
size_t valid_slab_rows(int H, int rb, int sh, int ns) {
    const size_t slab = rt_shard_rows((uint32_t)H, (uint32_t)rb, (uint32_t)ns);
    size_t v = 0;
    for (size_t blk = 0; blk * rb < slab; ++blk) {
        const long long base = ((long long)blk * ns + sh) * rb;
        v += (size_t)std::max(0LL, std::min((long long)rb, (long long)H - base));
    }
    return v;
}

// Does a wavefront pass write every pixel exactly once?  Yes with k_reflect_shade (the colours of
// records with a reflection hit are left to k_walk) and without reflections; no when k_light
// shades level 0 provisionally beside the chain (side streams, or levels requested).
bool wave_single_write(const rt_prepared *p, int D, bool levels) {
    const int nrefl = (p->hdr.n_light > 0 && D > 1) ? D - 1 : 0;
    const bool overlap = lit_overlap(p) && D > 1 && p->hdr.n_light > 0;
    return nrefl == 0 || (!overlap && !levels);
}

// acc (slab row 0, binary64, or null): supersampled passes fold their sample into it where each
// pixel is written (put_pixel) — only valid when wave_single_write holds.
template <int PREC, bool GENPOW>
int launch_wavefront(rt_prepared *p, int W, int H, int D, int rb, int sh, int ns, int row_begin, int row_end, void *out,
                     uint8_t *levels, hipStream_t st, int spp = 1, int sample = 0, unsigned long long seed = 0,
                     double *acc = nullptr, int levels_hit = 0) {
    // renders slab rows [row_begin, row_end) (row_begin a multiple of TILE); out / levels point at slab row 0.
    // levels_hit: k_primary writes the primary-hit mask (what it always writes: 1 on a hit, 0 on a
    // miss) and the later kernels do not count levels, so the fused path stays on
    uint8_t *const levels_primary = levels;
    if (levels_hit) levels = nullptr;
    const int slab_rows = row_end - row_begin;
    const int nlev = D > 0 ? D : 1;
    const size_t per_row = (size_t)W * nlev * sizeof(HitRec);
    int pass_rows = (int)std::min<size_t>((size_t)slab_rows, std::max<size_t>(TILE, queue_budget() / per_row));
    pass_rows = std::max(TILE, pass_rows / TILE * TILE);
    if (pass_rows > slab_rows) pass_rows = slab_rows;
    const int tiles_x = (W + TILE - 1) / TILE;
    const size_t max_tiles = (size_t)tiles_x * ((pass_rows + TILE - 1) / TILE);
    const size_t slots = max_tiles * TILE_SLOTS; // per level
    int rc = grow(&p->d_queue, &p->queue_bytes, slots * nlev * sizeof(HitRec), &p->gen);
    // colours of levels 1 .. depth-1, COL_W doubles per slot (level 0 goes straight to the
    // frame), and per level the has-a-child flags
    const size_t col_doubles = slots * COL_W * (size_t)std::max(1, nlev - 1);
    if (rc == RT_OK)
        rc = grow(reinterpret_cast<void **>(&p->d_colbuf), &p->colbuf_bytes, col_doubles * sizeof(double), &p->gen);
    if (rc == RT_OK) rc = grow(reinterpret_cast<void **>(&p->d_child), &p->child_bytes, slots * nlev, &p->gen);
    if (rc == RT_OK)
        rc = grow(reinterpret_cast<void **>(&p->d_lit), &p->lit_bytes, slots * nlev * sizeof(unsigned), &p->gen);
    if (rc == RT_OK)
        rc = grow(reinterpret_cast<void **>(&p->d_counts), &p->counts_bytes, max_tiles * nlev * sizeof(int), &p->gen);
    const bool overlap = lit_overlap(p) && D > 1 && p->hdr.n_light > 0;
    // dense work lists: 64 per-level record counts, then per level the slots of its records in tile order
    const size_t list0 = level_counts(nlev);
    const size_t items_ints = list0 + slots * nlev;
    if (rc == RT_OK)
        rc = grow(reinterpret_cast<void **>(&p->d_items), &p->items_bytes, items_ints * sizeof(int), &p->gen);
    if (rc == RT_OK && overlap) rc = side_stream(p, D);
    if (rc != RT_OK) return rc;
    // the primary rays' candidate masks of the whole slab (k_pmask), recomputed only when the
    // frame geometry or the scene changed (or after rt_trim)
    const unsigned long long *pmask = nullptr;
    if (p->hdr.beam_ok && D > 0) {
        const int slab_all = (int)rt_shard_rows(H, rb, ns);
        const size_t nhalf = (size_t)tiles_x * ((slab_all + TILE - 1) / TILE) * 2;
        const long long key[8] = {W, H, rb, sh, ns, spp > 1, (long long)p->scene_gen, slab_all};
        if (!(p->pmask_valid && std::memcmp(key, p->pmask_key, sizeof(key)) == 0)) {
            p->pmask_valid = false;
            // New masks (and perhaps a new buffer): a frame graph captured with the old ones holds
            // no k_pmask launch and would read these, so it is invalidated (gen).
            ++p->gen;
            if ((rc = grow(reinterpret_cast<void **>(&p->d_pmask), &p->pmask_bytes, nhalf * p->hdr.n_chunk * 8, &p->gen)) !=
                RT_OK)
                return rc;
            const dim3 pg((unsigned)std::min<size_t>(4096, (nhalf + 3) / 4));
            KtScope kt(p, RT_KT_PMASK, st);
            if (spp > 1)
                hipLaunchKernelGGL(k_pmask<true>, pg, dim3(256), 0, st, p->hdr, p->d_tab, p->d_itab, W, H, rb, sh, ns,
                                   slab_all, (int)nhalf, p->d_pmask);
            else
                hipLaunchKernelGGL(k_pmask<false>, pg, dim3(256), 0, st, p->hdr, p->d_tab, p->d_itab, W, H, rb, sh, ns,
                                   slab_all, (int)nhalf, p->d_pmask);
            HIPCHK(hipGetLastError());
            std::memcpy(p->pmask_key, key, sizeof(key));
            p->pmask_valid = true;
        }
        pmask = p->d_pmask;
    }
    // streams of the shading pass: level 0 (the bulk) beside the whole reflection chain, the
    // next levels each on their own, so no level waits for another's shading
    auto ls = [&](int k) { return overlap ? p->side[std::min(k, 1)] : st; };
    HitRec *q = static_cast<HitRec *>(p->d_queue);
    const int nrefl = (p->hdr.n_light > 0 && D > 1) ? D - 1 : 0;
    const int nshade = D > 0 ? 1 + nrefl : 0;
    // spheres only, culling on: every shadow target has occluder masks (lit_by<1>); their
    // per-lane-gathered tables staged in each workgroup's LDS when they fit (SPH = 2)
    const bool sph_only = p->hdr.n_tri == 0 && p->hdr.n_pl == 0 && p->hdr.cull_ok && p->hdr.occ_ok;
    const bool staged = sph_only && p->hdr.l_bytes > 0;
    const size_t lds = staged ? (size_t)p->hdr.l_bytes : 0;
    // Reflection kernels of levels that traverse the sphere BVH: after the staged tables in LDS,
    // the BVH nodes and sphere rows (when they fit BVH_LDS_MAX) and every lane's stack.
    SceneHdr rhdr = p->hdr;
    size_t lds_bvh = lds;
    if (rhdr.bvh_ok) {
        const size_t nb = (size_t)rhdr.n_bvh * BVH_NODE_DOUBLES * 8, sb = (size_t)rhdr.n_sph * SPH_W * 8;
        if (nb + sb <= (size_t)BVH_LDS_MAX) {
            rhdr.l_bvh = (int)lds_bvh;
            rhdr.l_bsph = (int)(lds_bvh + nb);
            lds_bvh += nb + sb;
        }
        rhdr.l_stack = (int)lds_bvh;
        lds_bvh += (size_t)BLOCK * rhdr.bvh_depth * sizeof(unsigned);
    }
    // (LDS-staged scenes keep the candidate walks: their tables and the BVH would not fit together)
    auto bvh_at = [&](int k) { return !staged && rhdr.bvh_ok && k >= rhdr.bvh_level; };
    auto lds_r = [&](int k) { return bvh_at(k) ? lds_bvh : lds; };
    // no side streams (frames in flight): each level's shading fused into the next reflection
    // pass (k_reflect_shade)
    const bool fuse = !overlap && !levels && nrefl > 0;
    // Inline walks (k_reflect_shade's iw, levels >= 1): every level is shaded by the launch that
    // reflects it; the chain of a shaded record without a child is walked by that launch, and the
    // deepest level's hits are shaded and walked by the launch that finds them (not queued) — what
    // k_walk did, minus its launch, the deepest level's k_items, the terminal records' colour entries
    // and their re-reads.  Needs the shadow answers in the records (<= 32 lights) and two reflection
    // levels or more (level 1's kernel, the dominant one, is left as is).  For S64 the dense
    // arrangement this implies measured the same as the sparse one (profiles/r05aa_ab_memset_dense.txt).
#ifndef RT_INLINE_WALK
#define RT_INLINE_WALK 1
#endif
    const bool iw = RT_INLINE_WALK && fuse && p->hdr.n_light <= 32 && nrefl >= 2;
    for (int row0 = row_begin; row0 < row_end; row0 += pass_rows) {
        const int rows = std::min(pass_rows, row_end - row0);
        const int ntiles = tiles_x * ((rows + TILE - 1) / TILE);
        // the pass covers slab rows [row0, row0 + rows): out/levels offset to row0; the
        // kernels map slab rows to image rows through the shard interleave themselves
        const size_t off = (size_t)row0 * W;
        void *o = static_cast<char *>(out) + off * 3 * (PREC == RT_OUT_F64 ? 8 : 4);
        uint8_t *lv = levels ? levels + off : nullptr;
        uint8_t *lv0 = levels_primary ? levels_primary + off : nullptr; // k_primary's
        double *acc_p = acc ? acc + off * 3 : nullptr;
        auto qk = [&](int k) { return q + (size_t)k * ntiles * TILE_SLOTS; };
        auto ck = [&](int k) { return p->d_counts + (size_t)k * ntiles; };
        int *nitems = p->d_items; // [0, 64): per-level record counts
        int *lists = p->d_items + list0;
        auto ik = [&](int k) { return lists + (size_t)k * ntiles * TILE_SLOTS; };
        auto colk = [&](int k) { return k > 0 ? p->d_colbuf + (size_t)(k - 1) * ntiles * TILE_SLOTS * COL_W : nullptr; };
        auto chk = [&](int k) { return p->d_child + (size_t)k * ntiles * TILE_SLOTS; };
        auto litk = [&](int k) { return p->d_lit + (size_t)k * ntiles * TILE_SLOTS; };
        const dim3 iblocks((ntiles + ITEMS_BLOCK - 1) / ITEMS_BLOCK);
        const PassGeom g{W, H, rb, sh, ns, row0, spp, sample, seed, acc_p}; // level-0 records are rebuilt from it
        const dim3 grid(std::min(ntiles, PRIMARY_GRID)); // k_primary: grid-stride loop over the tiles
        {
            KtScope kt(p, RT_KT_PRIMARY, st);
            if (lv0)
                hipLaunchKernelGGL((k_primary<PREC, true>), grid, dim3(PRIMARY_BLOCK), 0, st, p->hdr, p->d_tab, p->d_itab, W,
                                   H, D, rb, sh, ns, rows, row0, o, lv0, q, p->d_counts, ntiles, spp, sample, seed, acc_p,
                                   pmask, nitems);
            else
                hipLaunchKernelGGL((k_primary<PREC, false>), grid, dim3(PRIMARY_BLOCK), 0, st, p->hdr, p->d_tab, p->d_itab,
                                   W, H, D, rb, sh, ns, rows, row0, o, lv, q, p->d_counts, ntiles, spp, sample, seed, acc_p,
                                   pmask, nitems);
        }
        HIPCHK(hipGetLastError());
        const int sblocks = std::min<int>(STRIDE_BLOCKS, (ntiles * (TILE_SLOTS / 64) + BLOCK / 64 - 1) / (BLOCK / 64));
        const int sblocks1 = std::min<int>(STRIDE_BLOCKS_L1, (ntiles * (TILE_SLOTS / 64) + BLOCK / 64 - 1) / (BLOCK / 64));
        const int sblocksw = std::min<int>(STRIDE_BLOCKS_WALK, (ntiles * (TILE_SLOTS / 64) + BLOCK / 64 - 1) / (BLOCK / 64));
        const int sblocksb = std::min<int>(STRIDE_BLOCKS_BVH, (ntiles * (TILE_SLOTS / 64) + BLOCK / 64 - 1) / (BLOCK / 64));
        // level k's dense list, then its shading (k_light reads only level k: on a side stream
        // it starts as soon as the list exists and runs beside the next reflections)
        auto level_lists = [&](int k) -> int {
            // (inline walks: the deepest level is shaded by the launch that finds its hits, never queued)
            if (iw && k == nrefl) return RT_OK;
            hipLaunchKernelGGL(k_items, iblocks, dim3(ITEMS_BLOCK), 0, st, ck(k), ntiles, ik(k), nitems + k);
            HIPCHK(hipGetLastError());
            if (overlap) {
                HIPCHK(hipEventRecord(p->ev_level[k], st));
                HIPCHK(hipStreamWaitEvent(ls(k), p->ev_level[k], 0));
            }
            if (fuse && k < nrefl) return RT_OK; // shaded by k_reflect_shade(k + 1)
            if (k == nrefl && k >= 2) { // the deepest level >= 2: shaded by k_walk_deep / k_walk
                if (overlap) HIPCHK(hipEventRecord(p->ev_lit[k], ls(k)));
                return RT_OK;
            }
            // levels >= 2 are shaded here only when dense (decided on the device; otherwise the
            // launch exits at once): a smaller persistent grid keeps the empty launch cheap
            const int lblocks = k >= 2 ? std::min(sblocks, DEEP_LIGHT_BLOCKS) : sblocks;
            if (staged)
                hipLaunchKernelGGL((k_light<PREC, GENPOW, 2>), dim3(lblocks), dim3(BLOCK), lds, ls(k), p->hdr,
                                   p->d_tab, p->d_itab, k, o, qk(k), ik(k), nitems + k, colk(k), litk(k), g);
            else if (sph_only)
                hipLaunchKernelGGL((k_light<PREC, GENPOW, 1>), dim3(lblocks), dim3(BLOCK), 0, ls(k), p->hdr,
                                   p->d_tab, p->d_itab, k, o, qk(k), ik(k), nitems + k, colk(k), litk(k), g);
            else
                hipLaunchKernelGGL((k_light<PREC, GENPOW, 0>), dim3(lblocks), dim3(BLOCK), 0, ls(k), p->hdr,
                                   p->d_tab, p->d_itab, k, o, qk(k), ik(k), nitems + k, colk(k), litk(k), g);
            HIPCHK(hipGetLastError());
            if (overlap) HIPCHK(hipEventRecord(p->ev_lit[k], ls(k)));
            return RT_OK;
        };
        if (nshade > 0 && (rc = level_lists(0)) != RT_OK) return rc;
        for (int k = 1; k <= nrefl; ++k) {
            // level 1 (from the primary hits) is dense and throughput-bound; deeper levels are a few
            // waves each, bound by one wave's dependent chain: they walk two candidates per step
            KtScope kt(p, k == 1 ? RT_KT_LEVEL1 : 0, st);
            if (fuse) {
#define RT_RS_(SPHV, ILPV, LDSV, BVHV, LASTV)                                                                      \
    hipLaunchKernelGGL((k_reflect_shade<PREC, GENPOW, SPHV, ILPV, BVHV, LASTV>), dim3(k == 1 ? sblocks1 : BVHV ? sblocksb : sblocks), \
                       dim3(BLOCK), LDSV, st, rhdr,                                                                 \
                       p->d_tab, p->d_itab, k, o, qk(k - 1), ik(k - 1), nitems + (k - 1), qk(k), ck(k),                  \
                       iw ? nullptr : chk(k - 1), colk(k - 1), g, iw && k >= 2 ? (k == nrefl ? 2 : 1) : 0)
#define RT_RS(SPHV, ILPV, LDSV, BVHV)                                                                               \
    do {                                                                                                           \
        if (ILPV && iw && k == nrefl)                                                                              \
            RT_RS_(SPHV, ILPV, LDSV, BVHV, ILPV);                                                                  \
        else                                                                                                       \
            RT_RS_(SPHV, ILPV, LDSV, BVHV, false);                                                                 \
    } while (0)
                // levels traversing the sphere BVH (unstaged scenes only): the BVH instantiations
                const bool bvh_k = bvh_at(k);
                if (staged && k == 1) RT_RS(2, false, lds, false); // (staged: never the BVH, bvh_at)
                else if (staged) RT_RS(2, true, lds, false);
                else if (sph_only && bvh_k) RT_RS(1, true, lds_r(k), true);
                else if (sph_only && k == 1) RT_RS(1, false, lds, false);
                else if (sph_only) RT_RS(1, true, lds, false);
                else if (bvh_k) RT_RS(0, true, lds_r(k), true);
                else if (k == 1) RT_RS(0, false, lds, false);
                else RT_RS(0, true, lds, false);
#undef RT_RS
#undef RT_RS_
            } else if (lv && k == 1)
                hipLaunchKernelGGL((k_reflect<true, false>), dim3(sblocks), dim3(BLOCK), lds, st, rhdr, p->d_tab,
                                   p->d_itab, k, qk(k - 1), ik(k - 1), nitems + (k - 1), qk(k), ck(k), lv, chk(k - 1), g);
            else if (lv)
                hipLaunchKernelGGL((k_reflect<true, true>), dim3(sblocks), dim3(BLOCK), lds, st, rhdr, p->d_tab,
                                   p->d_itab, k, qk(k - 1), ik(k - 1), nitems + (k - 1), qk(k), ck(k), lv, chk(k - 1), g);
            else if (k == 1)
                hipLaunchKernelGGL((k_reflect<false, false>), dim3(sblocks), dim3(BLOCK), lds, st, rhdr, p->d_tab,
                                   p->d_itab, k, qk(k - 1), ik(k - 1), nitems + (k - 1), qk(k), ck(k), lv, chk(k - 1), g);
            else
                hipLaunchKernelGGL((k_reflect<false, true>), dim3(sblocks), dim3(BLOCK), lds, st, rhdr, p->d_tab,
                                   p->d_itab, k, qk(k - 1), ik(k - 1), nitems + (k - 1), qk(k), ck(k), lv, chk(k - 1), g);
            HIPCHK(hipGetLastError());
            if ((rc = level_lists(k)) != RT_OK) return rc;
        }
        // Without side streams one k_walk finishes every chain (sparse deep levels shaded on the
        // way).  With side streams (see deep_dense): k_walk_deep right after the chain; the chains
        // ending at level 1 (the bulk) are finished on side stream 0 as soon as levels 0 and 1 are
        // shaded, beside it; then the rest, once every level's shading is in (side stream 1
        // shades levels 1.. in order: its last level's event covers them all)
        if (nrefl > 0) {
            const size_t ls_ = (size_t)ntiles * TILE_SLOTS;
            const bool bits = p->hdr.n_light <= 32; // the shadow answers fit the record
            // deep: the merged walk (no k_walk_deep; without side streams); after k_reflect_shade
            // (fuse) the shadow answers are in the children's records (PAD)
            auto walk = [&](hipStream_t s_, int lo, int hi, bool deep) {
#define RT_WALK_K(SPHV, BITSV, DEEPV, PADV, LDSV)                                                                    \
    hipLaunchKernelGGL((k_walk<PREC, GENPOW, SPHV, BITSV, DEEPV, PADV>), dim3(sblocksw), dim3(BLOCK), LDSV, s_,      \
                       p->hdr, p->d_tab, p->d_itab, D, o, q, ls_, lists, nitems, p->d_colbuf, p->d_child,            \
                       p->d_lit, lo, hi, g)
#define RT_WALK(SPHV, BITSV, LDSV)                                                                                  \
    do {                                                                                                           \
        if (deep && fuse && BITSV)                                                                                 \
            RT_WALK_K(SPHV, BITSV, true, true, LDSV);                                                              \
        else if (deep)                                                                                             \
            RT_WALK_K(SPHV, BITSV, true, false, LDSV);                                                             \
        else                                                                                                       \
            RT_WALK_K(SPHV, BITSV, false, false, LDSV);                                                            \
    } while (0)
                if (staged && bits) RT_WALK(2, true, lds);
                else if (staged) RT_WALK(2, false, lds);
                else if (sph_only && bits) RT_WALK(1, true, 0);
                else if (sph_only) RT_WALK(1, false, 0);
                else if (bits) RT_WALK(0, true, 0);
                else RT_WALK(0, false, 0);
#undef RT_WALK
#undef RT_WALK_K
            };
            if (overlap) { // side stream 0 (after level 0's shading) waits for level 1's, and for
                           // k_reflect(2), which marks the level-1 records that have a child
                HIPCHK(hipStreamWaitEvent(p->side[0], p->ev_lit[1], 0));
                if (D > 2) HIPCHK(hipStreamWaitEvent(p->side[0], p->ev_level[2], 0));
                walk(p->side[0], 1, 2, false);
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(p->ev_lit[0], p->side[0]));
            }
            if (D > 2 && overlap) {
                if (staged)
                    hipLaunchKernelGGL((k_walk_deep<GENPOW, 2>), dim3(sblocks), dim3(BLOCK), lds, st, p->hdr,
                                       p->d_tab, p->d_itab, D, q, ls_, lists, nitems, p->d_child, colk(2));
                else if (sph_only)
                    hipLaunchKernelGGL((k_walk_deep<GENPOW, 1>), dim3(sblocks), dim3(BLOCK), 0, st, p->hdr,
                                       p->d_tab, p->d_itab, D, q, ls_, lists, nitems, p->d_child, colk(2));
                else
                    hipLaunchKernelGGL((k_walk_deep<GENPOW, 0>), dim3(sblocks), dim3(BLOCK), 0, st, p->hdr,
                                       p->d_tab, p->d_itab, D, q, ls_, lists, nitems, p->d_child, colk(2));
                HIPCHK(hipGetLastError());
            }
            if (overlap) {
                HIPCHK(hipStreamWaitEvent(st, p->ev_lit[nrefl], 0));
                HIPCHK(hipStreamWaitEvent(st, p->ev_lit[0], 0));
                if (D > 2) walk(st, 2, D, false);
            } else if (!iw) {
                walk(st, 1, D, true); // every chain in one launch, sparse deep levels shaded there too
            }
            HIPCHK(hipGetLastError());
        } else if (overlap && nshade > 0) {
            HIPCHK(hipStreamWaitEvent(st, p->ev_lit[0], 0));
        }
    }
    return RT_OK;
}

// RT_GRAPH=1 enables frame graphs.  Off by default: measured on MI355X (ROCm 7), replaying
// the captured frame ran its kernels slower than direct launches (S64 4096^2: 1.35 vs 0.94
// ms), the side stream's low priority does not survive capture.
bool graphs_on() {
    static bool on = [] {
        const char *s = std::getenv("RT_GRAPH");
        return s && std::strcmp(s, "1") == 0;
    }();
    return on;
}

// Run enqueue(stream) for a frame: directly, or through the cached graph of identical frames.
template <typename F>
int launch_frame(rt_prepared *p, const long long (&args)[12], hipStream_t st, F &&enqueue) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (!graphs_on() || hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
        return enqueue(st); // the caller is capturing (or graphs are off): plain launches
    long long key[12];
    std::memcpy(key, args, sizeof(key));
    key[11] = (long long)p->gen; // a reallocated work space invalidates captured pointers
    auto same = [&](const long long (&a)[12]) { return std::memcmp(a, key, sizeof(key)) == 0; };
    if (p->gexec && same(p->gkey)) {
        HIPCHK(hipGraphLaunch(p->gexec, st));
        return RT_OK;
    }
    if (!(p->last_valid && same(p->last_key))) { // first time with these arguments: run directly
        const int rc = enqueue(st);
        std::memcpy(p->last_key, key, sizeof(key));
        p->last_key[11] = (long long)p->gen;
        p->last_valid = rc == RT_OK;
        return rc;
    }
    // second identical frame (work space already sized): capture it on an internal stream
    if (!p->cap) HIPCHK(hipStreamCreateWithFlags(&p->cap, hipStreamNonBlocking));
    HIPCHK(hipStreamBeginCapture(p->cap, hipStreamCaptureModeRelaxed));
    const int rc = enqueue(p->cap);
    hipGraph_t gr = nullptr;
    const hipError_t e = hipStreamEndCapture(p->cap, &gr);
    if (rc == RT_OK && e == hipSuccess && (long long)p->gen != key[11]) {
        // the work space or the primary masks changed while capturing: no device work was run —
        // drop the graph and render this frame directly.  The host state the capture changed is
        // reset first: primary masks computed during the capture were never written (their k_pmask
        // launch is in the dropped graph), so the direct run must compute them again.
        (void)hipGraphDestroy(gr);
        p->last_valid = false;
        p->pmask_valid = false;
        return enqueue(st);
    }
    if (rc != RT_OK || e != hipSuccess) {
        if (gr) (void)hipGraphDestroy(gr);
        p->last_valid = false;
        return rc != RT_OK ? rc : RT_EHIP;
    }
    if (p->gexec) (void)hipGraphExecDestroy(p->gexec);
    p->gexec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&p->gexec, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (ei != hipSuccess) {
        p->gexec = nullptr;
        return RT_EHIP;
    }
    std::memcpy(p->gkey, key, sizeof(key));
    HIPCHK(hipGraphLaunch(p->gexec, st));
    return RT_OK;
}

// Engine.  Small mixed scenes are bound by per-level latency (every level of the wavefront
// pipeline costs its kernels' fixed ramp-up) and run fastest as the single fused kernel
// (default scene 1920x1080 d5: 15.1 vs 6.1 Gpx/s); larger ones by the scans, where the wavefront
// pipeline's coherent waves and overlap win (round 1, 4096^2 d5: wavefront ahead from 48
// objects), and spheres-only scenes with LDS-staged tables at any size (below).
// RT_ENGINE=fused | wave forces one.
constexpr int FUSED_MAX_OBJECTS = 40;
// The fused kernel's reference-order chain keeps each level's (t, object) per pixel in LDS (12 bytes
// per level and pixel): deeper frames in reference order take the wavefront engine, whose per-level
// queues are sized at run time (rt_render.hip launch_wavefront).
constexpr int FUSED_MAX_DEPTH = 16;
bool use_mega_engine(const rt_prepared *p, int depth = 0, int order = RT_ORDER_EXACT) {
    if (order == RT_ORDER_EXACT && depth > FUSED_MAX_DEPTH) return false;
    static const int mode = [] { // 0 auto, 1 fused, 2 wave
        const char *s = std::getenv("RT_ENGINE");
        if (s && (std::strcmp(s, "fused") == 0 || std::strcmp(s, "mega") == 0)) return 1;
        if (s && std::strcmp(s, "wave") == 0) return 2;
        return 0;
    }();
    if (mode) return mode == 1;
    // spheres-only scenes whose tables are staged in LDS: the wavefront engine at every size
    // (measured round 2, 4096^2 d5, 4 frames in flight: S4 115 vs 89 Gpx/s, S8 86 vs 70,
    // S16 58 vs 42, S24 49 vs 37, S32 52 vs 38).  Decided from the compiled header, not the one
    // RT_CFG_CULL = 0 strips, so the brute-force mode runs the production engine.
    const SceneHdr &h = p->hdr_full;
    if (h.n_tri == 0 && h.n_pl == 0 && h.cull_ok && h.l_bytes > 0) return false;
    return h.n_obj <= FUSED_MAX_OBJECTS;
}

} // namespace

extern "C" {

int rt_engine(rt_prepared *p, uint32_t spp) {
    if (!p || spp == 0) return RT_EBADARG;
    return (spp == 1 && use_mega_engine(p)) ? RT_ENGINE_FUSED : RT_ENGINE_WAVE;
}

int rt_launch(rt_prepared *p, uint32_t width, uint32_t height, uint32_t depth, uint32_t row_block, uint32_t shard,
              uint32_t nshards, int precision, int order, void *d_out, uint8_t *d_levels, void *stream) {
    return rt_launch_spp(p, width, height, depth, row_block, shard, nshards, precision, order, 1, 0, d_out, d_levels,
                         stream);
}

int rt_launch_spp(rt_prepared *p, uint32_t width, uint32_t height, uint32_t depth, uint32_t row_block,
                  uint32_t shard, uint32_t nshards, int precision, int order, uint32_t spp, uint64_t seed,
                  void *d_out, uint8_t *d_levels, void *stream) {
    return rt_launch_rows(p, width, height, depth, row_block, shard, nshards, precision, order, spp, seed, 0, ~0u,
                          d_out, d_levels, stream, 0);
}

} // extern "C"

// rt_launch_spp restricted to slab rows [row_begin, min(row_end, slab rows)): the boundary
// (rt_host.hip) renders a frame in row bands so that each band's copy to the host overlaps
// the next band's render.  row_begin must be a multiple of 16 (the tile height).
int rt_launch_rows(rt_prepared *p, uint32_t width, uint32_t height, uint32_t depth, uint32_t row_block,
                   uint32_t shard, uint32_t nshards, int precision, int order, uint32_t spp, uint64_t seed,
                   uint32_t row_begin, uint32_t row_end, void *d_out, uint8_t *d_levels, void *stream, int levels_hit) {
    if (!p || !d_out) return RT_EBADARG;
    if (width == 0 && height == 0) return RT_DONE;
    if (width == 0 || height == 0) return RT_EBADARG;
    if (row_block == 0 || nshards == 0 || shard >= nshards) return RT_EBADARG;
    if (precision != RT_OUT_F64 && precision != RT_OUT_F32) return RT_EBADARG;
    if (order != RT_ORDER_EXACT && order != RT_ORDER_FAST) return RT_EBADARG;
    if (spp == 0) return RT_EBADARG;
    if (spp > RT_MAX_SPP) return RT_ETOOBIG;
    if (width > (1u << 20) || height > (1u << 20)) return RT_ETOOBIG;
    uint32_t slab = rt_shard_rows(height, row_block, nshards);
    if ((uint64_t)slab > 65535ull * TILE) return RT_ETOOBIG;
    if (row_begin % TILE) return RT_EBADARG;
    if (row_end > slab) row_end = slab;
    if (row_begin >= row_end) return RT_OK;
    DevGuard g(p->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int W = (int)width, H = (int)height, D = (int)depth, rb = (int)row_block, sh = (int)shard, ns = (int)nshards;
    const int r0 = (int)row_begin, r1 = (int)row_end, slab_rows = (int)slab;
    if (spp > 1) { // RT_SUPERSAMPLING, on the wavefront engine: one pass per sample, summed in order
        // the slab rows inside the image (a prefix: global rows grow with slab rows)
        const size_t valid_rows = valid_slab_rows(H, rb, sh, ns);
        const size_t v1 = std::min<size_t>(valid_rows, (size_t)r1);
        if (v1 <= (size_t)r0) return RT_OK;
        const size_t e0 = (size_t)r0 * W * 3, n = (v1 - r0) * W * 3; // the band's elements
        const size_t n_slab = (size_t)slab_rows * W * 3;
        int rc = grow(reinterpret_cast<void **>(&p->d_sample), &p->sample_bytes, 2 * n_slab * sizeof(double), &p->gen);
        if (rc != RT_OK) return rc;
        double *smp = p->d_sample, *acc = p->d_sample + n_slab;
        const int blocks = (int)std::min<size_t>(8192, (n + 255) / 256);
        void *dst = static_cast<char *>(d_out) + e0 * (precision == RT_OUT_F64 ? 8 : 4);
        for (int s = 0; s < (int)spp; ++s) {
            uint8_t *lv = s == 0 ? d_levels : nullptr;
            if (wave_single_write(p, D, lv != nullptr && !levels_hit)) {
                // every pixel written once: the pass folds its sample into acc (and the last one
                // writes the output) itself — no sample slab, no k_accum
#define RT_SS(P) (p->hdr.int_pow ? launch_wavefront<P, false>(p, W, H, D, rb, sh, ns, r0, r1, d_out, lv, st, (int)spp, s, seed, acc, levels_hit) \
                                 : launch_wavefront<P, true>(p, W, H, D, rb, sh, ns, r0, r1, d_out, lv, st, (int)spp, s, seed, acc, levels_hit))
                rc = precision == RT_OUT_F64 ? RT_SS(RT_OUT_F64) : RT_SS(RT_OUT_F32);
#undef RT_SS
                if (rc != RT_OK) return rc;
                continue;
            }
            rc = p->hdr.int_pow ? launch_wavefront<RT_OUT_F64, false>(p, W, H, D, rb, sh, ns, r0, r1, smp, lv, st,
                                                                      (int)spp, s, seed, nullptr, levels_hit)
                                : launch_wavefront<RT_OUT_F64, true>(p, W, H, D, rb, sh, ns, r0, r1, smp, lv, st,
                                                                     (int)spp, s, seed, nullptr, levels_hit);
            if (rc != RT_OK) return rc;
            if (precision == RT_OUT_F64)
                hipLaunchKernelGGL(k_accum<RT_OUT_F64>, dim3(blocks), dim3(256), 0, st, n, smp + e0, acc + e0, dst, s,
                                   (int)spp);
            else
                hipLaunchKernelGGL(k_accum<RT_OUT_F32>, dim3(blocks), dim3(256), 0, st, n, smp + e0, acc + e0, dst, s,
                                   (int)spp);
            HIPCHK(hipGetLastError());
        }
        return RT_OK;
    }
    if (!use_mega_engine(p, D, order)) { // the wavefront engine always evaluates the reference's exact order
        const long long key[12] = {W, H, D, rb, sh, ns, precision, ((long long)r0 << 32) | r1,
                                   (long long)(intptr_t)d_out, (long long)(intptr_t)d_levels, levels_hit, 0};
        return launch_frame(p, key, st, [&](hipStream_t s) {
            if (precision == RT_OUT_F64)
                return p->hdr.int_pow
                           ? launch_wavefront<RT_OUT_F64, false>(p, W, H, D, rb, sh, ns, r0, r1, d_out, d_levels, s, 1, 0, 0,
                                                                 nullptr, levels_hit)
                           : launch_wavefront<RT_OUT_F64, true>(p, W, H, D, rb, sh, ns, r0, r1, d_out, d_levels, s, 1, 0, 0,
                                                                nullptr, levels_hit);
            return p->hdr.int_pow
                       ? launch_wavefront<RT_OUT_F32, false>(p, W, H, D, rb, sh, ns, r0, r1, d_out, d_levels, s, 1, 0, 0,
                                                             nullptr, levels_hit)
                       : launch_wavefront<RT_OUT_F32, true>(p, W, H, D, rb, sh, ns, r0, r1, d_out, d_levels, s, 1, 0, 0,
                                                            nullptr, levels_hit);
        });
    }
#define RT_DISPATCH(O, P)                                                                                          \
    return p->hdr.int_pow ? launch_t<O, P, false>(p, W, H, D, rb, sh, ns, r0, r1, d_out, d_levels, st, levels_hit)  \
                          : launch_t<O, P, true>(p, W, H, D, rb, sh, ns, r0, r1, d_out, d_levels, st, levels_hit)
    if (order == RT_ORDER_EXACT) {
        if (precision == RT_OUT_F64) RT_DISPATCH(RT_ORDER_EXACT, RT_OUT_F64);
        RT_DISPATCH(RT_ORDER_EXACT, RT_OUT_F32);
    }
    if (precision == RT_OUT_F64) RT_DISPATCH(RT_ORDER_FAST, RT_OUT_F64);
    RT_DISPATCH(RT_ORDER_FAST, RT_OUT_F32);
#undef RT_DISPATCH
}

extern "C" {

// Copy the blocks of one shard's slab to their rows in a row-major image.  dst_kind selects
// hipMemcpyDeviceToDevice or DeviceToHost.
static int scatter_slab(const char *slab, uint32_t rowbytes, uint32_t H, uint32_t rb, uint32_t shard,
                        uint32_t nshards, char *image, hipMemcpyKind kind, hipStream_t st) {
    uint64_t blk_bytes = (uint64_t)rb * rowbytes;
    uint32_t nfull = 0;
    while ((((uint64_t)nfull * nshards + shard) * rb + rb) <= H) nfull++;
    if (nfull)
        HIPCHK(hipMemcpy2DAsync(image + (uint64_t)shard * blk_bytes, (size_t)blk_bytes * nshards, slab,
                                (size_t)blk_bytes, (size_t)blk_bytes, nfull, kind, st));
    uint64_t g0 = ((uint64_t)nfull * nshards + shard) * rb;
    if (g0 < H) { // one partial block at the bottom of the image
        uint64_t rows = H - g0;
        HIPCHK(hipMemcpyAsync(image + g0 * rowbytes, slab + (uint64_t)nfull * blk_bytes, rows * rowbytes, kind, st));
    }
    return RT_OK;
}

int rt_unshard(const void *d_slabs, uint32_t width, uint32_t height, uint32_t row_block, uint32_t nshards,
               int precision, void *d_image, void *stream) {
    if (!d_slabs || !d_image || width == 0 || height == 0 || row_block == 0 || nshards == 0) return RT_EBADARG;
    if (precision != RT_OUT_F64 && precision != RT_OUT_F32) return RT_EBADARG;
    uint32_t rowbytes = width * 3 * (precision == RT_OUT_F64 ? 8 : 4);
    uint64_t slab_bytes = (uint64_t)rt_shard_rows(height, row_block, nshards) * rowbytes;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    for (uint32_t s = 0; s < nshards; s++) {
        int rc = scatter_slab(static_cast<const char *>(d_slabs) + s * slab_bytes, rowbytes, height, row_block, s,
                              nshards, static_cast<char *>(d_image), hipMemcpyDeviceToDevice, st);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}

} // extern "C"
