// rt_layout.h — the "compiled scene": how a reference scene list (raytracer.erl:618-665)
// lives in HBM for the render kernel.  Shared by the host scene compiler (rt_scene.cpp)
// and the kernel (rt_render.hip).
//
// The reference scans the scene list in order, dispatching on the record tag of every
// element (nearest_object_intersecting_ray/6, raytracer.erl:303-346; ray_object_intersect/2,
// :349-359).  Here objects are grouped by type so each type is a wave-uniform loop with no
// dispatch; the original list position survives as the compact object id (ids follow list
// order), and ties are broken by (t, id) lexicographically — which is exactly "keep the
// earlier object unless strictly nearer" (:319).
//
// Everything that depends only on the scene and a FIXED ray origin is precomputed on the
// host with the reference's own operation order (so the bits are identical): primary rays
// start at the camera, shadow rays at a light (shadow_factor/4, :259), so their
// per-object origin terms (sphere o-c and C, triangle T and Q, plane V0) are tabled per
// origin.  Origin slot 0 = camera, slot 1+i = point light i.
#pragma once
#include <stdint.h>

namespace rtl {

// double-table record widths (doubles)
constexpr int SPH_W = 4;     // cx cy cz r2                    (r2 = Radius*Radius, :374)
constexpr int SPH_ORG_W = 4; // ocx ocy ocz C  for one origin  (X0-Xc ..., C, :373-374)
constexpr int TRI_W = 12;    // v1(3) e1(3) e2(3) pad(3)       (Edge1, Edge2, :406-407)
constexpr int TRI_ORG_W = 8; // T(3) Q(3) pad(2)               (T = O - v1, Q = T x Edge1, :422, :431)
constexpr int PL_W = 4;      // nx ny nz distance
constexpr int PL_ORG_W = 1;  // V0 = -(N.O + distance)          (:465-466)
constexpr int OBJ_W = 12;    // n(3) or centre(3), colour(3), specular_power, shininess, reflectivity, pad
constexpr int LIGHT_W = 12;  // diffuse(3), location(3), specular(3), pad(3)
// wave culling (see rt_render.hip, "Beam culling"): sphere bounds and, per tabled origin, the
// sphere's direction cone as seen from that origin with conservative margins applied
constexpr int SPH_B_W = 4;   // cx cy cz r
constexpr int SPH_OB_W = 8;  // vx vy vz (= c - o), |v|, sin(rho) upper bound, cos(rho) lower bound, near(0/1),
                             // lower bound of |v| - r (no ray from o reaches the sphere before that distance)

constexpr int SPH_OB32_W = 8; // floats
constexpr float BEAM32_EPS = 1.0e-5f; // binary32 beams' margin (rt_render.hip, "Binary32 beams")

// Culling is exact only while every binary64 rounding error in the reference's sphere test is
// far below its 0.001 discriminant threshold: all scene coordinates within this bound.
constexpr double CULL_EXTENT = 1.0e4;
constexpr double CULL_EPS = 1.0e-9; // angular / relative safety margin of the cull tests
constexpr int BEAM_MIN_SPHERES = 8;  // fewer spheres: scans test every sphere (no wave beams)

// int-table record widths (ints)
constexpr int OBJ_META_W = 4; // kind, local index within its type, canon compact id, canon's local index

// Shadow rays from a light into the cone around a target sphere are split into OCC_CELLS
// direction cells (occ_cell); each cell has its own, smaller, occluder mask.
#ifndef RT_OCC_CELLS
#define RT_OCC_CELLS 16 // 4: signs only; 1: one mask per (light, target), as before the cells
#endif
constexpr int OCC_CELLS = RT_OCC_CELLS;
constexpr float OCC_CELL_EPS = 1.0e-4f; // cells overlap by this much (unit-vector components)
constexpr int OCC_CELLS_MIN_SPHERES = 128; // smaller scenes keep one cell
// Occluder masks cost the host one test per (light, target, sphere) triple: above this many the
// scene has none (SceneHdr::occ_ok = 0; shadow cones instead).  Above OCC_MAX_BYTES of masks,
// one cell.
constexpr double OCC_MAX_TESTS = 16777216.0; // 2^24: S2048 with 4 lights (~1.3 s of host time)
constexpr double OCC_MAX_BYTES = 64.0 * 1024 * 1024;

constexpr int LDS_STAGE_MAX = 32 * 1024; // 5 workgroups per CU keep their 32 KiB each

// Sphere BVH for incoherent reflection rays (see rt_render.hip, "Per-lane BVH"): a binary tree
// over the spheres, built on the host by SAH splits (depth <= ceil(log2 n_sph) + 2); one 64-byte
// node holds both children's binary32 boxes (rounded outwards and inflated, so the box test
// never rejects a sphere the binary64 test accepts), their links (>= 0: node, < 0: ~sphere) and,
// for a sphere child, the sphere's compact object id.
constexpr int BVH_NODE_DOUBLES = 8;  // 64 bytes
constexpr int BVH_LDS_MAX = 40 * 1024; // nodes + sphere rows staged in LDS up to this size
constexpr int BVH_STACK = 18;        // per-lane traversal stack entries (tree depth <= BVH_STACK)
constexpr int BVH_MAX_SPHERES = 1 << 16; // the stack words hold 16-bit node links: more spheres, no BVH
constexpr int BVH_MIN_SPHERES = 128; // below this the wave beams are cheaper (default; RT_BVH_MIN)
constexpr int BVH_LEVEL = 2;         // first reflection level traversing the BVH (default; RT_BVH_LEVEL)
constexpr int BVH_SAH_SLACK = 2;     // SAH trees may be this much deeper than ceil(log2 n_sph) (compile-time)
constexpr double BVH_BOX_REL = 1.0e-5; // box inflation, relative to the scene extent (+1)

enum ObjKind : int { K_SPHERE = 0, K_TRIANGLE = 1, K_PLANE = 2 };

// Scalar header passed to the kernel by value.  All offsets index the double table `tab`
// or the int table `itab` (both device allocations owned by an rt_prepared).
struct SceneHdr {
    int n_sph, n_tri, n_pl, n_obj, n_light, n_org; // n_org = 1 + n_light
    int cull_ok;                                   // scene within CULL_EXTENT: culling allowed (occluder masks)
    int beam_ok;                                   // cull_ok and enough spheres that wave beams pay
    int int_pow;                                   // every specular power is an integer in [0, 1024]
    // offsets into tab
    int o_sph, o_sph_org, o_tri, o_tri_org, o_pl, o_pl_org, o_obj, o_light, o_sph_b, o_sph_ob;
    // binary32 copy of the per-origin cone rows for the binary32 beams (SPH_OB32_W floats per row:
    // v (3), |v|, sin(rho) and cos(rho) bounds with BEAM32 margins, near, |v| - r lower bound)
    int o_sph_ob32;
    // offsets into itab
    int i_sph_id, i_tri_id, i_pl_id, i_obj_meta;
    // Occluder masks (only when cull_ok): for light i, target sphere t, direction cell e
    // (occ_cell; occ_cells of them: OCC_CELLS for scenes whose tables stay in L2, 1 for scenes
    // staged in LDS) and 64-sphere chunk k, the uint64 at
    // itab[i_occ + 2*(((i*n_sph + t)*occ_cells + e)*n_chunk + k)] has bit j set iff sphere 64k+j
    // can block a shadow ray from light i into cell e of the cone towards sphere t (rt_scene.cpp).
    int i_occ, n_chunk, occ_cells;
    int occ_ok; // the occluder masks exist (cull_ok, spheres, and within OCC_MAX_TESTS)
    // LDS staging (spheres-only scenes with culling whose per-lane-gathered tables fit
    // LDS_STAGE_MAX bytes; l_bytes = 0 otherwise): byte offsets in the workgroup's dynamic LDS of
    // the object rows (o_obj), object meta rows (i_obj_meta), the lights' per-origin sphere rows
    // (o_sph_org from origin 1 on), the occluder masks (i_occ), the sphere ids (i_sph_id) and
    // the sphere bounds of the reflection rays' beam culling (o_sph_b).
    int l_obj, l_meta, l_org, l_occ, l_id, l_sphb, l_bytes;
    // sphere BVH (bvh_ok: built and within its limits): nodes at tab[o_bvh], n_bvh of them, depth
    // bvh_depth; the reflection scans of levels >= bvh_level traverse it per lane (the wave beams
    // below that level).  Set per launch (the reflection kernels' dynamic LDS): byte offsets of the
    // nodes and the sphere rows (o_sph) staged there (l_bvh = -1: read from HBM) and of each
    // lane's stack (l_stack).
    int bvh_ok, o_bvh, n_bvh, bvh_level, bvh_depth, l_bvh, l_bsph, l_stack;
    // Range checks of normalize3 (rt_render.hip) proven unnecessary on the host for this scene:
    // norm_ok — spheres only, within CULL_EXTENT, every |radius| >= 1e-50 and every light off every
    // sphere's surface (| |L - c| - |r| | > 1e-9 (ext + 1)): the surface normals (hit - c) and the
    // light directions (L - hit) have squared lengths inside [2^-400, 2^400]; prim_ok — the same
    // for the primary rays' (Through - From) vectors.
    int norm_ok, prim_ok;
    // camera (point_on_screen/3, :486-503, with focal_length/2 :483-484 folded in)
    double cam_x, cam_y, cam_z; // Camera#camera.location
    double sx;   // 0*F + Lx            (first fold step, x)
    double sy;   // 0 + (0*F + Ly)      (first two fold steps, y)
    double dz;   // (0 + (0 + (1*F + Lz))) - Lz : z of Through - From
    double screen_w, screen_h;
    double n_light_d; // number of lights as a double (ORDER_FAST weight)
    double ext;       // largest |coordinate| (+ radius) of the origins and spheres (binary32 culling margins)
};

} // namespace rtl
