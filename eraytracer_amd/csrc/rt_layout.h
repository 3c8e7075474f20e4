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

// int-table record widths (ints)
constexpr int OBJ_META_W = 4; // kind, local index within its type, canon compact id, pad

enum ObjKind : int { K_SPHERE = 0, K_TRIANGLE = 1, K_PLANE = 2 };

// Scalar header passed to the kernel by value.  All offsets index the double table `tab`
// or the int table `itab` (both device allocations owned by an rt_prepared).
struct SceneHdr {
    int n_sph, n_tri, n_pl, n_obj, n_light, n_org; // n_org = 1 + n_light
    // offsets into tab
    int o_sph, o_sph_org, o_tri, o_tri_org, o_pl, o_pl_org, o_obj, o_light;
    // offsets into itab
    int i_sph_id, i_tri_id, i_pl_id, i_obj_meta;
    // camera (point_on_screen/3, :486-503, with focal_length/2 :483-484 folded in)
    double cam_x, cam_y, cam_z; // Camera#camera.location
    double sx;   // 0*F + Lx            (first fold step, x)
    double sy;   // 0 + (0*F + Ly)      (first two fold steps, y)
    double dz;   // (0 + (0 + (1*F + Lz))) - Lz : z of Through - From
    double screen_w, screen_h;
    double n_light_d; // number of lights as a double (ORDER_FAST weight)
};

} // namespace rtl
