// rt_scene.cpp — host-side scene compiler: validates an rt_elem list (the marshalled
// reference scene, raytracer.erl:618-665) and lays it out for the kernel (rt_layout.h).
//
// Every precomputed quantity is produced with the reference's operation order, in IEEE
// binary64, compiled with -ffp-contract=off, so the kernel sees bit-identical values to
// those the reference computes per ray.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_layout.h"
#include "rt_scene.h"

namespace rtl {

static bool finite3(const rt_vec3 &v) { return std::isfinite(v.x) && std::isfinite(v.y) && std::isfinite(v.z); }
static bool finite_mat(const rt_material &m) {
    return finite3(m.colour) && std::isfinite(m.specular_power) && std::isfinite(m.shininess) &&
           std::isfinite(m.reflectivity);
}

static bool elem_ok(const rt_elem &e) {
    switch (e.kind) {
    case RT_CAMERA:
        return finite3(e.u.camera.location) && finite3(e.u.camera.rotation) && std::isfinite(e.u.camera.fov) &&
               std::isfinite(e.u.camera.screen_width) && std::isfinite(e.u.camera.screen_height);
    case RT_POINT_LIGHT:
        return finite3(e.u.point_light.diffuse_colour) && finite3(e.u.point_light.location) &&
               finite3(e.u.point_light.specular_colour);
    case RT_SPHERE:
        return std::isfinite(e.u.sphere.radius) && finite3(e.u.sphere.center) && finite_mat(e.u.sphere.material);
    case RT_TRIANGLE:
        return finite3(e.u.triangle.v1) && finite3(e.u.triangle.v2) && finite3(e.u.triangle.v3) &&
               finite_mat(e.u.triangle.material);
    case RT_PLANE:
        return finite3(e.u.plane.normal) && std::isfinite(e.u.plane.distance) && finite_mat(e.u.plane.material);
    case RT_OTHER:
        return true;
    default:
        return false;
    }
}

static size_t payload_bytes(int kind) {
    switch (kind) {
    case RT_CAMERA: return sizeof(((rt_elem *)0)->u.camera);
    case RT_POINT_LIGHT: return sizeof(((rt_elem *)0)->u.point_light);
    case RT_SPHERE: return sizeof(((rt_elem *)0)->u.sphere);
    case RT_TRIANGLE: return sizeof(((rt_elem *)0)->u.triangle);
    case RT_PLANE: return sizeof(((rt_elem *)0)->u.plane);
    default: return 0;
    }
}

// No count limits: the reference's scans take any list (nearest_object_intersecting_ray/6,
// raytracer.erl:300-346; lighting_function/6 folds over every light, :209-252).  What does not
// fit the device (or the 32-bit table offsets) fails with RT_ENOMEM in compile_scene.
int check_scene(const rt_elem *e, uint32_t n) {
    if (!e || n < 1) return RT_EBADARG;         // [Camera|Rest] must match (raytracer.erl:180)
    if (e[0].kind != RT_CAMERA) return RT_EBADARG; // Camera#camera.location would crash (:488)
    if (n > (uint32_t)INT32_MAX / 2) return RT_ENOMEM; // object ids are 32-bit ints in the kernels
    for (uint32_t i = 0; i < n; i++) {
        if (!elem_ok(e[i])) return RT_EBADARG;
        if (e[i].canon < -1 || e[i].canon > (int32_t)i) return RT_EBADARG;
        if (e[i].canon >= 0 && e[e[i].canon].kind != e[i].kind) return RT_EBADARG;
    }
    return RT_OK;
}

// canon[i] = the first j <= i of the same kind that is its own canonical element and has the same
// payload bytes.  One hash lookup per element (the elements so far that are their own canonical
// element, keyed by kind and payload; the first one of each key kept), not a scan of the prefix.
int fill_canon(rt_elem *e, uint32_t n) {
    if (!e) return RT_EBADARG;
    struct Key {
        const rt_elem *p;
        size_t nb;
    };
    auto hash = [](const rt_elem *p, size_t nb) {
        uint64_t h = 1469598103934665603ull ^ (uint64_t)(uint32_t)p->kind;
        const unsigned char *b = reinterpret_cast<const unsigned char *>(&p->u);
        for (size_t k = 0; k < nb; ++k) h = (h ^ b[k]) * 1099511628211ull;
        return h;
    };
    // open addressing over indices (-1 = empty); 2x the element count, a power of two
    size_t cap = 16;
    while (cap < 2 * (size_t)n) cap <<= 1;
    std::vector<int32_t> slot(cap, -1);
    auto find_or_add = [&](uint32_t i, bool add) -> int32_t {
        const size_t nb = payload_bytes(e[i].kind);
        size_t s = hash(&e[i], nb) & (cap - 1);
        for (;; s = (s + 1) & (cap - 1)) {
            const int32_t j = slot[s];
            if (j < 0) {
                if (add) slot[s] = (int32_t)i;
                return -1;
            }
            if (e[j].kind == e[i].kind && std::memcmp(&e[j].u, &e[i].u, nb) == 0) return j;
        }
    };
    for (uint32_t i = 0; i < n; i++) {
        const bool has = payload_bytes(e[i].kind) != 0; // RT_OTHER terms are never matched
        if (e[i].canon < 0) {
            const int32_t j = has ? find_or_add(i, false) : -1;
            e[i].canon = j >= 0 ? j : (int32_t)i;
        }
        if (has && e[i].canon == (int32_t)i) (void)find_or_add(i, true); // keeps the first of its key
    }
    return RT_OK;
}

// resolve canon chains to the first element of each equality class
// Bytes of the LDS-staged tables of a spheres-only scene (the layout below, in rt_compile).
static long stage_bytes(const SceneHdr &h, int ncell) {
    auto up16 = [](long v) { return (v + 15) / 16 * 16; };
    long off = up16((long)h.n_obj * OBJ_W * 8);
    off = up16(off + (long)h.n_obj * OBJ_META_W * 4);
    off = up16(off + (long)h.n_light * h.n_sph * SPH_ORG_W * 8);
    off = up16(off + (long)h.n_light * h.n_sph * ncell * h.n_chunk * 8);
    off = up16(off + (long)h.n_sph * 4);
    return up16(off + (long)h.n_sph * SPH_B_W * 8);
}

static int root(const std::vector<rt_elem> &e, int i) {
    while (e[i].canon >= 0 && e[i].canon != i) i = e[i].canon;
    return i;
}

// binary32 bounds that contain the binary64 value: rounded down (lo) or up (hi)
static float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafterf(f, -INFINITY);
    return f;
}
static float f32_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafterf(f, INFINITY);
    return f;
}

// Sphere BVH for the reflection scans (rt_layout.h).  Binary, one sphere per leaf; splits by the
// surface area heuristic within a depth cap (or median splits along the longest axis of the
// centroids' bounds), so the depth is bounded and the per-lane stack never overflows.
// Each sphere's box is its centre +- |r| widened by m = BVH_BOX_REL * (extent + 1), far more than
// the binary32 rounding of the kernel's slab test (origins and directions rounded to binary32,
// relative error ~2^-22 in the slab distances) for scenes within CULL_EXTENT; the box test is only
// a filter, every sphere it lets through is tested by the reference's binary64 expressions.
static void build_bvh(const std::vector<rt_elem> &e, const std::vector<int> &sph, const std::vector<int> &compact,
                      const std::vector<rt_vec3> &org, SceneHdr &h, std::vector<double> &t) {
    h.bvh_ok = 0;
    h.o_bvh = 0;
    h.n_bvh = 0;
    h.bvh_level = 1 << 30;
    h.bvh_depth = 0;
    h.l_bvh = h.l_bsph = -1;
    h.l_stack = 0;
    static const int bvh_min = [] {
        const char *s = std::getenv("RT_BVH_MIN");
        return s ? std::atoi(s) : BVH_MIN_SPHERES;
    }();
    static const int bvh_level = [] {
        const char *s = std::getenv("RT_BVH_LEVEL");
        return s ? std::atoi(s) : BVH_LEVEL; // level 1 (coherent: from the primary hits) keeps the beams
    }();
    const int n = (int)sph.size();
    if (!h.cull_ok || n < 2 || n < bvh_min || n > BVH_MAX_SPHERES) return;
    int depth = 0;
    while ((1 << depth) < n) ++depth;
    if (depth > BVH_STACK) return; // a node at depth i holds at most i stack entries, pushes one more
    // Surface-area-heuristic splits among those that keep every leaf within ceil(log2 n) + slack
    // levels (the traversal stack's size; BVH_SAH_SLACK; 0: median splits).
    // Measured, config 5: slack 2 -2.2 % per frame against median splits; 1 or 3 neutral.
    constexpr int slack = BVH_SAH_SLACK;
    const int cap = slack > 0 && depth + 1 <= BVH_STACK ? std::min(depth + slack, BVH_STACK) : 0;
    double ext = 0;
    for (const rt_vec3 &o : org) ext = std::fmax(ext, std::fmax(std::fabs(o.x), std::fmax(std::fabs(o.y), std::fabs(o.z))));
    for (int i : sph) {
        const auto &s = e[i].u.sphere;
        ext = std::fmax(ext, std::fmax(std::fabs(s.center.x), std::fmax(std::fabs(s.center.y), std::fabs(s.center.z))) +
                                 std::fabs(s.radius));
    }
    const double m = BVH_BOX_REL * (ext + 1.0);
    struct Box {
        double lo[3], hi[3];
    };
    auto sbox = [&](int k) {
        const auto &s = e[sph[k]].u.sphere;
        const double c[3] = {s.center.x, s.center.y, s.center.z}, r = std::fabs(s.radius);
        Box b;
        for (int a = 0; a < 3; ++a) {
            b.lo[a] = c[a] - r - m;
            b.hi[a] = c[a] + r + m;
        }
        return b;
    };
    struct Node {
        Box b[2];
        int ch[2];
    };
    std::vector<Node> nodes;
    nodes.reserve(n);
    std::vector<int> items(n);
    for (int k = 0; k < n; ++k) items[k] = k;
    // returns the link of the subtree over items[b, e) and its box
    int max_depth = 0;
    auto area = [](const Box &x) {
        const double dx = x.hi[0] - x.lo[0], dy = x.hi[1] - x.lo[1], dz = x.hi[2] - x.lo[2];
        return dx * dy + dy * dz + dz * dx;
    };
    auto build = [&](auto &&self, int b, int en, int lvl, Box &box) -> int {
        if (en - b == 1) {
            box = sbox(items[b]);
            max_depth = std::max(max_depth, lvl);
            return ~items[b];
        }
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < en; ++i) {
            const auto &s = e[sph[items[i]]].u.sphere;
            const double c[3] = {s.center.x, s.center.y, s.center.z};
            for (int a = 0; a < 3; ++a) {
                clo[a] = std::fmin(clo[a], c[a]);
                chi[a] = std::fmax(chi[a], c[a]);
            }
        }
        int ax = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
        auto key = [&](int k) {
            const auto &s = e[sph[k]].u.sphere;
            return ax == 0 ? s.center.x : ax == 1 ? s.center.y : s.center.z;
        };
        std::sort(items.begin() + b, items.begin() + en, [&](int p, int q) {
            const double kp = key(p), kq = key(q);
            return kp < kq || (kp == kq && p < q);
        });
        int mid = b + (en - b) / 2;
        if (cap > 0) {
            const int cnt = en - b, lim = 1 << (cap - lvl - 1); // each side's leaves within the cap
            double best = INFINITY;
            int best_ax = ax, best_i = mid - b;
            std::vector<int> tmp(items.begin() + b, items.begin() + en);
            std::vector<Box> suf(cnt + 1);
            for (int a = 0; a < 3; ++a) {
                auto ka = [&](int k) {
                    const auto &sp = e[sph[k]].u.sphere;
                    return a == 0 ? sp.center.x : a == 1 ? sp.center.y : sp.center.z;
                };
                std::sort(tmp.begin(), tmp.end(), [&](int p, int q) { return ka(p) < ka(q) || (ka(p) == ka(q) && p < q); });
                suf[cnt] = Box{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
                for (int i = cnt - 1; i >= 0; --i) {
                    const Box sb = sbox(tmp[i]);
                    for (int c = 0; c < 3; ++c) {
                        suf[i].lo[c] = std::fmin(suf[i + 1].lo[c], sb.lo[c]);
                        suf[i].hi[c] = std::fmax(suf[i + 1].hi[c], sb.hi[c]);
                    }
                }
                Box pre = suf[cnt];
                for (int i = 1; i < cnt; ++i) {
                    const Box sb = sbox(tmp[i - 1]);
                    for (int c = 0; c < 3; ++c) {
                        pre.lo[c] = std::fmin(pre.lo[c], sb.lo[c]);
                        pre.hi[c] = std::fmax(pre.hi[c], sb.hi[c]);
                    }
                    if (i > lim || cnt - i > lim) continue;
                    const double cost = area(pre) * i + area(suf[i]) * (cnt - i);
                    if (cost < best) {
                        best = cost;
                        best_ax = a;
                        best_i = i;
                    }
                }
            }
            ax = best_ax;
            std::sort(items.begin() + b, items.begin() + en, [&](int p, int q) {
                const double kp = key(p), kq = key(q);
                return kp < kq || (kp == kq && p < q);
            });
            mid = b + best_i;
        }
        const int self_i = (int)nodes.size();
        nodes.push_back(Node{});
        Box bl, br;
        const int l = self(self, b, mid, lvl + 1, bl);
        const int r = self(self, mid, en, lvl + 1, br);
        nodes[self_i].b[0] = bl;
        nodes[self_i].b[1] = br;
        nodes[self_i].ch[0] = l;
        nodes[self_i].ch[1] = r;
        for (int a = 0; a < 3; ++a) {
            box.lo[a] = std::fmin(bl.lo[a], br.lo[a]);
            box.hi[a] = std::fmax(bl.hi[a], br.hi[a]);
        }
        return self_i;
    };
    Box root;
    build(build, 0, n, 0, root);
    while (t.size() % 2) t.push_back(0); // 16-byte aligned nodes
    h.o_bvh = (int)t.size();
    for (const Node &nd : nodes) {
        float f[16];
        const Box &b0 = nd.b[0], &b1 = nd.b[1];
        // (lx0 lx1 ly0 ly1) (lz0 lz1 ux0 ux1) (uy0 uy1 uz0 uz1): the two children's bounds side by
        // side, so the kernel's slab distances of both are packed binary32 pairs
        for (int a = 0; a < 3; ++a) {
            f[2 * a] = f32_down(b0.lo[a]);
            f[2 * a + 1] = f32_down(b1.lo[a]);
            f[6 + 2 * a] = f32_up(b0.hi[a]);
            f[6 + 2 * a + 1] = f32_up(b1.hi[a]);
        }
        std::memcpy(&f[12], &nd.ch[0], 4);
        std::memcpy(&f[13], &nd.ch[1], 4);
        const int id0 = nd.ch[0] < 0 ? compact[sph[~nd.ch[0]]] : -1, id1 = nd.ch[1] < 0 ? compact[sph[~nd.ch[1]]] : -1;
        std::memcpy(&f[14], &id0, 4);
        std::memcpy(&f[15], &id1, 4);
        double d[BVH_NODE_DOUBLES];
        std::memcpy(d, f, sizeof(d));
        t.insert(t.end(), d, d + BVH_NODE_DOUBLES);
    }
    h.n_bvh = (int)nodes.size();
    h.bvh_depth = max_depth;
    h.bvh_ok = 1;
    h.bvh_level = bvh_level < 1 ? 1 : bvh_level;
}

int compile_scene(const rt_elem *in, uint32_t n, Compiled &out) {
    int rc = check_scene(in, n);
    if (rc != RT_OK) return rc;
    std::vector<rt_elem> e(in, in + n);
    fill_canon(e.data(), n);

    const rt_elem &cam = e[0];
    std::vector<int> compact(n, -1);
    std::vector<int> objs, lights;
    for (uint32_t i = 1; i < n; i++) {
        int k = e[i].kind;
        if (k == RT_SPHERE || k == RT_TRIANGLE || k == RT_PLANE) {
            compact[i] = (int)objs.size();
            objs.push_back((int)i);
        } else if (k == RT_POINT_LIGHT) {
            lights.push_back((int)i);
        }
    }
    // The per-origin tables (camera and every light) hold ~16 doubles per (origin, sphere) pair: a
    // scene whose tables would not fit 32-bit offsets is refused before they are built.
    {
        const double per_origin = 16.0 * (double)objs.size();
        if ((double)(1 + lights.size()) * per_origin + 32.0 * (double)objs.size() >= (double)INT32_MAX / 2)
            return RT_ENOMEM;
    }
    std::vector<int> sph, tri, pl;
    for (int i : objs) {
        if (e[i].kind == RT_SPHERE) sph.push_back(i);
        else if (e[i].kind == RT_TRIANGLE) tri.push_back(i);
        else pl.push_back(i);
    }
    // The spheres' table order (their local index) decides only the order candidates and occluders
    // are visited in — nearest hits are broken by list position (compact id), shadow answers are
    // any-hit — so the spheres that cover most of the lights' view go first: a shadow ray's
    // occluder walk meets the likelier blockers early and its lane leaves sooner (measured against
    // list order: config 5 -4.5 % per frame, config 3 -1 %; ordering by radius alone: -3 %, and +1 %
    // on config 3).
    {
        // the spheres' solid angle summed over the lights (their radius when there are none)
        std::vector<double> w(e.size(), 0.0);
        for (int i : sph) {
            const auto &sp = e[i].u.sphere;
            const double r2 = sp.radius * sp.radius;
            double a = lights.empty() ? r2 : 0.0;
            for (int li : lights) {
                const rt_vec3 &L = e[li].u.point_light.location;
                const double dx = sp.center.x - L.x, dy = sp.center.y - L.y, dz = sp.center.z - L.z;
                a += r2 / std::fmax(dx * dx + dy * dy + dz * dz, 1e-300);
            }
            w[i] = a;
        }
        std::stable_sort(sph.begin(), sph.end(), [&](int a, int b) { return w[a] > w[b]; });
    }

    SceneHdr &h = out.hdr;
    std::memset(&h, 0, sizeof(h));
    h.n_sph = (int)sph.size();
    h.n_tri = (int)tri.size();
    h.n_pl = (int)pl.size();
    h.n_obj = (int)objs.size();
    h.n_light = (int)lights.size();
    h.n_org = 1 + h.n_light;

    // origins: slot 0 = camera location, slot 1+i = light i location
    std::vector<rt_vec3> org;
    org.push_back(cam.u.camera.location);
    for (int li : lights) org.push_back(e[li].u.point_light.location);

    std::vector<double> &t = out.tab;
    std::vector<int> &it = out.itab;
    t.clear();
    it.clear();

    // spheres (ray_sphere_intersect/2, :364-397)
    h.o_sph = (int)t.size();
    for (int i : sph) {
        const auto &s = e[i].u.sphere;
        double r = s.radius;
        t.insert(t.end(), {s.center.x, s.center.y, s.center.z, r * r});
    }
    h.o_sph_org = (int)t.size();
    for (const rt_vec3 &o : org) {
        for (int i : sph) {
            const auto &s = e[i].u.sphere;
            double X0 = o.x, Y0 = o.y, Z0 = o.z, Xc = s.center.x, Yc = s.center.y, Zc = s.center.z;
            double r = s.radius;
            double C = (X0 - Xc) * (X0 - Xc) + (Y0 - Yc) * (Y0 - Yc) + (Z0 - Zc) * (Z0 - Zc) - r * r;
            t.insert(t.end(), {X0 - Xc, Y0 - Yc, Z0 - Zc, C});
        }
    }
    // triangles (ray_triangle_intersect/2, :402-455)
    h.o_tri = (int)t.size();
    for (int i : tri) {
        const auto &tr = e[i].u.triangle;
        double e1x = tr.v2.x - tr.v1.x, e1y = tr.v2.y - tr.v1.y, e1z = tr.v2.z - tr.v1.z;
        double e2x = tr.v3.x - tr.v1.x, e2y = tr.v3.y - tr.v1.y, e2z = tr.v3.z - tr.v1.z;
        t.insert(t.end(), {tr.v1.x, tr.v1.y, tr.v1.z, e1x, e1y, e1z, e2x, e2y, e2z, 0, 0, 0});
    }
    h.o_tri_org = (int)t.size();
    for (const rt_vec3 &o : org) {
        for (int i : tri) {
            const auto &tr = e[i].u.triangle;
            double e1x = tr.v2.x - tr.v1.x, e1y = tr.v2.y - tr.v1.y, e1z = tr.v2.z - tr.v1.z;
            double Tx = o.x - tr.v1.x, Ty = o.y - tr.v1.y, Tz = o.z - tr.v1.z;
            // Q = vector_cross_product(T, Edge1) (:431, :549-552)
            double Qx = Ty * e1z - Tz * e1y, Qy = Tz * e1x - Tx * e1z, Qz = Tx * e1y - Ty * e1x;
            t.insert(t.end(), {Tx, Ty, Tz, Qx, Qy, Qz, 0, 0});
        }
    }
    // planes (ray_plane_intersect/2, :461-480)
    h.o_pl = (int)t.size();
    for (int i : pl) {
        const auto &p = e[i].u.plane;
        t.insert(t.end(), {p.normal.x, p.normal.y, p.normal.z, p.distance});
    }
    h.o_pl_org = (int)t.size();
    for (const rt_vec3 &o : org) {
        for (int i : pl) {
            const auto &p = e[i].u.plane;
            double V0 = -(p.normal.x * o.x + p.normal.y * o.y + p.normal.z * o.z + p.distance);
            t.push_back(V0);
        }
    }
    // per-object shading records, by compact id
    h.int_pow = 1;
    while (t.size() % 2) t.push_back(0); // every later section starts 16-byte aligned
    h.o_obj = (int)t.size();
    for (int i : objs) {
        const rt_elem &o = e[i];
        const rt_material *m;
        double a = 0, b = 0, c = 0;
        if (o.kind == RT_SPHERE) {
            m = &o.u.sphere.material;
            a = o.u.sphere.center.x; b = o.u.sphere.center.y; c = o.u.sphere.center.z;
        } else if (o.kind == RT_TRIANGLE) {
            m = &o.u.triangle.material;
            // Normal = vector_normalize(vector_cross_product(v1, v2)) (:448-451), a constant
            const rt_vec3 &v1 = o.u.triangle.v1, &v2 = o.u.triangle.v2;
            double nx = v1.y * v2.z - v1.z * v2.y, ny = v1.z * v2.x - v1.x * v2.z, nz = v1.x * v2.y - v1.y * v2.x;
            double mag = std::sqrt(nx * nx + ny * ny + nz * nz);
            if (mag == 0) {
                a = b = c = 0;
            } else {
                double s = 1 / std::sqrt(nx * nx + ny * ny + nz * nz);
                a = nx * s; b = ny * s; c = nz * s;
            }
        } else {
            m = &o.u.plane.material;
            a = o.u.plane.normal.x; b = o.u.plane.normal.y; c = o.u.plane.normal.z;
        }
        const double sp = m->specular_power;
        if (!(sp >= 0.0 && sp <= 1024.0 && sp == std::floor(sp))) h.int_pow = 0;
        t.insert(t.end(), {a, b, c, m->colour.x, m->colour.y, m->colour.z, m->specular_power, m->shininess,
                           m->reflectivity, 0, 0, 0});
    }
    h.o_light = (int)t.size();
    for (int li : lights) {
        const auto &L = e[li].u.point_light;
        t.insert(t.end(), {L.diffuse_colour.x, L.diffuse_colour.y, L.diffuse_colour.z, L.location.x, L.location.y,
                           L.location.z, L.specular_colour.x, L.specular_colour.y, L.specular_colour.z, 0, 0, 0});
    }
    // beam-culling tables (only consulted by the kernel when h.cull_ok); 16-byte aligned records
    while (t.size() % 2) t.push_back(0);
    h.o_sph_b = (int)t.size();
    for (int i : sph) {
        const auto &s = e[i].u.sphere;
        t.insert(t.end(), {s.center.x, s.center.y, s.center.z, std::fabs(s.radius)});
    }
    h.o_sph_ob = (int)t.size();
    for (const rt_vec3 &o : org) {
        for (int i : sph) {
            const auto &s = e[i].u.sphere;
            double vx = s.center.x - o.x, vy = s.center.y - o.y, vz = s.center.z - o.z;
            double vl = std::sqrt(vx * vx + vy * vy + vz * vz);
            double r = std::fabs(s.radius);
            double near = vl <= r * (1 + CULL_EPS) + CULL_EPS ? 1.0 : 0.0;
            double sr = near ? 1.0 : r / vl * (1 + CULL_EPS) + CULL_EPS;
            double cr = sr >= 1.0 ? 0.0 : std::sqrt(1 - sr * sr) - CULL_EPS;
            if (sr >= 1.0) near = 1.0;
            const double dlow = (vl - r) - CULL_EPS * (vl + r) - CULL_EPS;
            t.insert(t.end(), {vx, vy, vz, vl, sr, cr, near, dlow});
        }
    }
    // the same rows in binary32 for the binary32 beams: sin(rho) rounded up and widened, cos(rho)
    // rounded down and narrowed by BEAM32_EPS, |v| - r rounded down
    h.o_sph_ob32 = (int)t.size();
    for (const rt_vec3 &o : org) {
        for (int i : sph) {
            const auto &s = e[i].u.sphere;
            double vx = s.center.x - o.x, vy = s.center.y - o.y, vz = s.center.z - o.z;
            double vl = std::sqrt(vx * vx + vy * vy + vz * vz);
            double r = std::fabs(s.radius);
            const double eps = BEAM32_EPS;
            bool near = vl <= r * (1 + eps) + eps;
            double sr = near ? 1.0 : r / vl * (1 + eps) + eps;
            if (sr >= 1.0) near = true;
            double cr = near ? 0.0 : std::sqrt(1 - sr * sr) - eps;
            const double dlow = (vl - r) - eps * (vl + r) - eps;
            float f[SPH_OB32_W] = {(float)vx, (float)vy, (float)vz, (float)vl, f32_up(sr), f32_down(cr),
                                   near ? 1.0f : 0.0f, f32_down(dlow)};
            double d[SPH_OB32_W / 2];
            std::memcpy(d, f, sizeof(d));
            t.insert(t.end(), d, d + SPH_OB32_W / 2);
        }
    }
    {
        double ext = 0;
        auto grow = [&](double v) { ext = std::fmax(ext, std::fabs(v)); };
        for (const rt_vec3 &o : org) { grow(o.x); grow(o.y); grow(o.z); }
        for (int i : sph) {
            const auto &s = e[i].u.sphere;
            grow(s.center.x); grow(s.center.y); grow(s.center.z); grow(s.radius);
        }
        h.cull_ok = ext <= CULL_EXTENT ? 1 : 0;
        h.ext = ext;
    }
    {
        // normalize3's range checks that cannot fail (SceneHdr::norm_ok / prim_ok)
        bool ok = h.cull_ok && h.n_tri == 0 && h.n_pl == 0;
        const double tol = 1.0e-9 * (h.ext + 1.0);
        for (int i : sph) {
            if (!ok) break;
            const auto &s = e[i].u.sphere;
            const double r = std::fabs(s.radius);
            if (!(r >= 1.0e-50)) ok = false;
            for (int li : lights) {
                const rt_vec3 &L = e[li].u.point_light.location;
                const double dx = L.x - s.center.x, dy = L.y - s.center.y, dz = L.z - s.center.z;
                if (!(std::fabs(std::sqrt(dx * dx + dy * dy + dz * dz) - r) > tol)) ok = false;
            }
        }
        h.norm_ok = ok ? 1 : 0;
    }
    // Wave beams (a cone over the wave's rays, a candidate mask per 64 spheres) cost a few wave
    // reductions per scan; with a handful of spheres testing every one is cheaper
    // (RT_BEAM_MIN overrides the threshold, for A/B runs).
    {
        static const int beam_min = [] {
            const char *s = std::getenv("RT_BEAM_MIN");
            return s ? std::atoi(s) : BEAM_MIN_SPHERES;
        }();
        h.beam_ok = h.cull_ok && h.n_sph >= beam_min ? 1 : 0;
    }
    build_bvh(e, sph, compact, org, h, t);
    if (t.empty()) t.push_back(0);

    // int table
    h.i_sph_id = (int)it.size();
    for (int i : sph) it.push_back(compact[i]);
    h.i_tri_id = (int)it.size();
    for (int i : tri) it.push_back(compact[i]);
    h.i_pl_id = (int)it.size();
    for (int i : pl) it.push_back(compact[i]);
    while (it.size() % 4) it.push_back(0); // 16-byte rows
    h.i_obj_meta = (int)it.size();
    {
        // each element's index within its type's table
        std::vector<int> local_of(n, 0);
        for (const std::vector<int> *grp : {&sph, &tri, &pl})
            for (size_t q = 0; q < grp->size(); q++) local_of[(*grp)[q]] = (int)q;
        for (int i : objs) {
            int kind = e[i].kind == RT_SPHERE ? K_SPHERE : (e[i].kind == RT_TRIANGLE ? K_TRIANGLE : K_PLANE);
            // the canonical (first exactly equal) element is a record of the same type: its index
            // within the type is stored here too, so a shadow target resolves in one load
            const int r = root(e, i);
            it.insert(it.end(), {kind, local_of[i], compact[r], local_of[r]});
        }
    }
    // Occluder masks, per (light, target sphere, direction cell).  Shadow rays to a target
    // sphere t start at the light L and point into the cone from L around ball(c_t, r_t); the
    // target's own t* (its entry point) is at most |c_t - L|.  Sphere j can block such a ray only
    // if (a) it meets that cone (angular test as in the kernel's beam culling, with CULL_EPS
    // margins in the safe direction) and (b) some point of it is within |c_t - L| of L.  The
    // target itself never blocks (its t equals t* and its list position is not earlier).
    // Cells (the kernel's occ_cell): the cone is split by the signs of dir - a along two world
    // axes i, j (a = (c_t - L)/|c_t - L|; the axes on which a is shortest, chosen from the
    // binary32 components of L - c_t exactly as the kernel chooses them).  Sphere j stays in cell
    // (b_i, b_j) only if its cone of directions (axis w, sin of its half-angle sr) reaches the
    // half-spaces s*(dir_k - a_k) >= -OCC_CELL_EPS, s = +1 for b_k = 1 and -1 for b_k = 0: the
    // largest s*dir_k over the cone is cos(max(0, angle(w, s*e_k) - rho)).
    h.n_chunk = (h.n_sph + 63) / 64;
    // Small scenes and scenes whose tables are staged in LDS (below) keep one cell: their walks
    // are short (S64: 1.37 steps per test) and the cells' extra LDS and binary32 work cost more
    // than they save (measured: config 3 -5 %); large scenes get OCC_CELLS (config 5: +4 %).
    const bool stage_kind = h.cull_ok && h.n_tri == 0 && h.n_pl == 0 && h.n_sph > 0 && h.n_light > 0;
    h.occ_cells = (h.n_sph < OCC_CELLS_MIN_SPHERES || (stage_kind && stage_bytes(h, 1) <= LDS_STAGE_MAX)) ? 1 : OCC_CELLS;
    // The masks cost the host one (light, target, sphere) test per triple and the device
    // n_light * n_sph^2 * cells bits: beyond OCC_MAX_TESTS tests there are none (occ_ok = 0) and
    // the shadow rays take the shadow cones over the sphere chunks instead (lit_by); beyond
    // OCC_MAX_BYTES the masks keep one cell.
    const double occ_tests = (double)h.n_light * h.n_sph * h.n_sph;
    h.occ_ok = h.cull_ok && h.n_sph > 0 && occ_tests <= OCC_MAX_TESTS ? 1 : 0;
    if (h.occ_ok && (double)h.n_light * h.n_sph * h.occ_cells * h.n_chunk * 8 > OCC_MAX_BYTES) h.occ_cells = 1;
    const int ncell = h.occ_cells;
    while (it.size() % 2) it.push_back(0);
    h.i_occ = (int)it.size();
    if (h.occ_ok) {
        for (int li : lights) {
            const rt_vec3 &L = e[li].u.point_light.location;
            for (int ti : sph) {
                const auto &T = e[ti].u.sphere;
                const double ax = T.center.x - L.x, ay = T.center.y - L.y, az = T.center.z - L.z;
                const double D = std::sqrt(ax * ax + ay * ay + az * az);
                const double rt = std::fabs(T.radius);
                const bool wide = !(D > rt * (1 + CULL_EPS) + CULL_EPS); // light inside the target
                const double st = wide ? 1.0 : rt / D * (1 + CULL_EPS) + CULL_EPS;
                const double ct = st >= 1.0 ? 0.0 : std::sqrt(1 - st * st) - CULL_EPS;
                const double tmax = D * (1 + CULL_EPS) + CULL_EPS;
                // the kernel's cell axes, from the binary32 components of its row (L - c_t)
                const float qx = (float)(L.x - T.center.x), qy = (float)(L.y - T.center.y),
                            qz = (float)(L.z - T.center.z);
                const float fx = std::fabs(qx), fy = std::fabs(qy), fz = std::fabs(qz);
                const int drop = (fx >= fy && fx >= fz) ? 0 : (fy >= fz ? 1 : 2);
                const int axi = drop == 0 ? 1 : 0, axj = drop == 2 ? 1 : 2;
                const double a3[3] = {ax / D, ay / D, az / D};
                std::vector<uint64_t> m((size_t)ncell * h.n_chunk, 0);
                for (size_t j = 0; j < sph.size(); j++) {
                    if ((int)sph[j] == ti) continue;
                    const auto &S = e[sph[j]].u.sphere;
                    const double vx = S.center.x - L.x, vy = S.center.y - L.y, vz = S.center.z - L.z;
                    const double vl = std::sqrt(vx * vx + vy * vy + vz * vz);
                    const double r = std::fabs(S.radius);
                    bool keep, cells = false;
                    double sr = 1.0;
                    if (wide || st >= 1.0 || !(ct > 0.0) || vl <= r * (1 + CULL_EPS) + CULL_EPS) {
                        keep = true;
                    } else {
                        sr = r / vl * (1 + CULL_EPS) + CULL_EPS;
                        if (sr >= 1.0) {
                            keep = true;
                        } else {
                            const double cr = std::sqrt(1 - sr * sr) - CULL_EPS;
                            const double thr = ct * cr - st * sr;
                            const double av = (ax * vx + ay * vy + az * vz) / D;
                            keep = !(av + CULL_EPS * vl < thr * vl);
                            cells = true;
                        }
                    }
                    const double dlow = (vl - r) - CULL_EPS * (vl + r) - CULL_EPS;
                    if (!keep || dlow > tmax) continue;
                    const double w3[3] = {vx / vl, vy / vl, vz / vl};
                    const double rho = std::asin(sr) + CULL_EPS;
                    // the cone of sphere j reaches s*(dir_k - a_k) in [lo, hi] (widened by eps):
                    // its largest s*dir_k is cos(max(0, psi - rho)), its smallest cos(min(pi, psi + rho))
                    const double eps = OCC_CELL_EPS, tau = rt / D * 0.5; // the kernel's |sd - a| split
                    // does the cone reach s*(dir_k - a_k) in [t_lo, t_hi]?
                    auto reach = [&](int k, double s, double t_lo, double t_hi) {
                        const double psi = std::acos(std::max(-1.0, std::min(1.0, s * w3[k])));
                        const double top = psi <= rho ? 1.0 : std::cos(psi - rho);
                        const double bot = psi + rho >= M_PI ? -1.0 : std::cos(psi + rho);
                        if (top + 1e-7 < s * a3[k] + t_lo - eps) return false;
                        if (bot - 1e-7 > s * a3[k] + t_hi + eps) return false;
                        return true;
                    };
                    // the kernel's bins along one axis (occ_cell): the sign of dir_k - a_k and, with
                    // 16 cells, |dir_k - a_k| below / above tau; with 64, below tau/2, tau, 3 tau/2 or above
                    auto bin = [&](int b, double &s, double &t_lo, double &t_hi) {
                        const double inf = 1e300;
                        if (ncell == 4) {
                            s = (b & 1) ? 1.0 : -1.0; t_lo = 0; t_hi = inf;
                        } else if (ncell == 16) {
                            s = (b & 1) ? 1.0 : -1.0;
                            t_lo = (b & 2) ? tau : 0.0; t_hi = (b & 2) ? inf : tau;
                        } else {
                            s = (b & 4) ? 1.0 : -1.0;
                            const int g = b & 3;
                            t_lo = g * 0.5 * tau; t_hi = g == 3 ? inf : (g + 1) * 0.5 * tau;
                        }
                    };
                    for (int c = 0; c < ncell; c++) {
                        // cell -> the bins of axes i and j (occ_cell's numbering)
                        int bi = 0, bj = 0;
                        if (ncell == 4) { bi = c & 1; bj = (c >> 1) & 1; }
                        else if (ncell == 16) { bi = (c & 1) | ((c >> 1) & 2); bj = ((c >> 1) & 1) | ((c >> 2) & 2); }
                        else { bi = c & 7; bj = c >> 3; }
                        double si, li, hi_, sj, lj, hj;
                        bin(bi, si, li, hi_);
                        bin(bj, sj, lj, hj);
                        if (!cells || ncell == 1 || (reach(axi, si, li, hi_) && reach(axj, sj, lj, hj)))
                            m[(size_t)c * h.n_chunk + j / 64] |= 1ull << (j % 64);
                    }
                }
                for (uint64_t w : m) {
                    it.push_back((int)(uint32_t)(w & 0xffffffffu));
                    it.push_back((int)(uint32_t)(w >> 32));
                }
            }
        }
    }
    if (it.empty()) it.push_back(0);
    // the kernels index both tables with 32-bit ints
    if (t.size() >= (size_t)INT32_MAX / 2 || it.size() >= (size_t)INT32_MAX / 2) return RT_ENOMEM;

    // camera: point_on_screen/3 (:486-503) with focal_length/2 (:483-484).
    // Sum = foldl(fun(V, S) -> vector_add(V, S) end, Location, [ {0*F,0*F,1*F}, {(X-0.5)*SW,0,0},
    // {0,(Y-0.5)*SH,0} ]); the pixel-invariant parts are folded here in the same order.
    double SW = cam.u.camera.screen_width, SH = cam.u.camera.screen_height;
    double F = SW / (2 * std::tan(cam.u.camera.fov * (M_PI / 180) / 2));
    const rt_vec3 &L = cam.u.camera.location;
    h.cam_x = L.x; h.cam_y = L.y; h.cam_z = L.z;
    h.sx = 0 * F + L.x;                       // x after step 1; step 2 adds (X-0.5)*SW, step 3 adds 0
    h.sy = 0.0 + (0 * F + L.y);               // y after steps 1-2; step 3 adds (Y-0.5)*SH
    double pz = 0.0 + (0.0 + (1 * F + L.z));  // z after steps 1-3
    h.dz = pz - L.z;                          // vector_sub(Through, From).z (:507)
    if (!std::isfinite(F) || !std::isfinite(h.sx) || !std::isfinite(h.sy) || !std::isfinite(h.dz))
        return RT_EBADARG; // Erlang raises badarith where binary64 would overflow
    h.screen_w = SW;
    h.screen_h = SH;
    h.n_light_d = (double)h.n_light;
    {
        // primary rays: Through - From = (px - cx, py - cy, dz) with X, Y in [0, 1]: squared length
        // at least dz^2, at most (|sx| + |w| + |cx|)^2 + (|sy| + |h| + |cy|)^2 + dz^2 (prim_ok)
        const double bx = std::fabs(h.sx) + std::fabs(h.screen_w) + std::fabs(h.cam_x);
        const double by = std::fabs(h.sy) + std::fabs(h.screen_h) + std::fabs(h.cam_y);
        const double lo = h.dz * h.dz, hi = bx * bx + by * by + h.dz * h.dz;
        h.prim_ok = (lo >= 1.0e-100 && hi <= 1.0e100) ? 1 : 0;
    }
    // LDS staging layout (16-byte aligned sections)
    h.l_obj = h.l_meta = h.l_org = h.l_occ = h.l_id = h.l_sphb = -1;
    h.l_bytes = 0;
    if (stage_kind && h.occ_ok && h.occ_cells == 1) {
        auto up16 = [](long v) { return (v + 15) / 16 * 16; };
        long off = 0;
        const long l_obj = off; off = up16(off + (long)h.n_obj * OBJ_W * 8);
        const long l_meta = off; off = up16(off + (long)h.n_obj * OBJ_META_W * 4);
        const long l_org = off; off = up16(off + (long)h.n_light * h.n_sph * SPH_ORG_W * 8);
        const long l_occ = off; off = up16(off + (long)h.n_light * h.n_sph * h.n_chunk * 8);
        const long l_id = off; off = up16(off + (long)h.n_sph * 4);
        const long l_sphb = off; off = up16(off + (long)h.n_sph * SPH_B_W * 8);
        if (off <= LDS_STAGE_MAX) {
            h.l_obj = (int)l_obj; h.l_meta = (int)l_meta; h.l_org = (int)l_org; h.l_occ = (int)l_occ;
            h.l_id = (int)l_id; h.l_sphb = (int)l_sphb; h.l_bytes = (int)off;
        }
    }
    return RT_OK;
}

} // namespace rtl
