/*
 * rt_oracle.c — CPU ORACLE for the per-pixel render path.  TEST INFRASTRUCTURE
 * ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, never by the product path (eraytracer_amd/).
 *
 * An operation-for-operation restatement, in scalar IEEE binary64, of the
 * reference ray tracer plouj/eraytracer, raytracer.erl.  Every function cites
 * the reference lines it follows.  Compiled with -ffp-contract=off and no
 * fast-math: each Erlang float operation is one correctly rounded C double
 * operation, and math:sqrt/pow/tan are the host libm, as on BEAM.
 *
 * Erlang integers in the scene are small, so int arithmetic is exact in
 * double; the few places where the reference's int/float distinction shows
 * (lists:max([0,X]) returning int 0, structural =:= in shadow_factor) are
 * handled explicitly (see the comments there and rt_elem.canon).
 *
 * Two evaluation modes:
 *   ORC_LITERAL  — the reference's recursion as written: lighting_function
 *                  recomputes the reflection for EVERY light
 *                  (raytracer.erl:211-224), L^(depth-1) leaf calls per pixel.
 *   ORC_MEMO     — the reflection computed once per hit and reused for every
 *                  light.  Same sub-expression, same value: bit-identical to
 *                  ORC_LITERAL (checked by tests/test_oracle.py).
 * Both do the full nearest-object scan for shadows (raytracer.erl:261).
 *
 * Parity pin: the reference's own unit tests (raytracer.erl:735-1133) are
 * restated as KATs in tests/test_oracle.py; no reference-produced images exist
 * (the reference publishes none and Erlang is absent here), so image-level
 * parity is checked against an independent pure-Python restatement that works
 * on the Erlang terms themselves (oracle/erl_restatement.py).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt_mi355x.h"

typedef struct { double x, y, z; } V;

/* ---- vector math, raytracer.erl:524-573 ------------------------------------ */
static V v3(double x, double y, double z) { V r = {x, y, z}; return r; }
static V vector_add(V a, V b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }          /* :524-527 */
static V vector_sub(V a, V b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }          /* :529-532 */
static double vector_square_mag(V v) { return v.x * v.x + v.y * v.y + v.z * v.z; }    /* :534-535 */
static double vector_mag(V v) { return sqrt(vector_square_mag(v)); }                   /* :537-538 */
static V vector_scalar_mult(V v, double s) { return v3(v.x * s, v.y * s, v.z * s); }  /* :540-541 */
static V vector_component_mult(V a, V b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* :543-544 */
static double vector_dot_product(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :546-547 */
static V vector_cross_product(V a, V b) {                                              /* :549-552 */
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static V vector_normalize(V v) {                                                       /* :554-560 */
    double mag = vector_mag(v);
    if (mag == 0) return v3(0, 0, 0);
    return vector_scalar_mult(v, 1 / vector_mag(v));
}
static V vector_neg(V v) { return v3(-v.x, -v.y, -v.z); }                              /* :562-563 */
static V vector_bounce_off_plane(V vec, V n) {                                         /* :568-573 */
    return vector_add(vector_scalar_mult(n, 2 * vector_dot_product(n, vector_neg(vec))), vec);
}
static V from_rt(rt_vec3 a) { return v3(a.x, a.y, a.z); }

/* lists:max([0, X]) (raytracer.erl:275, :290): the int 0 unless X > 0.  The
 * int 0 multiplies to an exact 0.0 later, which is what 0.0 does here. */
static double max0(double x) { return x > 0 ? x : 0.0; }

/* ---- rays and hits ------------------------------------------------------------ */
typedef struct { V origin, direction; } Ray;              /* #ray{origin, direction} :74 */
typedef struct { int hit; double t; V loc, normal; } Hit; /* {Distance, Hit_location, Normal} | none */

/* ray_sphere_intersect/2, raytracer.erl:364-397 */
static Hit ray_sphere_intersect(Ray r, const rt_elem *s) {
    Hit h; h.hit = 0;
    const double epsilon = 0.001;
    double X0 = r.origin.x, Y0 = r.origin.y, Z0 = r.origin.z;
    double Xd = r.direction.x, Yd = r.direction.y, Zd = r.direction.z;
    double Xc = s->u.sphere.center.x, Yc = s->u.sphere.center.y, Zc = s->u.sphere.center.z;
    double radius = s->u.sphere.radius;
    double A = Xd * Xd + Yd * Yd + Zd * Zd;
    double B = 2 * (Xd * (X0 - Xc) + Yd * (Y0 - Yc) + Zd * (Z0 - Zc));
    double C = (X0 - Xc) * (X0 - Xc) + (Y0 - Yc) * (Y0 - Yc) + (Z0 - Zc) * (Z0 - Zc) - radius * radius;
    double disc = B * B - 4 * A * C;
    if (disc >= epsilon) {
        double T0 = (-B + sqrt(disc)) / 2;
        double T1 = (-B - sqrt(disc)) / 2;
        if ((T0 >= 0) && (T1 >= 0)) {
            double dist = (T1 < T0) ? T1 : T0; /* lists:min([T0, T1]) keeps T0 on ties */
            V inter = vector_add(v3(X0, Y0, Z0), vector_scalar_mult(v3(Xd, Yd, Zd), dist));
            h.hit = 1; h.t = dist; h.loc = inter;
            h.normal = vector_normalize(vector_sub(inter, v3(Xc, Yc, Zc)));
        }
    }
    return h;
}

/* ray_triangle_intersect/2, raytracer.erl:402-455 (Möller–Trumbore, no t >= 0 test,
 * normal = normalize(v1 x v2) as written). */
static Hit ray_triangle_intersect(Ray r, const rt_elem *tr) {
    Hit h; h.hit = 0;
    const double epsilon = 0.000001;
    V v1 = from_rt(tr->u.triangle.v1), v2 = from_rt(tr->u.triangle.v2), v3_ = from_rt(tr->u.triangle.v3);
    V edge1 = vector_sub(v2, v1);
    V edge2 = vector_sub(v3_, v1);
    V P = vector_cross_product(r.direction, edge2);
    double det = vector_dot_product(edge1, P);
    if (det < epsilon) return h;
    V T = vector_sub(r.origin, v1);
    double U = vector_dot_product(T, P);
    if ((U < 0) || (U > det)) return h;
    V Q = vector_cross_product(T, edge1);
    double Vv = vector_dot_product(r.direction, Q);
    if ((Vv < 0) || (U + Vv > det)) return h;
    double dist = vector_dot_product(edge2, Q) / det;
    h.hit = 1; h.t = dist;
    h.loc = vector_add(r.origin, vector_scalar_mult(r.direction, dist));
    h.normal = vector_normalize(vector_cross_product(v1, v2));
    return h;
}

/* ray_plane_intersect/2, raytracer.erl:461-480 */
static Hit ray_plane_intersect(Ray r, const rt_elem *p) {
    Hit h; h.hit = 0;
    const double epsilon = 0.001;
    V n = from_rt(p->u.plane.normal);
    double Vd = vector_dot_product(n, r.direction);
    if (Vd < 0) {
        double V0 = -(vector_dot_product(n, r.origin) + p->u.plane.distance);
        double dist = V0 / Vd;
        if (dist < epsilon) return h;
        h.hit = 1; h.t = dist;
        h.loc = vector_add(r.origin, vector_scalar_mult(r.direction, dist));
        h.normal = n;
    }
    return h;
}

/* ray_object_intersect/2, raytracer.erl:349-359 */
static Hit ray_object_intersect(Ray r, const rt_elem *o) {
    switch (o->kind) {
    case RT_SPHERE: return ray_sphere_intersect(r, o);
    case RT_TRIANGLE: return ray_triangle_intersect(r, o);
    case RT_PLANE: return ray_plane_intersect(r, o);
    default: { Hit h; h.hit = 0; return h; }
    }
}

/* nearest_object_intersecting_ray/2,6, raytracer.erl:300-346: linear scan in list
 * order starting from `infinity`; replace iff Distance > NewDistance (strict, so ties
 * keep the earlier object; negative distances win).  Returns the element index or -1. */
typedef struct { const rt_elem *e; uint32_t n; /* Rest_of_scene = elems[1..n) */ } Scene;

static int nearest_object_intersecting_ray(Ray r, const Scene *sc, Hit *out) {
    int best = -1;
    Hit bh = {0, 0, {0, 0, 0}, {0, 0, 0}};
    for (uint32_t i = 1; i < sc->n; i++) {
        Hit h = ray_object_intersect(r, &sc->e[i]);
        if (!h.hit) continue;
        if (best < 0 || bh.t > h.t) { best = (int)i; bh = h; }
    }
    if (out) *out = bh;
    return best;
}

/* exact (=:=) equality of two scene elements, via the host-supplied canon index */
static int same_term(const Scene *sc, int a, int b) { return sc->e[a].canon == sc->e[b].canon; }

/* shadow_factor/4, raytracer.erl:256-267: 1 iff the nearest object seen from the light
 * along normalize(Hit - Light) is (a copy of) the hit object. */
static double shadow_factor(V light_loc, V hit_loc, int object, const Scene *sc) {
    V light_vector = vector_sub(hit_loc, light_loc);
    V light_direction = vector_normalize(light_vector);
    Ray shadow_ray = {light_loc, light_direction};
    int j = nearest_object_intersecting_ray(shadow_ray, sc, NULL);
    if (j >= 0 && same_term(sc, j, object)) return 1;
    return 0;
}

/* diffuse_term/4, raytracer.erl:272-279 */
static V diffuse_term(const rt_material *m, V light_loc, V hit_loc, V hit_normal) {
    return vector_scalar_mult(from_rt(m->colour),
                              max0(vector_dot_product(hit_normal, vector_normalize(vector_sub(light_loc, hit_loc)))));
}

/* specular_term/7, raytracer.erl:285-297 */
static V specular_term(V eye, V light_loc, V hit_loc, V hit_normal, double spec_power, double shininess,
                       V spec_colour) {
    return vector_scalar_mult(
        spec_colour,
        shininess * pow(max0(vector_dot_product(
                            vector_normalize(vector_add(vector_normalize(vector_sub(light_loc, hit_loc)), vector_neg(eye))),
                            hit_normal)),
                        spec_power));
}

static const rt_material *object_material(const rt_elem *o) { /* object_*(), raytracer.erl:575-601 */
    switch (o->kind) {
    case RT_SPHERE: return &o->u.sphere.material;
    case RT_TRIANGLE: return &o->u.triangle.material;
    default: return &o->u.plane.material;
    }
}

enum { ORC_LITERAL = 0, ORC_MEMO = 1 };

static V pixel_colour_from_ray(Ray r, const Scene *sc, int depth, int mode, int *levels);

/* lighting_function/6, raytracer.erl:209-252: fold over the scene in list order; every
 * #point_light adds Reflection + (Lc (x) (diffuse + specular)) * shadow. */
static V lighting_function(Ray r, int object, V hit_loc, V hit_normal, const Scene *sc, int depth, int mode,
                           int *levels) {
    const rt_elem *obj = &sc->e[object];
    const rt_material *m = object_material(obj);
    V final_colour = v3(0, 0, 0);
    V memo_refl = v3(0, 0, 0);
    int have_memo = 0;
    for (uint32_t i = 1; i < sc->n; i++) {
        const rt_elem *L = &sc->e[i];
        if (L->kind != RT_POINT_LIGHT) continue; /* (_Not_a_point_light, F) -> F, :248-249 */
        V light_colour = from_rt(L->u.point_light.diffuse_colour);
        V light_loc = from_rt(L->u.point_light.location);
        V spec_colour = from_rt(L->u.point_light.specular_colour);
        V reflection;
        if (mode == ORC_MEMO && have_memo) {
            reflection = memo_refl;
        } else {
            Ray bounce = {hit_loc, vector_bounce_off_plane(r.direction, hit_normal)};
            /* only the first evaluation of the (identical) reflection reports the chain length */
            reflection = vector_scalar_mult(pixel_colour_from_ray(bounce, sc, depth - 1, mode, have_memo ? NULL : levels),
                                            m->reflectivity);
            memo_refl = reflection;
            have_memo = 1;
        }
        V light_contribution = vector_add(diffuse_term(m, light_loc, hit_loc, hit_normal),
                                          specular_term(r.direction, light_loc, hit_loc, hit_normal, m->specular_power,
                                                        m->shininess, spec_colour));
        final_colour = vector_add(
            final_colour,
            vector_add(reflection, vector_scalar_mult(vector_component_mult(light_colour, light_contribution),
                                                      shadow_factor(light_loc, hit_loc, object, sc))));
    }
    return final_colour;
}

/* pixel_colour_from_ray/3, raytracer.erl:186-203.  *levels (if given) is incremented
 * for every level of the reflection chain whose scan hits. */
static V pixel_colour_from_ray(Ray r, const Scene *sc, int depth, int mode, int *levels) {
    if (depth == 0) return v3(0, 0, 0);
    Hit h;
    int obj = nearest_object_intersecting_ray(r, sc, &h);
    if (obj < 0) return v3(0, 0, 0); /* ?BACKGROUND_COLOUR, :82 */
    if (levels) (*levels)++;
    return lighting_function(r, obj, h.loc, h.normal, sc, depth, mode, levels);
}

/* ---- camera, raytracer.erl:483-511 ------------------------------------------------ */
double orc_focal_length(double angle, double dimension) { /* :483-484 */
    return dimension / (2 * tan(angle * (M_PI / 180) / 2));
}

static V point_on_screen(double X, double Y, const rt_elem *cam) { /* :486-503 */
    double sw = cam->u.camera.screen_width, sh = cam->u.camera.screen_height;
    /* lists:foldl(fun(Vect, Sum) -> vector_add(Vect, Sum) end, Location, [...]) */
    V sum = from_rt(cam->u.camera.location);
    V l1 = vector_scalar_mult(v3(0, 0, 1), orc_focal_length(cam->u.camera.fov, sw));
    V l2 = v3((X - 0.5) * sw, 0, 0);
    V l3 = v3(0, (Y - 0.5) * sh, 0);
    sum = vector_add(l1, sum);
    sum = vector_add(l2, sum);
    sum = vector_add(l3, sum);
    return sum;
}

static Ray shoot_ray(V from, V through) { /* :506-507 */
    Ray r = {from, vector_normalize(vector_sub(through, from))};
    return r;
}

static Ray ray_through_pixel(double X, double Y, const rt_elem *cam) { /* :510-511 */
    return shoot_ray(from_rt(cam->u.camera.location), point_on_screen(X, Y, cam));
}

/* trace_ray_through_pixel/3, raytracer.erl:180-184 */
static V trace_ray_through_pixel(double X, double Y, const Scene *sc, int depth, int mode, int *levels) {
    return pixel_colour_from_ray(ray_through_pixel(X, Y, &sc->e[0]), sc, depth, mode, levels);
}

/* ---- exported helpers for the KATs (tests/test_oracle.py) ---------------------------- */
void orc_vec_op(int op, const double *a, const double *b, double s, double *out) {
    V A = v3(a[0], a[1], a[2]), B = v3(b[0], b[1], b[2]), R = v3(0, 0, 0);
    switch (op) {
    case 0: R = vector_add(A, B); break;
    case 1: R = vector_sub(A, B); break;
    case 2: R.x = vector_square_mag(A); break;
    case 3: R.x = vector_mag(A); break;
    case 4: R = vector_scalar_mult(A, s); break;
    case 5: R = vector_component_mult(A, B); break;
    case 6: R.x = vector_dot_product(A, B); break;
    case 7: R = vector_cross_product(A, B); break;
    case 8: R = vector_normalize(A); break;
    case 9: R = vector_neg(A); break;
    case 10: R = vector_bounce_off_plane(A, B); break;
    }
    out[0] = R.x; out[1] = R.y; out[2] = R.z;
}

/* Intersect one element: returns 1 and fills out[7] = {t, loc xyz, normal xyz} on a hit. */
int orc_intersect(const rt_elem *e, const double *origin, const double *dir, double *out) {
    Ray r = {v3(origin[0], origin[1], origin[2]), v3(dir[0], dir[1], dir[2])};
    Hit h = ray_object_intersect(r, e);
    if (!h.hit) return 0;
    out[0] = h.t; out[1] = h.loc.x; out[2] = h.loc.y; out[3] = h.loc.z;
    out[4] = h.normal.x; out[5] = h.normal.y; out[6] = h.normal.z;
    return 1;
}

/* nearest over a plain object list (no camera slot): returns the list index or -1 */
int orc_nearest(const rt_elem *objs, uint32_t n, const double *origin, const double *dir, double *out) {
    Ray r = {v3(origin[0], origin[1], origin[2]), v3(dir[0], dir[1], dir[2])};
    int best = -1;
    Hit bh = {0, 0, {0, 0, 0}, {0, 0, 0}};
    for (uint32_t i = 0; i < n; i++) {
        Hit h = ray_object_intersect(r, &objs[i]);
        if (!h.hit) continue;
        if (best < 0 || bh.t > h.t) { best = (int)i; bh = h; }
    }
    if (best >= 0 && out) {
        out[0] = bh.t; out[1] = bh.loc.x; out[2] = bh.loc.y; out[3] = bh.loc.z;
        out[4] = bh.normal.x; out[5] = bh.normal.y; out[6] = bh.normal.z;
    }
    return best;
}

void orc_point_on_screen(const rt_elem *cam, double X, double Y, double *out) {
    V p = point_on_screen(X, Y, cam);
    out[0] = p.x; out[1] = p.y; out[2] = p.z;
}

void orc_shoot_ray(const double *from, const double *through, double *out) {
    Ray r = shoot_ray(v3(from[0], from[1], from[2]), v3(through[0], through[1], through[2]));
    out[0] = r.direction.x; out[1] = r.direction.y; out[2] = r.direction.z;
}

void orc_trace_pixel(const rt_elem *scene, uint32_t n, double X, double Y, int depth, int mode, double *out,
                     int *levels) {
    Scene sc = {scene, n};
    int lv = 0;
    V c = trace_ray_through_pixel(X, Y, &sc, depth, mode, &lv);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
    if (levels) *levels = lv;
}

/* ---- whole-image render (the pixel loop of raytraced_pixel_list_simple/4, :86-99),
 * rows [row0, row0+nrows), threaded over rows. -------------------------------------- */
typedef struct {
    const Scene *sc;
    uint32_t W, H, row0, nrows;
    int depth, mode;
    double *out;
    uint8_t *levels;
    volatile uint32_t *next;
    uint32_t spp;
    uint64_t seed;
    const uint32_t *rows;      /* NULL: rows row0 .. row0+nrows-1; else the listed rows */
    volatile uint32_t *workers; /* threads that rendered at least one row */
} Job;

/* RT_SUPERSAMPLING (include/rt_mi355x.h; not part of the reference): the jitter hash. */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void *worker(void *arg) {
    Job *j = (Job *)arg;
    int worked = 0;
    for (;;) {
        uint32_t r = __sync_fetch_and_add(j->next, 1);
        if (r >= j->nrows) break;
        if (!worked && j->workers) __sync_fetch_and_add(j->workers, 1);
        worked = 1;
        uint32_t y = j->rows ? j->rows[r] : j->row0 + r;
        for (uint32_t x = 0; x < j->W; x++) {
            int lv = 0;
            V c;
            if (j->spp <= 1) {
                /* {X/Width, Y/Height}: float division of the integer pixel indices */
                c = trace_ray_through_pixel((double)x / (double)j->W, (double)y / (double)j->H, j->sc, j->depth,
                                            j->mode, &lv);
            } else {
                /* sample s at ((x+u)/W, (y+v)/H); the samples summed left to right, then / spp */
                const uint64_t pixel = (uint64_t)y * j->W + x;
                for (uint32_t s = 0; s < j->spp; s++) {
                    const uint64_t h = splitmix64(j->seed ^ (pixel * j->spp + s));
                    const double u = (double)(h >> 40) * 0x1p-24, v = (double)((h >> 16) & 0xFFFFFFull) * 0x1p-24;
                    int ls = 0;
                    const V cs = trace_ray_through_pixel(((double)x + u) / (double)j->W, ((double)y + v) / (double)j->H,
                                                         j->sc, j->depth, j->mode, &ls);
                    if (s == 0) {
                        c = cs;
                        lv = ls;
                    } else {
                        c.x = c.x + cs.x; c.y = c.y + cs.y; c.z = c.z + cs.z;
                    }
                }
                c.x = c.x / (double)j->spp; c.y = c.y / (double)j->spp; c.z = c.z / (double)j->spp;
            }
            size_t o = ((size_t)r * j->W + x);
            j->out[o * 3 + 0] = c.x; j->out[o * 3 + 1] = c.y; j->out[o * 3 + 2] = c.z;
            if (j->levels) j->levels[o] = (uint8_t)(lv > 255 ? 255 : lv); /* saturating, as rt_opts.out_levels */
        }
    }
    return NULL;
}

static void run_job(Job *job, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    for (int t = 1; t < threads; t++) pthread_create(&tid[t], NULL, worker, job);
    worker(job);
    for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
}

/* Render rows [row0, row0+nrows) of a W x H image into out (nrows*W*3 doubles), spp
 * samples per pixel (RT_SUPERSAMPLING; spp = 1 is the reference's pixel loop). */
int orc_render_spp(const rt_elem *scene, uint32_t n, uint32_t W, uint32_t H, uint32_t row0, uint32_t nrows,
                   int depth, int mode, int threads, uint32_t spp, uint64_t seed, double *out, uint8_t *levels) {
    if (n < 1 || scene[0].kind != RT_CAMERA) return RT_EBADARG;
    if (W == 0 || H == 0) return (W == 0 && H == 0) ? RT_DONE : RT_EBADARG;
    if (row0 + nrows > H) return RT_EBADARG;
    Scene sc = {scene, n};
    volatile uint32_t next = 0;
    Job job = {&sc, W, H, row0, nrows, depth, mode, out, levels, &next, spp ? spp : 1, seed, NULL, NULL};
    run_job(&job, threads);
    return RT_OK;
}

/* Render the listed rows rows[0..nrows) of a W x H image (out row i = image row rows[i]) on
 * `threads` threads, the rows shared out through one counter as in the `concurrent` strategy's
 * workers (raytracer.erl:101-119).  Returns the number of threads that rendered at least one
 * row (>= 1), or a negative RT_E* code. */
int orc_render_rows(const rt_elem *scene, uint32_t n, uint32_t W, uint32_t H, const uint32_t *rows, uint32_t nrows,
                    int depth, int mode, int threads, uint32_t spp, uint64_t seed, double *out, uint8_t *levels) {
    if (n < 1 || scene[0].kind != RT_CAMERA) return RT_EBADARG;
    if (W == 0 || H == 0 || rows == NULL || nrows == 0) return RT_EBADARG;
    for (uint32_t i = 0; i < nrows; i++)
        if (rows[i] >= H) return RT_EBADARG;
    Scene sc = {scene, n};
    volatile uint32_t next = 0, workers = 0;
    Job job = {&sc, W, H, 0, nrows, depth, mode, out, levels, &next, spp ? spp : 1, seed, rows, &workers};
    run_job(&job, threads);
    return (int)workers;
}

int orc_render(const rt_elem *scene, uint32_t n, uint32_t W, uint32_t H, uint32_t row0, uint32_t nrows,
               int depth, int mode, int threads, double *out, uint8_t *levels) {
    return orc_render_spp(scene, n, W, H, row0, nrows, depth, mode, threads, 1, 0, out, levels);
}
