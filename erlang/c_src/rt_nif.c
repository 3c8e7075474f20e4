/*
 * rt_nif.c — erl_nif shim between the reference's Erlang host (raytracer.erl) and the
 * MI355X render library (include/rt_mi355x.h, eraytracer_amd/librtmi355x.so).
 *
 * It replaces the pixel loop of raytraced_pixel_list_{simple,concurrent,distributed}/4
 * (raytracer.erl:86-178) with one call into the GPU library, and hands the frame back in
 * pieces the BEAM can take without one multi-million-element build:
 *
 *   rt_nif:render_frame(Width, Height, Scene, Depth, Opts) -> done | Frame
 *       Opts = #{spp => N, seed => S, devices => all | N}; dirty I/O scheduler.
 *       Frame = {rt_frame, Width, Height, Rgb, Levels, Mode}: Rgb is W*H*3 native-endian
 *       doubles, row-major, in pinned host memory (written by DMA; a resource binary);
 *       Mode says which pixels are the integer triple {0,0,0} (see below): true = those whose
 *       primary ray hits nothing (Levels: one byte per pixel, 0 there), false = every pixel
 *       (no #point_light{} in the scene; Levels is empty), floats = none (spp > 1, a
 *       supersampled frame, which the reference does not have: every pixel is an average of
 *       jittered samples, so always three floats; Levels is empty).
 *   rt_nif:pixels_chunk(Frame, Start, Count, KeyMode, Tail) -> [{Key, {R,G,B}} | Tail]
 *       pixels Start .. Start+Count-1 as the reference's list elements, consed onto Tail
 *       (KeyMode = simple: key 1, raytracer.erl:95 | indexed: X+Y*Width, :112, :173).  A normal
 *       scheduler call of bounded work: Count is at most PIXELS_CHUNK_MAX (4096 pixels, about
 *       20k terms, well under the 1 ms a normal-scheduler NIF may take), and it reports the
 *       share of its timeslice it used (enif_consume_timeslice).  raytracer_gpu builds the whole
 *       list from the end in chunks, or folds over it chunk by chunk (raytracer_gpu:fold_pixels/4).
 *   rt_nif:render_binary(Width, Height, Scene, Depth[, Opts]) -> done | binary()
 *   rt_nif:render_ppm_file(Width, Height, Scene, Depth, Filename) -> ok | done
 *
 * Term types follow the reference exactly: a pixel whose reference value is the integer
 * triple #colour{r=0,g=0,b=0} — no primary hit (?BACKGROUND_COLOUR, raytracer.erl:82, :201),
 * depth 0 (pixel_colour_from_ray/3 clause 1, :186-187), or no point light in the scene
 * (lighting_function/6 folds from #vector{0,0,0}, :250) — is returned as {0,0,0}; every other
 * pixel as three floats (specular_term's math:pow/2 always yields a float, :289).  The
 * primary-hit mask comes from rt_render's RT_LEVELS_HIT mode (rt_opts.flags), which keeps the
 * fused wavefront kernels that a full level count would turn off.
 *
 * The scene list is read record by record (raytracer.erl:72-81) accepting an integer or a
 * float in every numeric slot; exact equality (=:=) between list elements, which
 * shadow_factor/4's match relies on (raytracer.erl:263), is decided here with
 * enif_is_identical and passed down as rt_elem.canon.  A malformed scene raises badarg
 * instead of crashing a worker later.
 *
 * Build (needs erl_nif.h, i.e. an Erlang/OTP install; see erlang/Makefile and INTEGRATION.md):
 *   cc -O2 -fPIC -shared -I$ERL_ROOT/usr/include -I../../include rt_nif.c \
 *      -L../../eraytracer_amd -lrtmi355x -Wl,-rpath,'$ORIGIN' -o ../priv/rt_nif.so
 */
#include <erl_nif.h>
#include <string.h>

#include "rt_mi355x.h"

static ERL_NIF_TERM atom_done, atom_simple, atom_indexed, atom_error, atom_rt_frame, atom_true, atom_false,
    atom_floats, atom_spp, atom_seed, atom_devices, atom_all, atom_ok, atom_enomem;
static ErlNifResourceType *pinned_type;

/* a block of pinned host memory (rt_host_alloc) owned by the resource binaries made from it */
typedef struct {
    void *p;
    size_t n;
} pinned_buf;

static void pinned_dtor(ErlNifEnv *env, void *obj) {
    (void)env;
    pinned_buf *b = (pinned_buf *)obj;
    if (b->p) rt_host_free(b->p);
    b->p = NULL;
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)info;
    atom_done = enif_make_atom(env, "done");
    atom_simple = enif_make_atom(env, "simple");
    atom_indexed = enif_make_atom(env, "indexed");
    atom_error = enif_make_atom(env, "error");
    atom_rt_frame = enif_make_atom(env, "rt_frame");
    atom_true = enif_make_atom(env, "true");
    atom_false = enif_make_atom(env, "false");
    atom_floats = enif_make_atom(env, "floats");
    atom_spp = enif_make_atom(env, "spp");
    atom_seed = enif_make_atom(env, "seed");
    atom_devices = enif_make_atom(env, "devices");
    atom_all = enif_make_atom(env, "all");
    atom_ok = enif_make_atom(env, "ok");
    atom_enomem = enif_make_atom(env, "enomem");
    pinned_type = enif_open_resource_type(env, NULL, "rt_pinned", pinned_dtor, ERL_NIF_RT_CREATE, NULL);
    if (!pinned_type) return 1;
    return rt_abi_version() == RT_ABI_VERSION ? 0 : 1;
}

/* an Erlang number (int or float) as a double; ints beyond 2^53 are not exact: refuse */
static int get_num(ErlNifEnv *env, ERL_NIF_TERM t, double *out) {
    ErlNifSInt64 i;
    if (enif_get_double(env, t, out)) return 1;
    if (enif_get_int64(env, t, &i)) {
        if (i > (1LL << 53) || i < -(1LL << 53)) return 0;
        *out = (double)i;
        return 1;
    }
    return 0;
}

/* {Tag, ...} with the given arity (tag included) */
static int get_rec(ErlNifEnv *env, ERL_NIF_TERM t, const char *tag, int arity, const ERL_NIF_TERM **el) {
    int n;
    char a[16];
    if (!enif_get_tuple(env, t, &n, el) || n != arity) return 0;
    if (!enif_get_atom(env, (*el)[0], a, sizeof a, ERL_NIF_LATIN1)) return 0;
    return strcmp(a, tag) == 0;
}

/* #vector{x,y,z} or #colour{r,g,b} */
static int get_vec(ErlNifEnv *env, ERL_NIF_TERM t, const char *tag, rt_vec3 *v) {
    const ERL_NIF_TERM *e;
    return get_rec(env, t, tag, 4, &e) && get_num(env, e[1], &v->x) && get_num(env, e[2], &v->y) &&
           get_num(env, e[3], &v->z);
}

static int get_material(ErlNifEnv *env, ERL_NIF_TERM t, rt_material *m) {
    const ERL_NIF_TERM *e;
    return get_rec(env, t, "material", 5, &e) && get_vec(env, e[1], "colour", &m->colour) &&
           get_num(env, e[2], &m->specular_power) && get_num(env, e[3], &m->shininess) &&
           get_num(env, e[4], &m->reflectivity);
}

/* one scene element -> rt_elem; unknown terms become RT_OTHER (ignored, as the reference does) */
static int marshal_elem(ErlNifEnv *env, ERL_NIF_TERM t, rt_elem *out, int head) {
    const ERL_NIF_TERM *e;
    memset(out, 0, sizeof *out);
    if (get_rec(env, t, "camera", 5, &e)) {
        const ERL_NIF_TERM *s;
        out->kind = RT_CAMERA;
        if (!get_vec(env, e[1], "vector", &out->u.camera.location)) return 0;
        (void)get_vec(env, e[2], "vector", &out->u.camera.rotation); /* never read (:487) */
        if (!get_num(env, e[3], &out->u.camera.fov)) return 0;
        if (!get_rec(env, e[4], "screen", 3, &s)) return 0;
        return get_num(env, s[1], &out->u.camera.screen_width) && get_num(env, s[2], &out->u.camera.screen_height);
    }
    if (head) return 0; /* [Camera|Rest] (raytracer.erl:180) */
    if (get_rec(env, t, "point_light", 4, &e)) {
        out->kind = RT_POINT_LIGHT;
        return get_vec(env, e[1], "colour", &out->u.point_light.diffuse_colour) &&
               get_vec(env, e[2], "vector", &out->u.point_light.location) &&
               get_vec(env, e[3], "colour", &out->u.point_light.specular_colour);
    }
    if (get_rec(env, t, "sphere", 4, &e)) {
        out->kind = RT_SPHERE;
        return get_num(env, e[1], &out->u.sphere.radius) && get_vec(env, e[2], "vector", &out->u.sphere.center) &&
               get_material(env, e[3], &out->u.sphere.material);
    }
    if (get_rec(env, t, "triangle", 5, &e)) {
        out->kind = RT_TRIANGLE;
        return get_vec(env, e[1], "vector", &out->u.triangle.v1) && get_vec(env, e[2], "vector", &out->u.triangle.v2) &&
               get_vec(env, e[3], "vector", &out->u.triangle.v3) && get_material(env, e[4], &out->u.triangle.material);
    }
    if (get_rec(env, t, "plane", 4, &e)) {
        out->kind = RT_PLANE;
        return get_vec(env, e[1], "vector", &out->u.plane.normal) && get_num(env, e[2], &out->u.plane.distance) &&
               get_material(env, e[3], &out->u.plane.material);
    }
    out->kind = RT_OTHER;
    return 1;
}

/* Scene list -> rt_elem array (enif_alloc'd), canon by exact equality.  0 on badarg; the
 * arrays are freed by the caller in every case. */
static int marshal_scene(ErlNifEnv *env, ERL_NIF_TERM list, rt_elem **elems, ERL_NIF_TERM **terms,
                         unsigned *n_out, int *lights) {
    unsigned n, i = 0;
    ERL_NIF_TERM head, tail = list;
    *elems = NULL;
    *terms = NULL;
    *lights = 0;
    if (!enif_get_list_length(env, list, &n) || n == 0) return 0;
    *elems = enif_alloc(n * sizeof(rt_elem));
    *terms = enif_alloc(n * sizeof(ERL_NIF_TERM));
    if (!*elems || !*terms) return 0;
    while (enif_get_list_cell(env, tail, &head, &tail)) {
        (*terms)[i] = head;
        if (!marshal_elem(env, head, &(*elems)[i], i == 0)) return 0;
        if ((*elems)[i].kind == RT_POINT_LIGHT) *lights = 1;
        (*elems)[i].canon = (int32_t)i;
        for (unsigned j = 0; j < i; j++) {
            if ((*elems)[j].canon == (int32_t)j && enif_is_identical((*terms)[j], head)) {
                (*elems)[i].canon = (int32_t)j;
                break;
            }
        }
        i++;
    }
    *n_out = n;
    return 1;
}

static ERL_NIF_TERM rt_error(ErlNifEnv *env, int rc) {
    return enif_raise_exception(
        env, enif_make_tuple2(env, atom_error, enif_make_string(env, rt_strerror(rc), ERL_NIF_LATIN1)));
}

/* W*H*3 doubles in pinned memory as a resource binary (falls back to a plain binary) */
static int frame_binary(ErlNifEnv *env, size_t bytes, void **data, ERL_NIF_TERM *bin) {
    pinned_buf *b = enif_alloc_resource(pinned_type, sizeof(pinned_buf));
    if (!b) return 0;
    b->n = bytes;
    b->p = rt_host_alloc(bytes);
    if (b->p) {
        *data = b->p;
        *bin = enif_make_resource_binary(env, b, b->p, bytes);
        enif_release_resource(b); /* the binary keeps it */
        return 1;
    }
    enif_release_resource(b);
    ErlNifBinary eb;
    if (!enif_alloc_binary(bytes, &eb)) return 0;
    *data = eb.data;
    *bin = enif_make_binary(env, &eb);
    return 1;
}

/* Opts map: spp, seed, devices (all | N) */
static int get_opts(ErlNifEnv *env, ERL_NIF_TERM m, unsigned *spp, ErlNifUInt64 *seed, int *ndev) {
    ERL_NIF_TERM v;
    *spp = 1;
    *seed = 0;
    *ndev = 1;
    if (!enif_is_map(env, m)) return 0;
    if (enif_get_map_value(env, m, atom_spp, &v) && (!enif_get_uint(env, v, spp) || *spp == 0)) return 0;
    if (enif_get_map_value(env, m, atom_seed, &v) && !enif_get_uint64(env, v, seed)) return 0;
    if (enif_get_map_value(env, m, atom_devices, &v)) {
        if (enif_is_identical(v, atom_all))
            *ndev = -1;
        else if (!enif_get_int(env, v, ndev) || *ndev <= 0)
            return 0;
    }
    return 1;
}

/* Parse (W, H, Scene, Depth), render into *rgb (a new binary) and *lv (levels, optional).
 * Returns 0 with *ret set (done, badarg or an exception) when there is nothing more to do. */
static int render_common(ErlNifEnv *env, const ERL_NIF_TERM argv[], unsigned spp, ErlNifUInt64 seed, int ndev,
                         int want_levels, unsigned *W, unsigned *H, ERL_NIF_TERM *rgb, ERL_NIF_TERM *lv,
                         int *lights, ERL_NIF_TERM *ret) {
    unsigned D, n = 0;
    rt_elem *elems = NULL;
    ERL_NIF_TERM *terms = NULL;
    void *data = NULL;
    ErlNifBinary lvb;
    int ok = 0, have_lv = 0;
    if (!enif_get_uint(env, argv[0], W) || !enif_get_uint(env, argv[1], H) || !enif_get_uint(env, argv[3], &D)) {
        *ret = enif_make_badarg(env);
        return 0;
    }
    if (*W == 0 && *H == 0) {
        *ret = atom_done;
        return 0;
    }
    if (*W == 0 || *H == 0) { /* function_clause in the reference */
        *ret = enif_make_badarg(env);
        return 0;
    }
    if (!marshal_scene(env, argv[2], &elems, &terms, &n, lights)) {
        *ret = enif_make_badarg(env);
        goto out;
    }
    if (!frame_binary(env, (size_t)*W * *H * 3 * sizeof(double), &data, rgb)) {
        *ret = enif_raise_exception(env, atom_enomem);
        goto out;
    }
    /* the primary-hit mask, only where it decides a term type: spp = 1 and a lit scene */
    want_levels = want_levels && spp == 1 && *lights;
    if (!want_levels) (void)enif_make_new_binary(env, 0, lv); /* an empty Levels binary */
    if (want_levels) {
        if (!enif_alloc_binary((size_t)*W * *H, &lvb)) {
            *ret = enif_raise_exception(env, atom_enomem);
            goto out;
        }
        have_lv = 1;
    }
    rt_opts o;
    memset(&o, 0, sizeof o);
    o.struct_size = sizeof o;
    o.ndev = ndev;
    o.precision = RT_OUT_F64;
    o.order = RT_ORDER_EXACT;
    o.row_block = 16;
    o.out_levels = have_lv ? lvb.data : NULL;
    o.flags = RT_LEVELS_HIT; /* a hit mask, not level counts: the fused kernels stay on */
    o.spp = spp; /* RT_SUPERSAMPLING (include/rt_mi355x.h); 1 = the reference's pixel */
    o.seed = seed;
    int rc = rt_render(elems, n, *W, *H, D, &o, data, NULL);
    if (rc < 0) {
        *ret = rt_error(env, rc);
        goto out;
    }
    if (have_lv) {
        *lv = enif_make_binary(env, &lvb);
        have_lv = 0;
    }
    ok = 1;
out:
    if (have_lv) enif_release_binary(&lvb);
    if (elems) enif_free(elems);
    if (terms) enif_free(terms);
    return ok;
}

/* render_frame(W, H, Scene, Depth, Opts) -> done | {rt_frame, W, H, Rgb, Levels, Lights} */
static ERL_NIF_TERM render_frame_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned W, H, spp;
    ErlNifUInt64 seed;
    int ndev, lights;
    ERL_NIF_TERM rgb, lv, ret;
    (void)argc;
    if (!get_opts(env, argv[4], &spp, &seed, &ndev)) return enif_make_badarg(env);
    if (!render_common(env, argv, spp, seed, ndev, 1, &W, &H, &rgb, &lv, &lights, &ret)) return ret;
    ERL_NIF_TERM t[6] = {atom_rt_frame, enif_make_uint(env, W), enif_make_uint(env, H), rgb, lv,
                         spp > 1 ? atom_floats : lights ? atom_true : atom_false};
    return enif_make_tuple_from_array(env, t, 6);
}

/* pixels_chunk(Frame, Start, Count, KeyMode, Tail) -> [{Key, {R,G,B}} | Tail] */
#define PIXELS_CHUNK_MAX 4096
static ERL_NIF_TERM pixels_chunk_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    const ERL_NIF_TERM *f;
    int arity, keyed;
    unsigned W, H;
    ErlNifUInt64 start, count;
    ErlNifBinary rgb, lv;
    (void)argc;
    if (!enif_get_tuple(env, argv[0], &arity, &f) || arity != 6 || !enif_is_identical(f[0], atom_rt_frame) ||
        !enif_get_uint(env, f[1], &W) || !enif_get_uint(env, f[2], &H) || !enif_inspect_binary(env, f[3], &rgb) ||
        !enif_inspect_binary(env, f[4], &lv))
        return enif_make_badarg(env);
    /* mode: true = {0,0,0} where the primary ray misses, false = everywhere, floats = nowhere */
    const int by_hit = enif_is_identical(f[5], atom_true), floats = enif_is_identical(f[5], atom_floats);
    if (!by_hit && !floats && !enif_is_identical(f[5], atom_false)) return enif_make_badarg(env);
    const ErlNifUInt64 npx = (ErlNifUInt64)W * H;
    if (rgb.size != npx * 3 * sizeof(double) || lv.size != (by_hit ? npx : 0)) return enif_make_badarg(env);
    if (!enif_get_uint64(env, argv[1], &start) || !enif_get_uint64(env, argv[2], &count) || start > npx ||
        count > npx - start || count > PIXELS_CHUNK_MAX)
        return enif_make_badarg(env);
    if (enif_is_identical(argv[3], atom_simple)) keyed = 0;
    else if (enif_is_identical(argv[3], atom_indexed)) keyed = 1;
    else return enif_make_badarg(env);
    if (!enif_is_list(env, argv[4])) return enif_make_badarg(env);
    const double *px = (const double *)rgb.data;
    ERL_NIF_TERM list = argv[4], one = enif_make_int(env, 1), zero = enif_make_int(env, 0);
    ERL_NIF_TERM ints = enif_make_tuple3(env, zero, zero, zero);
    for (ErlNifUInt64 i = start + count; i-- > start;) {
        ERL_NIF_TERM c;
        if (!floats && (!by_hit || lv.data[i] == 0)) {
            c = ints;
        } else {
            const double *p = px + 3 * i;
            c = enif_make_tuple3(env, enif_make_double(env, p[0]), enif_make_double(env, p[1]),
                                 enif_make_double(env, p[2]));
        }
        list = enif_make_list_cell(env, enif_make_tuple2(env, keyed ? enif_make_uint64(env, i) : one, c), list);
    }
    /* the share of a 1 ms timeslice this call used (~PIXELS_CHUNK_MAX pixels per slice) */
    int pct = (int)(count * 100 / PIXELS_CHUNK_MAX);
    (void)enif_consume_timeslice(env, pct < 1 ? 1 : pct > 100 ? 100 : pct);
    return list;
}

/* render_binary(W, H, Scene, Depth[, Opts]) -> <<R:64/float-native, G, B, ...>> row-major */
static ERL_NIF_TERM render_binary_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned W, H, spp = 1;
    ErlNifUInt64 seed = 0;
    int ndev = 1, lights;
    ERL_NIF_TERM rgb, lv, ret;
    if (argc == 5 && !get_opts(env, argv[4], &spp, &seed, &ndev)) return enif_make_badarg(env);
    if (!render_common(env, argv, spp, seed, ndev, 0, &W, &H, &rgb, &lv, &lights, &ret)) return ret;
    return rgb;
}

/* render_ppm_file(W, H, Scene, Depth, Filename) -> ok | done: raytrace/5's render and
 * write_pixels_to_ppm/5 (MaxValue 255) in one call; the P3 text is made on the GPU. */
static ERL_NIF_TERM render_ppm_file_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned W, H, D, n = 0;
    int lights;
    char path[4096];
    rt_elem *elems = NULL;
    ERL_NIF_TERM *terms = NULL, ret;
    (void)argc;
    if (!enif_get_uint(env, argv[0], &W) || !enif_get_uint(env, argv[1], &H) || !enif_get_uint(env, argv[3], &D))
        return enif_make_badarg(env);
    if (enif_get_string(env, argv[4], path, sizeof path, ERL_NIF_LATIN1) <= 0) return enif_make_badarg(env);
    if (W == 0 && H == 0) return atom_done;
    if (W == 0 || H == 0) return enif_make_badarg(env);
    if (!marshal_scene(env, argv[2], &elems, &terms, &n, &lights)) {
        ret = enif_make_badarg(env);
    } else {
        int rc = rt_render_ppm_file(elems, n, W, H, D, NULL, 255, path, NULL);
        ret = rc == RT_OK ? atom_ok : rt_error(env, rc);
    }
    if (elems) enif_free(elems);
    if (terms) enif_free(terms);
    return ret;
}

static ErlNifFunc funcs[] = {
    {"render_frame", 5, render_frame_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"pixels_chunk", 5, pixels_chunk_nif, 0},
    {"render_binary", 4, render_binary_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"render_binary", 5, render_binary_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"render_ppm_file", 5, render_ppm_file_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

ERL_NIF_INIT(rt_nif, funcs, load, NULL, NULL, NULL)
