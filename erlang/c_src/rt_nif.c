/*
 * rt_nif.c — erl_nif shim between the reference's Erlang host (raytracer.erl) and the
 * MI355X render library (include/rt_mi355x.h, eraytracer_amd/librtmi355x.so).
 *
 * It replaces the pixel loop of raytraced_pixel_list_{simple,concurrent,distributed}/4
 * (raytracer.erl:86-178) with one call into the GPU library:
 *
 *   rt_nif:render(Width, Height, Scene, Depth, KeyMode) -> done | [{Key, {R,G,B}}]
 *       KeyMode = simple (every key 1, raytracer.erl:95) | indexed (X+Y*Width, :112, :173)
 *               | distributed (indexed keys, rows shared over every visible GPU, :121-149)
 *   rt_nif:render_binary(Width, Height, Scene, Depth) -> done | binary()   (W*H*3 native doubles)
 *
 * Runs on a dirty I/O scheduler (it blocks while the GPU renders).  The scene list is read
 * record by record (raytracer.erl:72-81) accepting an integer or a float in every numeric
 * slot; exact equality (=:=) between list elements, which shadow_factor/4's match relies on
 * (raytracer.erl:263), is decided here with enif_is_identical and passed down as rt_elem.canon.
 * A malformed scene raises badarg instead of crashing a worker later.
 *
 * Build (needs erl_nif.h, i.e. an Erlang/OTP install; see erlang/Makefile and INTEGRATION.md):
 *   cc -O2 -fPIC -shared -I$ERL_ROOT/usr/include -I../../include rt_nif.c \
 *      -L../../eraytracer_amd -lrtmi355x -Wl,-rpath,'$ORIGIN' -o ../priv/rt_nif.so
 */
#include <erl_nif.h>
#include <string.h>

#include "rt_mi355x.h"

static ERL_NIF_TERM atom_done, atom_simple, atom_indexed, atom_distributed, atom_error;

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)info;
    atom_done = enif_make_atom(env, "done");
    atom_simple = enif_make_atom(env, "simple");
    atom_indexed = enif_make_atom(env, "indexed");
    atom_distributed = enif_make_atom(env, "distributed");
    atom_error = enif_make_atom(env, "error");
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

/* Scene list -> rt_elem array (enif_alloc'd), canon by exact equality.  0 on badarg. */
static int marshal_scene(ErlNifEnv *env, ERL_NIF_TERM list, rt_elem **elems, ERL_NIF_TERM **terms,
                         unsigned *n_out) {
    unsigned n, i = 0;
    ERL_NIF_TERM head, tail = list;
    if (!enif_get_list_length(env, list, &n) || n == 0) return 0;
    *elems = enif_alloc(n * sizeof(rt_elem));
    *terms = enif_alloc(n * sizeof(ERL_NIF_TERM));
    while (enif_get_list_cell(env, tail, &head, &tail)) {
        (*terms)[i] = head;
        if (!marshal_elem(env, head, &(*elems)[i], i == 0)) return 0;
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

/* shared front half: parse args, render into a double buffer */
static ERL_NIF_TERM render_common(ErlNifEnv *env, const ERL_NIF_TERM argv[], unsigned *W, unsigned *H,
                                  double **buf, int *done, int all_devices, unsigned spp, ErlNifUInt64 seed) {
    unsigned D, n = 0;
    rt_elem *elems = NULL;
    ERL_NIF_TERM *terms = NULL, err = 0;
    int rc;
    *done = 0;
    *buf = NULL;
    if (!enif_get_uint(env, argv[0], W) || !enif_get_uint(env, argv[1], H) || !enif_get_uint(env, argv[3], &D))
        return enif_make_badarg(env);
    if (*W == 0 && *H == 0) {
        *done = 1;
        return atom_done;
    }
    if (*W == 0 || *H == 0) return enif_make_badarg(env); /* function_clause in the reference */
    if (!marshal_scene(env, argv[2], &elems, &terms, &n)) {
        err = enif_make_badarg(env);
        goto out;
    }
    *buf = enif_alloc((size_t)*W * *H * 3 * sizeof(double));
    if (!*buf) {
        err = enif_raise_exception(env, enif_make_atom(env, "enomem"));
        goto out;
    }
    rt_opts o;
    memset(&o, 0, sizeof o);
    o.struct_size = sizeof o;
    o.ndev = all_devices ? -1 : 1;
    o.precision = RT_OUT_F64;
    o.order = RT_ORDER_EXACT;
    o.row_block = 16;
    o.spp = spp;   /* RT_SUPERSAMPLING (include/rt_mi355x.h); 1 = the reference's pixel */
    o.seed = seed;
    rc = rt_render(elems, n, *W, *H, D, &o, *buf, NULL);
    if (rc < 0) {
        enif_free(*buf);
        *buf = NULL;
        err = rt_error(env, rc);
    }
out:
    if (elems) enif_free(elems);
    if (terms) enif_free(terms);
    return err;
}

/* render(W, H, Scene, Depth, KeyMode) -> [{Key, {R,G,B}}] in row-major order */
static ERL_NIF_TERM render_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned W, H;
    double *buf;
    int done, keyed, all = 0;
    (void)argc;
    if (enif_is_identical(argv[4], atom_simple)) keyed = 0;
    else if (enif_is_identical(argv[4], atom_indexed)) keyed = 1;
    else if (enif_is_identical(argv[4], atom_distributed)) keyed = all = 1;
    else return enif_make_badarg(env);
    ERL_NIF_TERM r = render_common(env, argv, &W, &H, &buf, &done, all, 1, 0);
    if (done || !buf) return r;
    ERL_NIF_TERM list = enif_make_list(env, 0), one = enif_make_int(env, 1);
    for (size_t i = (size_t)W * H; i-- > 0;) {
        const double *p = buf + 3 * i;
        ERL_NIF_TERM rgb = enif_make_tuple3(env, enif_make_double(env, p[0]), enif_make_double(env, p[1]),
                                            enif_make_double(env, p[2]));
        ERL_NIF_TERM key = keyed ? enif_make_uint64(env, i) : one;
        list = enif_make_list_cell(env, enif_make_tuple2(env, key, rgb), list);
    }
    enif_free(buf);
    return list;
}

/* render_binary(W, H, Scene, Depth) -> <<R:64/float-native, G, B, ...>> row-major
 * render_binary(W, H, Scene, Depth, #{spp => N, seed => S}) -> the same, supersampled */
static ERL_NIF_TERM render_binary_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned W, H, spp = 1;
    ErlNifUInt64 seed = 0;
    double *buf;
    int done;
    ErlNifBinary bin;
    if (argc == 5) {
        ERL_NIF_TERM v;
        if (!enif_is_map(env, argv[4])) return enif_make_badarg(env);
        if (enif_get_map_value(env, argv[4], enif_make_atom(env, "spp"), &v) && !enif_get_uint(env, v, &spp))
            return enif_make_badarg(env);
        if (enif_get_map_value(env, argv[4], enif_make_atom(env, "seed"), &v) && !enif_get_uint64(env, v, &seed))
            return enif_make_badarg(env);
        if (spp == 0) return enif_make_badarg(env);
    }
    ERL_NIF_TERM r = render_common(env, argv, &W, &H, &buf, &done, 0, spp, seed);
    if (done || !buf) return r;
    size_t nb = (size_t)W * H * 3 * sizeof(double);
    if (!enif_alloc_binary(nb, &bin)) {
        enif_free(buf);
        return enif_raise_exception(env, enif_make_atom(env, "enomem"));
    }
    memcpy(bin.data, buf, nb);
    enif_free(buf);
    return enif_make_binary(env, &bin);
}

/* render_ppm_file(W, H, Scene, Depth, Filename) -> ok | done: raytrace/5's render and
 * write_pixels_to_ppm/5 (MaxValue 255) in one call; the P3 text is made on the GPU. */
static ERL_NIF_TERM render_ppm_file_nif(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned W, H, D, n = 0;
    char path[4096];
    rt_elem *elems = NULL;
    ERL_NIF_TERM *terms = NULL, ret;
    (void)argc;
    if (!enif_get_uint(env, argv[0], &W) || !enif_get_uint(env, argv[1], &H) || !enif_get_uint(env, argv[3], &D))
        return enif_make_badarg(env);
    if (enif_get_string(env, argv[4], path, sizeof path, ERL_NIF_LATIN1) <= 0) return enif_make_badarg(env);
    if (W == 0 && H == 0) return atom_done;
    if (W == 0 || H == 0) return enif_make_badarg(env);
    if (!marshal_scene(env, argv[2], &elems, &terms, &n)) {
        ret = enif_make_badarg(env);
    } else {
        int rc = rt_render_ppm_file(elems, n, W, H, D, NULL, 255, path, NULL);
        ret = rc == RT_OK ? enif_make_atom(env, "ok") : rt_error(env, rc);
    }
    if (elems) enif_free(elems);
    if (terms) enif_free(terms);
    return ret;
}

static ErlNifFunc funcs[] = {
    {"render", 5, render_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"render_binary", 4, render_binary_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"render_binary", 5, render_binary_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"render_ppm_file", 5, render_ppm_file_nif, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

ERL_NIF_INIT(rt_nif, funcs, load, NULL, NULL, NULL)
