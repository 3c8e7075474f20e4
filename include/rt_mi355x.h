/*
 * rt_mi355x.h — C-ABI boundary of the MI355X-native per-pixel render path.
 *
 * This library replaces the pixel loop of the reference ray tracer
 * (plouj/eraytracer, raytracer.erl).  The reference's strategy interface is
 *
 *     F(Width, Height, Scene, Recursion_depth) -> done | [{Key, {R,G,B}}]
 *
 * implemented by raytraced_pixel_list_simple/4      (raytracer.erl:86-99),
 *                raytraced_pixel_list_concurrent/4  (raytracer.erl:101-119),
 *                raytraced_pixel_list_distributed/4 (raytracer.erl:121-149),
 * chosen by tracing_function/1 (raytracer.erl:714-719) and called once by
 * raytrace/5 (raytracer.erl:723-733).  Every pixel runs
 * trace_ray_through_pixel/3 (raytracer.erl:180-184) and the shading /
 * intersection functions below it (raytracer.erl:186-511).
 *
 * The host (an erl_nif shim, a ctypes binding, a C++ program) marshals the
 * scene list (raytracer.erl:618-665 for the default one) into an array of
 * rt_elem records in LIST ORDER, element 0 being the camera, and calls
 * rt_render().  The result is the W*H*3 framebuffer in row-major order, i.e.
 * exactly the {R,G,B} values of the reference's list, in the list's order.
 * The keys are implied: simple uses key 1 for every pixel (raytracer.erl:95),
 * concurrent/distributed use X+Y*Width (raytracer.erl:112,173) and sort by it.
 *
 * All arithmetic is IEEE binary64 in the reference's operation order
 * (Erlang floats are doubles).  No pointer passed in is retained after a call
 * returns.  Every entry point returns 0 (RT_OK), RT_DONE, or a negative RT_E*
 * code; rt_strerror() names it.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 5

/* ---- return codes ------------------------------------------------------- */
#define RT_OK 0
#define RT_DONE 1          /* W = H = 0: the reference returns the atom `done` (raytracer.erl:86,101,121) */
#define RT_EBADARG (-1)    /* malformed scene / sizes: the reference crashes (function_clause, badrecord) */
#define RT_ENODEV (-2)     /* no HIP device, or device index out of range */
#define RT_EHIP (-3)       /* a HIP runtime call failed */
#define RT_ENOMEM (-4)     /* host or device allocation failed */
#define RT_ETOOBIG (-5)    /* a frame size, spp or shard count above its documented limit (RT_MAX_*) */
#define RT_ERANGE (-6)     /* rt_ppm_format: a channel below -2^31 after scaling (see there) */

/* No limit on the recursion depth or on the number of objects or lights: the reference recurses
 * to any depth (pixel_colour_from_ray/3, raytracer.erl:186-203), folds over every light
 * (lighting_function/6, :209-252) and scans any list (nearest_object_intersecting_ray/6,
 * :300-346).  Frames whose work space (per-level hit queues, ~100 bytes per pixel and level, in
 * row passes of at least 16 rows) or scene tables (32-bit offsets: about 16 doubles per
 * (origin, object) pair, the origins being the camera and every light) do not fit fail with
 * RT_ENOMEM.  out_levels saturates at 255. */

/* ---- scene records, mirroring the reference's records (raytracer.erl:72-81) -- */
enum rt_kind {
    RT_CAMERA = 0,      /* #camera{location, rotation, fov, screen}             :76 */
    RT_POINT_LIGHT = 1, /* #point_light{diffuse_colour, location, specular_colour} :81 */
    RT_SPHERE = 2,      /* #sphere{radius, center, material}                    :78 */
    RT_TRIANGLE = 3,    /* #triangle{v1, v2, v3, material}                      :79 */
    RT_PLANE = 4,       /* #plane{normal, distance, material}                   :80 */
    RT_OTHER = 5        /* any other term: ray_object_intersect/2 -> none (:357),
                           lighting_function skips it (:248) */
};

typedef struct rt_vec3 {
    double x, y, z; /* #vector{x, y, z} / #colour{r, g, b} (:72-73) */
} rt_vec3;

typedef struct rt_material { /* #material{colour, specular_power, shininess, reflectivity} (:77) */
    rt_vec3 colour;
    double specular_power;
    double shininess;
    double reflectivity;
} rt_material;

typedef struct rt_elem {
    int32_t kind;  /* enum rt_kind */
    /* canon: index (into this array) of the FIRST element that is exactly equal
     * (=:=, so 4 and 4.0 differ) to this one; shadow_factor/4 (raytracer.erl:
     * 256-267) lights a hit iff the nearest object seen from the light MATCHES
     * the hit object term, so duplicates count as the same object.  Pass -1 to
     * let the library decide by bitwise equality of kind and every field. */
    int32_t canon;
    union {
        struct { rt_vec3 location, rotation; double fov, screen_width, screen_height; } camera;
        struct { rt_vec3 diffuse_colour, location, specular_colour; } point_light;
        struct { double radius; rt_vec3 center; rt_material material; } sphere;
        struct { rt_vec3 v1, v2, v3; rt_material material; } triangle;
        struct { rt_vec3 normal; double distance; rt_material material; } plane;
        double raw[12];
    } u;
} rt_elem;

/* ---- options / statistics ---------------------------------------------------- */
#define RT_OUT_F64 0   /* out_rgb is double[H][W][3] (the reference's values, exact) */
#define RT_OUT_F32 1   /* out_rgb is float[H][W][3]  (the "float3 framebuffer") */

#define RT_ORDER_EXACT 0 /* reflection added once per light, reference fold order (bit-identical colour sums) */
#define RT_ORDER_FAST 1  /* forward-only reassociated accumulation (|delta| ~ 1e-15, same hit decisions) */

typedef struct rt_opts {
    uint32_t struct_size; /* sizeof(rt_opts); 0 or a NULL opts pointer selects every default */
    int32_t first_dev;    /* first HIP device (default 0) */
    int32_t ndev;         /* devices used by rt_render in this process (default 1; -1 = all visible).
                             Test hook: the environment variable RT_DEVICE_ALIAS=N (1..4, read once
                             per process) makes rt_render see N devices that are all first_dev; one
                             call then holds N of the device's 4 contexts, so the hook supports one
                             rt_render caller at a time (concurrent callers with N >= 3 can deadlock) */
    int32_t precision;    /* RT_OUT_F64 (default) or RT_OUT_F32 */
    int32_t order;        /* RT_ORDER_EXACT (default) or RT_ORDER_FAST */
    uint32_t row_block;   /* multi-device interleave granularity in rows (default 16) */
    uint8_t *out_levels;  /* optional host W*H bytes: reflection-chain levels that hit, per pixel */
    /* appended in ABI 2 (older callers' smaller struct_size leaves the defaults) */
    uint32_t spp;         /* samples per pixel (default 1 = the reference; see RT_SUPERSAMPLING) */
    uint32_t nshards;     /* rt_render: row shards (default 0 = one per device used); shard s runs on
                             device first_dev + s % ndev, so more shards than devices runs the
                             distributed strategy's split (raytracer.erl:121-149) on fewer GPUs */
    uint64_t seed;        /* jitter seed for spp > 1 */
    /* appended in ABI 4 */
    uint32_t flags;       /* RT_LEVELS_HIT: out_levels gets 1 where the pixel's primary ray hits an
                             object (depth > 0), 0 elsewhere, instead of the chain's level count —
                             all a host needs for the reference's integer {0,0,0} pixels, and it keeps
                             the fused shading kernels that a full level count turns off */
} rt_opts;
#define RT_LEVELS_HIT 1

/* RT_SUPERSAMPLING — stochastic supersampling (BASELINE.json config 5; the reference has
 * none, so this definition is the contract and the oracle restates it).  With spp > 1,
 * sample s (0 <= s < spp) of pixel (x, y), pixel = y*W + x in the whole image:
 *     r = splitmix64(seed ^ (pixel*spp + s)),
 *         splitmix64(z): z += 0x9E3779B97F4A7C15; z = (z ^ z>>30) * 0xBF58476D1CE4E5B9;
 *                        z = (z ^ z>>27) * 0x94D049BB133111EB; return z ^ z>>31;
 *     u = (r >> 40) * 2^-24,  v = ((r >> 16) & 0xFFFFFF) * 2^-24      (24-bit fractions)
 *     X = (x + u) / W,  Y = (y + v) / H                                 (binary64)
 * and the pixel is (c_0 + c_1 + ... + c_{spp-1}) / spp, summed left to right in binary64.
 * spp = 1 is the reference's X = x/W, Y = y/H exactly.  out_levels / d_levels report
 * sample 0 (its chain's level count, or with RT_LEVELS_HIT its primary-hit mask).
 * Levels count the objects a pixel's reflection chain hit (0 = background).  A scene without
 * point lights traces no reflections (the reference's fold over the lights never recurses,
 * raytracer.erl:209-252), so there a pixel's level is at most 1 with or without RT_LEVELS_HIT;
 * so it is at depth 1. */
#define RT_MAX_SPP 4096

typedef struct rt_stats {
    double kernel_ms;   /* device time of the render kernels (max over devices) */
    double total_ms;    /* wall time of the whole call, boundary to boundary */
    uint64_t pixels;    /* W*H */
    int32_t ndev;       /* devices actually used */
    int32_t flags;      /* bit 0: out_rgb was pinned host memory (written by DMA directly) */
} rt_stats;

/* ---- library / device ------------------------------------------------------------ */
int rt_abi_version(void);
const char *rt_strerror(int code);
int rt_device_count(int *count);

/* Diagnostic: the kernels' correctly rounded sqrt / division fast paths (rt_render.hip,
 * sqrt_n / div_n: the device library's sequences without their range handling, used only
 * where every operand of the wave is in range) against the library, bit for bit, on n random
 * operands; *mismatches = the count of differing results (0 expected). */
int rt_selftest_math(int device, uint64_t n, uint64_t seed, uint64_t *mismatches);

/* Validate a scene list without rendering (0 = a scene the reference would
 * trace without crashing for a pixel that hits any object). */
int rt_scene_check(const rt_elem *scene, uint32_t n_elems);

/* Fill canon[] for elems whose canon is -1 (bitwise-equality rule). */
int rt_scene_canon(rt_elem *scene, uint32_t n_elems);

/* ---- one-shot render: the drop-in for raytraced_pixel_list_{simple,concurrent,distributed} --
 * Replaces the whole pixel loop (raytracer.erl:86-178): for every pixel (x,y),
 * row-major, out = trace_ray_through_pixel({x/W, y/H}, Scene, Depth).
 * out_rgb: caller-owned host memory, W*H*3 elements of the chosen precision.
 * Returns RT_DONE for W = H = 0, RT_EBADARG if exactly one of them is 0.
 * The process keeps a pool of render contexts per device (streams, device frame buffers, the
 * wavefront work space, the last scene compiled — recompiled only when the scene's bytes
 * change), created on first use: the reference calls its strategy once per frame
 * (raytracer.erl:723-733), and repeated calls pay only the render and the copy.  The frame is
 * rendered in row bands whose copies to the host overlap the next band's render; memory from
 * rt_host_alloc (or registered with HIP) is written by DMA directly, other memory through a
 * pinned staging ring.  Thread-safe: concurrent callers get separate contexts (up to 4 per
 * device; more wait).  Device memory per context: the wavefront work space of the largest frame
 * it rendered (~5 GB at 4096^2 depth 5: 64-byte hit records per level and 16x16-tile slot,
 * colours, flags, lists; spp > 1 adds the binary64 sums, 24 B per pixel) plus its output
 * buffers (the frame, 201 MB at 4096^2 f32); it is kept while the context is idle.  An
 * allocation that fails while other contexts of the device are idle is retried once after their
 * memory is freed (a busy context's is never touched); rt_reset_contexts frees it all. */
int rt_render(const rt_elem *scene, uint32_t n_elems, uint32_t width, uint32_t height,
              uint32_t depth, const rt_opts *opts, void *out_rgb, rt_stats *stats);

/* Pinned (page-locked) host memory for rt_render's out_rgb: the frame is written by DMA
 * straight into it (a NIF can wrap it in a resource binary; the Python host uses it for its
 * frames).  rt_host_alloc returns NULL on failure.  Freed blocks are kept for reuse (up to 8
 * blocks / 4 GiB; a request reuses a block at most twice its size), so allocating one per
 * frame costs nothing after the first; rt_host_free of a pointer not from rt_host_alloc
 * returns RT_EBADARG. */
void *rt_host_alloc(size_t bytes);
int rt_host_free(void *p);
/* Free the idle render contexts of the process (device memory, streams) and the cached
 * pinned blocks; returns the number of contexts still in use by other threads.  The next
 * rt_render creates them again. */
int rt_reset_contexts(void);

/* ---- resident-scene API (device buffers, caller's HIP stream) -------------------
 * rt_prepare uploads the scene (and its per-origin constant tables) to one device.
 * rt_launch renders shard `shard` of `nshards` into device memory, asynchronously
 * on `stream` (a hipStream_t; NULL = the null stream).  Rows are dealt to shards
 * in interleaved blocks of `row_block` rows: global row g belongs to shard
 * (g / row_block) % nshards.  d_out receives the shard's rows packed in order,
 * rt_shard_rows(height,row_block,nshards) rows of width*3 elements; slab rows past
 * the image (the tail of the last row block) are not written, so with nshards = 1 a buffer
 * of `height` rows suffices.  d_levels (optional) gets one byte per slab pixel. */
typedef struct rt_prepared rt_prepared;

int rt_prepare(const rt_elem *scene, uint32_t n_elems, int device, rt_prepared **out);
uint32_t rt_shard_rows(uint32_t height, uint32_t row_block, uint32_t nshards);
int rt_launch(rt_prepared *p, uint32_t width, uint32_t height, uint32_t depth,
              uint32_t row_block, uint32_t shard, uint32_t nshards, int precision, int order,
              void *d_out, uint8_t *d_levels, void *stream);
/* rt_launch with spp samples per pixel (RT_SUPERSAMPLING); spp = 1 is rt_launch. */
int rt_launch_spp(rt_prepared *p, uint32_t width, uint32_t height, uint32_t depth,
                  uint32_t row_block, uint32_t shard, uint32_t nshards, int precision, int order,
                  uint32_t spp, uint64_t seed, void *d_out, uint8_t *d_levels, void *stream);
/* Reassemble nshards gathered slabs (d_slabs = [nshards][shard_rows][W*3]) into the
 * row-major image d_image ([H][W*3]), on `stream`. */
int rt_unshard(const void *d_slabs, uint32_t width, uint32_t height, uint32_t row_block,
               uint32_t nshards, int precision, void *d_image, void *stream);
int rt_release(rt_prepared *p);
/* Replace the scene of a prepared context in place (an animated scene: the next rt_launch renders
 * the new one): the scene is compiled and uploaded as by rt_prepare, the context's work space,
 * streams and options are kept.  No launch of p may be in flight (synchronise its stream first). */
int rt_update_scene(rt_prepared *p, const rt_elem *scene, uint32_t n_elems);
/* Per-context launch options.
 * RT_CFG_SIDE_STREAMS: 1 = a frame's shading runs on two low-priority side streams of the
 *   context beside its reflection chain (the fastest for ONE frame in flight); 0 = every
 *   kernel on the caller's stream (for callers that keep several frames in flight on
 *   their own streams, one context each: the frames then fill each other's latency-bound
 *   tails); -1 = the default (on, unless the environment sets RT_LIT_STREAM=0). */
#define RT_CFG_SIDE_STREAMS 1
/* RT_CFG_KERNEL_TIMING: value = a mask of RT_KT_* kernels; every later launch of those kernels
 *   by this context is bracketed by HIP timing events on the stream it runs on (0 = off, the
 *   default).  rt_kernel_time reports their summed duration and launch count (it waits for
 *   the events recorded so far).  Used by bench.py for the roofline of the dominant kernel. */
#define RT_CFG_KERNEL_TIMING 2
#define RT_KT_PRIMARY 1  /* k_primary: camera rays and their nearest scan (wavefront engine) */
#define RT_KT_LEVEL1 2   /* the level-0 shading + level-1 reflection pass (k_reflect_shade(1); with
                            side streams or levels: k_reflect(1)) */
#define RT_KT_RENDER 4   /* k_render: the fused engine's one kernel per frame */
#define RT_KT_PMASK 8    /* k_pmask: the primary rays' candidate masks, computed when the scene, the culling
                            mode or the frame geometry changes (the wavefront engine, culled scenes) */
/* RT_CFG_CULL: 1 = the default: scans skip objects a conservative filter proves cannot be hit
 *   (wave beams and shadow cones, per-light occluder masks, the sphere BVH); 0 = brute force,
 *   every nearest scan and every shadow test visits every object of the scene, as the
 *   reference's scans do (raytracer.erl:303-346, :256-267).  Both give the same bits; 0 exists
 *   to check that (it is many times slower). */
#define RT_CFG_CULL 3
int rt_configure(rt_prepared *p, int option, int64_t value);
/* Which engine rt_launch_spp runs for this context's scene at `spp` samples per pixel:
 * RT_ENGINE_WAVE (the wavefront kernels) or RT_ENGINE_FUSED (k_render, one kernel per frame);
 * negative on a bad argument.  bench.py names the dominant kernel from it. */
#define RT_ENGINE_WAVE 0
#define RT_ENGINE_FUSED 1
int rt_engine(rt_prepared *p, uint32_t spp);
int rt_kernel_time(rt_prepared *p, int kernel, double *total_ms, uint64_t *launches, int reset);
/* ---- compact slab transfer (the multi-GPU gather; raytracer.erl:151-161 collects pixels) --
 * A slab (as rt_launch writes it) is mostly background pixels, +0.0 in all three channels.
 * For the gather it is sent as a fixed-size header (count of non-zero pixels, u64 at byte
 * 0; per 256 slab pixels the non-zero pixels before them; one bit per slab pixel) plus
 * count*3 values of the slab's precision, the non-zero pixels in slab order.  The round trip
 * is exact (bit patterns are copied; a pixel is zero iff its three channels are all-zero
 * bits).  Slab rows past the image are not read and decode as zero.
 * rt_slab_header_bytes: header size for one shard of this frame (0 for bad arguments).
 * rt_slab_pack: encode shard `shard`'s slab on `stream`; d_values needs room for every slab
 *   pixel (shard_rows*width*3 elements) in the worst case.
 * rt_slab_unpack: decode nshards (<= RT_MAX_SHARDS) shards into the row-major image
 *   ([H][W*3]) on `stream` — rt_unshard fused with the decode; d_headers[s] / d_values[s]
 *   are device pointers to shard s's header and values. */
#define RT_MAX_SHARDS 64
size_t rt_slab_header_bytes(uint32_t width, uint32_t height, uint32_t row_block, uint32_t nshards);
int rt_slab_pack(const void *d_slab, uint32_t width, uint32_t height, uint32_t row_block, uint32_t shard,
                 uint32_t nshards, int precision, void *d_header, void *d_values, void *stream);
int rt_slab_unpack(const void *const *d_headers, const void *const *d_values, uint32_t width, uint32_t height,
                   uint32_t row_block, uint32_t nshards, int precision, void *d_image, void *stream);

/* ---- P3 output: write_pixels_to_ppm/5 (raytracer.erl:667-685) -----------------------
 * The file is "P3\nW H\nMaxValue\n" followed, for every pixel in row order, by
 * "R G B " where each channel is min(trunc(C*MaxValue), MaxValue) printed in decimal
 * (C*MaxValue in binary64; no lower clamp, so a negative colour prints a negative
 * number).  Byte-exact for RT_OUT_F64 frames; an RT_OUT_F32 frame is formatted from its
 * float values.
 * rt_ppm_bound: a byte count that always suffices for rt_ppm_format's output.
 * rt_ppm_format: formats a device frame (precision as rt_launch writes it) into the device
 *   buffer d_text (text_cap bytes) on `stream`, then synchronises it to report *text_len.
 *   RT_ERANGE if a channel is below -2^31 (BEAM prints such values as bignums; the file
 *   API below formats them on the host), RT_ETOOBIG if text_cap is too small.
 * rt_render_ppm_file: raytrace/5 without the strategy fun — render (opts as rt_render) and
 *   write the P3 file at `path`; the text is produced on the GPU. */
size_t rt_ppm_bound(uint32_t width, uint32_t height, uint32_t max_value);
int rt_ppm_format(const void *d_rgb, int precision, uint32_t width, uint32_t height, uint32_t max_value,
                  char *d_text, size_t text_cap, size_t *text_len, void *stream);
int rt_render_ppm_file(const rt_elem *scene, uint32_t n_elems, uint32_t width, uint32_t height,
                       uint32_t depth, const rt_opts *opts, uint32_t max_value, const char *path,
                       rt_stats *stats);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
