// rt_host.hip — the host side of the boundary: the process's render contexts and rt_render,
// the one-shot drop-in for raytraced_pixel_list_{simple,concurrent,distributed}/4
// (raytracer.erl:86-178).
//
// The reference calls its strategy fun once per frame (raytrace/5, raytracer.erl:723-733), so
// what a call costs besides the kernels matters: compiling and uploading the scene, allocating
// the device frame and the wavefront work space (GBs at 4096^2), and moving the frame to the
// caller's host memory.  Here:
//  * contexts persist for the life of the process (per device, up to RT_CTX_PER_DEVICE
//    concurrent callers): streams, events, device buffers and work space are created once and
//    grown on demand; the scene is recompiled only when its bytes change;
//  * the frame is rendered in row bands, and each band's copy to the host runs on a second
//    stream while the next band renders;
//  * a pinned destination (rt_host_alloc, or memory the caller registered with HIP) is written
//    by DMA directly; a pageable one goes through a pinned staging ring of two bands, copied
//    out by host threads while the next band's DMA is in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_internal.h"
#include "rt_scene.h"

namespace {

constexpr int RT_CTX_PER_DEVICE = 4;
constexpr int MAX_BANDS = 64;
// target output bytes per band (RT_BAND_MB overrides, for A/B runs)
size_t band_bytes() {
    static const size_t b = [] {
        const char *e = std::getenv("RT_BAND_MB");
        const long v = e ? std::atol(e) : 24;
        return (size_t)(v > 0 ? v : 24) << 20;
    }();
    return b;
}
// Test hook: RT_DEVICE_ALIAS=N makes rt_render see N devices that are all device first_dev, so
// its multi-device path (a context, work space and band pipeline per device, every device's
// slabs scattered into the one frame) runs on a one-GPU machine (0, the default: off)
int device_alias() {
    static const int n = [] {
        const char *e = std::getenv("RT_DEVICE_ALIAS");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 && v <= RT_CTX_PER_DEVICE ? v : 0;
    }();
    return n;
}
// DMA queues a pinned frame's band copies alternate over (RT_COPY_STREAMS = 1, the default, or 2)
int copy_streams() {
    static const int n = [] {
        const char *e = std::getenv("RT_COPY_STREAMS");
        return e && std::atoi(e) == 2 ? 2 : 1;
    }();
    return n;
}
// the contexts' shading side streams: off (RT_CTX_SIDE_STREAMS=1 turns them on, for A/B runs)
int side_streams_env() {
    static const int v = [] {
        const char *e = std::getenv("RT_CTX_SIDE_STREAMS");
        return e && std::strcmp(e, "1") == 0 ? 1 : 0;
    }();
    return v;
}

} // namespace

struct rt_ctx {
    int device = -1;
    bool busy = false;
    hipStream_t render = nullptr, copy = nullptr, copy2 = nullptr; // copy2: a second DMA queue for pinned frames
    hipEvent_t e0 = nullptr, e1 = nullptr;      // timing: around the render launches
    hipEvent_t band[MAX_BANDS] = {};             // band i rendered
    hipEvent_t copied[MAX_BANDS] = {};           // band i copied to the host (staging or pinned)
    rt_prepared *p = nullptr;
    std::vector<unsigned char> key;              // bytes of the scene p was prepared from
    void *d_buf[3] = {};
    size_t d_cap[3] = {};
    void *h_stage = nullptr;
    size_t h_cap = 0;
};

namespace {

std::mutex g_mu;
std::condition_variable g_cv;
std::vector<rt_ctx *> &pool() {
    static std::vector<rt_ctx *> *v = new std::vector<rt_ctx *>(); // never destroyed: contexts live with the process
    return *v;
}

void destroy_ctx(rt_ctx *c) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(c->device);
    if (c->p) rt_release(c->p);
    for (void *b : c->d_buf)
        if (b) (void)hipFree(b);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    for (hipEvent_t e : c->band)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->copied)
        if (e) (void)hipEventDestroy(e);
    if (c->e0) (void)hipEventDestroy(c->e0);
    if (c->e1) (void)hipEventDestroy(c->e1);
    if (c->render) (void)hipStreamDestroy(c->render);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->copy2) (void)hipStreamDestroy(c->copy2);
    if (prev >= 0) (void)hipSetDevice(prev);
    delete c;
}

int create_ctx(int device, rt_ctx **out) {
    rt_ctx *c = new (std::nothrow) rt_ctx();
    if (!c) return RT_ENOMEM;
    c->device = device;
    int prev = -1;
    (void)hipGetDevice(&prev);
    int rc = RT_OK;
    if (hipSetDevice(device) != hipSuccess) rc = RT_ENODEV;
    if (rc == RT_OK && (hipStreamCreateWithFlags(&c->render, hipStreamNonBlocking) != hipSuccess ||
                        hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) != hipSuccess ||
                        hipStreamCreateWithFlags(&c->copy2, hipStreamNonBlocking) != hipSuccess ||
                        hipEventCreate(&c->e0) != hipSuccess || hipEventCreate(&c->e1) != hipSuccess))
        rc = RT_EHIP;
    for (int i = 0; rc == RT_OK && i < MAX_BANDS; ++i)
        if (hipEventCreateWithFlags(&c->band[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->copied[i], hipEventDisableTiming) != hipSuccess)
            rc = RT_EHIP;
    if (prev >= 0) (void)hipSetDevice(prev);
    if (rc != RT_OK) {
        destroy_ctx(c);
        return rc;
    }
    *out = c;
    return RT_OK;
}

// The pinned staging ring's copy-out: rows [0, rows) of `src` (slab rows b0.., row pitch
// rowbytes) to their image rows in `dst` through the shard interleave, split over host threads.
void host_scatter(const char *src, uint32_t b0, uint32_t rows, uint32_t rowbytes, uint32_t H, uint32_t rb,
                  uint32_t shard, uint32_t ns, char *dst) {
    auto body = [=](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) {
            const uint64_t r = (uint64_t)b0 + i;
            const uint64_t g = (r / rb * ns + shard) * rb + r % rb;
            if (g < H) std::memcpy(dst + g * rowbytes, src + (uint64_t)i * rowbytes, rowbytes);
        }
    };
    const uint64_t bytes = (uint64_t)rows * rowbytes;
    unsigned nt = std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()));
    if (bytes < (4u << 20) || nt <= 1 || rows < 2 * nt) {
        body(0, rows);
        return;
    }
    std::vector<std::thread> th;
    const uint32_t per = (rows + nt - 1) / nt;
    for (unsigned t = 1; t < nt && t * per < rows; ++t) th.emplace_back(body, t * per, std::min(rows, (t + 1) * per));
    body(0, std::min(rows, per));
    for (std::thread &x : th) x.join();
}

// Async copy of slab rows [b0, b1) of shard `shard` (device slab, row pitch rowbytes) to their
// rows of the row-major host image (pinned), on `st`.  Row-block runs become 2D copies.
int scatter_rows_async(const char *slab, uint32_t b0, uint32_t b1, uint32_t rowbytes, uint32_t H, uint32_t rb,
                       uint32_t shard, uint32_t ns, char *image, hipStream_t st) {
    uint32_t r = b0;
    while (r < b1) {
        const uint32_t q = r / rb, rr = r % rb;
        const uint64_t g = ((uint64_t)q * ns + shard) * rb + rr;
        if (g >= H) break; // later slab rows map further down: all past the image
        if (rr == 0 && ns > 1) {
            // whole row blocks inside [r, b1) and inside the image: one strided copy
            uint32_t nblk = (b1 - r) / rb;
            while (nblk > 0 && (((uint64_t)(q + nblk - 1) * ns + shard) * rb + rb) > H) --nblk;
            if (nblk > 0) {
                const size_t w = (size_t)rb * rowbytes;
                if (hipMemcpy2DAsync(image + g * rowbytes, w * ns, slab + (uint64_t)r * rowbytes, w, w, nblk,
                                     hipMemcpyDeviceToHost, st) != hipSuccess)
                    return RT_EHIP;
                r += nblk * rb;
                continue;
            }
        }
        // the rest of this row block (contiguous in both), clipped to the image and the band
        uint32_t n = std::min(b1 - r, rb - rr);
        if (ns == 1) n = b1 - r; // one shard: slab rows are image rows
        n = (uint32_t)std::min<uint64_t>(n, H - g);
        if (hipMemcpyAsync(image + g * rowbytes, slab + (uint64_t)r * rowbytes, (size_t)n * rowbytes,
                           hipMemcpyDeviceToHost, st) != hipSuccess)
            return RT_EHIP;
        r += n;
    }
    return RT_OK;
}

bool is_pinned(const void *p, size_t bytes) {
    auto one = [](const void *q) {
        hipPointerAttribute_t a;
        std::memset(&a, 0, sizeof a);
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError(); // pageable memory: not an error of the call
            return false;
        }
        return a.type == hipMemoryTypeHost;
    };
    return bytes > 0 && one(p) && one(static_cast<const char *>(p) + bytes - 1);
}

uint32_t lcm_u(uint32_t a, uint32_t b) {
    uint32_t x = a, y = b;
    while (y) {
        const uint32_t t = x % y;
        x = y;
        y = t;
    }
    return a / x * b;
}

} // namespace

int rt_ctx_acquire(int device, const rt_elem *scene, uint32_t n, rt_ctx **out) {
    *out = nullptr;
    rt_ctx *c = nullptr;
    {
        std::unique_lock<std::mutex> lk(g_mu);
        for (;;) {
            rt_ctx *free_any = nullptr;
            int count = 0;
            const size_t kb = (size_t)n * sizeof(rt_elem);
            for (rt_ctx *x : pool()) {
                if (x->device != device) continue;
                ++count;
                if (x->busy) continue;
                if (x->key.size() == kb && std::memcmp(x->key.data(), scene, kb) == 0) {
                    c = x; // same scene already prepared
                    break;
                }
                if (!free_any) free_any = x;
            }
            if (!c) c = free_any;
            if (c) {
                c->busy = true;
                break;
            }
            if (count < RT_CTX_PER_DEVICE) {
                const int rc = create_ctx(device, &c);
                if (rc != RT_OK) return rc;
                c->busy = true;
                pool().push_back(c);
                break;
            }
            g_cv.wait(lk);
        }
    }
    const size_t kb = (size_t)n * sizeof(rt_elem);
    if (!(c->p && c->key.size() == kb && std::memcmp(c->key.data(), scene, kb) == 0)) {
        // a different scene: compile and upload it; the context's work space is kept
        int rc = c->p ? rt_prepare_scene(c->p, scene, n) : rt_prepare(scene, n, device, &c->p);
        // every kernel on the context's render stream: with the library's two shading side
        // streams beside the render and copy streams a process exceeds its 4 hardware queues,
        // and streams sharing a queue serialise behind each other's event waits (measured:
        // each row band then cost ~0.7 ms of render time whatever its size)
        if (rc == RT_OK) rc = rt_configure(c->p, RT_CFG_SIDE_STREAMS, side_streams_env());
        if (rc != RT_OK) {
            c->key.clear();
            rt_ctx_release(c);
            return rc;
        }
        c->key.assign(reinterpret_cast<const unsigned char *>(scene), reinterpret_cast<const unsigned char *>(scene) + kb);
    }
    *out = c;
    return RT_OK;
}

void rt_ctx_release(rt_ctx *c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        c->busy = false;
    }
    g_cv.notify_all();
}

rt_prepared *rt_ctx_prepared(rt_ctx *c) { return c->p; }
hipStream_t rt_ctx_stream(rt_ctx *c) { return c->render; }

int rt_ctx_device_buffer(rt_ctx *c, int which, size_t bytes, void **out) {
    if (which < 0 || which > 2) return RT_EBADARG;
    if (c->d_cap[which] < bytes) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(c->device);
        if (c->d_buf[which]) {
            (void)hipStreamSynchronize(c->render);
            (void)hipStreamSynchronize(c->copy);
            (void)hipStreamSynchronize(c->copy2);
            (void)hipFree(c->d_buf[which]);
        }
        c->d_buf[which] = nullptr;
        c->d_cap[which] = 0;
        const hipError_t e = hipMalloc(&c->d_buf[which], bytes);
        if (prev >= 0) (void)hipSetDevice(prev);
        if (e != hipSuccess) {
            c->d_buf[which] = nullptr;
            return RT_ENOMEM;
        }
        c->d_cap[which] = bytes;
    }
    *out = c->d_buf[which];
    return RT_OK;
}

int rt_ctx_host_buffer(rt_ctx *c, size_t bytes, void **out) {
    if (c->h_cap < bytes) {
        if (c->h_stage) {
            (void)hipStreamSynchronize(c->copy);
            (void)hipHostFree(c->h_stage);
        }
        c->h_stage = nullptr;
        c->h_cap = 0;
        if (hipHostMalloc(&c->h_stage, bytes, hipHostMallocPortable) != hipSuccess) {
            c->h_stage = nullptr;
            return RT_ENOMEM;
        }
        c->h_cap = bytes;
    }
    *out = c->h_stage;
    return RT_OK;
}

// rt_host_alloc keeps freed blocks for reuse (pinning is slow: a fresh 200 MB block costs
// milliseconds to tens of them, a NIF allocates one per frame): up to HOST_CACHE_BLOCKS blocks
// and HOST_CACHE_BYTES in all; a request takes the smallest cached block that fits and is at
// most twice its size.
namespace {
constexpr size_t HOST_CACHE_BLOCKS = 8;
constexpr size_t HOST_CACHE_BYTES = (size_t)4 << 30;
struct HostBlock {
    void *p;
    size_t n;
};
std::mutex g_host_mu;
std::vector<HostBlock> &host_live() { // blocks handed out (their sizes)
    static std::vector<HostBlock> *v = new std::vector<HostBlock>();
    return *v;
}
std::vector<HostBlock> &host_free() {
    static std::vector<HostBlock> *v = new std::vector<HostBlock>();
    return *v;
}
} // namespace

extern "C" {

void *rt_host_alloc(size_t bytes) {
    if (bytes == 0) return nullptr;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto &fr = host_free();
        int best = -1;
        for (size_t i = 0; i < fr.size(); ++i)
            if (fr[i].n >= bytes && fr[i].n / 2 <= bytes && (best < 0 || fr[i].n < fr[best].n)) best = (int)i;
        if (best >= 0) {
            HostBlock b = fr[best];
            fr.erase(fr.begin() + best);
            host_live().push_back(b);
            return b.p;
        }
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_host_mu);
    host_live().push_back(HostBlock{p, bytes});
    return p;
}

int rt_host_free(void *p) {
    if (!p) return RT_OK;
    std::vector<void *> release;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto &lv = host_live();
        auto it = std::find_if(lv.begin(), lv.end(), [&](const HostBlock &b) { return b.p == p; });
        if (it == lv.end()) return RT_EBADARG; // not from rt_host_alloc (or freed twice)
        const HostBlock b = *it;
        lv.erase(it);
        auto &fr = host_free();
        fr.push_back(b);
        size_t total = 0;
        for (const HostBlock &x : fr) total += x.n;
        while (!fr.empty() && (fr.size() > HOST_CACHE_BLOCKS || total > HOST_CACHE_BYTES)) {
            total -= fr.front().n; // oldest first
            release.push_back(fr.front().p);
            fr.erase(fr.begin());
        }
    }
    for (void *q : release) (void)hipHostFree(q);
    return RT_OK;
}

// Device memory held by the idle contexts of `device` (their work space and output buffers), freed
// so that a caller whose allocation failed can retry: the pool caps contexts by count, and each
// keeps what its largest frame needed (about 5 GB at 4096^2 depth 5), so idle ones can crowd out
// a busy one.  Returns the bytes freed (0: nothing to free, the failure stands).
static size_t trim_idle(int device) {
    std::vector<rt_ctx *> idle;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (rt_ctx *c : pool())
            if (c->device == device && !c->busy) {
                c->busy = true; // claimed while trimmed
                idle.push_back(c);
            }
    }
    size_t freed = 0;
    for (rt_ctx *c : idle) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->render);
        (void)hipStreamSynchronize(c->copy);
        (void)hipStreamSynchronize(c->copy2);
        if (c->p) freed += rt_trim(c->p);
        for (int i = 0; i < 3; ++i) {
            if (c->d_buf[i]) (void)hipFree(c->d_buf[i]);
            freed += c->d_cap[i];
            c->d_buf[i] = nullptr;
            c->d_cap[i] = 0;
        }
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    if (!idle.empty()) {
        {
            std::lock_guard<std::mutex> lk(g_mu);
            for (rt_ctx *c : idle) c->busy = false;
        }
        g_cv.notify_all();
    }
    return freed;
}

int rt_reset_contexts(void) {
    std::vector<rt_ctx *> dead;
    int busy = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        std::vector<rt_ctx *> keep;
        for (rt_ctx *c : pool()) (c->busy ? keep : dead).push_back(c);
        busy = (int)keep.size();
        pool().swap(keep);
    }
    {
        std::vector<HostBlock> fr;
        {
            std::lock_guard<std::mutex> lk(g_host_mu);
            fr.swap(host_free());
        }
        for (const HostBlock &b : fr) (void)hipHostFree(b.p);
    }
    for (rt_ctx *c : dead) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->render);
        (void)hipStreamSynchronize(c->copy);
        (void)hipStreamSynchronize(c->copy2);
        destroy_ctx(c);
    }
    return busy;
}

int rt_render(const rt_elem *scene, uint32_t n, uint32_t width, uint32_t height, uint32_t depth, const rt_opts *opts,
              void *out_rgb, rt_stats *stats) {
    auto t_begin = std::chrono::steady_clock::now();
    if (width == 0 && height == 0) return RT_DONE;
    if (width == 0 || height == 0) return RT_EBADARG;
    if (!out_rgb) return RT_EBADARG;
    rt_opts o;
    std::memset(&o, 0, sizeof(o));
    o.ndev = 1;
    o.row_block = 16;
    o.spp = 1;
    if (opts && opts->struct_size) {
        std::memcpy(&o, opts, opts->struct_size < sizeof(o) ? opts->struct_size : sizeof(o));
        if (o.row_block == 0) o.row_block = 16;
        if (o.ndev == 0) o.ndev = 1;
        if (opts->struct_size < offsetof(rt_opts, spp) + sizeof(o.spp) || o.spp == 0) o.spp = 1; // ABI 1 callers
    }
    if (o.precision != RT_OUT_F64 && o.precision != RT_OUT_F32) return RT_EBADARG;
    if (o.order != RT_ORDER_EXACT && o.order != RT_ORDER_FAST) return RT_EBADARG;
    if (o.spp > RT_MAX_SPP) return RT_ETOOBIG;
    if (width > (1u << 20) || height > (1u << 20)) return RT_ETOOBIG;
    int rc = rtl::check_scene(scene, n);
    if (rc != RT_OK) return rc;
    int navail = 0;
    if (hipGetDeviceCount(&navail) != hipSuccess || navail <= 0) return RT_ENODEV;
    const int alias = device_alias();
    if (alias > 0) {
        if (o.first_dev < 0 || o.first_dev >= navail) return RT_ENODEV;
        navail = o.first_dev + alias;
    }
    if (o.ndev < 0) o.ndev = navail - o.first_dev;
    if (o.first_dev < 0 || o.ndev <= 0 || o.first_dev + o.ndev > navail) return RT_ENODEV;
    const uint32_t ns = o.nshards ? o.nshards : (uint32_t)o.ndev, rb = o.row_block;
    if (ns > RT_MAX_SHARDS) return RT_ETOOBIG;
    const uint32_t nd = std::min<uint32_t>(ns, (uint32_t)o.ndev); // devices used; shard s on device s % nd
    const uint32_t slab = rt_shard_rows(height, rb, ns);
    const size_t esz = o.precision == RT_OUT_F32 ? 4 : 8;
    const uint32_t rowbytes = width * 3 * (uint32_t)esz;
    const size_t frame_bytes = (size_t)height * rowbytes, slab_bytes = (size_t)slab * rowbytes;
    const bool pinned = is_pinned(out_rgb, frame_bytes);
    // bands: whole row blocks and whole tiles, about band_bytes() of output each, at most
    // MAX_BANDS per device over all of its shards
    const uint32_t per_dev = (ns + nd - 1) / nd;
    const uint32_t max_nb = std::max<uint32_t>(1, MAX_BANDS / per_dev);
    const uint32_t gran = lcm_u(rb, 16);
    uint32_t band = (uint32_t)std::max<size_t>(1, band_bytes() / rowbytes) / gran * gran;
    band = std::max(band, gran);
    if ((slab + band - 1) / band > max_nb) band = ((slab + max_nb - 1) / max_nb + gran - 1) / gran * gran;
    const uint32_t nb = (slab + band - 1) / band;

    int prev = -1;
    (void)hipGetDevice(&prev);
    std::vector<rt_ctx *> ctx(nd, nullptr);
    std::vector<char *> d_out(nd, nullptr), stage(nd, nullptr);
    std::vector<uint8_t *> d_lv(nd, nullptr);
    int err = RT_OK;
    auto shards_of = [&](uint32_t d) { return (ns - d + nd - 1) / nd; }; // shards d, d + nd, ...
    for (uint32_t d = 0; d < nd && err == RT_OK; ++d) {
        const int dev = alias > 0 ? o.first_dev : o.first_dev + (int)d;
        err = rt_ctx_acquire(dev, scene, n, &ctx[d]);
        if (err != RT_OK) break;
        rt_ctx *c = ctx[d];
        (void)hipSetDevice(dev);
        const uint32_t k = shards_of(d);
        // an allocation that fails while other contexts of the device sit idle on their memory is
        // retried once after those are trimmed (trim_idle)
        err = rt_ctx_device_buffer(c, 0, k * slab_bytes, reinterpret_cast<void **>(&d_out[d]));
        if (err == RT_ENOMEM && trim_idle(dev) > 0)
            err = rt_ctx_device_buffer(c, 0, k * slab_bytes, reinterpret_cast<void **>(&d_out[d]));
        if (err == RT_OK && o.out_levels) {
            err = rt_ctx_device_buffer(c, 1, (size_t)k * slab * width, reinterpret_cast<void **>(&d_lv[d]));
            if (err == RT_ENOMEM && trim_idle(dev) > 0)
                err = rt_ctx_device_buffer(c, 1, (size_t)k * slab * width, reinterpret_cast<void **>(&d_lv[d]));
        }
        if (err == RT_OK && !pinned) err = rt_ctx_host_buffer(c, 2 * (size_t)band * rowbytes, reinterpret_cast<void **>(&stage[d]));
        if (err != RT_OK) break;
        if (hipEventRecord(c->e0, c->render) != hipSuccess) err = RT_EHIP;
        // every band's render on the render stream, its copy on the copy stream behind it
        for (uint32_t i = 0; i < k && err == RT_OK; ++i) {
            const uint32_t s = d + i * nd;
            char *slab_out = d_out[d] + i * slab_bytes;
            uint8_t *slab_lv = o.out_levels ? d_lv[d] + (size_t)i * slab * width : nullptr;
            for (uint32_t b = 0; b < nb && err == RT_OK; ++b) {
                const uint32_t b0 = b * band, b1 = std::min(slab, b0 + band);
                err = rt_launch_rows(c->p, width, height, depth, rb, s, ns, o.precision, o.order, o.spp, o.seed, b0,
                                     b1, slab_out, slab_lv, c->render, (o.flags & RT_LEVELS_HIT) ? 1 : 0);
                if (err == RT_ENOMEM && trim_idle(dev) > 0) // (a failed grow launches nothing)
                    err = rt_launch_rows(c->p, width, height, depth, rb, s, ns, o.precision, o.order, o.spp, o.seed,
                                         b0, b1, slab_out, slab_lv, c->render, (o.flags & RT_LEVELS_HIT) ? 1 : 0);
                if (err == RT_OK && hipEventRecord(c->band[i * nb + b], c->render) != hipSuccess) err = RT_EHIP;
                if (err == RT_OK && pinned) {
                    hipStream_t cs = ((i * nb + b) % copy_streams()) ? c->copy2 : c->copy;
                    if (hipStreamWaitEvent(cs, c->band[i * nb + b], 0) != hipSuccess) err = RT_EHIP;
                    if (err == RT_OK)
                        err = scatter_rows_async(slab_out, b0, b1, rowbytes, height, rb, s, ns,
                                                 static_cast<char *>(out_rgb), cs);
                }
            }
        }
        if (err == RT_OK && hipEventRecord(c->e1, c->render) != hipSuccess) err = RT_EHIP;
    }
    // pageable destination: DMA into a ring of two staging bands, copied out by host threads
    // while the next band's DMA runs
    for (uint32_t d = 0; d < nd && err == RT_OK && !pinned; ++d) {
        rt_ctx *c = ctx[d];
        (void)hipSetDevice(c->device);
        const uint32_t total = shards_of(d) * nb; // bands j = i * nb + b
        auto rows_of = [&](uint32_t j, uint32_t &b0, uint32_t &b1) {
            b0 = (j % nb) * band;
            b1 = std::min(slab, b0 + band);
        };
        auto enqueue = [&](uint32_t j) -> int {
            uint32_t b0, b1;
            rows_of(j, b0, b1);
            char *dst = stage[d] + (size_t)(j & 1) * band * rowbytes;
            const char *src = d_out[d] + (j / nb) * slab_bytes + (size_t)b0 * rowbytes;
            if (hipStreamWaitEvent(c->copy, c->band[j], 0) != hipSuccess ||
                hipMemcpyAsync(dst, src, (size_t)(b1 - b0) * rowbytes, hipMemcpyDeviceToHost, c->copy) != hipSuccess ||
                hipEventRecord(c->copied[j], c->copy) != hipSuccess)
                return RT_EHIP;
            return RT_OK;
        };
        for (uint32_t j = 0; j < total && j < 2 && err == RT_OK; ++j) err = enqueue(j);
        for (uint32_t j = 0; j < total && err == RT_OK; ++j) {
            if (hipEventSynchronize(c->copied[j]) != hipSuccess) {
                err = RT_EHIP;
                break;
            }
            uint32_t b0, b1;
            rows_of(j, b0, b1);
            host_scatter(stage[d] + (size_t)(j & 1) * band * rowbytes, b0, b1 - b0, rowbytes, height, rb,
                         d + (j / nb) * nd, ns, static_cast<char *>(out_rgb));
            if (j + 2 < total) err = enqueue(j + 2);
        }
    }
    // levels (1 byte per pixel) after the frame
    for (uint32_t d = 0; d < nd && err == RT_OK && o.out_levels; ++d) {
        rt_ctx *c = ctx[d];
        (void)hipSetDevice(c->device);
        const uint32_t k = shards_of(d);
        std::vector<uint8_t> tmp((size_t)k * slab * width);
        if (hipStreamSynchronize(c->render) != hipSuccess ||
            hipMemcpy(tmp.data(), d_lv[d], tmp.size(), hipMemcpyDeviceToHost) != hipSuccess) {
            err = RT_EHIP;
            break;
        }
        for (uint32_t i = 0; i < k; ++i)
            host_scatter(reinterpret_cast<const char *>(tmp.data()) + (size_t)i * slab * width, 0, slab, width, height,
                         rb, d + i * nd, ns, reinterpret_cast<char *>(o.out_levels));
    }
    double kms = 0;
    for (uint32_t d = 0; d < nd; ++d) {
        rt_ctx *c = ctx[d];
        if (!c) continue;
        (void)hipSetDevice(c->device);
        if (hipStreamSynchronize(c->render) != hipSuccess && err == RT_OK) err = RT_EHIP;
        if (hipStreamSynchronize(c->copy) != hipSuccess && err == RT_OK) err = RT_EHIP;
        if (hipStreamSynchronize(c->copy2) != hipSuccess && err == RT_OK) err = RT_EHIP;
        float ms = 0;
        if (err == RT_OK && hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess && ms > kms) kms = ms;
        rt_ctx_release(c);
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    if (stats) {
        stats->kernel_ms = kms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count();
        stats->pixels = (uint64_t)width * height;
        stats->ndev = (int32_t)nd;
        stats->flags = pinned ? 1 : 0;
    }
    return err;
}

} // extern "C"
