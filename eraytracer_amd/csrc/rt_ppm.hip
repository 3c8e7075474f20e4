// rt_ppm.hip — P3 output on the GPU: write_pixels_to_ppm/5 (raytracer.erl:667-685).
//
// Every channel becomes min(trunc(C*MaxValue), MaxValue) (binary64; no lower clamp) printed
// in decimal and followed by one space, after the header "P3\nW H\nMaxValue\n".  The text
// is variable-length, so three kernels: per pixel the channel values and the text length
// with a block sum (k_ppm_count), one workgroup scanning the block sums into offsets
// (k_ppm_scan), and every pixel writing its digits at its offset (k_ppm_write).  A 4096^2
// frame is ~150 MB of text: formatting it on the GPU and copying the text down is cheaper
// than copying the 400 MB binary64 frame and formatting it on the host.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_internal.h"

namespace {

constexpr int PPM_BLOCK = 256;

#define PPMCHK(x)                                                                                                  \
    do {                                                                                                           \
        hipError_t e_ = (x);                                                                                       \
        if (e_ != hipSuccess) {                                                                                    \
            std::fprintf(stderr, "rt_mi355x: %s failed: %s\n", #x, hipGetErrorString(e_));                        \
            return RT_EHIP;                                                                                        \
        }                                                                                                          \
    } while (0)

// min(trunc(c * maxv), maxv) as a 64-bit integer; *wide when below -2^31 (or not a number)
__host__ __device__ inline long long quantise(double c, double maxv, bool *wide) {
    const double x = c * maxv;
    if (!(x < maxv)) {                // also +inf; NaN falls through to the check below
        if (x == x) return (long long)maxv;
    }
    const double t = trunc(x);
    if (!(t >= -2147483648.0)) {      // below -2^31, or NaN
        *wide = true;
        return 0;
    }
    return (long long)t;
}

__host__ __device__ inline int ndigits(long long v) { // decimal characters of v (with a '-')
    int n = v < 0 ? 2 : 1;
    unsigned long long u = v < 0 ? (unsigned long long)(-v) : (unsigned long long)v;
    while (u >= 10) {
        u /= 10;
        ++n;
    }
    return n;
}

template <int PREC>
__device__ inline double channel(const void *rgb, size_t i) {
    return PREC == RT_OUT_F64 ? reinterpret_cast<const double *>(rgb)[i]
                              : (double)reinterpret_cast<const float *>(rgb)[i];
}

template <int PREC>
__device__ inline int pixel_len(const void *rgb, size_t pix, double maxv, long long q[3], bool *wide) {
    int len = 0;
    for (int c = 0; c < 3; ++c) {
        q[c] = quantise(channel<PREC>(rgb, pix * 3 + c), maxv, wide);
        len += ndigits(q[c]) + 1;
    }
    return len;
}

// inclusive block scan of v over PPM_BLOCK threads (4 waves: shuffles, then LDS)
__device__ inline unsigned block_scan(unsigned v, unsigned *s_wave, unsigned *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned u = __shfl_up(v, off);
        if (lane >= off) v += u;
    }
    if (lane == 63) s_wave[wave] = v;
    __syncthreads();
    unsigned before = 0, all = 0;
    for (int w = 0; w < PPM_BLOCK / 64; ++w) {
        const unsigned x = s_wave[w];
        before += w < wave ? x : 0;
        all += x;
    }
    *total = all;
    return before + v;
}

template <int PREC>
__global__ __launch_bounds__(PPM_BLOCK) void k_ppm_count(const void *__restrict__ rgb, size_t npix, double maxv,
                                                         unsigned *__restrict__ partial, int *__restrict__ wide) {
    __shared__ unsigned s_wave[PPM_BLOCK / 64];
    const size_t pix = (size_t)blockIdx.x * PPM_BLOCK + threadIdx.x;
    long long q[3];
    bool w = false;
    const unsigned len = pix < npix ? (unsigned)pixel_len<PREC>(rgb, pix, maxv, q, &w) : 0u;
    if (w) atomicOr(wide, 1);
    unsigned total;
    block_scan(len, s_wave, &total);
    if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// exclusive scan of the block sums in place (one workgroup, any count); total at partial[n]
__global__ __launch_bounds__(1024) void k_ppm_scan(unsigned *__restrict__ partial, unsigned n,
                                                   unsigned long long *__restrict__ total) {
    __shared__ unsigned long long s_sum[1024];
    const unsigned t = threadIdx.x, per = (n + 1023) / 1024;
    const unsigned lo = t * per, hi = lo + per < n ? lo + per : n;
    unsigned long long acc = 0;
    for (unsigned i = lo; i < hi; ++i) acc += partial[i];
    s_sum[t] = acc;
    __syncthreads();
    if (t == 0) { // 1024 sums: serial is fine
        unsigned long long run = 0;
        for (int i = 0; i < 1024; ++i) {
            const unsigned long long x = s_sum[i];
            s_sum[i] = run;
            run += x;
        }
        *total = run;
    }
    __syncthreads();
    unsigned long long run = s_sum[t];
    for (unsigned i = lo; i < hi; ++i) {
        const unsigned x = partial[i];
        partial[i] = (unsigned)run; // offsets fit: the caller checks total < 2^32
        run += x;
    }
}

__device__ inline char *put(char *o, long long v) {
    char buf[24];
    int n = 0;
    const bool neg = v < 0;
    unsigned long long u = neg ? (unsigned long long)(-v) : (unsigned long long)v;
    do {
        buf[n++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (neg) *o++ = '-';
    while (n) *o++ = buf[--n];
    *o++ = ' ';
    return o;
}

template <int PREC>
__global__ __launch_bounds__(PPM_BLOCK) void k_ppm_write(const void *__restrict__ rgb, size_t npix, double maxv,
                                                         const unsigned *__restrict__ offset, char *__restrict__ text,
                                                         size_t header) {
    __shared__ unsigned s_wave[PPM_BLOCK / 64];
    const size_t pix = (size_t)blockIdx.x * PPM_BLOCK + threadIdx.x;
    long long q[3] = {0, 0, 0};
    bool w = false;
    const unsigned len = pix < npix ? (unsigned)pixel_len<PREC>(rgb, pix, maxv, q, &w) : 0u;
    unsigned total;
    const unsigned incl = block_scan(len, s_wave, &total);
    if (pix >= npix) return;
    char *o = text + header + offset[blockIdx.x] + (incl - len);
    o = put(o, q[0]);
    o = put(o, q[1]);
    put(o, q[2]);
}

std::string header_of(uint32_t W, uint32_t H, uint32_t maxv) {
    char h[64];
    std::snprintf(h, sizeof h, "P3\n%u %u\n%u\n", W, H, maxv);
    return h;
}

// Exact decimal of trunc(x) for any finite x (BEAM integers are unbounded): |x| < 2^63 as
// int64, larger values from the binary64 bits with a small base-1e9 bignum.
std::string int_text(double x) {
    const double t = std::trunc(x);
    if (std::fabs(t) < 9.2e18) return std::to_string((long long)t);
    int e = 0;
    const double m = std::frexp(std::fabs(t), &e); // |t| = m * 2^e, m in [0.5, 1)
    unsigned long long mant = (unsigned long long)std::ldexp(m, 53);
    e -= 53;
    std::vector<unsigned> limbs; // little-endian base 1e9
    while (mant) {
        limbs.push_back((unsigned)(mant % 1000000000ull));
        mant /= 1000000000ull;
    }
    for (int i = 0; i < e; ++i) { // times 2^e
        unsigned long long carry = 0;
        for (unsigned &l : limbs) {
            const unsigned long long v = (unsigned long long)l * 2 + carry;
            l = (unsigned)(v % 1000000000ull);
            carry = v / 1000000000ull;
        }
        if (carry) limbs.push_back((unsigned)carry);
    }
    std::string s = t < 0 ? "-" : "";
    s += std::to_string(limbs.back());
    for (size_t i = limbs.size() - 1; i-- > 0;) {
        char b[16];
        std::snprintf(b, sizeof b, "%09u", limbs[i]);
        s += b;
    }
    return s;
}

// Host formatter for frames the device formatter declines (RT_ERANGE) — same rules.
template <typename T>
int host_ppm(const T *rgb, uint32_t W, uint32_t H, uint32_t maxv, FILE *f) {
    const std::string h = header_of(W, H, maxv);
    if (std::fwrite(h.data(), 1, h.size(), f) != h.size()) return RT_EBADARG;
    const double mv = (double)maxv;
    std::string line;
    for (size_t p = 0; p < (size_t)W * H; ++p) {
        line.clear();
        for (int c = 0; c < 3; ++c) {
            const double x = (double)rgb[p * 3 + c] * mv;
            line += (x < mv || x != x) ? int_text(x) : std::to_string(maxv);
            line += ' ';
        }
        if (std::fwrite(line.data(), 1, line.size(), f) != line.size()) return RT_EBADARG;
    }
    return RT_OK;
}

} // namespace

extern "C" {

size_t rt_ppm_bound(uint32_t width, uint32_t height, uint32_t max_value) {
    // a channel is at most max(digits(max_value), 11 = '-' + 10 digits of 2^31) + 1 chars
    const int d = ndigits((long long)max_value);
    const size_t per = (size_t)(d > 11 ? d : 11) + 1;
    return header_of(width, height, max_value).size() + (size_t)width * height * 3 * per;
}

int rt_ppm_format(const void *d_rgb, int precision, uint32_t width, uint32_t height, uint32_t max_value, char *d_text,
                  size_t text_cap, size_t *text_len, void *stream) {
    if (!d_rgb || !d_text || !text_len) return RT_EBADARG;
    if (precision != RT_OUT_F64 && precision != RT_OUT_F32) return RT_EBADARG;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const std::string h = header_of(width, height, max_value);
    const size_t npix = (size_t)width * height;
    const unsigned nblk = (unsigned)((npix + PPM_BLOCK - 1) / PPM_BLOCK);
    if (npix == 0) {
        if (text_cap < h.size()) return RT_ETOOBIG;
        PPMCHK(hipMemcpyAsync(d_text, h.data(), h.size(), hipMemcpyHostToDevice, st));
        PPMCHK(hipStreamSynchronize(st));
        *text_len = h.size();
        return RT_OK;
    }
    unsigned *partial = nullptr;
    unsigned long long *total = nullptr;
    int *wide = nullptr;
    // one allocation: block sums, the total and the range flag
    char *ws = nullptr;
    const size_t ws_bytes = (size_t)nblk * sizeof(unsigned) + 64;
    PPMCHK(hipMallocAsync(reinterpret_cast<void **>(&ws), ws_bytes, st));
    partial = reinterpret_cast<unsigned *>(ws);
    total = reinterpret_cast<unsigned long long *>(ws + (((size_t)nblk * sizeof(unsigned) + 15) / 16) * 16);
    wide = reinterpret_cast<int *>(total + 1);
    int rc = RT_OK;
    unsigned long long h_total = 0;
    int h_wide = 0;
    const double mv = (double)max_value;
    do {
        if (hipMemsetAsync(wide, 0, sizeof(int), st) != hipSuccess) { rc = RT_EHIP; break; }
        if (precision == RT_OUT_F64)
            hipLaunchKernelGGL(k_ppm_count<RT_OUT_F64>, dim3(nblk), dim3(PPM_BLOCK), 0, st, d_rgb, npix, mv, partial, wide);
        else
            hipLaunchKernelGGL(k_ppm_count<RT_OUT_F32>, dim3(nblk), dim3(PPM_BLOCK), 0, st, d_rgb, npix, mv, partial, wide);
        hipLaunchKernelGGL(k_ppm_scan, dim3(1), dim3(1024), 0, st, partial, nblk, total);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(&h_total, total, sizeof h_total, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(&h_wide, wide, sizeof h_wide, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) { rc = RT_EHIP; break; }
        if (h_wide) { rc = RT_ERANGE; break; }
        if (h_total >= (1ull << 32) || h.size() + h_total > text_cap) { rc = RT_ETOOBIG; break; }
        if (hipMemcpyAsync(d_text, h.data(), h.size(), hipMemcpyHostToDevice, st) != hipSuccess) { rc = RT_EHIP; break; }
        if (precision == RT_OUT_F64)
            hipLaunchKernelGGL(k_ppm_write<RT_OUT_F64>, dim3(nblk), dim3(PPM_BLOCK), 0, st, d_rgb, npix, mv, partial,
                               d_text, h.size());
        else
            hipLaunchKernelGGL(k_ppm_write<RT_OUT_F32>, dim3(nblk), dim3(PPM_BLOCK), 0, st, d_rgb, npix, mv, partial,
                               d_text, h.size());
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) { rc = RT_EHIP; break; }
        *text_len = h.size() + (size_t)h_total;
    } while (0);
    (void)hipFreeAsync(ws, st);
    (void)hipStreamSynchronize(st);
    return rc;
}

int rt_render_ppm_file(const rt_elem *scene, uint32_t n, uint32_t width, uint32_t height, uint32_t depth,
                       const rt_opts *opts, uint32_t max_value, const char *path, rt_stats *stats) {
    if (!path) return RT_EBADARG;
    if (width == 0 && height == 0) return RT_DONE;
    if (width == 0 || height == 0) return RT_EBADARG;
    rt_opts o;
    std::memset(&o, 0, sizeof o);
    o.ndev = 1;
    o.row_block = 16;
    o.spp = 1;
    if (opts && opts->struct_size) std::memcpy(&o, opts, opts->struct_size < sizeof o ? opts->struct_size : sizeof o);
    if (o.spp == 0) o.spp = 1;
    if (o.row_block == 0) o.row_block = 16;
    o.precision = RT_OUT_F64; // the reference's values: the text is byte-exact
    o.out_levels = nullptr;
    FILE *f = nullptr;
    int rc = RT_OK;
    if (o.ndev != 1) { // several devices: rt_render assembles the frame on the host
        std::vector<double> img((size_t)width * height * 3);
        rc = rt_render(scene, n, width, height, depth, &o, img.data(), stats);
        if (rc != RT_OK) return rc;
        f = std::fopen(path, "wb");
        if (!f) return RT_EBADARG;
        rc = host_ppm(img.data(), width, height, max_value, f);
        std::fclose(f);
        return rc;
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || o.first_dev < 0 || o.first_dev >= nd) return RT_ENODEV;
    // the process's render context for this device (rt_host.hip): scene, streams, frame and text
    // buffers and the pinned host buffer persist across calls
    rt_ctx *ctx = nullptr;
    rc = rt_ctx_acquire(o.first_dev, scene, n, &ctx);
    if (rc != RT_OK) return rc;
    (void)hipSetDevice(o.first_dev);
    const size_t frame_bytes = (size_t)width * height * 3 * sizeof(double);
    const size_t cap = rt_ppm_bound(width, height, max_value);
    void *d_rgb = nullptr, *d_text = nullptr, *h_text = nullptr;
    hipStream_t st = rt_ctx_stream(ctx);
    size_t len = 0;
    do {
        if ((rc = rt_ctx_device_buffer(ctx, 0, frame_bytes, &d_rgb)) != RT_OK) break;
        if ((rc = rt_ctx_device_buffer(ctx, 2, cap, &d_text)) != RT_OK) break;
        rc = rt_launch_spp(rt_ctx_prepared(ctx), width, height, depth, o.row_block, 0, 1, RT_OUT_F64, o.order, o.spp,
                           o.seed, d_rgb, nullptr, st);
        if (rc != RT_OK) break;
        rc = rt_ppm_format(d_rgb, RT_OUT_F64, width, height, max_value, static_cast<char *>(d_text), cap, &len, st);
        if (rc == RT_ERANGE) { // a colour BEAM would print as a bignum: format on the host
            std::vector<double> img((size_t)width * height * 3);
            if (hipMemcpy(img.data(), d_rgb, frame_bytes, hipMemcpyDeviceToHost) != hipSuccess) { rc = RT_EHIP; break; }
            f = std::fopen(path, "wb");
            if (!f) { rc = RT_EBADARG; break; }
            rc = host_ppm(img.data(), width, height, max_value, f);
            break;
        }
        if (rc != RT_OK) break;
        // the text to pinned memory by DMA, written to the file from there
        if ((rc = rt_ctx_host_buffer(ctx, len ? len : 1, &h_text)) != RT_OK) break;
        if (hipMemcpyAsync(h_text, d_text, len, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) { rc = RT_EHIP; break; }
        f = std::fopen(path, "wb");
        if (!f) { rc = RT_EBADARG; break; }
        if (std::fwrite(h_text, 1, len, f) != len) rc = RT_EBADARG;
    } while (0);
    if (f) std::fclose(f);
    (void)hipStreamSynchronize(st);
    rt_ctx_release(ctx);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (stats && rc == RT_OK) {
        stats->pixels = (uint64_t)width * height;
        stats->ndev = 1;
    }
    return rc;
}

} // extern "C"
