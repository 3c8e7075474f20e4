// rt_slab.hip — compact slabs for the multi-GPU frame gather (include/rt_mi355x.h, "compact
// slab transfer").
//
// The reference's master collects every pixel from its workers (raytracer.erl:151-161,
// :169-178); here each rank renders its interleaved rows into a slab in HBM and rank 0
// gathers the slabs over xGMI.  Rendering runs at ~27 Gpx/s per MI355X, i.e. ~325 GB/s of
// f32 RGB per GPU, so with 8 ranks the gather into rank 0 (7 inbound links) and not the
// render bounds a frame.  Most pixels are background (the reference's BACKGROUND_COLOUR,
// raytracer.erl:186-203, exactly +0.0 in every channel: 73 % of S64's pixels), so a slab
// is sent as
//     header (fixed size):  u64 count | u32 block_off[nblk] | u64 mask[4*nblk]
//     values (count*3 elements of the slab's precision): the non-zero pixels in slab order
// with one mask bit per slab pixel (a pixel is "zero" iff all three channels are +0.0
// bit for bit, so the round trip is exact) and, per 256-pixel block, the number of
// non-zero pixels before it.  Slab rows past the image are never written by rt_launch and
// are encoded as zero without being read.
//
// Pack: k_mask (one wave per 64 pixels: ballot -> mask word, block popcount), k_scan (one
// workgroup, exclusive scan of the block counts -> offsets and the count), k_compact
// (non-zero pixels copied to their rank).  Unpack on rank 0 is fused with the reorder of
// rt_unshard: one workgroup per image row and 256 columns (the row's shard and slab row are
// wave-uniform), one thread per pixel finds its mask bit and reads its value, so the full
// frame is written once.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../../include/rt_mi355x.h"

namespace {

constexpr int SLAB_BLOCK = 256;       // pixels per offset entry = threads per pack workgroup
constexpr size_t HDR_OFFS = 64;       // block offsets start here (the count sits at 0)

#define SLABCHK(x)                                                                                                 \
    do {                                                                                                           \
        hipError_t e_ = (x);                                                                                       \
        if (e_ != hipSuccess) {                                                                                    \
            std::fprintf(stderr, "rt_mi355x: %s failed: %s\n", #x, hipGetErrorString(e_));                        \
            return RT_EHIP;                                                                                        \
        }                                                                                                          \
    } while (0)

struct Layout {
    uint64_t px;      // slab pixels (rows * width)
    uint64_t nblk;    // 256-pixel blocks
    uint64_t mask_at; // byte offset of the mask words
    uint64_t bytes;   // header size
};

__host__ __device__ inline Layout layout(uint32_t width, uint32_t rows) {
    Layout l;
    l.px = (uint64_t)width * rows;
    l.nblk = (l.px + SLAB_BLOCK - 1) / SLAB_BLOCK;
    l.mask_at = (HDR_OFFS + l.nblk * 4 + 255) / 256 * 256;
    l.bytes = l.mask_at + l.nblk * (SLAB_BLOCK / 8);
    return l;
}

// slab rows inside the image: a prefix of the slab (rt_launch's interleave)
uint64_t valid_rows(uint32_t height, uint32_t rb, uint32_t shard, uint32_t ns, uint32_t rows) {
    uint64_t n = 0;
    for (uint64_t b = 0; b * rb < rows; ++b) {
        const uint64_t g0 = (b * ns + shard) * rb;
        if (g0 >= height) break;
        n += (g0 + rb <= height) ? rb : height - g0;
    }
    return n;
}

template <typename T>
__device__ inline bool nonzero(const T *__restrict__ slab, uint64_t p) {
    return (slab[p * 3] | slab[p * 3 + 1] | slab[p * 3 + 2]) != 0;
}

// one thread per slab pixel: mask words (one per wave) and the block's non-zero count.  The slab
// rows inside the image are a prefix of the slab (global rows grow with slab rows), so a pixel
// is in the image iff p < valid_px.
template <typename T>
__global__ __launch_bounds__(SLAB_BLOCK) void k_mask(const T *__restrict__ slab, uint64_t valid_px,
                                                     uint32_t *__restrict__ blk_cnt, uint64_t *__restrict__ mask) {
    __shared__ uint32_t s_cnt[SLAB_BLOCK / 64];
    const uint64_t p = (uint64_t)blockIdx.x * SLAB_BLOCK + threadIdx.x;
    const bool nz = p < valid_px && nonzero(slab, p);
    const uint64_t m = __ballot(nz);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        mask[p / 64] = m;
        s_cnt[wave] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

// exclusive scan of the block counts in place (one workgroup, any count); the total to *count.
// Tiles of SCAN_T * 1024 counts go through LDS: loaded and stored coalesced, each thread sums and
// rewrites SCAN_T consecutive counts there, and a wave scan (shuffles) plus the 16 wave totals
// ranks the threads (4096^2 / 8192^2 shards at N = 8: one / four tiles).  4096^2 / 8192^2 shard
// packs 0.024 -> 0.017 / 0.103 -> 0.061 ms against one thread walking 8 / 32 counts twice
// (profiles/r06ak_codec_ab.txt).  The counts and the
// total are < 2^32: the host checks px < 2^32.
constexpr int SCAN_T = 8, SCAN_TILE = 1024 * SCAN_T;
__device__ inline uint32_t scan_pad(uint32_t i) { return i + (i >> 5); } // (spreads a thread's run over banks)
__global__ __launch_bounds__(1024) void k_scan(uint32_t *__restrict__ blk, uint64_t n, uint64_t *__restrict__ count) {
    __shared__ uint32_t s[SCAN_TILE + SCAN_TILE / 32];
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t carry = 0;
    for (uint64_t base = 0; base < n; base += SCAN_TILE) {
#pragma unroll
        for (int j = 0; j < SCAN_T; ++j) {
            const uint64_t i = base + j * 1024 + t;
            s[scan_pad(j * 1024 + t)] = i < n ? blk[i] : 0u;
        }
        __syncthreads();
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < SCAN_T; ++j) acc += s[scan_pad(t * SCAN_T + j)];
        uint32_t inc = acc; // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(inc, o);
            if (lane >= (uint32_t)o) inc += u;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t wpre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t x = s_w[k];
            wpre += (uint32_t)k < w ? x : 0u;
            tot += x;
        }
        uint32_t run = carry + wpre + inc - acc;
#pragma unroll
        for (int j = 0; j < SCAN_T; ++j) {
            const uint32_t q = scan_pad(t * SCAN_T + j), x = s[q];
            s[q] = run;
            run += x;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SCAN_T; ++j) {
            const uint64_t i = base + j * 1024 + t;
            if (i < n) blk[i] = s[scan_pad(j * 1024 + t)];
        }
        carry += tot;
        __syncthreads(); // (s and s_w are refilled by the next tile)
    }
    if (t == 0) *count = carry;
}

// rank of slab pixel p among the non-zero pixels (its mask bit is set)
__device__ inline uint64_t rank_of(const uint32_t *__restrict__ off, const uint64_t *__restrict__ mask, uint64_t p) {
    const uint64_t w = p / 64, w0 = (p / SLAB_BLOCK) * (SLAB_BLOCK / 64);
    uint64_t r = off[p / SLAB_BLOCK];
    for (uint64_t i = w0; i < w; ++i) r += __popcll(mask[i]);
    const uint64_t below = (1ull << (p % 64)) - 1ull;
    return r + __popcll(mask[w] & below);
}

// non-zero pixels to their rank: the wave's mask word gives each lane its place
template <typename T>
__global__ __launch_bounds__(SLAB_BLOCK) void k_compact(const T *__restrict__ slab, uint64_t px,
                                                        const uint32_t *__restrict__ off,
                                                        const uint64_t *__restrict__ mask, T *__restrict__ vals) {
    const uint64_t p = (uint64_t)blockIdx.x * SLAB_BLOCK + threadIdx.x;
    if (p >= px) return;
    if (!((mask[p / 64] >> (p % 64)) & 1ull)) return;
    const uint64_t r = rank_of(off, mask, p);
    if (r >= px) return; // a consistent header never ranks past the slab (values hold px pixels)
    vals[r * 3] = slab[p * 3];
    vals[r * 3 + 1] = slab[p * 3 + 1];
    vals[r * 3 + 2] = slab[p * 3 + 2];
}

struct ShardPtrs {
    const unsigned char *hdr[RT_MAX_SHARDS];
    const void *vals[RT_MAX_SHARDS];
};

// one workgroup per (image row g, 256 columns): the row's shard and slab row are wave-uniform
// (no per-lane division), each lane finds its pixel's mask bit and value
template <typename T>
__global__ __launch_bounds__(SLAB_BLOCK) void k_unpack(ShardPtrs sp, uint64_t mask_at, uint64_t px, uint32_t W,
                                                       uint32_t ncol, uint32_t rb, uint32_t ns, T *__restrict__ image) {
    const uint32_t g = blockIdx.x / ncol, c = blockIdx.x - g * ncol;
    const uint32_t x = c * SLAB_BLOCK + threadIdx.x;
    if (x >= W) return;
    const uint32_t blk = g / rb, s = blk % ns;
    const uint64_t lr = (uint64_t)(blk / ns) * rb + (g - blk * rb);
    const uint64_t p = lr * W + x;
    const unsigned char *h = sp.hdr[s];
    const uint32_t *off = reinterpret_cast<const uint32_t *>(h + HDR_OFFS);
    const uint64_t *mask = reinterpret_cast<const uint64_t *>(h + mask_at);
    T c0 = 0, c1 = 0, c2 = 0;
    const uint64_t r = ((mask[p / 64] >> (p % 64)) & 1ull) ? rank_of(off, mask, p) : px;
    if (r < px) { // (a consistent header never ranks past the slab: values hold px pixels)
        const T *v = static_cast<const T *>(sp.vals[s]) + r * 3;
        c0 = v[0];
        c1 = v[1];
        c2 = v[2];
    }
    T *o = image + ((uint64_t)g * W + x) * 3;
    o[0] = c0;
    o[1] = c1;
    o[2] = c2;
}

// Frames whose width is a multiple of 4: each thread decodes 4 consecutive pixels of an image row
// (their mask bits share one word: p is a multiple of 4), one workgroup per (row, 1024 columns).
// The frame is the bulk of the decode's traffic (201 MB at 4096^2 f32 against ~55 MB of values
// for S64), so the stores decide its speed: each thread's 3 (binary32) or 6 (binary64) 16-byte
// pieces are staged in LDS and the workgroup writes its contiguous stretch of the frame with lane i
// of a store instruction at 16 i bytes (1 KiB per wave instruction instead of 16 B every 48 B),
// non-temporal (the frame is not read back on the device).  4096^2 f32, 8 shards: 0.068 -> 0.035 ms,
// 7.4 TB/s of algorithmic bytes (profiles/r06aj_codec_ab.txt).
constexpr int UNPACK_PX = 4;
template <typename T>
__global__ __launch_bounds__(SLAB_BLOCK) void k_unpack4(ShardPtrs sp, uint64_t mask_at, uint64_t px, uint32_t W,
                                                         uint32_t ncol, uint32_t rb, uint32_t ns, T *__restrict__ image) {
    constexpr int Q = 3 * UNPACK_PX * (int)sizeof(T) / 16; // 16-byte pieces per thread
    __shared__ uint4 s_out[SLAB_BLOCK * Q];
    const uint32_t g = blockIdx.x / ncol, c = blockIdx.x - g * ncol;
    const uint32_t x0 = c * SLAB_BLOCK * UNPACK_PX, x = x0 + threadIdx.x * UNPACK_PX;
    const uint32_t nact = (W - x0 < SLAB_BLOCK * UNPACK_PX ? W - x0 : SLAB_BLOCK * UNPACK_PX) / UNPACK_PX;
    if (x < W) {
        const uint32_t blk = g / rb, s = blk % ns;
        const uint64_t lr = (uint64_t)(blk / ns) * rb + (g - blk * rb);
        const uint64_t p = lr * W + x; // a multiple of 4 (W is)
        const unsigned char *h = sp.hdr[s];
        const uint32_t *off = reinterpret_cast<const uint32_t *>(h + HDR_OFFS);
        const uint64_t *mask = reinterpret_cast<const uint64_t *>(h + mask_at);
        const unsigned bits = (unsigned)(mask[p / 64] >> (p % 64)) & 0xFu;
        T v[3 * UNPACK_PX];
#pragma unroll
        for (int k = 0; k < 3 * UNPACK_PX; ++k) v[k] = 0;
        if (bits) {
            uint64_t r = rank_of(off, mask, p);
            if (r + __popc(bits) <= px) { // (a consistent header never ranks past the slab)
                const T *src = static_cast<const T *>(sp.vals[s]);
#pragma unroll
                for (int k = 0; k < UNPACK_PX; ++k) {
                    if ((bits >> k) & 1u) {
                        v[3 * k] = src[r * 3];
                        v[3 * k + 1] = src[r * 3 + 1];
                        v[3 * k + 2] = src[r * 3 + 2];
                        ++r;
                    }
                }
            }
        }
        uint4 *so = s_out + threadIdx.x * Q;
        if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
                so[k] = make_uint4((unsigned)v[4 * k], (unsigned)v[4 * k + 1], (unsigned)v[4 * k + 2], (unsigned)v[4 * k + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                so[k] = make_uint4((unsigned)v[2 * k], (unsigned)(v[2 * k] >> 32), (unsigned)v[2 * k + 1],
                                   (unsigned)(v[2 * k + 1] >> 32));
        }
    }
    __syncthreads();
    uint4 *o = reinterpret_cast<uint4 *>(image + ((uint64_t)g * W + x0) * 3);
    const uint32_t n16 = nact * Q;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
        const uint32_t i = k * SLAB_BLOCK + threadIdx.x;
        if (i < n16) {
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const uint4 w = s_out[i];
            __builtin_nontemporal_store(v4u{w.x, w.y, w.z, w.w}, reinterpret_cast<v4u *>(o + i));
        }
    }
}

bool args_ok(uint32_t width, uint32_t height, uint32_t row_block, uint32_t nshards, int precision) {
    if (width == 0 || height == 0 || row_block == 0 || nshards == 0 || nshards > RT_MAX_SHARDS) return false;
    if (precision != RT_OUT_F64 && precision != RT_OUT_F32) return false;
    return true;
}

} // namespace

extern "C" {

size_t rt_slab_header_bytes(uint32_t width, uint32_t height, uint32_t row_block, uint32_t nshards) {
    if (width == 0 || row_block == 0 || nshards == 0) return 0;
    return (size_t)layout(width, rt_shard_rows(height, row_block, nshards)).bytes;
}

int rt_slab_pack(const void *d_slab, uint32_t width, uint32_t height, uint32_t row_block, uint32_t shard,
                 uint32_t nshards, int precision, void *d_header, void *d_values, void *stream) {
    if (!d_slab || !d_header || !d_values || !args_ok(width, height, row_block, nshards, precision) ||
        shard >= nshards)
        return RT_EBADARG;
    const Layout l = layout(width, rt_shard_rows(height, row_block, nshards));
    if (l.px >= (1ull << 32)) return RT_ETOOBIG;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    unsigned char *h = static_cast<unsigned char *>(d_header);
    uint64_t *count = reinterpret_cast<uint64_t *>(h);
    uint32_t *off = reinterpret_cast<uint32_t *>(h + HDR_OFFS);
    uint64_t *mask = reinterpret_cast<uint64_t *>(h + l.mask_at);
    const dim3 grid((unsigned)l.nblk), blk(SLAB_BLOCK);
    const uint64_t valid_px =
        valid_rows(height, row_block, shard, nshards, rt_shard_rows(height, row_block, nshards)) * width;
    if (precision == RT_OUT_F32)
        hipLaunchKernelGGL(k_mask<uint32_t>, grid, blk, 0, st, static_cast<const uint32_t *>(d_slab), valid_px, off,
                           mask);
    else
        hipLaunchKernelGGL(k_mask<uint64_t>, grid, blk, 0, st, static_cast<const uint64_t *>(d_slab), valid_px, off,
                           mask);
    SLABCHK(hipGetLastError());
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, off, l.nblk, count);
    SLABCHK(hipGetLastError());
    if (precision == RT_OUT_F32)
        hipLaunchKernelGGL(k_compact<uint32_t>, grid, blk, 0, st, static_cast<const uint32_t *>(d_slab), l.px, off,
                           mask, static_cast<uint32_t *>(d_values));
    else
        hipLaunchKernelGGL(k_compact<uint64_t>, grid, blk, 0, st, static_cast<const uint64_t *>(d_slab), l.px, off,
                           mask, static_cast<uint64_t *>(d_values));
    SLABCHK(hipGetLastError());
    return RT_OK;
}

int rt_slab_unpack(const void *const *d_headers, const void *const *d_values, uint32_t width, uint32_t height,
                   uint32_t row_block, uint32_t nshards, int precision, void *d_image, void *stream) {
    if (!d_headers || !d_values || !d_image || !args_ok(width, height, row_block, nshards, precision))
        return RT_EBADARG;
    const Layout l = layout(width, rt_shard_rows(height, row_block, nshards));
    if (l.px >= (1ull << 32)) return RT_ETOOBIG;
    ShardPtrs sp = {};
    for (uint32_t s = 0; s < nshards; ++s) {
        if (!d_headers[s] || !d_values[s]) return RT_EBADARG;
        sp.hdr[s] = static_cast<const unsigned char *>(d_headers[s]);
        sp.vals[s] = d_values[s];
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (width % UNPACK_PX == 0) { // 4 pixels per thread, 16-byte stores
        const uint32_t ncol = (width + SLAB_BLOCK * UNPACK_PX - 1) / (SLAB_BLOCK * UNPACK_PX);
        const uint64_t nblocks = (uint64_t)ncol * height;
        if (nblocks >= (1ull << 31)) return RT_ETOOBIG;
        if (precision == RT_OUT_F32)
            hipLaunchKernelGGL(k_unpack4<uint32_t>, dim3((unsigned)nblocks), dim3(SLAB_BLOCK), 0, st, sp, l.mask_at,
                               l.px, width, ncol, row_block, nshards, static_cast<uint32_t *>(d_image));
        else
            hipLaunchKernelGGL(k_unpack4<uint64_t>, dim3((unsigned)nblocks), dim3(SLAB_BLOCK), 0, st, sp, l.mask_at,
                               l.px, width, ncol, row_block, nshards, static_cast<uint64_t *>(d_image));
        SLABCHK(hipGetLastError());
        return RT_OK;
    }
    const uint32_t ncol = (width + SLAB_BLOCK - 1) / SLAB_BLOCK;
    const uint64_t nblocks = (uint64_t)ncol * height;
    if (nblocks >= (1ull << 31)) return RT_ETOOBIG;
    const dim3 grid((unsigned)nblocks);
    if (precision == RT_OUT_F32)
        hipLaunchKernelGGL(k_unpack<uint32_t>, grid, dim3(SLAB_BLOCK), 0, st, sp, l.mask_at, l.px, width, ncol, row_block,
                           nshards, static_cast<uint32_t *>(d_image));
    else
        hipLaunchKernelGGL(k_unpack<uint64_t>, grid, dim3(SLAB_BLOCK), 0, st, sp, l.mask_at, l.px, width, ncol, row_block,
                           nshards, static_cast<uint64_t *>(d_image));
    SLABCHK(hipGetLastError());
    return RT_OK;
}

} // extern "C"
