// Calibration of rocprofv3's FETCH_SIZE / TCC_EA0_RDREQ* counters on gfx950 for the access patterns
// of the wavefront engine (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated").
// Each kernel reads a known number of bytes from a buffer far larger than L2 + Infinity Cache:
//   k_stream   16 B per lane, coalesced (the calibrated pattern: FETCH_SIZE reads half of it)
//   k_gather64 one 64-byte record per lane at a random 64-B aligned slot (HitRec reads)
//   k_gather16 16 B per lane at a random 16-B aligned slot (Rec0 / colour reads)
//   k_gather8  8 B per lane at a random 8-B aligned slot ((parent, pbits) words)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/hbm_calib.hip -o gpurun_out/hbm_calib
// Run:   rocprofv3 --pmc FETCH_SIZE -- gpurun_out/hbm_calib   (and TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
//        TCC_BUBBLE_sum in a second pass); the program prints each kernel's known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_stream(const int4 *__restrict__ a, size_t n, int *__restrict__ sink) {
    int4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int4 v = a[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345) sink[0] = 1;
}

template <int BYTES>
__global__ void k_gather(const int4 *__restrict__ a, size_t slots, size_t n, int *__restrict__ sink) {
    int acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t s = mix(i) % slots; // slot of BYTES bytes
        if (BYTES == 64) {
            const int4 *p = a + s * 4;
            const int4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
            acc ^= v0.x ^ v1.y ^ v2.z ^ v3.w;
        } else if (BYTES == 16) {
            const int4 v = a[s];
            acc ^= v.x ^ v.w;
        } else {
            const int2 v = reinterpret_cast<const int2 *>(a)[s];
            acc ^= v.x ^ v.y;
        }
    }
    if (acc == 0x12345) sink[0] = 1;
}

int main() {
    const size_t bytes = (size_t)8 << 30; // 8 GiB: far beyond L2 (32 MiB) and the Infinity Cache (256 MiB)
    int4 *a = nullptr;
    int *sink = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipDeviceSynchronize();
    const size_t n_stream = ((size_t)1 << 30) / 16; // 1 GiB streamed
    const size_t n_g = (size_t)1 << 24;             // 16.8 M gathers each
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, a, n_stream, sink);
    (void)hipDeviceSynchronize();
    std::printf("k_stream bytes %zu\n", n_stream * 16);
    hipLaunchKernelGGL(k_gather<64>, dim3(8192), dim3(256), 0, 0, a, bytes / 64, n_g, sink);
    (void)hipDeviceSynchronize();
    std::printf("k_gather64 bytes %zu\n", n_g * 64);
    hipLaunchKernelGGL(k_gather<16>, dim3(8192), dim3(256), 0, 0, a, bytes / 16, n_g, sink);
    (void)hipDeviceSynchronize();
    std::printf("k_gather16 bytes %zu\n", n_g * 16);
    hipLaunchKernelGGL(k_gather<8>, dim3(8192), dim3(256), 0, 0, a, bytes / 8, n_g, sink);
    (void)hipDeviceSynchronize();
    std::printf("k_gather8 bytes %zu\n", n_g * 8);
    (void)hipFree(a);
    (void)hipFree(sink);
    return 0;
}
