// Microbenchmark: does a just-written buffer read back from the Infinity Cache (MALL) faster than from HBM?
// For each size S: stream-write S bytes, then stream-read them back (each timed on its own); then the same with an
// R-byte streaming read of unrelated input inside the writing kernel (the k_part shape: read input, write staging).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_mall tools/mb_mall.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(512) void k_write(uint4* buf, int64_t n16, uint32_t v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
        buf[i] = make_uint4(v, (uint32_t)i, v ^ 1u, (uint32_t)(i >> 32));
}
// read `in` (n_in16) and write `buf` (n16): the input/staging ratio of k_part
__global__ __launch_bounds__(512) void k_rw(const uint4* in, int64_t n_in16, uint4* buf, int64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    const int64_t st = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    // both streams advance proportionally
    for (int64_t i = i0; i < n_in16; i += st) {
        const uint4 a = in[i];
        acc += a.x ^ a.y ^ a.z ^ a.w;
        const int64_t j = (int64_t)((double)i * n16 / n_in16);
        if (j < n16) buf[j] = a;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(512) void k_read(const uint4* buf, int64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 a = buf[i];
        acc += a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const int64_t MB = 1 << 20;
    const int64_t maxS = 2048 * MB;
    uint4 *buf, *flush, *in;
    uint32_t* sink;
    CK(hipMalloc(&buf, maxS));
    CK(hipMalloc(&flush, 1024 * MB));
    CK(hipMalloc(&in, 2048 * MB));
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    const int G = 2048;
    hipLaunchKernelGGL(k_write, dim3(G), dim3(512), 0, 0, in, 2048 * MB / 16, 7u);
    for (int64_t s : {16, 32, 64, 96, 128, 192, 256, 384, 512, 1024, 2048}) {
        const int64_t S = s * MB;
        float tw = 0, tr = 0, tr2 = 0;
        for (int rep = 0; rep < 4; ++rep) {
            // evict: write + read 1 GB of unrelated data
            hipLaunchKernelGGL(k_write, dim3(G), dim3(512), 0, 0, flush, 1024 * MB / 16, 3u);
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, flush, 1024 * MB / 16, sink);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_write, dim3(G), dim3(512), 0, 0, buf, S / 16, (uint32_t)rep);
            CK(hipEventRecord(e1));
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, buf, S / 16, sink);
            CK(hipEventRecord(e2));
            CK(hipEventSynchronize(e2));
            float a, b;
            CK(hipEventElapsedTime(&a, e0, e1));
            CK(hipEventElapsedTime(&b, e1, e2));
            if (rep) { tw += a; tr += b; }
            // cold read for comparison
            hipLaunchKernelGGL(k_write, dim3(G), dim3(512), 0, 0, flush, 1024 * MB / 16, 5u);
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, flush, 1024 * MB / 16, sink);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, buf, S / 16, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&a, e0, e1));
            if (rep) tr2 += a;
        }
        tw /= 3; tr /= 3; tr2 /= 3;
        printf("S=%5lld MB  write %.4f ms (%5.0f GB/s)  read-after-write %.4f ms (%5.0f GB/s)  cold read %.4f ms (%5.0f GB/s)\n",
               (long long)s, tw, S / tw / 1e6, tr, S / tr / 1e6, tr2, S / tr2 / 1e6);
    }
    // k_part shape: read R of input while writing S = 0.9 R of staging, then read the staging back
    for (int64_t s : {32, 64, 128, 192, 256, 512}) {
        const int64_t S = s * MB, R = S * 10 / 9;
        float t1 = 0, t2 = 0;
        for (int rep = 0; rep < 4; ++rep) {
            hipLaunchKernelGGL(k_write, dim3(G), dim3(512), 0, 0, flush, 1024 * MB / 16, 3u);
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, flush, 1024 * MB / 16, sink);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_rw, dim3(G), dim3(512), 0, 0, in, R / 16, buf, S / 16, sink);
            CK(hipEventRecord(e1));
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, buf, S / 16, sink);
            CK(hipEventRecord(e2));
            CK(hipEventSynchronize(e2));
            float a, b;
            CK(hipEventElapsedTime(&a, e0, e1));
            CK(hipEventElapsedTime(&b, e1, e2));
            if (rep) { t1 += a; t2 += b; }
        }
        t1 /= 3; t2 /= 3;
        printf("k_part shape: read %4lld MB + write %4lld MB: %.4f ms (%5.0f GB/s)   read-back %.4f ms (%5.0f GB/s)\n",
               (long long)(R / MB), (long long)s, t1, (R + S) / t1 / 1e6, t2, S / t2 / 1e6);
    }
    // steady-state ring: repeatedly rewrite + reread the same S-byte buffer while streaming fresh input
    for (int64_t s : {64, 128, 192}) {
        const int64_t S = s * MB, R = S * 10 / 9;
        const int rounds = (int)(2048 * MB / R);
        CK(hipEventRecord(e0));
        for (int r = 0; r < rounds; ++r) {
            hipLaunchKernelGGL(k_rw, dim3(G), dim3(512), 0, 0, in + (r * R) / 16, R / 16, buf, S / 16, sink);
            hipLaunchKernelGGL(k_read, dim3(G), dim3(512), 0, 0, buf, S / 16, sink);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float a;
        CK(hipEventElapsedTime(&a, e0, e1));
        printf("ring S=%lld MB x %d rounds: %.3f ms total, %.0f GB/s of input (input %.0f MB)\n", (long long)s, rounds, a,
               rounds * R / a / 1e6, rounds * R / (double)MB);
    }
    printf("done\n");
    return 0;
}
