// Microbenchmark: are plain stores to a small, L2-resident, per-XCD footprint absorbed by the XCD's L2 (write-back),
// or do they all leave L2 (write-through to the Infinity Cache / HBM)? Each workgroup rewrites its own S-byte region
// `iters` times. An absorbing L2 runs at the L2 rate (tens of TB/s); a write-through one at the fabric write rate.
// A second kernel adds the k_part shape: a streamed HBM read beside the rewrites.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_l2wb tools/mb_l2wb.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_rewrite(uint4* buf, int64_t s16, int iters) {
    uint4* r = buf + (int64_t)blockIdx.x * s16;
    for (int it = 0; it < iters; ++it) {
        for (int64_t i = threadIdx.x; i < s16; i += 256) r[i] = make_uint4(it, (uint32_t)i, blockIdx.x, it ^ 7);
        asm volatile("" ::: "memory");
    }
}
// streamed read of `in` (n_in16 per block) while rewriting the block's region once per `chunk16` of input
__global__ __launch_bounds__(256) void k_stream_rewrite(const uint4* in, int64_t n_in16, uint4* buf, int64_t s16, uint32_t* sink) {
    uint4* r = buf + (int64_t)blockIdx.x * s16;
    const uint4* src = in + (int64_t)blockIdx.x * n_in16;
    uint32_t acc = 0;
    int64_t w = 0;
    for (int64_t i = threadIdx.x; i < n_in16; i += 256) {
        const uint4 a = src[i];
        acc += a.x ^ a.y ^ a.z ^ a.w;
        // ~0.9 bytes of staging per input byte, like k_part
        if ((i & 15) < 14) { r[w] = a; w += 256; if (w >= s16) w = threadIdx.x; }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_read(const uint4* in, int64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const uint4 a = in[i];
        acc += a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;   // run one case (for PMC passes)
    const int G = 512;
    const int64_t KB = 1024;
    uint4 *buf, *in;
    uint32_t* sink;
    CK(hipMalloc(&buf, (int64_t)G * 1024 * KB));
    CK(hipMalloc(&in, (int64_t)2048 * 1024 * KB));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 1, (int64_t)2048 * 1024 * KB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cs = 0;
    for (int64_t s : {4, 8, 16, 64, 1024}) {
        const int64_t S = s * KB;
        const int iters = (int)(512 * 1024 * KB / (S * G)) * 4 + 1;
        ++cs;
        if (only >= 0 && only != cs) continue;
        float t = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_rewrite, dim3(G), dim3(256), 0, 0, buf, S / 16, iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float a;
            CK(hipEventElapsedTime(&a, e0, e1));
            if (rep) t += a;
        }
        t /= 2;
        const double bytes = (double)S * G * iters;
        printf("case %d rewrite: %4lld KB per block (%6.1f MB total) x %5d: %.4f ms  %7.0f GB/s stored\n", cs, (long long)s,
               S * G / 1e6, iters, t, bytes / t / 1e6);
    }
    for (int64_t s : {8, 32, 128}) {
        const int64_t S = s * KB;
        const int64_t nin = (int64_t)2048 * 1024 * KB / 16 / G;
        ++cs;
        if (only >= 0 && only != cs) continue;
        float t = 0, tr = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_stream_rewrite, dim3(G), dim3(256), 0, 0, in, nin, buf, S / 16, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float a;
            CK(hipEventElapsedTime(&a, e0, e1));
            if (rep) t += a;
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, in, nin * G, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&a, e0, e1));
            if (rep) tr += a;
        }
        t /= 2;
        tr /= 2;
        printf("case %d stream+rewrite: read 2048 MB + store %.0f MB into %lld KB per block: %.4f ms (read alone %.4f ms, %.0f GB/s)\n",
               cs, 2048.0 * 14 / 16, (long long)s, t, tr, 2048.0 * 1.048576 / tr);
    }
    printf("done\n");
    return 0;
}
