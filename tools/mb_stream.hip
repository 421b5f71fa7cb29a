// mb_stream.hip — HBM ceilings on this part for the C2 step's access shapes: read-only (k_stats), read + write of
// about the same size (k_part: 20 B in, 18 B out), write-only, and a copy; blocks per CU and bytes in flight swept.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_stream tools/mb_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int U>
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ a, int64_t n16, unsigned long long* sink) {
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { const int64_t i = b + u * 256; v[u] = i < n16 ? a[i] : make_uint4(0, 0, 0, 0); }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}
template <int U>
__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ a, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) { const int64_t i = b + u * 256; if (i < n16) a[i] = make_uint4((uint32_t)i, 1, 2, 3); }
    }
}
template <int U>
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ c, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { const int64_t i = b + u * 256; v[u] = i < n16 ? a[i] : make_uint4(0, 0, 0, 0); }
#pragma unroll
        for (int u = 0; u < U; ++u) { const int64_t i = b + u * 256; if (i < n16) c[i] = v[u]; }
    }
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    const int64_t bytes = 800ll << 20;   // C2's ts column (1e8 x 8 B)
    const int64_t n16 = bytes / 16;
    uint4 *a, *c;
    unsigned long long* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&c, bytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(c, 2, bytes));
    for (int grid : {512, 1024, 2048, 4096, 8192}) {
        float r2 = timeit([&] { hipLaunchKernelGGL(k_read<2>, dim3(grid), dim3(256), 0, 0, a, n16, sink); }, 20);
        float r4 = timeit([&] { hipLaunchKernelGGL(k_read<4>, dim3(grid), dim3(256), 0, 0, a, n16, sink); }, 20);
        float r8 = timeit([&] { hipLaunchKernelGGL(k_read<8>, dim3(grid), dim3(256), 0, 0, a, n16, sink); }, 20);
        float w4 = timeit([&] { hipLaunchKernelGGL(k_write<4>, dim3(grid), dim3(256), 0, 0, c, n16); }, 20);
        float c4 = timeit([&] { hipLaunchKernelGGL(k_copy<4>, dim3(grid), dim3(256), 0, 0, a, c, n16); }, 20);
        printf("grid %5d  read U2 %.4f ms %.2f TB/s | U4 %.4f %.2f | U8 %.4f %.2f | write U4 %.4f %.2f | copy U4 %.4f %.2f (r+w)\n",
               grid, r2, bytes / r2 / 1e9, r4, bytes / r4 / 1e9, r8, bytes / r8 / 1e9, w4, bytes / w4 / 1e9, c4, 2 * bytes / c4 / 1e9);
    }
    return 0;
}
