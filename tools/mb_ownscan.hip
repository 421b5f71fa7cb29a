// Microbenchmark: C2-shaped owner-scan aggregation (no staging). Each group of NO workgroups on one XCD streams
// the same contiguous slice of the batch; workgroup o keeps the LDS partial table of keys [o*KPO, (o+1)*KPO) and
// folds in only the events of its keys. The slice is read from HBM once and served NO times from the XCD's L2.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mb_ownscan tools/mb_ownscan.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t f64_to_ord(double x) {
    uint64_t u = (uint64_t)__double_as_longlong(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ void k_fill(uint32_t* key, int64_t* ts, double* t, double* h, int64_t n, uint32_t K) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + 12345;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        key[i] = (uint32_t)(z % K);
        ts[i] = 1541152480000ll + i / 100;
        t[i] = (double)((z >> 11) & 0xFFFFF) / 10000.0;
        h[i] = (double)((z >> 33) & 0xFFFFF) / 10000.0;
    }
}

// plain streaming read of the four columns: the achievable HBM rate for the same bytes
__global__ __launch_bounds__(512) void k_stream4(const uint32_t* key, const int64_t* ts, const double* t, const double* h,
                                                 int64_t n, double* out) {
    double acc = 0;
    int64_t s = 0;
    const int64_t n4 = n / 4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        uint4 k = ((const uint4*)key)[i];
        const longlong2 a = ((const longlong2*)ts)[2 * i], b = ((const longlong2*)ts)[2 * i + 1];
        const double2 c = ((const double2*)t)[2 * i], d = ((const double2*)t)[2 * i + 1];
        const double2 e = ((const double2*)h)[2 * i], f = ((const double2*)h)[2 * i + 1];
        s += k.x + k.y + k.z + k.w + a.x + a.y + b.x + b.y;
        acc += c.x + c.y + d.x + d.y + e.x + e.y + f.x + f.y;
    }
    if (acc == 1234.5 && s == 7) out[0] = acc;
}

// MODE 0: full (values + LDS atomics), 1: keys only (no value loads, count atomics), 2: values loaded, no atomics
template <int NO, int KPO, int BLK, int EPT, int MODE>
__global__ __launch_bounds__(BLK) void k_own(const uint32_t* __restrict__ key, const double* __restrict__ t,
                                             const double* __restrict__ h, int64_t n, const int64_t* __restrict__ pb,
                                             int npanes, int ngroups, uint32_t* out_cnt, double* out_sum,
                                             unsigned long long* out_mx) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double* lsum = (double*)lds;
    unsigned long long* lmx = (unsigned long long*)(lds + 8 * KPO);
    uint32_t* lcnt = (uint32_t*)(lds + 16 * KPO);
    const int b = blockIdx.x;
    const int x = b & 7, i = b >> 3;
    const int grp = i / NO, o = i % NO;
    const int gid = grp * 8 + x;
    if (gid >= ngroups) return;
    int64_t slice = ((n + ngroups - 1) / ngroups + 4095) & ~(int64_t)4095;
    const int64_t lo = gid * slice, hi = min(n, lo + slice);
    const uint32_t klo = (uint32_t)o * KPO;
    double dsink = 0;
    for (int q = 0; q < npanes; ++q) {
        const int64_t a = max(lo, pb[q]), e = min(hi, pb[q + 1]);
        if (a >= e) continue;
        for (int k = threadIdx.x; k < KPO; k += BLK) { lsum[k] = 0; lmx[k] = 0; lcnt[k] = 0; }
        __syncthreads();
        // a..e are multiples of 4 here (1e6-event panes, 4096-aligned slices)
        constexpr int SPAN = BLK * 4 * EPT;
        for (int64_t base = a; base < e; base += SPAN) {
            uint4 kv[EPT];
#pragma unroll
            for (int u = 0; u < EPT; ++u) {
                const int64_t j = base + ((int64_t)u * BLK + threadIdx.x) * 4;
                kv[u] = j < e ? *(const uint4*)(key + j) : make_uint4(~0u, ~0u, ~0u, ~0u);
            }
            double tv[EPT][4], hv[EPT][4];
            uint32_t kl[EPT][4];
#pragma unroll
            for (int u = 0; u < EPT; ++u) {
                const int64_t j = base + ((int64_t)u * BLK + threadIdx.x) * 4;
                const uint32_t kk[4] = {kv[u].x, kv[u].y, kv[u].z, kv[u].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    kl[u][c] = kk[c] - klo;
                    const bool m = kl[u][c] < (uint32_t)KPO;
                    tv[u][c] = 0; hv[u][c] = 0;
                    if ((MODE == 0 || MODE == 2) && m) { tv[u][c] = t[j + c]; hv[u][c] = h[j + c]; }
                }
                if (MODE >= 3 && j < e) {   // coalesced: every lane loads its 4 events' values
                    const double2 t0 = ((const double2*)(t + j))[0], t1 = ((const double2*)(t + j))[1];
                    const double2 h0 = ((const double2*)(h + j))[0], h1 = ((const double2*)(h + j))[1];
                    tv[u][0] = t0.x; tv[u][1] = t0.y; tv[u][2] = t1.x; tv[u][3] = t1.y;
                    hv[u][0] = h0.x; hv[u][1] = h0.y; hv[u][2] = h1.x; hv[u][3] = h1.y;
                }
            }
#pragma unroll
            for (int u = 0; u < EPT; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (kl[u][c] >= (uint32_t)KPO) continue;
                    if (MODE == 2 || MODE == 4) { dsink += tv[u][c] + hv[u][c]; continue; }
                    atomicAdd(&lcnt[kl[u][c]], 1u);
                    if (MODE == 0 || MODE == 3) {
                        atomicAdd(&lsum[kl[u][c]], tv[u][c]);
                        atomicMax(&lmx[kl[u][c]], (unsigned long long)f64_to_ord(hv[u][c]));
                    }
                }
        }
        __syncthreads();
        // flush: this owner's rows of pane q
        for (int k = threadIdx.x; k < KPO; k += BLK) {
            const int64_t r = (int64_t)q * NO * KPO + (int64_t)o * KPO + k;
            if (lcnt[k]) { out_cnt[r] = lcnt[k]; out_sum[r] = lsum[k]; out_mx[r] = lmx[k]; }
        }
        __syncthreads();
    }
    if (dsink == 1234.5) out_sum[0] = dsink;
}

template <int NO, int KPO, int BLK, int EPT, int MODE>
float run_own(const char* name, uint32_t* key, double* t, double* h, int64_t n, int64_t* d_pb, int np, uint32_t* oc, double* os,
              unsigned long long* om, int groups_per_xcd, int reps) {
    const int ngroups = 8 * groups_per_xcd;
    const int grid = 8 * groups_per_xcd * NO;
    const size_t lds = (size_t)KPO * 20;
    CK(hipFuncSetAttribute((const void*)k_own<NO, KPO, BLK, EPT, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_own<NO, KPO, BLK, EPT, MODE>), dim3(grid), dim3(BLK), lds, 0, key, t, h, n, d_pb, np, ngroups, oc, os, om);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_own<NO, KPO, BLK, EPT, MODE>), dim3(grid), dim3(BLK), lds, 0, key, t, h, n, d_pb, np, ngroups, oc, os, om);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-44s grid %4d lds %6zu  %.3f ms  (%.0f GB/s of 20 B/event)\n", name, grid, lds, ms, n * 20.0 / ms / 1e6);
    return ms;
}

int main(int argc, char** argv) {
    const int64_t n = 100000000;
    const uint32_t K = 65536;
    uint32_t* key;
    int64_t* ts;
    double *t, *h;
    CK(hipMalloc(&key, n * 4));
    CK(hipMalloc(&ts, n * 8));
    CK(hipMalloc(&t, n * 8));
    CK(hipMalloc(&h, n * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, key, ts, t, h, n, K);
    const int np = 100;
    std::vector<int64_t> pb(np + 1);
    for (int q = 0; q <= np; ++q) pb[q] = std::min<int64_t>(n, (int64_t)q * 1000000);
    int64_t* d_pb;
    CK(hipMalloc(&d_pb, (np + 1) * 8));
    CK(hipMemcpy(d_pb, pb.data(), (np + 1) * 8, hipMemcpyHostToDevice));
    uint32_t* oc;
    double* os;
    unsigned long long* om;
    const size_t rows = (size_t)np * 70000;
    CK(hipMalloc(&oc, rows * 4));
    CK(hipMalloc(&os, rows * 8));
    CK(hipMalloc(&om, rows * 8));
    double* sink;
    CK(hipMalloc(&sink, 64));
    CK(hipDeviceSynchronize());
    const int reps = 10;
    {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int g : {1024, 2048, 4096}) {
            hipLaunchKernelGGL(k_stream4, dim3(g), dim3(512), 0, 0, key, ts, t, h, n, sink);
            CK(hipEventRecord(a));
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_stream4, dim3(g), dim3(512), 0, 0, key, ts, t, h, n, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ms /= reps;
            printf("stream 4 columns (28 B/event) grid %d: %.3f ms  %.0f GB/s\n", g, ms, n * 28.0 / ms / 1e6);
        }
    }
    // NO owners x KPO keys per owner must cover K = 65536
    run_own<8, 8192, 1024, 2, 3>("NO8 KPO8192 coalesced full", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<8, 8192, 1024, 2, 4>("NO8 KPO8192 coalesced no atomics", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<8, 8192, 1024, 4, 3>("NO8 KPO8192 coalesced full EPT4", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<8, 8192, 1024, 1, 3>("NO8 KPO8192 coalesced full EPT1", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<10, 6554, 1024, 2, 3>("NO10 KPO6554 coalesced full", key, t, h, n, d_pb, np, oc, os, om, 3, reps);
    run_own<10, 6554, 1024, 2, 4>("NO10 KPO6554 coalesced no atomics", key, t, h, n, d_pb, np, oc, os, om, 3, reps);
    run_own<16, 4096, 512, 2, 3>("NO16 KPO4096 coalesced full", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<16, 4096, 512, 2, 4>("NO16 KPO4096 coalesced no atomics", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<8, 8192, 1024, 2, 1>("NO8 KPO8192 keys-only(count)", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<8, 8192, 1024, 2, 2>("NO8 KPO8192 values, no atomics", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<10, 6554, 1024, 2, 0>("NO10 KPO6554 full (3 grp/XCD)", key, t, h, n, d_pb, np, oc, os, om, 3, reps);
    run_own<16, 4096, 512, 2, 0>("NO16 KPO4096 full (4 grp/XCD, 2 WG/CU)", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    run_own<16, 4096, 512, 2, 1>("NO16 KPO4096 keys-only(count)", key, t, h, n, d_pb, np, oc, os, om, 4, reps);
    printf("done\n");
    return 0;
}
