// mb_lockstep.hip — microbenchmark of a staging-free C2 layout.
//
// C2 today is two passes: k_part reads the batch (key 4 B + two f64 values) and writes an 18 B/event staging copy
// partitioned by (pane, key bucket); k_agg reads it back and aggregates each partition in LDS. The staging round trip
// is 3.6 GB of the 7 GB a step moves. The layout measured here never stages: the 32 CUs of one XCD all stream the
// SAME row tiles (HBM -> that XCD's L2 once), each CU owning 1/32 of the key space in LDS (2048 keys x count / f64 sum /
// f64 max = 40 KB). A row is aggregated by the one CU whose key range holds it; the other 31 only read its key.
// XCD x takes rows [x N / 8, (x + 1) N / 8); workgroup w runs on XCD w % 8 (the dispatcher's round robin), so
// lane = w / 8 picks the key range. The per-XCD tables are merged at the end (8 x 64 Ki keys, negligible).
//
// Reported: lockstep kernel time, a plain streaming read of the same 20 B/row (the HBM floor of any one-pass design),
// and the two-pass staging equivalent (read 20 B + write 18 B + read 18 B per row, as plain streams). Run under
// rocprofv3 --pmc FETCH_SIZE to see whether HBM is really read once (L2 serving the other 31 CUs).
//
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mb_lockstep tools/mb_lockstep.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kKeys = 65536;
constexpr int kLanes = 32;                  // CUs per XCD
constexpr int kXcd = 8;
constexpr int kRange = kKeys / kLanes;      // keys per CU: 2048
constexpr int kBlock = 1024;
constexpr int kTile = 16384;                // rows per tile step

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t f64_ord(double d) {
    const uint64_t u = (uint64_t)__double_as_longlong(d);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__global__ void k_init(uint32_t* key, double* v0, double* v1, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix((uint64_t)i);
        key[i] = (uint32_t)(h % kKeys);
        v0[i] = (double)(h >> 40) * 1e-4;
        v1[i] = (double)((h >> 12) & 0xFFFFF) * 1e-3;
    }
}

// one workgroup per CU: XCD x = blockIdx.x % 8 streams its eighth of the rows; lane = blockIdx.x / 8 owns keys
// [lane * kRange, + kRange) in LDS
__global__ __launch_bounds__(kBlock) void k_lockstep(const uint32_t* __restrict__ key, const double* __restrict__ v0,
                                                     const double* __restrict__ v1, int64_t n, uint64_t* __restrict__ out) {
    __shared__ uint32_t s_cnt[kRange];
    __shared__ double s_sum[kRange];
    __shared__ unsigned long long s_max[kRange];
    for (int k = threadIdx.x; k < kRange; k += kBlock) { s_cnt[k] = 0; s_sum[k] = 0.0; s_max[k] = 0ull; }
    __syncthreads();
    const int xcd = blockIdx.x % kXcd, lane = blockIdx.x / kXcd;
    const int64_t r0 = n * xcd / kXcd, r1 = n * (xcd + 1) / kXcd;
    const uint32_t lo = (uint32_t)lane * kRange;
    for (int64_t t = r0; t < r1; t += kTile)
        for (int64_t i = t + threadIdx.x; i < min(t + kTile, r1); i += kBlock) {
            const uint32_t k = key[i] - lo;
            if (k >= (uint32_t)kRange) continue;
            atomicAdd(&s_cnt[k], 1u);
            atomicAdd(&s_sum[k], v0[i]);
            atomicMax(&s_max[k], (unsigned long long)f64_ord(v1[i]));
        }
    __syncthreads();
    uint64_t* o = out + ((size_t)xcd * kKeys + lo) * 3;
    for (int k = threadIdx.x; k < kRange; k += kBlock) {
        o[3 * k] = s_cnt[k];
        o[3 * k + 1] = (uint64_t)__double_as_longlong(s_sum[k]);
        o[3 * k + 2] = s_max[k];
    }
}

// streaming reference: every row's 20 B read once (the floor of any one-pass layout)
__global__ void k_stream(const uint4* __restrict__ key, const double2* __restrict__ v0, const double2* __restrict__ v1,
                         int64_t n4, int64_t n2, unsigned long long* sink) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 k = key[i];
        acc += k.x ^ k.y ^ k.z ^ k.w;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        const double2 a = v0[i], b = v1[i];
        acc += (unsigned long long)__double_as_longlong(a.x + b.y) ^ (unsigned long long)__double_as_longlong(a.y + b.x);
    }
    if (acc == 0x1234567ull) atomicAdd(sink, acc);   // keeps the loads
}

// the staging round trip as plain streams: write 18 B/row then read it back
__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    uint32_t* key;
    double *v0, *v1;
    uint64_t* out;
    unsigned long long* sink;
    uint4 *stg, *stg_src;
    CK(hipMalloc(&key, n * 4));
    CK(hipMalloc(&v0, n * 8));
    CK(hipMalloc(&v1, n * 8));
    CK(hipMalloc(&out, (size_t)kXcd * kKeys * 3 * 8));
    CK(hipMalloc(&sink, 8));
    const int64_t stg16 = n * 18 / 16;
    CK(hipMalloc(&stg, stg16 * 16));
    CK(hipMalloc(&stg_src, stg16 * 16));
    CK(hipMemset(stg_src, 0, stg16 * 16));
    hipLaunchKernelGGL(k_init, dim3(8192), dim3(256), 0, 0, key, v0, v1, n);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](auto launch, int reps) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    };
    const float t_lock = timeit([&] { hipLaunchKernelGGL(k_lockstep, dim3(kXcd * kLanes), dim3(kBlock), 0, 0, key, v0, v1, n, out); }, 5);
    const float t_stream = timeit([&] { hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)key, (const double2*)v0,
                                                           (const double2*)v1, n / 4, n / 2, sink); }, 5);
    const float t_stage = timeit([&] {
        // write 18 B/row (read from a second staging-sized buffer: the copy's read stands in for k_part's batch read)
        hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, (const uint4*)stg_src, stg, stg16);
        hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)stg, (const double2*)stg, (const double2*)stg,
                           stg16, 0, sink);                                                       // read it back
    }, 5);
    // check: total count over the per-XCD tables == n
    std::vector<uint64_t> h((size_t)kXcd * kKeys * 3);
    CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t total = 0;
    for (size_t k = 0; k < (size_t)kXcd * kKeys; ++k) total += h[3 * k];
    printf("{\"rows\": %lld, \"rows_counted\": %llu, \"lockstep_ms\": %.4f, \"stream_read_20B_ms\": %.4f, "
           "\"staging_roundtrip_36B_ms\": %.4f, \"lockstep_GBps_of_20B\": %.1f, \"stream_GBps\": %.1f}\n",
           (long long)n, (unsigned long long)total, t_lock, t_stream, t_stage, n * 20.0 / t_lock / 1e6, n * 20.0 / t_stream / 1e6);
    return total == (uint64_t)n ? 0 : 2;
}
