// Microbenchmark: LDS atomic throughput on gfx950 for the ops k_agg uses (random keys in a 1024-entry table).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int OP>
__global__ __launch_bounds__(512) void kern(const uint32_t* keys, const double* vals, int iters, double* out) {
    __shared__ unsigned long long tab[1024];
    __shared__ unsigned int tabc[1024];
    for (int k = threadIdx.x; k < 1024; k += 512) { tab[k] = 0; tabc[k] = 0; }
    __syncthreads();
    uint32_t kk = keys[(blockIdx.x * 512 + threadIdx.x) & 65535];
    double v = vals[threadIdx.x];
    for (int i = 0; i < iters; ++i) {
        int kl = (kk + i * 2654435761u) >> 22;   // pseudo-random 10-bit key
        if (OP == 0) atomicAdd(&tabc[kl], 1u);
        if (OP == 1) atomicAdd((double*)&tab[kl], v);
        if (OP == 2) atomicMax(&tab[kl], (unsigned long long)__double_as_longlong(v));
        if (OP == 3) { double* d = (double*)&tab[kl]; *d += v; }   // non-atomic RMW (racy, speed reference)
        if (OP == 4) atomicAdd(&tabc[kl & ~63 | (threadIdx.x & 63)], 1u);  // conflict-free u32
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (double)tab[threadIdx.x & 1023] + tabc[0];
}
int main() {
    uint32_t* keys; double* vals; double* out;
    hipMalloc(&keys, 65536 * 4); hipMalloc(&vals, 512 * 8); hipMalloc(&out, 4096 * 8);
    uint32_t hk[65536]; for (int i = 0; i < 65536; ++i) hk[i] = i * 2654435761u;
    hipMemcpy(keys, hk, sizeof hk, hipMemcpyHostToDevice);
    hipMemset(vals, 0, 512 * 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = 1024, iters = 4096;
    const char* names[] = {"ds_add_u32 random", "ds_add_f64 random", "ds_max_u64 random", "plain f64 RMW", "ds_add_u32 no-conflict"};
    for (int op = 0; op < 5; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            switch (op) {
            case 0: kern<0><<<blocks, 512>>>(keys, vals, iters, out); break;
            case 1: kern<1><<<blocks, 512>>>(keys, vals, iters, out); break;
            case 2: kern<2><<<blocks, 512>>>(keys, vals, iters, out); break;
            case 3: kern<3><<<blocks, 512>>>(keys, vals, iters, out); break;
            case 4: kern<4><<<blocks, 512>>>(keys, vals, iters, out); break;
            }
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            double ops = (double)blocks * 512 * iters;
            if (rep) printf("%-26s %8.3f ms  %8.2f Gop/s  (%.2f lane-ops/clk/CU @2.4GHz)\n", names[op], ms, ops / ms / 1e6,
                            ops / (ms * 1e-3) / 256 / 2.4e9);
        }
    }
    return 0;
}
