// ek_route.hip — the key-hash router of a multi-GPU rule (gpu = hash(key) mod G per micro-batch).
//
// Every rank ingests a contiguous slice of the global stream (its rows carry consecutive global arrival indices);
// ek_route_partition splits that slice by owner rank, mix64(key) mod G (the same hash as ekgpu.shard.key_owner), into
// G destination segments of one output batch, stably (each segment keeps arrival order), and renames each key to
// its owner's dense id (the shard's dictionary, ekgpu.shard / keys.py, as a device table global key -> local id). The
// segments are then exchanged with one all_to_all per column (RCCL over xGMI, ekgpu.dist.route_exchange); a rank
// receives its rows in source-rank order, i.e. in global arrival order, as ek_push_batch_global requires.
//
// Bound: HBM. One read of the key column for the count pass, then one read and one write of every row for the
// scatter (the rows of one 4096-row tile bound for one destination land on consecutive addresses).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "../../include/ekgpu.h"

namespace {

constexpr int kRouteBlock = 256;
constexpr int kRouteTile = 4096;
constexpr int kRouteMaxDest = 64;

__device__ __forceinline__ uint32_t route_dest(uint32_t key, int G) {
    uint64_t x = (uint64_t)key;   // ek_mix64 (include/ekgpu.h), & (2^62 - 1), mod G: ekgpu.shard.key_owner
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (uint32_t)((x & ((1ull << 62) - 1ull)) % (uint64_t)G);
}

// per tile: rows bound for each destination -> cnt[tile][d]
__global__ __launch_bounds__(kRouteBlock) void k_route_count(const uint32_t* __restrict__ key, int64_t n, int G,
                                                             uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[kRouteMaxDest];
    for (int d = threadIdx.x; d < G; d += kRouteBlock) h[d] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kRouteTile;
    for (int k = threadIdx.x; k < kRouteTile; k += kRouteBlock) {
        const int64_t i = t0 + k;
        if (i < n) atomicAdd(&h[route_dest(key[i], G)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < G; d += kRouteBlock) cnt[(int64_t)blockIdx.x * G + d] = h[d];
}

// one workgroup: per destination, the exclusive prefix over tiles (in place) and the segment bases dbase[0..G]
__global__ __launch_bounds__(1024) void k_route_scan(uint32_t* __restrict__ cnt, int64_t nt, int G, int64_t* __restrict__ dbase) {
    __shared__ int64_t tot[kRouteMaxDest];
    for (int d = threadIdx.x >> 6; d < G; d += 1024 / 64) {   // one wave per destination
        const int lane = threadIdx.x & 63;
        int64_t run = 0;
        for (int64_t c0 = 0; c0 < nt; c0 += 64) {
            const int64_t t = c0 + lane;
            const uint32_t v = t < nt ? cnt[t * G + d] : 0u;
            uint32_t x = v;
            for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
            if (t < nt) cnt[t * G + d] = (uint32_t)(run + x - v);   // (per-destination totals < 2^31: host-checked)
            run += __shfl(x, 63, 64);
        }
        if (lane == 0) tot[d] = run;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t b = 0;
        for (int d = 0; d < G; ++d) { dbase[d] = b; b += tot[d]; }
        dbase[G] = b;
    }
}

struct RouteCols {
    const void* in[EK_MAX_COLUMNS];
    void* out[EK_MAX_COLUMNS];
    int32_t width[EK_MAX_COLUMNS];   // 4 or 8 bytes
    int32_t n_cols;
    int32_t key_col;
    const uint32_t* key_map;         // global key -> owner's dense id (nullptr: keep the key)
    uint32_t key_map_size;           // keys at or past it are left as they are and flagged (bad_key)
    int32_t* bad_key;
    int64_t* out_arrival;            // global arrival of every routed row (nullptr: none)
    int64_t arrival_base;
};

// stable scatter: the tile's rows in order, 256 at a time; a row's slot = its destination's base + the tile's offset
// + the rows of that destination before it in the tile (ballot ranks inside the wave, LDS prefix across waves)
__global__ __launch_bounds__(kRouteBlock) void k_route_scatter(RouteCols rc, int64_t n, int G, const uint32_t* __restrict__ toff,
                                                               const int64_t* __restrict__ dbase) {
    __shared__ uint32_t run[kRouteMaxDest];
    __shared__ uint32_t wcnt[kRouteBlock / 64][kRouteMaxDest];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int d = threadIdx.x; d < G; d += kRouteBlock) run[d] = toff[(int64_t)blockIdx.x * G + d];
    const uint32_t* key = (const uint32_t*)rc.in[rc.key_col];
    const int64_t t0 = (int64_t)blockIdx.x * kRouteTile;
    const unsigned long long lt = (1ull << lane) - 1ull;
    __syncthreads();
    for (int k0 = 0; k0 < kRouteTile; k0 += kRouteBlock) {
        const int64_t i = t0 + k0 + threadIdx.x;
        const bool valid = i < n;
        const uint32_t kv = valid ? key[i] : 0u;
        const int d = valid ? (int)route_dest(kv, G) : -1;
        uint32_t rank = 0;
        for (int q = 0; q < G; ++q) {
            const unsigned long long m = __ballot(d == q);
            if (d == q) rank = (uint32_t)__popcll(m & lt);
            if (lane == 0) wcnt[wv][q] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if (valid) {
            uint32_t before = run[d];
            for (int w = 0; w < wv; ++w) before += wcnt[w][d];
            const int64_t pos = dbase[d] + (int64_t)before + rank;
            for (int c = 0; c < rc.n_cols; ++c) {
                if (c == rc.key_col) {
                    uint32_t kk = kv;
                    if (rc.key_map) {
                        if (kv < rc.key_map_size) kk = rc.key_map[kv];
                        else atomicOr(rc.bad_key, 1);
                    }
                    ((uint32_t*)rc.out[c])[pos] = kk;
                } else if (rc.width[c] == 4) {
                    ((uint32_t*)rc.out[c])[pos] = ((const uint32_t*)rc.in[c])[i];
                } else {
                    ((int64_t*)rc.out[c])[pos] = ((const int64_t*)rc.in[c])[i];
                }
            }
            if (rc.out_arrival) rc.out_arrival[pos] = rc.arrival_base + i;
        }
        __syncthreads();
        for (int q = threadIdx.x; q < G; q += kRouteBlock) {
            uint32_t s = 0;
            for (int w = 0; w < kRouteBlock / 64; ++w) s += wcnt[w][q];
            run[q] += s;
        }
        __syncthreads();
    }
}

struct RouteScratch {
    int device = -1;
    void* cnt = nullptr;
    size_t cnt_bytes = 0;
    int64_t* dbase = nullptr;        // [kRouteMaxDest + 1] segment bases, then the bad-key flag
    int64_t* h_base = nullptr;
};
thread_local RouteScratch g_route;

}  // namespace

extern "C" int ek_route_partition(int device, void* stream, const ek_batch* batch, const int32_t* column_type,
                                  int32_t key_column, int32_t n_dest, const uint32_t* key_map, uint32_t key_map_size,
                                  int64_t arrival_base,
                                  void* const* out_columns, int64_t* out_arrival, int64_t* dest_counts) {
    if (!batch || !column_type || !out_columns || !dest_counts) return EK_ERR_INVALID;
    if (n_dest < 1 || n_dest > kRouteMaxDest) return EK_ERR_UNSUPPORTED;
    if (batch->memory != EK_MEM_DEVICE) return EK_ERR_INVALID;
    const int64_t n = batch->n_rows;
    if (n < 0 || n > ((int64_t)1 << 31) - 1) return EK_ERR_UNSUPPORTED;
    if (n == 0) {   // (an empty slice: nothing to route, every segment empty)
        for (int d = 0; d < n_dest; ++d) dest_counts[d] = 0;
        return EK_OK;
    }
    int nc = 0;
    while (nc < EK_MAX_COLUMNS && batch->columns[nc]) ++nc;
    if (key_column < 0 || key_column >= nc || column_type[key_column] != EK_COL_U32) return EK_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return EK_ERR_DEVICE;
    hipStream_t s = (hipStream_t)stream;
    RouteScratch& R = g_route;
    if (R.device != device) {
        if (R.cnt) { hipFree(R.cnt); hipFree(R.dbase); hipHostFree(R.h_base); }
        R = RouteScratch{};
        R.device = device;
        if (hipMalloc((void**)&R.dbase, (kRouteMaxDest + 2) * 8) != hipSuccess) return EK_ERR_NOMEM;
        if (hipHostMalloc((void**)&R.h_base, (kRouteMaxDest + 2) * 8) != hipSuccess) return EK_ERR_NOMEM;
    }
    const int64_t nt = std::max<int64_t>(1, (n + kRouteTile - 1) / kRouteTile);
    const size_t cb = (size_t)nt * n_dest * 4;
    if (cb > R.cnt_bytes) {
        if (R.cnt) { hipStreamSynchronize(s); hipFree(R.cnt); }
        if (hipMalloc(&R.cnt, cb) != hipSuccess) { R.cnt = nullptr; R.cnt_bytes = 0; return EK_ERR_NOMEM; }
        R.cnt_bytes = cb;
    }
    RouteCols rc{};
    rc.n_cols = nc;
    rc.key_col = key_column;
    rc.key_map = key_map;
    rc.key_map_size = key_map_size;
    rc.bad_key = (int32_t*)(R.dbase + kRouteMaxDest + 1);
    rc.out_arrival = out_arrival;
    rc.arrival_base = arrival_base;
    for (int c = 0; c < nc; ++c) {
        if (!out_columns[c]) return EK_ERR_INVALID;
        rc.in[c] = batch->columns[c];
        rc.out[c] = out_columns[c];
        rc.width[c] = column_type[c] == EK_COL_U32 ? 4 : 8;
    }
    if (n > 0) {
        hipMemsetAsync(rc.bad_key, 0, 8, s);
        hipLaunchKernelGGL(k_route_count, dim3((unsigned)nt), dim3(kRouteBlock), 0, s, (const uint32_t*)batch->columns[key_column], n,
                           n_dest, (uint32_t*)R.cnt);
        hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, s, (uint32_t*)R.cnt, nt, n_dest, R.dbase);
        hipLaunchKernelGGL(k_route_scatter, dim3((unsigned)nt), dim3(kRouteBlock), 0, s, rc, n, n_dest, (const uint32_t*)R.cnt,
                           (const int64_t*)R.dbase);
        hipMemcpyAsync(R.h_base, R.dbase, (size_t)(n_dest + 1) * 8, hipMemcpyDeviceToHost, s);
        hipMemcpyAsync(R.h_base + kRouteMaxDest + 1, R.dbase + kRouteMaxDest + 1, 8, hipMemcpyDeviceToHost, s);
    } else {
        memset(R.h_base, 0, (size_t)(n_dest + 1) * 8);
    }
    if (hipStreamSynchronize(s) != hipSuccess) return EK_ERR_DEVICE;
    for (int d = 0; d < n_dest; ++d) dest_counts[d] = R.h_base[d + 1] - R.h_base[d];
    return R.h_base[kRouteMaxDest + 1] ? EK_ERR_INVALID : EK_OK;   // a key outside the dictionary
}
