// ek_global.h — gfx950 kernels of the SHARD (global watermark) mode.
//
// A key-hash shard of a rule sees only its own rows, each tagged with its global arrival index; the rule's
// WatermarkOp runs over the whole stream on the host that assigns the arrival order, and its WatermarkTuples
// (global arrival after which the watermark advanced, new watermark) reach every shard (ek_push_batch_global,
// include/ekgpu.h). Per row the shard then needs the last tuple before its arrival (late drop,
// watermark_op.go:144-155; hopping empty-window discard, window_op.go:605-655) and the tuple that releases it
// (watermark_op.go:157-204: the first tuple at or after its arrival whose watermark reaches its ts). Both are
// binary searches over the batch's tuple list, which is small next to the rows (one tuple per advance of the
// stream max).
#pragma once
#include "ek_kernels.h"

namespace ek {

struct WmList {
    const int64_t* arr;   // arrival index of each WatermarkTuple's event (strictly increasing)
    const int64_t* ts;    // its watermark (strictly increasing)
    int64_t n;
    int64_t carry;        // watermark before the list (INT64_MIN: none yet)
};

// last watermark emitted before global arrival a
__device__ __forceinline__ int64_t wm_before(const WmList& w, int64_t a) {
    int64_t lo = 0, hi = w.n;   // first k with arr[k] >= a
    while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (w.arr[m] < a) lo = m + 1; else hi = m; }
    return lo > 0 ? w.ts[lo - 1] : w.carry;
}

// Acceptance of the rows of a shard batch: ts >= the watermark before the row's arrival; for hopping windows
// with lateTolerance 0 (hop != 0) also the empty-window discard of k_hop_drop with that watermark as W_{i-1}.
// Counts accepted rows, their min ts and the discarded rows into st (zeroed by k_stats_reduce).
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_accept_global(const int64_t* __restrict__ ts, const int64_t* __restrict__ arr,
                                                          int64_t n, WmList w, int hop, int64_t E1, int64_t H, int64_t L,
                                                          uint8_t* __restrict__ acc, BatchStats* st) {
    int64_t cnt = 0, mn = INT64_MAX, drops = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = ts[i];
        const int64_t wp = wm_before(w, arr[i]);
        bool ok = wp == INT64_MIN || t >= wp;
        if (ok && hop && wp != INT64_MIN && t > wp && t >= E1) {
            const int64_t e_max = E1 + ((t - E1) / H) * H;
            if (e_max - L > wp) { ok = false; drops++; }
        }
        acc[i] = ok ? 1 : 0;
        if (ok) { cnt++; mn = min(mn, t); }
    }
    mn = wave_min64(mn);
    for (int o = 32; o > 0; o >>= 1) { cnt += __shfl_xor(cnt, o, 64); drops += __shfl_xor(drops, o, 64); }
    if ((threadIdx.x & 63) == 0) {
        if (cnt) atomicAdd((unsigned long long*)&st->n_accepted, (unsigned long long)cnt);
        if (mn != INT64_MAX) atomicMin((long long*)&st->min_accepted, (long long)mn);
        if (drops) atomicAdd((unsigned long long*)&st->n_dropped, (unsigned long long)drops);
    }
}
#endif

// Release step of buffer rows [i0, i1) (all released by this batch's tuples): the arrival index of the first
// tuple at or after the row's arrival whose watermark reaches its ts (INT64_MAX if none).
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_release_step_global(const int64_t* __restrict__ bts, const int64_t* __restrict__ barr, int64_t i0,
                                      int64_t i1, WmList w, int64_t* __restrict__ brel) {
    for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = barr[i], t = bts[i];
        int64_t lo = 0, hi = w.n;
        while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (w.arr[m] < a) lo = m + 1; else hi = m; }
        int64_t k = lo;
        lo = 0; hi = w.n;
        while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (w.ts[m] < t) lo = m + 1; else hi = m; }
        k = max(k, lo);
        brel[i] = k < w.n ? w.arr[k] : INT64_MAX;
    }
}
#endif

// flags[i] &= acc[i] (trigger rows that the global watermark accepts)
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_and_flags(uint8_t* __restrict__ flags, const uint8_t* __restrict__ acc, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flags[i] = flags[i] && acc[i];
}
#endif

}  // namespace ek
