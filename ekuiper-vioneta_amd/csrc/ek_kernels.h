// ek_kernels.h — gfx950 kernels of the window/aggregate engine (pane-partial mode).
//
// Data path for one micro-batch (columnar, HBM resident):
//   k_stats         one pass over ts: min/max, arrival sortedness           (watermark_op.go:144-155 inputs)
//   k_chunk_max / k_scan_max / k_accept   late-event drop for out-of-order batches
//                   accept(i) = ts_i >= max(ts_<i) - lateTol                (watermark_op.go:144-155)
//   k_pane_bounds   sorted batches: first event index of each pane (binary search)
//   k_hist          per chunk histogram over partitions (pane, key bucket) after WHERE
//   k_scan_*        exclusive scan of the partition-major histogram
//   k_scatter       route rows into contiguous per-partition staging runs (key low bits + values)
//   k_agg           one workgroup per partition: LDS aggregation (count/sum/min/max, then the
//                   two-pass M2 for var/stddev), merged into the per-(pane,key) partial state
//   k_finalize      per closed window: merge its panes, finalise aggregates (funcs_agg.go), HAVING,
//                   compact result rows
// Everything is bandwidth-bound integer/f64 scan work: no MFMA.
#pragma once
#include "ek_device.h"

// The non-template kernels of the ek_*.h headers are compiled by the engine's unit only: the units that instantiate the
// big template kernel families (ek_tpl_*.hip, compiled in parallel) define EK_NO_PLAIN_KERNELS before including them.

namespace ek {

struct BatchStats {
    int64_t min_ts;
    int64_t max_ts;
    int64_t n_accepted;
    int64_t min_accepted;
    int32_t unsorted;
    int32_t pad;
    int64_t max_gap;    // max over arrival-adjacent pairs of ts[i] - ts[i-1] (ts[0] - seed when seeded)
    int64_t n_dropped;  // events removed by the hopping empty-window discard (k_hop_drop)
};

// What the fused sorted pass (k_part MODE 3) found: the batch is used only if it is ts-sorted, no chunk spans more
// than fz_mp panes, and (hopping, lateTolerance 0) no arrival gap exceeds the window
struct FzStatus {
    int32_t unsorted;
    int32_t overflow;
    unsigned long long max_gap;
};

struct PaneGrid {
    int64_t origin;     // tumbling: E1 (pane 0 = (-inf,E1)); hopping: E1 - L (pane 0 = [origin, origin+P))
    int64_t P;          // pane length (ms)
    int32_t tumbling;
};

__device__ __forceinline__ int64_t pane_of(const PaneGrid& g, int64_t ts) {
    if (g.tumbling) return ts < g.origin ? 0 : floordiv64(ts - g.origin, g.P) + 1;
    return ts < g.origin ? -1 : floordiv64(ts - g.origin, g.P);
}

// ---------------------------------------------------------------- wave / block reductions
__device__ __forceinline__ int64_t wave_min64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
    return v;
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
    return v;
}

// ---------------------------------------------------------------- k_stats
// One streaming pass over ts (16 B per lane per load): min, max and "arrival order is non-decreasing".
// GAP (hopping, lateTolerance 0 only): also the widest arrival gap, for the empty-window discard check.
template <bool GAP>
__global__ __launch_bounds__(kBlock) void k_stats(const int64_t* __restrict__ ts, int64_t n, int64_t seed, BatchStats* part) {
    int64_t mn = INT64_MAX, mx = INT64_MIN, mg = INT64_MIN;
    int uns = 0;
    const int64_t npair = n >> 1;
    const longlong2* t2 = (const longlong2*)ts;
    const int lane = threadIdx.x & 63;
    constexpr int U = 4;   // pairs in flight per thread
    const int64_t stride = (int64_t)gridDim.x * kBlock * U;
    for (int64_t base = (int64_t)blockIdx.x * kBlock * U; base < npair; base += stride) {
        longlong2 v[U];
        int64_t lp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t pi = base + u * kBlock + threadIdx.x;
            v[u] = pi < npair ? t2[pi] : make_longlong2(INT64_MAX, INT64_MAX);
            lp[u] = (lane == 0 && pi > 0 && pi < npair) ? ts[2 * pi - 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t pi = base + u * kBlock + threadIdx.x;
            // previous element of this pair = .y of the lane below; lane 0 reads it from memory
            int64_t prev = __shfl_up(v[u].y, 1, 64);
            if (lane == 0) prev = pi > 0 ? lp[u] : v[u].x;
            if (pi < npair) {
                uns |= (v[u].x < prev) | (v[u].y < v[u].x);
                if (GAP) mg = max(mg, max(v[u].x - prev, v[u].y - v[u].x));
                mn = min(mn, min(v[u].x, v[u].y));
                mx = max(mx, max(v[u].x, v[u].y));
            }
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // odd tail element
        int64_t last = ts[n - 1];
        mn = min(mn, last);
        mx = max(mx, last);
        if (n > 1) { uns |= last < ts[n - 2]; if (GAP) mg = max(mg, last - ts[n - 2]); }
    }
    // the gap between the carried stream max and the first event (hopping empty-window check)
    if (GAP && blockIdx.x == 0 && threadIdx.x == 0 && n > 0 && seed != INT64_MIN) mg = max(mg, ts[0] - seed);
    mn = wave_min64(mn);
    mx = wave_max64(mx);
    if (GAP) mg = wave_max64(mg);
    uns = __any(uns);
    // one partial per block (same-address atomics from every wave would serialise at the memory side)
    __shared__ int64_t smn[kBlock / 64], smx[kBlock / 64];
    __shared__ int64_t smg[kBlock / 64];
    __shared__ int suns[kBlock / 64];
    if (lane == 0) { smn[threadIdx.x >> 6] = mn; smx[threadIdx.x >> 6] = mx; smg[threadIdx.x >> 6] = mg; suns[threadIdx.x >> 6] = uns; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) { mn = min(mn, smn[w]); mx = max(mx, smx[w]); mg = max(mg, smg[w]); uns |= suns[w]; }
        part[blockIdx.x] = BatchStats{mn, mx, 0, INT64_MAX, uns, 0, mg, 0};
    }
}

#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(1024) void k_stats_reduce(const BatchStats* __restrict__ part, int nb, BatchStats* st) {
    int64_t mn = INT64_MAX, mx = INT64_MIN, mg = INT64_MIN;
    int uns = 0;
    for (int k = threadIdx.x; k < nb; k += 1024) {
        mn = min(mn, part[k].min_ts); mx = max(mx, part[k].max_ts); mg = max(mg, part[k].max_gap); uns |= part[k].unsorted;
    }
    mn = wave_min64(mn);
    mx = wave_max64(mx);
    mg = wave_max64(mg);
    uns = __any(uns);
    __shared__ int64_t smn[16], smx[16], smg[16];
    __shared__ int su[16];
    if ((threadIdx.x & 63) == 0) { smn[threadIdx.x >> 6] = mn; smx[threadIdx.x >> 6] = mx; smg[threadIdx.x >> 6] = mg; su[threadIdx.x >> 6] = uns; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) { mn = min(mn, smn[w]); mx = max(mx, smx[w]); mg = max(mg, smg[w]); uns |= su[w]; }
        st->min_ts = mn;
        st->max_ts = mx;
        st->max_gap = mg;
        st->n_dropped = 0;
        st->unsorted = uns;
        st->n_accepted = 0;
        st->min_accepted = INT64_MAX;
    }
}
#endif

// ---------------------------------------------------------------- late-event drop (out-of-order batches)
constexpr int kAccPerThread = 16;
constexpr int kAccChunk = kBlock * kAccPerThread;  // 4096 events per block

#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_chunk_max(const int64_t* __restrict__ ts, int64_t n, int64_t* cmax) {
    int64_t base = (int64_t)blockIdx.x * kAccChunk;
    int64_t mx = INT64_MIN;
    for (int k = threadIdx.x; k < kAccChunk; k += kBlock) {
        int64_t i = base + k;
        if (i < n) mx = max(mx, ts[i]);
    }
    mx = wave_max64(mx);
    __shared__ int64_t s[kBlock / 64];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) cmax[blockIdx.x] = max(max(s[0], s[1]), max(s[2], s[3]));
}
#endif

// exclusive prefix max over chunk maxima, seeded with the carried stream max (single workgroup; the threads' partial
// maxima are scanned with wave shuffles, not by one thread)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(1024) void k_scan_max(int64_t* cmax, int nch, int64_t seed) {
    __shared__ int64_t s_w[16];
    const int per = (nch + 1023) / 1024;
    const int b = threadIdx.x * per, e = min(nch, b + per);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int64_t m = INT64_MIN;
    for (int i = b; i < e; ++i) m = max(m, cmax[i]);
    int64_t x = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x = max(x, y);
    }
    int64_t run = __shfl_up(x, 1, 64);
    if (lane == 0) run = INT64_MIN;
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    run = max(run, seed);
    for (int w = 0; w < wv; ++w) run = max(run, s_w[w]);
    for (int i = b; i < e; ++i) { const int64_t v = cmax[i]; cmax[i] = run; run = max(run, v); }
}
#endif

// per-event acceptance of a 4096-event chunk; the chunk's (accepted count, min accepted ts) go to part[2 * chunk]
// (reduced by k_accept_reduce: one atomic per wave on two counters serialised ~1.5 M atomics per 1e8 events)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_accept(const int64_t* __restrict__ ts, int64_t n, const int64_t* excl,
                                                   int64_t late_tol, uint8_t* acc, int64_t* __restrict__ part) {
    __shared__ int64_t s_w[kBlock / 64], s_c[kBlock / 64], s_m[kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kAccChunk + (int64_t)threadIdx.x * kAccPerThread;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int64_t v[kAccPerThread];
    int64_t lm = INT64_MIN;
    if (base + kAccPerThread <= n && ((uintptr_t)ts & 15) == 0) {
#pragma unroll
        for (int k = 0; k < kAccPerThread; k += 2) {   // 16-B loads (base is 16-event aligned)
            const longlong2 q = *(const longlong2*)(ts + base + k);
            v[k] = q.x;
            v[k + 1] = q.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kAccPerThread; ++k) v[k] = base + k < n ? ts[base + k] : INT64_MIN;
    }
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) lm = max(lm, v[k]);
    // exclusive prefix max of the threads' maxima over the block (wave shuffles + one LDS step)
    int64_t x = lm;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x = max(x, y);
    }
    int64_t run = __shfl_up(x, 1, 64);
    if (lane == 0) run = INT64_MIN;
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    run = max(run, excl[blockIdx.x]);
    for (int w = 0; w < wv; ++w) run = max(run, s_w[w]);
    int64_t cnt = 0, mn = INT64_MAX;
    uint32_t pk[kAccPerThread / 4] = {};
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) {
        if (base + k < n) {
            // W_{i-1} = M_{i-1} - lateTol; no watermark yet (run == INT64_MIN) accepts everything
            const bool ok = (run == INT64_MIN) || (v[k] >= run - late_tol);
            pk[k >> 2] |= (ok ? 1u : 0u) << ((k & 3) * 8);
            if (ok) { cnt++; mn = min(mn, v[k]); }
            run = max(run, v[k]);
        }
    }
    if (base + kAccPerThread <= n) {
        *(uint4*)(acc + base) = make_uint4(pk[0], pk[1], pk[2], pk[3]);   // one 16-B store
    } else {
        for (int k = 0; k < kAccPerThread; ++k)
            if (base + k < n) acc[base + k] = (uint8_t)((pk[k >> 2] >> ((k & 3) * 8)) & 1u);
    }
    mn = wave_min64(mn);
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) { s_c[wv] = cnt; s_m[wv] = mn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t c = 0, m = INT64_MAX;
        for (int w = 0; w < kBlock / 64; ++w) { c += s_c[w]; m = min(m, s_m[w]); }
        part[2 * blockIdx.x] = c;
        part[2 * blockIdx.x + 1] = m;
    }
}
#endif

#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(1024) void k_accept_reduce(const int64_t* __restrict__ part, int nch, BatchStats* st) {
    __shared__ int64_t s_c[16], s_m[16];
    int64_t c = 0, m = INT64_MAX;
    for (int i = threadIdx.x; i < nch; i += 1024) { c += part[2 * i]; m = min(m, part[2 * i + 1]); }
    m = wave_min64(m);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) { s_c[threadIdx.x >> 6] = c; s_m[threadIdx.x >> 6] = m; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t tc = 0, tm = INT64_MAX;
        for (int w = 0; w < 16; ++w) { tc += s_c[w]; tm = min(tm, s_m[w]); }
        st->n_accepted = tc;
        st->min_accepted = tm;
    }
}
#endif

// Hopping windows with lateTolerance 0: the empty-window discard of window_op.go:605-655 (handleInputs). When the
// watermark step of event i triggers a hopping window [e - L, e) that holds no released event, handleInputs finds
// no member (nextleft < 0) and returns inputs[:0]: every buffered input is dropped. With lateTolerance 0 the only
// buffered input that is not expired at that step is event i itself (events released earlier are <= the previous
// watermark < e - L, and the watermark rises to ts_i exactly at i), so event i reaches no window. Window ends lie on
// the grid E1 + k H; the largest one <= ts_i is e_max, and some triggered window is empty iff
// e_max - L > W_{i-1} (the watermark before i, the exclusive running max of ts seeded with the carried stream max).
// acc_out[i] = accepted(i) && !dropped(i); accepted = acc_in[i] (out-of-order batches) or i >= start (sorted).
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_hop_drop(const int64_t* __restrict__ ts, int64_t n, const int64_t* excl,
                                                     int64_t start, const uint8_t* acc_in, int64_t E1, int64_t H,
                                                     int64_t L, uint8_t* acc_out, BatchStats* st) {
    __shared__ int64_t tmax[kBlock];
    const int64_t base = (int64_t)blockIdx.x * kAccChunk + (int64_t)threadIdx.x * kAccPerThread;
    int64_t v[kAccPerThread];
    int64_t lm = INT64_MIN;
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) {
        const int64_t i = base + k;
        v[k] = i < n ? ts[i] : INT64_MIN;
        lm = max(lm, v[k]);
    }
    tmax[threadIdx.x] = lm;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = excl[blockIdx.x];
        for (int t = 0; t < kBlock; ++t) { int64_t x = tmax[t]; tmax[t] = run; run = max(run, x); }
    }
    __syncthreads();
    int64_t run = tmax[threadIdx.x];
    int64_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) {
        const int64_t i = base + k;
        if (i < n) {
            const bool a = acc_in ? acc_in[i] != 0 : i >= start;
            bool drop = false;
            if (a && run != INT64_MIN && v[k] > run && v[k] >= E1) {
                const int64_t e_max = E1 + ((v[k] - E1) / H) * H;
                drop = e_max - L > run;
            }
            acc_out[i] = (a && !drop) ? 1 : 0;
            cnt += drop;
            run = max(run, v[k]);
        }
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd((unsigned long long*)&st->n_dropped, (unsigned long long)cnt);
}
#endif

// first index in [lo, hi) with ts >= start of pane q_lo + k (sorted batches; k = 0 -> lo for pane 0 of tumbling).
// One wave per pane, 64-ary search: each round the 64 lanes probe 64 evenly spaced rows of the bracket and a ballot
// narrows it 65-fold, so a 1e8-row batch costs 5 dependent load rounds instead of 27.
constexpr int kBoundsBlock = 256;
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBoundsBlock) void k_pane_bounds(const int64_t* __restrict__ ts, int64_t lo, int64_t hi,
                                                              PaneGrid g, int64_t q_lo, int nb, int64_t* out) {
    const int lane = threadIdx.x & 63;
    const int k = blockIdx.x * (kBoundsBlock / 64) + (threadIdx.x >> 6);
    if (k >= nb) return;
    if (k == nb - 1) { if (lane == 0) out[k] = hi; return; }
    const int64_t q = q_lo + k;
    int64_t x;
    if (g.tumbling) x = q == 0 ? INT64_MIN : g.origin + (q - 1) * g.P;
    else x = g.origin + q * g.P;
    int64_t a = lo, b = hi;   // the answer lies in [a, b]
    while (b - a > 64) {
        const int64_t m = a + ((b - a) * (lane + 1)) / 65;
        const unsigned long long below = __ballot(ts[m] < x);
        const int c = __popcll(below);   // probes 0 .. c-1 are below x (ts is non-decreasing)
        const int64_t mlo = __shfl(m, c > 0 ? c - 1 : 0, 64);
        const int64_t mhi = __shfl(m, c < 64 ? c : 63, 64);
        if (c > 0) a = mlo + 1;
        if (c < 64) b = mhi;
    }
    const int64_t m = a + lane;
    const unsigned long long below = __ballot(m < b && ts[m] < x);
    if (lane == 0) out[k] = a + __popcll(below);
}
#endif

// The fused sorted pass's first look at a batch: its first and last ts (the pane range, if it is sorted) and a
// cleared verdict block — one tiny launch and one 16-byte read-back instead of the whole ts pass
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_fz_prep(const int64_t* __restrict__ ts, int64_t n, FzStatus* st, int64_t* ends) {
    if (threadIdx.x == 0) {
        ends[0] = ts[0];
        ends[1] = ts[n - 1];
        st->unsorted = 0;
        st->overflow = 0;
        st->max_gap = 0;
    }
}
#endif

// per-window result counters of the windows handed out by a poll: one launch instead of four fills
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_zero_wins(int64_t n, int64_t* wcnt, int32_t* werr, int64_t* wmc, int64_t* wmh) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        wcnt[i] = 0;
        werr[i] = 0;
        wmc[i] = 0;
        wmh[i] = 0;
    }
}
#endif

// Panes no group touched (bound by a window before any event reached them): their ring slots are zeroed — the count
// row (per_words u64) plus the per-slot error / membership / witness words — in one launch, blockIdx.y = list entry
// (instead of five fills per slot, most of them of a few bytes)
constexpr int kZeroSlotsMax = 64;
struct SlotList { int32_t n; int32_t s[kZeroSlotsMax]; };
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_zero_slots(SlotList L, uint64_t* __restrict__ cnt, int64_t per_words, int32_t* __restrict__ perr,
                             int64_t* __restrict__ pmc, uint64_t* __restrict__ pmh, uint8_t* __restrict__ pwit, int wit_bytes) {
    if ((int)blockIdx.y >= L.n) return;
    const int64_t s = L.s[blockIdx.y];
    uint64_t* row = cnt + s * per_words;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < per_words; i += (int64_t)gridDim.x * blockDim.x)
        row[i] = 0;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) { perr[s] = 0; pmc[s] = 0; pmh[s] = 0; }
        if (pwit)
            for (int b = threadIdx.x; b < wit_bytes; b += blockDim.x) pwit[s * wit_bytes + b] = 0;
    }
}
#endif

// first index in [lo, hi) with ts >= bound[k] (sorted batches)
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_lower_bound(const int64_t* __restrict__ ts, int64_t lo, int64_t hi, const int64_t* bound, int nb,
                              int64_t* out) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nb) return;
    int64_t x = bound[k], a = lo, b = hi;
    while (a < b) { int64_t m = (a + b) >> 1; if (ts[m] < x) a = m + 1; else b = m; }
    out[k] = a;
}
#endif

// ---------------------------------------------------------------- error witnesses
// Error witness (ek_window_error, ek_errmsg.h): the earliest offender of one window / pane — a row whose WHERE failed
// (v / tag: the columns the program reads, by column id) or a group whose HAVING did (the aggregate slots it reads,
// by slot) — in (o1, o2) order. Offers serialise on a per-record lock, so the record is the minimum whatever the
// order of the offers; zeroed = empty. Tags are Val tags (V_NULL .. V_ERR).
struct WitRec {
    unsigned long long o1, o2;
    int32_t lock, set;
    int64_t v[EK_MAX_AGGS];
    uint8_t tag[EK_MAX_AGGS];
};
static_assert(EK_MAX_AGGS >= EK_MAX_COLUMNS, "witness slots cover the columns");

// One lane at a time offers (o1, o2) to r; fill(r) writes the values under the lock when the offer is the new minimum.
// Divergent callers are fine: the active lanes take turns (a lane spinning on the lock never waits on its own wave).
template <typename F>
__device__ __forceinline__ void wit_offer(WitRec* r, unsigned long long o1, unsigned long long o2, F fill) {
    unsigned long long m = __ballot(1);
    const int lane = (int)__lane_id();
    while (m) {
        const int l = __ffsll((long long)m) - 1;
        if (lane == l) {
            while (atomicCAS(&r->lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
            __threadfence();
            const int set = __hip_atomic_load(&r->set, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long a1 = __hip_atomic_load(&r->o1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long a2 = __hip_atomic_load(&r->o2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!set || o1 < a1 || (o1 == a1 && o2 < a2)) {
                fill(r);
                r->o1 = o1;
                r->o2 = o2;
                r->set = 1;
            }
            __threadfence();
            atomicExch(&r->lock, 0);
        }
        m &= m - 1;
    }
}
__device__ __forceinline__ void wit_put(WitRec* r, int k, const Val& v) {
    r->tag[k] = (uint8_t)v.tag;
    r->v[k] = v.tag == V_F64 ? (int64_t)__double_as_longlong(v.f) : v.i;
}
// a failed WHERE row: the columns its program reads
__device__ inline void wit_where_row(WitRec* r, unsigned long long o1, unsigned long long o2, const DPlan& p,
                                     const DBatch& b, int64_t row) {
    wit_offer(r, o1, o2, [&](WitRec* w) {
        for (int k = 0; k < p.n_where; ++k) {
            if (p.where_prog[k].op != EK_OP_COL) continue;
            const int c = p.where_prog[k].arg;
            wit_put(w, c, col_val(p, b, c, row));
        }
    });
}
// copy a set record (one thread)
__device__ inline void wit_copy(WitRec* dst, const WitRec* src) {
    if (!src->set) return;
    dst->o1 = src->o1;
    dst->o2 = src->o2;
    for (int k = 0; k < EK_MAX_AGGS; ++k) { dst->v[k] = src->v[k]; dst->tag[k] = src->tag[k]; }
    dst->set = 1;
}

// ---------------------------------------------------------------- partition pass
struct GroupDesc {
    int64_t lo, hi;        // event index range in the batch
    int64_t q_lo;          // first pane of the group
    int32_t n_panes;       // panes in the group
    int32_t nb;            // key buckets per pane
    int32_t kbits;         // keys per bucket = 1 << kbits
    int32_t chunk;         // events per chunk (one workgroup)
    int32_t nch;           // chunks in the group
    int32_t np;            // partitions = n_panes * nb
    int32_t ring;          // pane-slot ring size
    int32_t has_accept;    // acc[] valid
    int32_t sorted;        // ts non-decreasing: pane of event i from the pane index boundaries pbnd[]
    int32_t pad;           // diagnostic knobs (0 in production)
    int64_t abase;         // chunk grid origin: lo rounded down to 16 rows (chunk k = [abase + k*chunk, +chunk) ∩ [lo, hi))
    int64_t nbatch;        // rows in the batch (vector loads never read past it)
    // hot plan scalars (kernel arguments stay in SGPRs; DPlan loads inside LDS-atomic loops re-issue)
    int32_t key_col, ts_col, n_where;
    uint32_t num_keys;
    // per-pane descriptors (device arrays, one upload per group)
    const int64_t* pbnd;   // sorted groups: pbnd[k] = first event of pane q_lo + k (k <= n_panes)
    const int64_t* dbase;  // direct emission: result row base of pane r's window, or -1
    const int32_t* didx;   // direct emission: window index of pane r
    const uint8_t* fresh;  // 1: pane r was claimed for this group (its partials are written, not merged)
    const int64_t* voff;   // range mode (virtual panes): physical row of virtual row v in pane r = v + voff[r]
    int32_t* cpa;          // first pane (group-relative) of every chunk, written by k_part for k_agg
    // WHERE error witnesses (nullptr: the plan's WHERE cannot fail): per pane slot like pane_err, ordered by
    // (ts, wit_o2 + row) in pane mode (release order), by buffer row in range mode (wit_ts = 0)
    WitRec* pwit;
    int64_t wit_o2;
    int32_t wit_ts;
    int32_t pad2;          // layout variants (EKGPU_VARIANT; results stay valid)
    int32_t mruns;         // k_agg: most chunk runs one partition of the launch holds (sizes its LDS run tables)
    // k_part MODE 3 (the fused sorted pass, FzStatus): panes per chunk the ctab rows hold, 1 = also the widest
    // arrival gap, the device pane bounds it writes (pbnd_out[k] = first row of pane q_lo + k, 0 < k < n_panes)
    int32_t fz_mp, fz_gap;
    int64_t* pbnd_out;
    FzStatus* fz_st;
};


constexpr int kMaxGroupPanes = 64;
#ifndef EK_PART_BLOCK
#define EK_PART_BLOCK 512
#endif
#ifndef EK_PART_TILE
#define EK_PART_TILE 4096
#endif
constexpr int kPartBlock = EK_PART_BLOCK;    // k_part workgroup (8 wave64s)
constexpr int kTile = EK_PART_TILE;          // events staged and sorted in LDS per k_part tile
constexpr int kTileE = kTile / kPartBlock;   // events per thread per tile
constexpr int kMaxLocalParts = 2048;         // chunk-local partitions sorted through LDS

__device__ __forceinline__ void chunk_range(const GroupDesc& gd, int64_t* a0, int64_t* c0, int64_t* c1) {
    *a0 = gd.abase + (int64_t)blockIdx.x * gd.chunk;
    *c0 = max(gd.lo, *a0);
    *c1 = min(gd.hi, *a0 + gd.chunk);
}

// Pane range [pa, pb] touched by the chunk [c0, c1). pbnd[k] = first event of pane q_lo + k (k <= n_panes).
__device__ __forceinline__ void chunk_panes(const GroupDesc& gd, int64_t c0, int64_t c1, int* pa, int* pb) {
    const int64_t* pbnd = gd.pbnd;
    if (!gd.sorted) { *pa = 0; *pb = gd.n_panes - 1; return; }
    // pa = last pane whose first row <= c0; pb = last pane whose first row < c1 (binary searches)
    int lo = 0, hi = gd.n_panes - 1;
    while (lo < hi) { int m = (lo + hi + 1) >> 1; if (pbnd[m] <= c0) lo = m; else hi = m - 1; }
    *pa = lo;
    hi = gd.n_panes - 1;
    while (lo < hi) { int m = (lo + hi + 1) >> 1; if (pbnd[m] < c1) lo = m; else hi = m - 1; }
    *pb = lo;
}

constexpr int kMaxChunkBnd = 64;
// boundaries strictly inside the chunk -> LDS (sorted groups): event i's pane is pa + #(lb <= i)
__device__ __forceinline__ int chunk_bounds(const GroupDesc& gd, int pa, int pb, int64_t* lb) {
    const int64_t* pbnd = gd.pbnd;
    if (!gd.sorted) return 0;
    const int n = min(pb - pa, kMaxChunkBnd);
    for (int k = threadIdx.x; k < n; k += blockDim.x) lb[k] = pbnd[pa + 1 + k];
    return n;
}

// Pane (group-relative) of virtual row v inside a sorted chunk: pa + #(boundaries <= v).
__device__ __forceinline__ int chunk_rel(const int64_t* lb, int nlb, int pa, int64_t v) {
    int rel = pa;
    for (int k = 0; k < nlb; ++k) rel += (v >= lb[k]) ? 1 : 0;
    return rel;
}

// MODE 3: group-relative pane of a timestamp, clamped to the group's panes (rows before pane q_lo belong to the
// first pane's index range, as pbnd[0] = lo makes them in MODE 1)
__device__ __forceinline__ int fz_rel(const GroupDesc& gd, const PaneGrid& g, int64_t t) {
    const int64_t q = pane_of(g, t);
    return q <= gd.q_lo ? 0 : (q >= gd.q_lo + gd.n_panes - 1 ? gd.n_panes - 1 : (int)(q - gd.q_lo));
}

// MODE 3: start of group pane r (INT64_MAX past the group's last pane) — multiplications only: the per-row pane of a
// chunk is counted against these bounds, never divided out (64-bit division is a long VALU sequence on gfx950)
__device__ __forceinline__ int64_t fz_start(const GroupDesc& gd, const PaneGrid& g, int r) {
    if (r > gd.n_panes - 1) return INT64_MAX;
    const int64_t q = gd.q_lo + r;
    if (g.tumbling) return q == 0 ? INT64_MIN : g.origin + (q - 1) * g.P;
    return g.origin + q * g.P;
}

// Local partition of event row `i` (-1: dropped: late, outside the group's panes, or filtered by WHERE).
// MODE 0 (unsorted): the pane comes from the event's ts. MODE 1 (sorted) / 2 (virtual panes): the
// caller passes the pane `rel` derived from the (virtual) row index; `i` is the physical row.
template <int MODE, bool WHERE>
__device__ __forceinline__ int local_part(const DPlan& p, const DBatch& b, const PaneGrid& g, const GroupDesc& gd,
                                          int rel, const uint8_t* acc, int64_t i, int pa, uint32_t key,
                                          int32_t* pane_err, bool check_where) {
    if (MODE == 0) {
        if (gd.has_accept && !acc[i]) return -1;
        int64_t q = pane_of(g, ((const int64_t*)b.col[gd.ts_col])[i]);
        int64_t r = q - gd.q_lo;
        if (q < 0 || r < 0 || r >= gd.n_panes) return -1;
        rel = (int)r;
    } else if (MODE == 1 || MODE == 3) {
        if (gd.has_accept && !acc[i]) return -1;   // hopping empty-window discard (k_hop_drop)
    }
    if (gd.key_col >= 0 && key >= gd.num_keys) return -1;
    if (WHERE) {
        int w = where_decide_slow(p, b, i);
        if (w < 0) {
            if (check_where) {
                const int64_t slot = (gd.q_lo + rel) % gd.ring;
                atomicOr(&pane_err[slot], EK_WIN_WHERE_ERROR);
                if (gd.pwit)
                    wit_where_row(&gd.pwit[slot], gd.wit_ts ? i64_to_ord(((const int64_t*)b.col[gd.ts_col])[i]) : 0ull,
                                  (unsigned long long)(gd.wit_o2 + i), p, b, i);
            }
            return -1;
        }
        if (w == 0) return -1;
    }
    return (rel - pa) * gd.nb + (int)(key >> gd.kbits);
}

__device__ __forceinline__ uint32_t load_key(const DPlan& p, const DBatch& b, int64_t i) {
    return p.key_col >= 0 ? ((const uint32_t*)b.col[p.key_col])[i] : 0u;
}

// Per chunk: histogram over its chunk-local partitions (pane, key bucket) of the rows that pass WHERE,
// stored compactly as chist[chunk][lp] (lp < lp_stride), plus the group-wide totals per partition.
struct Staging {
    uint16_t* klo;
    int64_t* val[kMaxVC];
    uint8_t* valid[kMaxVC];
    uint32_t nullable_mask;   // bit v: staging carries validity for value column v
};

// Block-wide exclusive scan of cnt[0..n) in LDS; cnt[n] receives the total (B threads, wsum[B / 64]).
template <int B>
__device__ inline void block_excl_scan(uint32_t* cnt, int n, uint32_t* wsum) {
    const int per = (n + B - 1) / B;
    const int b = threadIdx.x * per, e = min(n, b + per);
    uint32_t s = 0;
    for (int k = b; k < e; ++k) s += cnt[k];
    uint32_t x = s;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wv; ++w) wbase += wsum[w];
    uint32_t run = wbase + x - s;
    for (int k = b; k < e; ++k) { uint32_t c = cnt[k]; cnt[k] = run; run += c; }
    if (threadIdx.x == B - 1) cnt[n] = run;
    __syncthreads();
}

// LDS bytes of k_part for `nvc` value columns and `lp` chunk-local partitions
// (single-tile chunks need no per-row partition array: their runs come straight from the tile sort)
// (value columns are staged through LDS one at a time, so the footprint does not grow with their number)
// MODE 3 (single-tile chunks): the tile's ts in LDS past the single-tile layout with its validity bytes
__host__ __device__ inline size_t fz_lds_off(int lp) {
    const size_t lpp = ((size_t)lp + 4 + 3) & ~(size_t)3;
    return (((size_t)kTile * 8 + 2 * lpp * 4 + (size_t)kTile * 2 + (size_t)kTile) + 15) & ~(size_t)15;
}
inline size_t fz_lds_bytes(int lp) { return fz_lds_off(lp) + (size_t)kTile * 8; }
inline size_t part_lds_bytes(int nvc, int lp, bool nullable, bool single_tile) {
    size_t lpp = ((size_t)lp + 4 + 3) & ~(size_t)3;
    return (size_t)kTile * 8 + 2 * lpp * 4 + (size_t)kTile * (single_tile ? 2 : 4) + (nullable ? (size_t)kTile : 0);
}

// One workgroup per chunk: partition the chunk's rows by (pane, key bucket) into the chunk's OWN
// staging region [chunk * rs, chunk * rs + rows): (1) count rows per chunk-local partition (16-byte
// key loads), (2) exclusive scan -> run offsets, published in ctab[chunk][0..lp_n], (3) per tile of
// kTile rows: load, counting-sort by partition in LDS, write runs with consecutive lanes on
// consecutive addresses. No global atomics, no global scan: k_agg walks the per-chunk runs.
// A chunk of at most one tile skips (1)-(2): the tile's own sort yields its runs, so the keys are read
// once and the tile is written as one block of runs at region + sorted position.
// MODE 0: unsorted batch (pane from ts); 1: ts-sorted batch (pane from the row index);
// 2: virtual panes (range mode): the group's rows are the concatenation of possibly overlapping
//    index ranges of the event buffer, virtual row v of pane r lives at physical row v + voff[r].
// 3: the fused sorted pass (single-tile chunks of a batch presumed ts-sorted): the pane of each row comes from its
//    own ts, and the same read of ts checks the presumption (arrival order non-decreasing, watermark_op.go:144-155:
//    then no row is late and the running max is the row's own ts), finds the widest arrival gap when asked, and
//    writes the pane bounds (pbnd_out) that k_agg walks — so no separate ts pass and no pane-bounds search precede
//    it. Its verdict goes to fz_st; the host discards the pass and takes the general path when the batch is not sorted.
template <int MODE, bool WHERE, int NVC>
__global__ __launch_bounds__(kPartBlock) __attribute__((amdgpu_waves_per_eu(EK_PART_WAVES_PER_EU))) void k_part(DPlan* __restrict__ pp, DBatch b, PaneGrid g, GroupDesc gd,
                                                 const uint8_t* __restrict__ acc, Staging st, uint32_t* __restrict__ ctab,
                                                 int ls, int64_t rs, int32_t* __restrict__ pane_err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const DPlan& p = *pp;
    int64_t a0, c0, c1;
    chunk_range(gd, &a0, &c0, &c1);
    int pa, pb;
    const int64_t* tsc = (const int64_t*)b.col[gd.ts_col];
    if (MODE == 3) {
        pa = fz_rel(gd, g, tsc[c0]);
        pb = pa + gd.fz_mp - 1;
    } else {
        chunk_panes(gd, c0, c1, &pa, &pb);
    }
    const int lp_n = (pb - pa + 1) * gd.nb;
    __shared__ int64_t lb[kMaxChunkBnd];
    __shared__ int64_t loff[kMaxChunkBnd + 1];
    __shared__ uint32_t wsum[kPartBlock / 64];
    __shared__ int s_fz_bad[2];                 // MODE 3: unsorted, pane overflow
    __shared__ unsigned long long s_fz_gap;     // MODE 3: widest arrival gap
    const int64_t fz_before = (MODE == 3 && c0 > 0) ? tsc[c0 - 1] : 0;              // MODE 3: the row before the chunk
    const int fz_rp0 = (MODE == 3 && c0 > 0) ? fz_rel(gd, g, fz_before) : 0;         // ... and its pane (one division)
    if (MODE == 3 && threadIdx.x == 0) { s_fz_bad[0] = 0; s_fz_bad[1] = 0; s_fz_gap = 0; }
    const int nlb = MODE == 3 ? 0 : chunk_bounds(gd, pa, pb, lb);
    // MODE 3: lb[k] = start of pane pa + 1 + k (k < fz_mp - 1); a row at or past the start of pane pa + fz_mp overflows
    int64_t fz_ovf = INT64_MAX;
    if constexpr (MODE == 3) {
        for (int k = threadIdx.x; k < gd.fz_mp - 1; k += kPartBlock) lb[k] = fz_start(gd, g, pa + 1 + k);
        fz_ovf = fz_start(gd, g, pa + gd.fz_mp);
    }
    auto fz_relb = [&](int64_t t) {   // group pane of a row of this chunk (t >= the chunk's first ts)
        int r = pa;
        for (int k = 0; k < gd.fz_mp - 1; ++k) r += t >= lb[k] ? 1 : 0;
        return r;
    };
    if (threadIdx.x == 0) gd.cpa[blockIdx.x] = pa;
    if (MODE == 2)
        for (int k = threadIdx.x; k <= pb - pa; k += kPartBlock) loff[k] = gd.voff[pa + k];
    const int lpp = (lp_n + 4 + 3) & ~3;
    int64_t* s_val = (int64_t*)smem;                                          // [kTile] one value column at a time
    uint32_t* cur = (uint32_t*)(smem + (size_t)kTile * 8);                    // [lpp]
    uint32_t* tcnt = cur + lpp;                                               // [lpp]
    const bool single = gd.chunk <= kTile;
    uint16_t* s_klo = (uint16_t*)(tcnt + lpp);                                // [kTile]
    uint16_t* s_lp = s_klo + kTile;                                           // [kTile] (multi-tile chunks)
    uint8_t* s_vd = (uint8_t*)(s_klo + (single ? 1 : 2) * kTile);             // [kTile] validity of that column
    int64_t* s_ts = (int64_t*)(smem + fz_lds_off(lp_n));                       // MODE 3: [kTile] the tile's ts, row order
    const uint32_t* kcol = gd.key_col >= 0 ? (const uint32_t*)b.col[gd.key_col] : nullptr;
    const int64_t region = (int64_t)blockIdx.x * rs;

    // ---- (1) count
    for (int k = threadIdx.x; k <= lp_n; k += kPartBlock) tcnt[k] = 0;
    __syncthreads();
    if (single) {
        // runs come from the tile sort below
    } else if (MODE == 2) {
        // physical rows are contiguous only inside one pane: scalar (still coalesced) key loads
        for (int64_t v = c0 + threadIdx.x; v < c1; v += kPartBlock) {
            const int rel = chunk_rel(lb, nlb, pa, v);
            const int64_t i = v + loff[rel - pa];
            const uint32_t key = kcol ? kcol[i] : (p.pseudo_keys ? (uint32_t)(i & (kPseudoKeys - 1)) : 0u);
            const int lp = local_part<MODE, WHERE>(p, b, g, gd, rel, acc, i, pa, key, pane_err, true);
            if (lp >= 0) atomicAdd(&tcnt[lp], 1u);
        }
    } else if (!(gd.pad & 4)) {   // (diagnostic knob 4: skip the count pass; timing only)
        constexpr int V = 4;   // 16-byte key loads in flight per thread
        for (int64_t base = a0 + (int64_t)threadIdx.x * 4; base < c1; base += (int64_t)kPartBlock * 4 * V) {
            uint4 kv[V];
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int64_t i = base + (int64_t)u * kPartBlock * 4;
                if (kcol && i + 3 < gd.nbatch && i < c1) kv[u] = *(const uint4*)(kcol + i);
                else if (kcol && i < c1) {
                    kv[u].x = kcol[i];
                    kv[u].y = i + 1 < gd.nbatch ? kcol[i + 1] : 0u;
                    kv[u].z = i + 2 < gd.nbatch ? kcol[i + 2] : 0u;
                    kv[u].w = i + 3 < gd.nbatch ? kcol[i + 3] : 0u;
                } else kv[u] = make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < V; ++u) {
                uint32_t kk[4] = {kv[u].x, kv[u].y, kv[u].z, kv[u].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int64_t i = base + (int64_t)u * kPartBlock * 4 + e;
                    if (i < c0 || i >= c1) continue;
                    if (p.pseudo_keys) kk[e] = (uint32_t)(i & (kPseudoKeys - 1));
                    const int rel = MODE == 1 ? chunk_rel(lb, nlb, pa, i) : 0;
                    const int lp = local_part<MODE, WHERE>(p, b, g, gd, rel, acc, i, pa, kk[e], pane_err, true);
                    if (lp >= 0) atomicAdd(&tcnt[lp], 1u);
                }
            }
        }
    }
    __syncthreads();
    // ---- (2) run offsets of this chunk
    if (!single) {
        block_excl_scan<kPartBlock>(tcnt, lp_n, wsum);
        for (int k = threadIdx.x; k < ls; k += kPartBlock) ctab[(int64_t)blockIdx.x * ls + k] = k <= lp_n ? tcnt[k] : tcnt[lp_n];
        for (int k = threadIdx.x; k < lp_n; k += kPartBlock) cur[k] = tcnt[k];
        __syncthreads();
    }
    // ---- (3) tiles: load, LDS counting sort, coalesced run writes
    const uint32_t kmask = (1u << gd.kbits) - 1u;
    if (gd.pad & 16) return;   // diagnostic knob 16: count pass only
    for (int64_t t0 = a0; t0 < c1; t0 += kTile) {
        uint32_t key[kTileE];
        int64_t val[NVC][kTileE];
        int64_t phys[kTileE];   // MODE 2: physical row of each element (-1 outside the chunk)
        int rel[kTileE];
        if (MODE == 2) {
#pragma unroll
            for (int j = 0; j < kTileE; ++j) {
                const int64_t v = t0 + (int64_t)(j >> 1) * 2 * kPartBlock + 2 * threadIdx.x + (j & 1);
                rel[j] = 0;
                phys[j] = -1;
                if (v >= c0 && v < c1) {
                    rel[j] = chunk_rel(lb, nlb, pa, v);
                    phys[j] = v + loff[rel[j] - pa];
                }
                key[j] = (kcol && phys[j] >= 0) ? kcol[phys[j]] : (p.pseudo_keys && phys[j] >= 0 ? (uint32_t)(phys[j] & (kPseudoKeys - 1)) : 0u);
#pragma unroll
                for (int c = 0; c < NVC; ++c)
                    val[c][j] = (c < p.n_vc && phys[j] >= 0) ? ((const int64_t*)b.col[p.vc_col[c]])[phys[j]] : 0;
            }
        } else {
#pragma unroll
            for (int m = 0; m < kTileE / 2; ++m) {
                const int64_t i = t0 + (int64_t)m * 2 * kPartBlock + 2 * threadIdx.x;
                const bool full = i + 1 < gd.nbatch && i < c1;
                if (full) {
                    uint2 kp = kcol ? *(const uint2*)(kcol + i) : make_uint2(0, 0);
                    key[2 * m] = kp.x;
                    key[2 * m + 1] = kp.y;
                } else {
                    key[2 * m] = (kcol && i < gd.nbatch) ? kcol[i] : 0u;
                    key[2 * m + 1] = 0u;
                }
                if (p.pseudo_keys) {   // un-grouped rule: partial slot from the row index
                    key[2 * m] = (uint32_t)(i & (kPseudoKeys - 1));
                    key[2 * m + 1] = (uint32_t)((i + 1) & (kPseudoKeys - 1));
                }
                if constexpr (MODE == 3) {
                    // ts straight into LDS (global_load_lds, no VGPRs: k_part is at its register cap), in row order:
                    // a wave's 64 lanes x 16 B land at its 128 rows of this pair group (destination = wave base +
                    // lane x 16); the barrier after the loads drains them
                    int64_t* s_tm = s_ts + (int64_t)m * 2 * kPartBlock;
                    if (full)
                        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(tsc + i),
                                                         (__attribute__((address_space(3))) void*)(s_tm + 2 * (threadIdx.x & ~63)),
                                                         16, 0, 0);
                    else if (i < gd.nbatch) {
                        s_tm[2 * threadIdx.x] = tsc[i];
                        s_tm[2 * threadIdx.x + 1] = 0;
                    }
                }
#pragma unroll
                for (int v = 0; v < NVC; ++v) {
                    if (v < p.n_vc && full) {
                        longlong2 vp = *(const longlong2*)((const int64_t*)b.col[p.vc_col[v]] + i);
                        val[v][2 * m] = vp.x;
                        val[v][2 * m + 1] = vp.y;
                    } else {
                        val[v][2 * m] = (v < p.n_vc && i < gd.nbatch) ? ((const int64_t*)b.col[p.vc_col[v]])[i] : 0;
                        val[v][2 * m + 1] = 0;
                    }
                }
            }
        }
        for (int k = threadIdx.x; k <= lp_n; k += kPartBlock) tcnt[k] = 0;
        __syncthreads();
        int lp[kTileE];
        uint32_t rank[kTileE];
        if constexpr (MODE == 3) {
            // each row's pane from its ts in LDS, counted against the chunk's pane starts (a row past fz_mp panes —
            // overflow: the pass is discarded — is not staged); the order check runs after the tile's writes
#pragma unroll
            for (int j = 0; j < kTileE; ++j) {
                const int64_t i = t0 + (int64_t)(j >> 1) * 2 * kPartBlock + 2 * threadIdx.x + (j & 1);
                const int loc = (j >> 1) * 2 * kPartBlock + 2 * threadIdx.x + (j & 1);
                lp[j] = -1;
                if (i < c1) {
                    const int64_t t = s_ts[loc];
                    if (t < fz_ovf) lp[j] = local_part<MODE, WHERE>(p, b, g, gd, fz_relb(t), acc, i, pa, key[j], pane_err, single);
                }
                if (lp[j] >= 0) rank[j] = atomicAdd(&tcnt[lp[j]], 1u);
            }
        }
#pragma unroll
        for (int j = 0; j < kTileE; ++j) {
            if (MODE == 3) break;   // (MODE 3: partitioned in the check loop above)
            const int64_t i = t0 + (int64_t)(j >> 1) * 2 * kPartBlock + 2 * threadIdx.x + (j & 1);
            // (single-tile chunks flag WHERE errors here: there was no count pass)
            if (MODE == 2) {
                lp[j] = phys[j] >= 0 ? local_part<MODE, WHERE>(p, b, g, gd, rel[j], acc, phys[j], pa, key[j], pane_err, single) : -1;
            } else {
                const int r = (MODE == 1 && i >= c0 && i < c1) ? chunk_rel(lb, nlb, pa, i) : 0;
                lp[j] = (i >= c0 && i < c1) ? local_part<MODE, WHERE>(p, b, g, gd, r, acc, i, pa, key[j], pane_err, single) : -1;
            }
            if (lp[j] >= 0) rank[j] = atomicAdd(&tcnt[lp[j]], 1u);
        }
        __syncthreads();
        block_excl_scan<kPartBlock>(tcnt, lp_n, wsum);
        if (single)
            for (int k = threadIdx.x; k < ls; k += kPartBlock) ctab[(int64_t)blockIdx.x * ls + k] = k <= lp_n ? tcnt[k] : tcnt[lp_n];
        uint32_t spos[kTileE];   // sorted position of each element (its partition run + rank)
#pragma unroll
        for (int j = 0; j < kTileE; ++j) {
            if (lp[j] < 0) continue;
            spos[j] = tcnt[lp[j]] + rank[j];
            s_klo[spos[j]] = (uint16_t)(key[j] & kmask);
            if (!single) s_lp[spos[j]] = (uint16_t)lp[j];
        }
        __syncthreads();
        const uint32_t total = (gd.pad & 8) ? 0u : tcnt[lp_n];   // diagnostic knob 8: no global stores
        auto gpos_of = [&](uint32_t s) -> int64_t {
            if (single) return region + s;
            const int l = s_lp[s];
            return region + cur[l] + (s - tcnt[l]);
        };
        for (uint32_t s = threadIdx.x; s < total; s += kPartBlock) st.klo[gpos_of(s)] = s_klo[s];
        // value columns: one LDS staging buffer, reused column by column
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            if (v >= p.n_vc) break;
            const bool vnull = (st.nullable_mask >> v) & 1u;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kTileE; ++j) {
                if (lp[j] < 0) continue;
                s_val[spos[j]] = val[v][j];
                if (vnull) {
                    const int64_t i = MODE == 2 ? phys[j] : t0 + (int64_t)(j >> 1) * 2 * kPartBlock + 2 * threadIdx.x + (j & 1);
                    s_vd[spos[j]] = col_valid(b, p.vc_col[v], i) ? 1 : 0;
                }
            }
            __syncthreads();
            for (uint32_t s = threadIdx.x; s < total; s += kPartBlock) {
                const int64_t gp = gpos_of(s);
                st.val[v][gp] = s_val[s];
                if (vnull) st.valid[v][gp] = s_vd[s];
            }
        }
        if (single) break;
        __syncthreads();
        for (int k = threadIdx.x; k < lp_n; k += kPartBlock) cur[k] += tcnt[k + 1] - tcnt[k];
        __syncthreads();
    }
    if constexpr (MODE == 3) {
        // the presumption check on the tile's ts (still in LDS): row i against row i - 1 (the chunk's first row against
        // the row before the chunk), pane bounds at every pane change, the widest gap
        {
            bool bad = false, ovf = false;
            int64_t gap = 0;
#pragma unroll
            for (int m = 0; m < kTileE / 2; ++m) {
                const int64_t i = a0 + (int64_t)m * 2 * kPartBlock + 2 * threadIdx.x;
                const int loc = m * 2 * kPartBlock + 2 * threadIdx.x;
                if (i >= c1) continue;
                const int64_t x = s_ts[loc];
                const int rx = fz_relb(x);
                ovf |= x >= fz_ovf;
                if (i > 0) {
                    const int64_t prev = loc > 0 ? s_ts[loc - 1] : fz_before;
                    bad |= x < prev;
                    gap = max(gap, x - prev);
                    const int rp = loc > 0 ? fz_relb(prev) : fz_rp0;
                    for (int k = rp + 1; k <= rx; ++k) gd.pbnd_out[k] = i;
                }
                if (i + 1 < c1) {
                    const int64_t y = s_ts[loc + 1];
                    const int ry = fz_relb(y);
                    ovf |= y >= fz_ovf;
                    bad |= y < x;
                    gap = max(gap, y - x);
                    for (int k = rx + 1; k <= ry; ++k) gd.pbnd_out[k] = i + 1;
                }
            }
            if (bad) s_fz_bad[0] = 1;
            if (ovf) s_fz_bad[1] = 1;
            if (gd.fz_gap) {
                gap = wave_max64(gap);
                if ((threadIdx.x & 63) == 0 && gap > 0) atomicMax(&s_fz_gap, (unsigned long long)gap);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (s_fz_bad[0]) atomicOr(&gd.fz_st->unsorted, 1);
            if (s_fz_bad[1]) atomicOr(&gd.fz_st->overflow, 1);
            if (s_fz_gap) atomicMax(&gd.fz_st->max_gap, s_fz_gap);
        }
    }
}

// per group: zero the per-pane scalars (WHERE error flag, membership fingerprint) of freshly
// claimed ring slots
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_group_prep(GroupDesc gd, int32_t* pane_err, int64_t* pane_mcnt, unsigned long long* pane_mhash) {
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < gd.n_panes && gd.fresh[r]) {
        int64_t s = (gd.q_lo + r) % gd.ring;
        pane_err[s] = 0;
        pane_mcnt[s] = 0;
        pane_mhash[s] = 0;
        if (gd.pwit) { gd.pwit[s].set = 0; gd.pwit[s].lock = 0; }
    }
}
#endif

// ---------------------------------------------------------------- per-partition aggregation
// LDS layout per partition (kk = 1 << kbits keys): 8-byte fields first, then u32 counts.
struct LdsLayout {
    int32_t off_cnt;
    int32_t off_vcnt[kMaxVC];
    int32_t off_sum[kMaxVC];
    int32_t off_min[kMaxVC];
    int32_t off_max[kMaxVC];
    int32_t off_m2[kMaxVC];
    int32_t off_fsum[kMaxVC];
    int32_t off_koff, off_kcur, off_sres, off_stag;   // sort aggregates: key offsets/cursors, results, tags
    int32_t bytes;
};

struct WinDesc {
    int64_t q_first, q_last;   // panes merged into the window
    int64_t out_base;          // first result row of this window's region
    int32_t idx;               // index into win_cnt / win_err
    int32_t pad;
};

struct Results {
    uint32_t* key;
    int64_t* val[EK_MAX_AGGS];
    uint8_t* tag[EK_MAX_AGGS];
    int64_t* win_cnt;      // rows per window
    int32_t* win_err;      // EK_WIN_* per window
    // error witnesses (nullptr when the plan cannot fail): wwit[2 w] the window's WHERE offender, wwit[2 w + 1] its
    // HAVING offender (smallest key), aslot[w] the smallest order-statistic index whose value failed; pwit: the pane
    // slots' WHERE offenders (GroupDesc::pwit), read when a window takes its panes' errors
    WitRec* wwit;
    const WitRec* pwit;
    int32_t* aslot;
};

// Merged partial aggregate of one (window, key), kept in registers (all indices compile-time).
template <int NVC>
struct Part {
    int64_t cnt;
    int64_t vcnt[NVC];
    int64_t isum[NVC];
    double fsum[NVC];    // f64 sum (float columns) or f64 shadow sum (int columns with var)
    double m2[NVC];
    uint64_t omn[NVC], omx[NVC];
};

template <int N, typename T>
__device__ __forceinline__ T sel(const T (&a)[N], int v) {
    T r = a[0];
#pragma unroll
    for (int u = 1; u < N; ++u) if (v == u) r = a[u];
    return r;
}

__device__ __forceinline__ double chan_m2(double m2a, double sa, int64_t na, double m2b, double sb, int64_t nb) {
    // Chan et al. pairwise merge of (n, sum, M2) partials
    double d = __dsub_rn(__ddiv_rn(sb, (double)nb), __ddiv_rn(sa, (double)na));
    double w = __ddiv_rn(__dmul_rn((double)na, (double)nb), (double)(na + nb));
    return __dadd_rn(__dadd_rn(m2a, m2b), __dmul_rn(__dmul_rn(d, d), w));
}

// merge partial b (count c, fields from arrays) into a
template <int NVC>
__device__ __forceinline__ void part_merge(const DPlan& p, Part<NVC>& a, int64_t c, const int64_t (&vc)[NVC],
                                           const int64_t (&is)[NVC], const double (&fs)[NVC], const double (&m2)[NVC],
                                           const uint64_t (&mn)[NVC], const uint64_t (&mx)[NVC]) {
    int64_t cprev = a.cnt;
    a.cnt += c;
#pragma unroll
    for (int v = 0; v < NVC; ++v) {
        const int f = p.vc_flags[v];
        int64_t nb = (f & NEED_CNT) ? vc[v] : c;
        if (nb == 0) continue;
        int64_t na = (f & NEED_CNT) ? a.vcnt[v] : cprev;
        a.vcnt[v] = na + nb;
        a.isum[v] = (int64_t)((uint64_t)a.isum[v] + (uint64_t)is[v]);
        if (f & NEED_M2) a.m2[v] = na ? chan_m2(a.m2[v], a.fsum[v], na, m2[v], fs[v], nb) : m2[v];
        a.fsum[v] = na ? __dadd_rn(a.fsum[v], fs[v]) : fs[v];
        a.omn[v] = (na == 0 || mn[v] < a.omn[v]) ? mn[v] : a.omn[v];
        a.omx[v] = (na == 0 || mx[v] > a.omx[v]) ? mx[v] : a.omx[v];
    }
}

// funcs_agg.go: the value (and Go type) of aggregate slot k for a merged group partial
// Order-statistic results (median / percentile_*) come from the per-key LDS table of k_agg's sort pass:
// sres[slot * kk + kl] value bits, stag[...] EK_TAG_* or kTagErr.
constexpr uint8_t kTagErr = 0xFF;
struct SortRes {
    const uint64_t* sres;
    const uint8_t* stag;
    int kl, kk;
};
template <int NVC>
__device__ __forceinline__ Val agg_value(const DPlan& p, const Part<NVC>& s, int k, const SortRes* sr = nullptr) {
    const int fn = p.agg_fn[k];
    if (fn == EK_AGG_COUNT_STAR) return Val{V_I64, s.cnt, 0.0};
    if (fn == EK_AGG_FIRST) {   // the group's first row: min event-buffer position (k_first_fetch swaps in the value)
        const int v = p.agg_vc[k];
        return sel(s.vcnt, v) ? Val{V_I64, ord_to_i64(sel(s.omn, v)), 0.0} : Val{V_NULL, 0, 0.0};
    }
    if (fn >= EK_AGG_MEDIAN) {
        if (!sr) return Val{V_ERR, 0, 0.0};
        const int e = p.agg_sidx[k] * sr->kk + sr->kl;
        const uint8_t t = sr->stag[e];
        if (t == kTagErr) return Val{V_ERR, 0, 0.0};
        if (t == EK_TAG_NULL) return Val{V_NULL, 0, 0.0};
        if (t == EK_TAG_I64) return Val{V_I64, (int64_t)sr->sres[e], 0.0};
        return Val{V_F64, 0, __longlong_as_double((long long)sr->sres[e])};
    }
    const int v = p.agg_vc[k];
    const int64_t n = sel(s.vcnt, v);
    if (fn == EK_AGG_COUNT) return Val{V_I64, n, 0.0};
    if (n == 0) return Val{V_NULL, 0, 0.0};      // every value nil
    const bool fl = p.vc_is_float[v];
    switch (fn) {
    case EK_AGG_SUM: return (fl || p.inc) ? Val{V_F64, 0, sel(s.fsum, v)} : Val{V_I64, sel(s.isum, v), 0.0};
    case EK_AGG_AVG: {   // funcs_agg.go:56-86: int -> truncating int64 division; inc_avg: float64 (funcs_inc_agg.go:56-75)
        if (fl || p.inc) return Val{V_F64, 0, __ddiv_rn(sel(s.fsum, v), (double)n)};
        int64_t t = sel(s.isum, v);
        return Val{V_I64, (t == INT64_MIN && n == -1) ? t : t / n, 0.0};
    }
    case EK_AGG_MIN: return fl ? Val{V_F64, 0, ord_to_f64(sel(s.omn, v))} : Val{V_I64, ord_to_i64(sel(s.omn, v)), 0.0};
    case EK_AGG_MAX: return fl ? Val{V_F64, 0, ord_to_f64(sel(s.omx, v))} : Val{V_I64, ord_to_i64(sel(s.omx, v)), 0.0};
    case EK_AGG_VAR: return Val{V_F64, 0, __ddiv_rn(sel(s.m2, v), (double)n)};
    case EK_AGG_VARS: return Val{V_F64, 0, __ddiv_rn(sel(s.m2, v), (double)(n - 1))};
    case EK_AGG_STDDEV: return Val{V_F64, 0, __dsqrt_rn(__ddiv_rn(sel(s.m2, v), (double)n))};
    case EK_AGG_STDDEVS: return Val{V_F64, 0, __dsqrt_rn(__ddiv_rn(sel(s.m2, v), (double)(n - 1)))};
    }
    return Val{V_NULL, 0, 0.0};
}

// HAVING (having_operator.go:41-56): true keeps the group, false drops it, anything else is an error.
// Aggregate slots are evaluated on demand from the group's partial (no per-lane array).
// A failed HAVING group becomes the window's HAVING witness when its key is the smallest failed one (the reference's
// groups come out of a Go map, aggregate_operator.go:44-72, so any failed group's error is one it can report).
template <typename AGGF>
__device__ inline void wit_having(WitRec* r, uint32_t key, const DPlan& p, AGGF aggf) {
    wit_offer(r, key, 0ull, [&](WitRec* w) {
        for (int k = 0; k < p.n_having; ++k)
            if (p.having_prog[k].op == EK_OP_AGG) wit_put(w, p.having_prog[k].arg, aggf(p.having_prog[k].arg));
    });
}
template <int NVC>
__device__ __forceinline__ bool having_keep(const DPlan& p, const Part<NVC>& s, const Results& res, int32_t widx, uint32_t key,
                                            const SortRes* sr = nullptr) {
    if (p.n_having <= 0) return true;
    auto aggf = [&](int k) { return agg_value(p, s, k, sr); };
    const Val h = eval_prog(p.having_prog, p.n_having, p, nullptr, 0, aggf);
    if (h.tag != V_BOOL) {
        atomicOr(&res.win_err[widx], EK_WIN_HAVING_ERROR);
        if (res.wwit) wit_having(&res.wwit[2 * widx + 1], key, p, aggf);
        return false;
    }
    return h.i != 0;
}

// Block-compacted emission of result rows: ONE returning atomic per workgroup on the window's row
// counter (per-wave atomics from thousands of waves on one address serialise for tens of µs).
// Every thread of the block must call it (sh: >= 17 u32 of LDS).
template <int NVC>
__device__ __forceinline__ void emit_rows(const DPlan& p, bool present, const Part<NVC>& s, int64_t key, int64_t out_base,
                                          int32_t widx, Results& res, uint32_t* sh, const SortRes* sr = nullptr) {
    const unsigned long long mask = __ballot(present);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0) sh[wv] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < nw; ++w) { uint32_t c = sh[w]; sh[w] = run; run += c; }
        sh[16] = run ? (uint32_t)atomicAdd((unsigned long long*)&res.win_cnt[widx], (unsigned long long)run) : 0u;
    }
    __syncthreads();
    const uint32_t wbase = sh[wv], bbase = sh[16];
    __syncthreads();   // sh is reused by the caller's next round
    if (!present) return;
    const int64_t pos = out_base + (int64_t)bbase + wbase + __popcll(mask & ((1ull << lane) - 1ull));
    res.key[pos] = (uint32_t)key;
#pragma unroll
    for (int k = 0; k < EK_MAX_AGGS; ++k) {
        if (k >= p.n_aggs) break;
        Val a = agg_value(p, s, k, sr);
        res.tag[k][pos] = a.tag == V_NULL ? EK_TAG_NULL : (a.tag == V_I64 ? EK_TAG_I64 : EK_TAG_F64);
        res.val[k][pos] = a.tag == V_F64 ? __double_as_longlong(a.f) : a.i;
    }
}

constexpr int kAggBlock = 512;

// One workgroup per partition (pane, key bucket): LDS aggregation of the partition's staged run,
// then either (a) direct emission of the final rows when the pane is a whole tumbling window that
// closes in this batch (direct[2*rel] = out_base >= 0), or (b) write / merge into the pane state.
constexpr int kMaxRuns = 1024;
#ifndef EK_AGG_PIPE
#define EK_AGG_PIPE 0
#endif
// k_agg's run tables in dynamic LDS after the aggregation tables: r_start[mr], r_pre[mr + 1]
inline size_t agg_run_lds_bytes(int mruns) { return ((size_t)(2 * mruns + 1) * 4 + 15) & ~(size_t)15; }
constexpr int kMaxBucketKeys = 8192;   // keys per bucket (1 << kbits) the direct emission's present mask covers

// Runs of partition (rel, bucket): chunk c in [c_lo, c_hi] holds ctab[c][lp .. lp+1) of it.
__device__ __forceinline__ void part_chunks(const GroupDesc& gd, int rel, int* c_lo, int* c_hi) {
    *c_lo = 0;
    *c_hi = gd.nch - 1;
    if (gd.sorted) {
        const int64_t e0 = gd.pbnd[rel], e1 = gd.pbnd[rel + 1];
        if (e1 <= e0) { *c_lo = 0; *c_hi = -1; }
        else { *c_lo = (int)((e0 - gd.abase) / gd.chunk); *c_hi = (int)((e1 - 1 - gd.abase) / gd.chunk); }
    }
}
// (k_part wrote the chunk's first pane pa into cpa[c]; ctab rows are padded with the chunk total past its
// last local partition, so a pane beyond the chunk's last one reads an empty run)
__device__ __forceinline__ void part_run(const GroupDesc& gd, const uint32_t* ctab, int ls, int rel, int bucket, int c,
                                         uint32_t* o0, uint32_t* o1) {
    const int pa = gd.cpa[c];
    const int lp = (rel - pa) * gd.nb + bucket;
    *o0 = *o1 = 0;
    if (rel >= pa && lp + 1 < ls) { *o0 = ctab[(int64_t)c * ls + lp]; *o1 = ctab[(int64_t)c * ls + lp + 1]; }
}

// Rows per partition (sort aggregates: the key-grouped scratch region of each partition), one thread each.
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_part_sizes(GroupDesc gd, const uint32_t* __restrict__ ctab, int ls, int64_t* __restrict__ out) {
    const int pid = blockIdx.x * blockDim.x + threadIdx.x;
    if (pid >= gd.np) return;
    const int rel = pid / gd.nb, bucket = pid % gd.nb;
    int c_lo, c_hi;
    part_chunks(gd, rel, &c_lo, &c_hi);
    int64_t t = 0;
    for (int c = c_lo; c <= c_hi; ++c) {
        uint32_t o0, o1;
        part_run(gd, ctab, ls, rel, bucket, c, &o0, &o1);
        t += o1 - o0;
    }
    out[pid] = t;
}
#endif

// ---------------------------------------------------------------- order statistics (median, percentile_*)
// Element of rank r (0-based, ascending) of a short segment of ordered keys: O(n^2) counting, one thread.
__device__ __forceinline__ uint64_t seg_select(const uint64_t* seg, int n, int r) {
    for (int i = 0; i < n; ++i) {
        const uint64_t x = seg[i];
        int less = 0, eq = 0;
        for (int j = 0; j < n; ++j) { const uint64_t y = seg[j]; less += y < x; eq += y == x; }
        if (less <= r && r < less + eq) return x;
    }
    return 0;
}
// Same for a long segment, by the whole workgroup: MSD radix select, 8 bits per pass (all threads call it).
__device__ inline uint64_t block_select(const uint64_t* seg, int64_t n, int64_t r, uint32_t* hist, uint64_t* sh) {
    uint64_t prefix = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int d = threadIdx.x; d < 256; d += blockDim.x) hist[d] = 0;
        __syncthreads();
        const uint64_t hm = shift == 56 ? 0ull : (~0ull << (shift + 8));
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t x = seg[i];
            if ((x & hm) == prefix) atomicAdd(&hist[(x >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t c = 0;
            for (int d = 0; d < 256; ++d) {
                if (r < c + hist[d]) { prefix |= (uint64_t)d << shift; r -= c; break; }
                c += hist[d];
            }
            sh[0] = prefix;
            sh[1] = (uint64_t)r;
        }
        __syncthreads();
        prefix = sh[0];
        r = (int64_t)sh[1];
        __syncthreads();
    }
    return prefix;
}

// funcs_agg.go:29-55 (median), :298-370 with stats v0.7.1 Percentile / PercentileNearestRank over the n
// values of one group; sel(r) returns the ordered bits of the rank-r value. Tag kTagErr = "Input is outside of range".
template <typename SEL>
__device__ __forceinline__ void order_stat(int fn, bool isf, double param, int64_t n, SEL sel, uint64_t* out, uint8_t* tag) {
    auto val = [&](uint64_t o) { return isf ? ord_to_f64(o) : (double)ord_to_i64(o); };
    *out = 0;
    if (n <= 0) { *tag = EK_TAG_NULL; return; }
    if (fn == EK_AGG_MEDIAN) {
        if (n & 1) {
            const uint64_t o = sel(n / 2);
            *tag = isf ? EK_TAG_F64 : EK_TAG_I64;
            *out = isf ? (uint64_t)__double_as_longlong(ord_to_f64(o)) : (uint64_t)ord_to_i64(o);
        } else {
            const uint64_t a = sel(n / 2 - 1), b = sel(n / 2);
            double m;
            if (isf) m = __ddiv_rn(__dadd_rn(ord_to_f64(a), ord_to_f64(b)), 2.0);
            else m = __ddiv_rn((double)(int64_t)((uint64_t)ord_to_i64(a) + (uint64_t)ord_to_i64(b)), 2.0);
            *tag = EK_TAG_F64;
            *out = (uint64_t)__double_as_longlong(m);
        }
        return;
    }
    const double percent = __dmul_rn(param, 100.0);
    double res;
    if (fn == EK_AGG_PERCENTILE_CONT) {
        if (n == 1) res = val(sel(0));
        else {
            if (percent <= 0 || percent > 100) { *tag = kTagErr; return; }
            const double index = __dmul_rn(__ddiv_rn(percent, 100.0), (double)n);
            const int64_t i = (int64_t)index;
            if (index == (double)i) res = val(sel(i - 1));
            else if (index > 1) {
                const double a = val(sel(i - 1)), b = val(sel(i));
                res = __ddiv_rn(__dadd_rn(__dadd_rn(0.0, a), b), 2.0);
            } else { *tag = kTagErr; return; }
        }
    } else {
        if (percent < 0 || percent > 100) { *tag = kTagErr; return; }
        if (percent == 100.0) res = val(sel(n - 1));
        else {
            const int64_t r = (int64_t)ceil(__ddiv_rn(__dmul_rn((double)n, percent), 100.0));
            res = val(sel(r == 0 ? 0 : r - 1));
        }
    }
    *tag = EK_TAG_F64;
    *out = (uint64_t)__double_as_longlong(res);
}

constexpr int kSmallSeg = 32;   // segments up to this length are selected by one thread

// ---------------------------------------------------------------- sparse partitions
// A directly emitted partition with at most kSparseRows rows (windows much smaller than the key space, e.g. a
// 1000-event COUNTWINDOW over 1 M keys spreads ~2 rows over each 2048-key bucket): instead of zeroing and
// scanning the dense 2^kbits-key LDS table, the rows are staged in LDS, the first row of every key leads its
// group, and the leader folds the group's rows in staging order (exact two-pass M2 per group).
constexpr int kSparseRows = kAggBlock;
inline size_t sparse_lds_bytes(int nvc) { return (size_t)kSparseRows * (4 + 9 * (size_t)(nvc > 0 ? nvc : 1)); }

template <int NVC, bool HV>
__device__ inline void agg_sparse(const DPlan& p, const GroupDesc& gd, const Staging& st, unsigned char* lds,
                                  const uint32_t* r_start, const uint32_t* r_pre, int nruns, uint32_t total, int bucket,
                                  int kk, int64_t slot, int rel, int64_t dbase, const int32_t* pane_err, Results& res) {
    uint32_t* s_klo = (uint32_t*)lds;                                  // [kSparseRows]
    int64_t* s_val = (int64_t*)(lds + kSparseRows * 4);                // [NVC][kSparseRows]
    uint8_t* s_vd = (uint8_t*)(s_val + (size_t)NVC * kSparseRows);     // [NVC][kSparseRows]
    const int t = threadIdx.x;
    if ((uint32_t)t < total) {
        int lo = 0, hi = nruns - 1;
        while (lo < hi) { int m = (lo + hi + 1) >> 1; if (r_pre[m] <= (uint32_t)t) lo = m; else hi = m - 1; }
        const int64_t i = (int64_t)r_start[lo] + ((uint32_t)t - r_pre[lo]);
        s_klo[t] = st.klo[i];
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            s_val[v * kSparseRows + t] = v < p.n_vc ? st.val[v][i] : 0;
            s_vd[v * kSparseRows + t] = (v < p.n_vc && ((st.nullable_mask >> v) & 1u)) ? st.valid[v][i] : (uint8_t)1;
        }
    }
    __syncthreads();
    const int32_t widx = gd.didx[rel];
    const int32_t perr = pane_err[slot];
    if (perr) {   // a WHERE error replaces the window's output (filter_operator.go:63-77)
        if (t == 0 && bucket == 0) {
            atomicOr(&res.win_err[widx], perr);
            if (res.wwit) wit_copy(&res.wwit[2 * widx], &res.pwit[slot]);
        }
        return;
    }
    Part<NVC> s{};
    bool present = false;
    uint32_t kl = 0;
    if ((uint32_t)t < total) {
        kl = s_klo[t];
        bool leader = true;
        for (int u = 0; u < t && leader; ++u) leader = s_klo[u] != kl;
        if (leader) {
            int64_t c = 0, vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
#pragma unroll
            for (int v = 0; v < NVC; ++v) { vc[v] = 0; is[v] = 0; fs[v] = 0.0; m2[v] = 0.0; mn[v] = ~0ull; mx[v] = 0ull; }
            for (uint32_t u = t; u < total; ++u) {
                if (s_klo[u] != kl) continue;
                c++;
#pragma unroll
                for (int v = 0; v < NVC; ++v) {
                    if (v >= p.n_vc || !s_vd[v * kSparseRows + u]) continue;
                    const int64_t raw = s_val[v * kSparseRows + u];
                    const bool fl = p.vc_is_float[v];
                    const double x = fl ? __longlong_as_double(raw) : (double)raw;
                    const uint64_t o = fl ? f64_to_ord(x) : i64_to_ord(raw);
                    vc[v]++;
                    is[v] = (int64_t)((uint64_t)is[v] + (uint64_t)raw);
                    fs[v] = __dadd_rn(fs[v], x);
                    mn[v] = o < mn[v] ? o : mn[v];
                    mx[v] = o > mx[v] ? o : mx[v];
                }
            }
#pragma unroll
            for (int v = 0; v < NVC; ++v) {   // centred second pass (stats._variance shape)
                if (v >= p.n_vc || !(p.vc_flags[v] & NEED_M2) || vc[v] == 0) continue;
                const double mean = __ddiv_rn(fs[v], (double)vc[v]);
                for (uint32_t u = t; u < total; ++u) {
                    if (s_klo[u] != kl || !s_vd[v * kSparseRows + u]) continue;
                    const int64_t raw = s_val[v * kSparseRows + u];
                    const double d = __dsub_rn(p.vc_is_float[v] ? __longlong_as_double(raw) : (double)raw, mean);
                    m2[v] = __dadd_rn(m2[v], __dmul_rn(d, d));
                }
            }
            part_merge(p, s, c, vc, is, fs, m2, mn, mx);
            present = !HV || having_keep(p, s, res, widx, (uint32_t)((int64_t)bucket * kk + kl));
        }
    }
    __shared__ uint32_t esh[20];
    emit_rows(p, present, s, (int64_t)bucket * kk + kl, dbase, widx, res, esh);
}

// HV: the plan has a HAVING clause (without one, the emission carries no expression evaluator: fewer registers)
// NUL: some staged value column carries validity (without, the fold keeps no per-row validity bytes in registers)
// UR: rows in flight per lane in the fold (EK_AGG_U; 4 for launches whose partitions average under 8 192 rows, where a
// 512-thread span of 8 rows per lane leaves most lanes idle: C3 0.262 -> 0.222 ms)
template <int NVC, bool SORT, bool HV, bool NUL = true, int UR = EK_AGG_U>
__global__ __launch_bounds__(kAggBlock) __attribute__((amdgpu_waves_per_eu(EK_AGG_WAVES_PER_EU))) void k_agg(DPlan* __restrict__ pp, GroupDesc gd, LdsLayout lay,
                                                   const uint32_t* __restrict__ ctab, int ls, int64_t rs,
                                                   Staging st, DState ds, Results res, const int32_t* __restrict__ pane_err,
                                                   const int64_t* __restrict__ pbase, uint64_t* __restrict__ scratch,
                                                   int64_t scr_stride) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const DPlan& p = *pp;
    // XCD-aware order: dispatch slot b runs on XCD b % 8, which takes a contiguous share of the partitions, so the
    // neighbours (pane, bucket) and (pane, bucket + 1) — whose runs share a 128-B line at every chunk's run boundary —
    // are in flight together on one XCD and read that line once from its L2 (FETCH 2.15 -> 1.87 GB on C2)
    int pid = blockIdx.x;
    {
        const int xcd = pid % 8, q8 = (int)gridDim.x / 8, r8 = (int)gridDim.x % 8;
        pid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pid / 8;
    }
    const int kk = 1 << gd.kbits;
    const int rel = pid / gd.nb, bucket = pid % gd.nb;
    const int64_t q = gd.q_lo + rel;
    const int64_t slot = q % gd.ring;
    const bool fresh = gd.fresh[rel] != 0;
    const int64_t dbase = gd.dbase[rel];
    // ---- the partition's rows are one run per chunk that holds rows of this pane (k_part)
    // run tables in dynamic LDS past the aggregation tables, sized by the launch's longest run list (gd.mruns):
    // staging index of each run (staging < 2^32 rows, host-checked) and the exclusive prefix of the run lengths
    const int mr = gd.mruns;
    uint32_t* r_start = (uint32_t*)(lds + lay.bytes);
    uint32_t* r_pre = r_start + mr;
    __shared__ uint32_t r_wsum[kAggBlock / 64];
    int c_lo, c_hi;
    part_chunks(gd, rel, &c_lo, &c_hi);
    const int nruns = min(c_hi - c_lo + 1, mr);
    for (int j = threadIdx.x; j < nruns; j += kAggBlock) {
        const int c = c_lo + j;
        uint32_t o0, o1;
        part_run(gd, ctab, ls, rel, bucket, c, &o0, &o1);
        r_start[j] = (uint32_t)((int64_t)c * rs + o0);
        r_pre[j] = o1 - o0;
    }
    __syncthreads();
    {   // exclusive prefix of run lengths (512 threads)
        const int per = (nruns + kAggBlock - 1) / kAggBlock;
        const int b0 = threadIdx.x * per, b1 = min(nruns, b0 + per);
        uint32_t sm = 0;
        for (int k = b0; k < b1; ++k) sm += r_pre[k];
        uint32_t x = sm;
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) r_wsum[wv] = x;
        __syncthreads();
        uint32_t wb = 0;
        for (int w = 0; w < wv; ++w) wb += r_wsum[w];
        uint32_t run = wb + x - sm;
        for (int k = b0; k < b1; ++k) { uint32_t c = r_pre[k]; r_pre[k] = run; run += c; }
        if (threadIdx.x == kAggBlock - 1) r_pre[nruns] = run;
        __syncthreads();
    }
    const uint32_t total = nruns > 0 ? r_pre[nruns] : 0u;
    if (total == 0 && (!fresh || dbase >= 0)) {   // nothing to merge / no rows to emit
        // a directly emitted pane whose every row failed WHERE still carries the window's error
        if (dbase >= 0 && bucket == 0 && threadIdx.x == 0 && pane_err[slot]) {
            const int32_t widx = gd.didx[rel];
            atomicOr(&res.win_err[widx], pane_err[slot]);
            if (res.wwit) wit_copy(&res.wwit[2 * widx], &res.pwit[slot]);
        }
        return;
    }
    if (!SORT && dbase >= 0 && total <= (uint32_t)kSparseRows) {
        agg_sparse<NVC, HV>(p, gd, st, lds, r_start, r_pre, nruns, total, bucket, kk, slot, rel, dbase, pane_err, res);
        return;
    }

    uint32_t* lcnt = (uint32_t*)(lds + lay.off_cnt);
    for (int k = threadIdx.x; k < lay.bytes / 4; k += kAggBlock) ((uint32_t*)lds)[k] = 0;
    // plan fields in registers (scalar reloads inside the atomic loop would serialise on lgkmcnt)
    int fl[NVC];
    bool isf[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) { fl[v] = p.vc_flags[v]; isf[v] = p.vc_is_float[v] != 0; }
    const uint32_t nullm = st.nullable_mask;
    __syncthreads();
    // rows of the partition as one virtual array: row v lives in run j = max{j : r_pre[j] <= v}.
    // Each wave takes a span of 64*U consecutive rows (coalesced loads); its first run is found by
    // one binary search, and every lane then advances its run pointer monotonically.
    constexpr int U = UR;   // rows in flight per lane (per pipeline stage with EK_AGG_PIPE)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    auto run_of = [&](uint32_t v) {
        int lo = 0, hi = nruns - 1;
        while (lo < hi) { int m = (lo + hi + 1) >> 1; if (r_pre[m] <= v) lo = m; else hi = m - 1; }
        return lo;
    };
    int64_t dbg_sink = 0;
    struct Span {
        int klu[U];
        int64_t rv[NVC][U];
        uint8_t vd[NVC][U];
    };
    // the rows [span, span + 64 U) of this lane: key low bits (-1 past the end), values, validity
    auto load_span = [&](uint32_t span, Span& sp) {
        int j = run_of(span);
        int64_t pos[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = span + u * 64 + lane;
            pos[u] = -1;
            if (v < total) {
                while (j + 1 < nruns && r_pre[j + 1] <= v) ++j;
                pos[u] = (int64_t)r_start[j] + (v - r_pre[j]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            sp.klu[u] = pos[u] >= 0 ? (int)st.klo[pos[u]] : -1;
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                sp.rv[v][u] = (pos[u] >= 0 && fl[v]) ? st.val[v][pos[u]] : 0;
                sp.vd[v][u] = (NUL && pos[u] >= 0 && (nullm & (1u << v))) ? st.valid[v][pos[u]] : (uint8_t)1;
            }
        }
    };
    auto fold_span = [&](const Span& sp) {
        if (gd.pad & 32) {   // diagnostic knob 32: loads only, no LDS atomics (timing only)
#pragma unroll
            for (int u = 0; u < U; ++u) { dbg_sink += sp.klu[u]; for (int v = 0; v < NVC; ++v) dbg_sink += sp.rv[v][u]; }
            return;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int kl = sp.klu[u];
            if (kl < 0) break;
            atomicAdd(&lcnt[kl], 1u);
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = fl[v];
                if (f == 0 || !sp.vd[v][u]) continue;
                const int64_t raw = sp.rv[v][u];
                if (f & NEED_CNT) atomicAdd(&((uint32_t*)(lds + lay.off_vcnt[v]))[kl], 1u);
                if (isf[v]) {
                    const double x = __longlong_as_double(raw);
                    if (f & NEED_SUM) atomicAdd(&((double*)(lds + lay.off_sum[v]))[kl], x);
                    if (f & NEED_MIN) atomicMax(&((unsigned long long*)(lds + lay.off_min[v]))[kl], (unsigned long long)~f64_to_ord(x));
                    if (f & NEED_MAX) atomicMax(&((unsigned long long*)(lds + lay.off_max[v]))[kl], (unsigned long long)f64_to_ord(x));
                } else {
                    if (f & NEED_SUM) atomicAdd(&((unsigned long long*)(lds + lay.off_sum[v]))[kl], (unsigned long long)raw);
                    if (f & NEED_FSUM) atomicAdd(&((double*)(lds + lay.off_fsum[v]))[kl], (double)raw);
                    if (f & NEED_MIN) atomicMax(&((unsigned long long*)(lds + lay.off_min[v]))[kl], (unsigned long long)~i64_to_ord(raw));
                    if (f & NEED_MAX) atomicMax(&((unsigned long long*)(lds + lay.off_max[v]))[kl], (unsigned long long)i64_to_ord(raw));
                }
            }
        }
    };
    constexpr uint32_t kSpanStep = (uint32_t)kAggBlock * U;
#if EK_AGG_PIPE
    // software pipeline: the next span's loads are in flight while this span's rows are folded into LDS
    {
        uint32_t span = (uint32_t)wave * 64u * U;
        Span a, b;
        if (span < total) load_span(span, a);
        for (; span < total; span += 2 * kSpanStep) {
            if (span + kSpanStep < total) load_span(span + kSpanStep, b);
            fold_span(a);
            if (span + kSpanStep >= total) break;
            if (span + 2 * kSpanStep < total) load_span(span + 2 * kSpanStep, a);
            fold_span(b);
        }
    }
#else
    for (uint32_t span = (uint32_t)wave * 64u * U; span < total; span += kSpanStep) {
        Span a;
        load_span(span, a);
        fold_span(a);
    }
#endif
    if ((gd.pad & 32) && dbg_sink == 0x5A5A5A5A5A5ALL) lcnt[0] = 1;   // keeps the knob-32 loads alive
    __syncthreads();
    bool need_m2 = false;
#pragma unroll
    for (int v = 0; v < NVC; ++v) need_m2 |= (p.vc_flags[v] & NEED_M2) != 0;
    if (need_m2) {
        // second pass over the (L2-resident) run: Σ (x - mean)^2 with this partial's mean (stats._variance shape)
        for (uint32_t span = (uint32_t)wave * 64u; span < total; span += (uint32_t)kAggBlock) {
            const uint32_t vv = span + lane;
            if (vv >= total) continue;
            int lo = run_of(span);
            while (lo + 1 < nruns && r_pre[lo + 1] <= vv) ++lo;
            const int64_t i = (int64_t)r_start[lo] + (vv - r_pre[lo]);
            const int kl = st.klo[i];
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                if (!(p.vc_flags[v] & NEED_M2)) continue;
                if ((st.nullable_mask & (1u << v)) && !st.valid[v][i]) continue;
                const int64_t raw = st.val[v][i];
                const double x = p.vc_is_float[v] ? __longlong_as_double(raw) : (double)raw;
                const double n = (p.vc_flags[v] & NEED_CNT) ? (double)((uint32_t*)(lds + lay.off_vcnt[v]))[kl] : (double)lcnt[kl];
                const double sm = p.vc_is_float[v] ? ((double*)(lds + lay.off_sum[v]))[kl] : ((double*)(lds + lay.off_fsum[v]))[kl];
                const double d = __dsub_rn(x, __ddiv_rn(sm, n));
                atomicAdd(&((double*)(lds + lay.off_m2[v]))[kl], __dmul_rn(d, d));
            }
        }
        __syncthreads();
    }
    // ---- order statistics: group the partition's values by key into its scratch region, then select
    if constexpr (SORT) {
        uint32_t* koff = (uint32_t*)(lds + lay.off_koff);   // [kk + 1]
        uint32_t* kcur = (uint32_t*)(lds + lay.off_kcur);   // [kk]
        uint64_t* sres = (uint64_t*)(lds + lay.off_sres);   // [n_sagg][kk]
        uint8_t* stag = (uint8_t*)(lds + lay.off_stag);     // [n_sagg][kk]
        __shared__ uint32_t s_hist[256];
        __shared__ uint64_t s_sel[2];
        __shared__ uint32_t s_nbig;
        __shared__ uint32_t s_wsum[kAggBlock / 64];
        const int64_t pbs = pbase[pid];
        for (int sc = 0; sc < p.n_scol; ++sc) {
            const int v = p.scol_vc[sc];
            const bool vnull = (nullm >> v) & 1u;
            uint64_t* seg0 = scratch + (int64_t)sc * scr_stride + pbs;
            // values per key (nil values are ignored, cast.ToFloat64Slice IGNORE_NIL) -> exclusive offsets
            for (int k = threadIdx.x; k < kk; k += kAggBlock)
                koff[k] = (p.vc_flags[v] & NEED_CNT) ? ((uint32_t*)(lds + lay.off_vcnt[v]))[k] : lcnt[k];
            if (threadIdx.x == 0) s_nbig = 0;
            __syncthreads();
            {
                const int per = (kk + kAggBlock - 1) / kAggBlock;
                const int b0 = threadIdx.x * per, b1 = min(kk, b0 + per);
                uint32_t sm = 0;
                for (int k = b0; k < b1; ++k) sm += koff[k];
                uint32_t x = sm;
                for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
                if (lane == 63) s_wsum[wave] = x;
                __syncthreads();
                uint32_t wb = 0;
                for (int w = 0; w < wave; ++w) wb += s_wsum[w];
                uint32_t run = wb + x - sm;
                for (int k = b0; k < b1; ++k) { uint32_t c = koff[k]; koff[k] = run; kcur[k] = 0; run += c; }
                if (threadIdx.x == kAggBlock - 1) koff[kk] = run;
                __syncthreads();
            }
            // scatter the ordered bits of every valid value to its key's segment
            for (uint32_t span = (uint32_t)wave * 64u; span < total; span += (uint32_t)kAggBlock) {
                const uint32_t vv = span + lane;
                if (vv >= total) continue;
                int j = run_of(span);
                while (j + 1 < nruns && r_pre[j + 1] <= vv) ++j;
                const int64_t i = (int64_t)r_start[j] + (vv - r_pre[j]);
                if (vnull && !st.valid[v][i]) continue;
                const int kl = st.klo[i];
                const int64_t raw = st.val[v][i];
                const uint64_t o = isf[v] ? f64_to_ord(__longlong_as_double(raw)) : i64_to_ord(raw);
                seg0[koff[kl] + atomicAdd(&kcur[kl], 1u)] = o;
            }
            __threadfence();
            __syncthreads();
            // short segments: one thread per key; long ones are queued for the whole workgroup
            for (int kl = threadIdx.x; kl < kk; kl += kAggBlock) {
                const int n = (int)(koff[kl + 1] - koff[kl]);
                const uint64_t* seg = seg0 + koff[kl];
                const bool big = n > kSmallSeg;
                for (int a = 0; a < p.n_sagg; ++a) {
                    if (p.sagg_scol[a] != sc) continue;
                    const int k = p.sagg_agg[a];
                    if (big) continue;
                    order_stat(p.agg_fn[k], isf[v], p.agg_p[k], n, [&](int64_t r) { return seg_select(seg, n, (int)r); },
                               &sres[a * kk + kl], &stag[a * kk + kl]);
                }
                if (big) kcur[atomicAdd(&s_nbig, 1u)] = (uint32_t)kl;
            }
            __syncthreads();
            const uint32_t nbig = s_nbig;
            for (uint32_t t = 0; t < nbig; ++t) {
                const int kl = (int)kcur[t];
                const int64_t n = koff[kl + 1] - koff[kl];
                const uint64_t* seg = seg0 + koff[kl];
                for (int a = 0; a < p.n_sagg; ++a) {
                    if (p.sagg_scol[a] != sc) continue;
                    const int k = p.sagg_agg[a];
                    uint64_t o;
                    uint8_t tg;
                    order_stat(p.agg_fn[k], isf[v], p.agg_p[k], n,
                               [&](int64_t r) { return block_select(seg, n, r, s_hist, s_sel); }, &o, &tg);
                    if (threadIdx.x == 0) { sres[a * kk + kl] = o; stag[a * kk + kl] = tg; }
                }
            }
            __syncthreads();
        }
    }
    // this partition's partial for key kl, read back from LDS
    auto lds_part = [&](int kl, int64_t& c, int64_t (&vc)[NVC], int64_t (&is)[NVC], double (&fs)[NVC], double (&m2)[NVC],
                        uint64_t (&mn)[NVC], uint64_t (&mx)[NVC]) {
        c = lcnt[kl];
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            const int f = p.vc_flags[v];
            vc[v] = (f & NEED_CNT) ? (int64_t)((uint32_t*)(lds + lay.off_vcnt[v]))[kl] : c;
            is[v] = (!p.vc_is_float[v] && (f & NEED_SUM)) ? ((int64_t*)(lds + lay.off_sum[v]))[kl] : 0;
            fs[v] = p.vc_is_float[v] ? ((f & NEED_SUM) ? ((double*)(lds + lay.off_sum[v]))[kl] : 0.0)
                                     : ((f & NEED_FSUM) ? ((double*)(lds + lay.off_fsum[v]))[kl] : 0.0);
            m2[v] = (f & NEED_M2) ? ((double*)(lds + lay.off_m2[v]))[kl] : 0.0;
            mn[v] = (f & NEED_MIN) ? ~((unsigned long long*)(lds + lay.off_min[v]))[kl] : 0ull;
            mx[v] = (f & NEED_MAX) ? ((unsigned long long*)(lds + lay.off_max[v]))[kl] : 0ull;
        }
    };
    if (gd.pad & 2) return;   // diagnostic build knob: no emission / merge
    __shared__ uint32_t esh[20];
    if (dbase >= 0) {
        const int32_t widx = gd.didx[rel];
        const int32_t perr = pane_err[slot];
        if (perr) {   // a WHERE error replaces the window's output (filter_operator.go:63-77)
            if (threadIdx.x == 0 && bucket == 0) {
                atomicOr(&res.win_err[widx], perr);
                if (res.wwit) wit_copy(&res.wwit[2 * widx], &res.pwit[slot]);
            }
            return;
        }
        // (1) decide every key of the bucket (aggregate errors, HAVING) into a present bitmask, (2) one result-row
        // reservation for the workgroup, (3) each present key's row at its rank among the present keys (key order)
        const uint32_t K = p.key_col >= 0 ? p.num_keys : 1u;
        __shared__ uint32_t pmask[kMaxBucketKeys / 32];     // present keys of the bucket
        __shared__ uint32_t ppre[kMaxBucketKeys / 64 + 1];  // present keys before each 64-key chunk
        for (int kb = 0; kb < kk; kb += kAggBlock) {
            const int kl = kb + threadIdx.x;
            const int64_t key = (int64_t)bucket * kk + kl;
            bool present = false;
            if (kl < kk && key < K) {
                int64_t c, vc[NVC], is[NVC];
                double fs[NVC], m2[NVC];
                uint64_t mn[NVC], mx[NVC];
                lds_part(kl, c, vc, is, fs, m2, mn, mx);
                if (c > 0) {
                    Part<NVC> s{};
                    part_merge(p, s, c, vc, is, fs, m2, mn, mx);
                    int ea = -1;   // the first order statistic that failed
                    if constexpr (SORT) {
                        for (int a = p.n_sagg - 1; a >= 0; --a) if (((uint8_t*)(lds + lay.off_stag))[a * kk + kl] == kTagErr) ea = a;
                    }
                    const bool err = ea >= 0;
                    if (err) {   // "run Select error: ..." replaces the window
                        atomicOr(&res.win_err[widx], EK_WIN_AGG_ERROR);
                        if (res.aslot) atomicMax(&res.aslot[widx], kMaxSortAggs - ea);
                    }
                    else {
                        const SortRes sr{(const uint64_t*)(lds + lay.off_sres), (const uint8_t*)(lds + lay.off_stag), kl, kk};
                        present = !HV || having_keep(p, s, res, widx, (uint32_t)key, SORT ? &sr : nullptr);
                    }
                }
            }
            const unsigned long long m = __ballot(present);
            const int ch = (kb >> 6) + wave;
            if (lane == 0 && kb + wave * 64 < kk) { pmask[2 * ch] = (uint32_t)m; pmask[2 * ch + 1] = (uint32_t)(m >> 32); }
        }
        __syncthreads();
        const int nchk = (kk + 63) >> 6;
        if (wave == 0) {
            uint32_t run = 0;
            for (int c0 = 0; c0 < nchk; c0 += 64) {
                const int c = c0 + lane;
                const uint32_t n = c < nchk ? (uint32_t)(__popc(pmask[2 * c]) + __popc(pmask[2 * c + 1])) : 0u;
                uint32_t x = n;
                for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
                if (c < nchk) ppre[c] = run + x - n;
                run += __shfl(x, 63, 64);
            }
            if (lane == 0) esh[16] = run ? (uint32_t)atomicAdd((unsigned long long*)&res.win_cnt[widx], (unsigned long long)run) : 0u;
        }
        __syncthreads();
        const int64_t rbase = dbase + (int64_t)esh[16];
        for (int kl = threadIdx.x; kl < kk; kl += kAggBlock) {
            const int c = kl >> 6;
            const unsigned long long m = (unsigned long long)pmask[2 * c] | ((unsigned long long)pmask[2 * c + 1] << 32);
            if (!((m >> (kl & 63)) & 1ull) || (gd.pad & 64)) continue;   // (diagnostic knob 64: no row stores)
            const int64_t pos = rbase + ppre[c] + __popcll(m & ((1ull << (kl & 63)) - 1ull));
            int64_t cc, vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
            lds_part(kl, cc, vc, is, fs, m2, mn, mx);
            Part<NVC> s{};
            part_merge(p, s, cc, vc, is, fs, m2, mn, mx);
            const SortRes sr{(const uint64_t*)(lds + lay.off_sres), (const uint8_t*)(lds + lay.off_stag), kl, kk};
            res.key[pos] = (uint32_t)((int64_t)bucket * kk + kl);
#pragma unroll
            for (int k = 0; k < EK_MAX_AGGS; ++k) {
                if (k >= p.n_aggs) break;
                const Val a = agg_value(p, s, k, SORT ? &sr : nullptr);
                res.tag[k][pos] = a.tag == V_NULL ? EK_TAG_NULL : (a.tag == V_I64 ? EK_TAG_I64 : EK_TAG_F64);
                res.val[k][pos] = a.tag == V_F64 ? __double_as_longlong(a.f) : a.i;
            }
        }
        return;
    }
    // write (fresh pane) or merge into the pane state; the workgroup owns these (pane, key) entries
    for (int kl = threadIdx.x; kl < kk; kl += kAggBlock) {
        const int64_t e = slot * ds.K + (int64_t)bucket * kk + kl;
        int64_t c, vc[NVC], is[NVC];
        double fs[NVC], m2[NVC];
        uint64_t mn[NVC], mx[NVC];
        lds_part(kl, c, vc, is, fs, m2, mn, mx);
        if (fresh) {
            ds.cnt[e] = c;       // count 0 marks an absent key
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = p.vc_flags[v];
                if (f & NEED_CNT) ds.vcnt[v][e] = vc[v];
                if (f & NEED_SUM) ds.sum[v][e] = p.vc_is_float[v] ? __double_as_longlong(fs[v]) : is[v];
                if (f & NEED_FSUM) ds.fsum[v][e] = fs[v];
                if (f & NEED_M2) ds.m2[v][e] = m2[v];
                if (f & NEED_MIN) ds.mn[v][e] = (int64_t)mn[v];
                if (f & NEED_MAX) ds.mx[v][e] = (int64_t)mx[v];
            }
            continue;
        }
        if (c == 0) continue;
        Part<NVC> a{};
        int64_t avc[NVC], ais[NVC];
        double afs[NVC], am2[NVC];
        uint64_t amn[NVC], amx[NVC];
        const int64_t ac = ds.cnt[e];
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            const int f = p.vc_flags[v];
            avc[v] = (f & NEED_CNT) ? ds.vcnt[v][e] : ac;
            ais[v] = (!p.vc_is_float[v] && (f & NEED_SUM)) ? ds.sum[v][e] : 0;
            afs[v] = p.vc_is_float[v] ? ((f & NEED_SUM) ? __longlong_as_double(ds.sum[v][e]) : 0.0) : ((f & NEED_FSUM) ? ds.fsum[v][e] : 0.0);
            am2[v] = (f & NEED_M2) ? ds.m2[v][e] : 0.0;
            amn[v] = (f & NEED_MIN) ? (uint64_t)ds.mn[v][e] : 0ull;
            amx[v] = (f & NEED_MAX) ? (uint64_t)ds.mx[v][e] : 0ull;
        }
        if (ac) part_merge(p, a, ac, avc, ais, afs, am2, amn, amx);
        part_merge(p, a, c, vc, is, fs, m2, mn, mx);
        ds.cnt[e] = a.cnt;
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            const int f = p.vc_flags[v];
            if (f & NEED_CNT) ds.vcnt[v][e] = a.vcnt[v];
            if (f & NEED_SUM) ds.sum[v][e] = p.vc_is_float[v] ? __double_as_longlong(a.fsum[v]) : a.isum[v];
            if (f & NEED_FSUM) ds.fsum[v][e] = a.fsum[v];
            if (f & NEED_M2) ds.m2[v][e] = a.m2[v];
            if (f & NEED_MIN) ds.mn[v][e] = (int64_t)a.omn[v];
            if (f & NEED_MAX) ds.mx[v][e] = (int64_t)a.omx[v];
        }
    }
}

// ---------------------------------------------------------------- finalize closed windows
// Per (window, key): merge the window's panes from the pane state, finalise, HAVING, emit.
template <int NVC>
__global__ __launch_bounds__(kBlock) void k_finalize(DPlan* __restrict__ pp, const WinDesc* __restrict__ wins,
                                                     DState ds, int32_t ring, const int32_t* __restrict__ pane_err,
                                                     Results res) {
    const DPlan& p = *pp;
    // XCD-aware order: dispatch slot `orig` runs on the XCD labelled orig % 8; the bijective swizzle gives every XCD
    // a contiguous run of (key block-major, window-minor) work, so the consecutive windows of a key block — which
    // share all but one (hopping: ppw - 1 of ppw) panes — are merged on one XCD and re-read its L2
    const int64_t nwg = (int64_t)gridDim.x * gridDim.y;
    const int64_t orig = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
    const int64_t xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int64_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const WinDesc w = wins[wgid % gridDim.y];
    const int64_t key = (wgid / gridDim.y) * kBlock + threadIdx.x;
    int32_t werr = 0;
    for (int64_t q = w.q_first; q <= w.q_last; ++q) werr |= pane_err[q % ring];
    if (werr) {
        if (key == 0) {
            atomicOr(&res.win_err[w.idx], werr);
            if (res.wwit)   // the first pane with an error holds the window's first failed row
                for (int64_t q = w.q_first; q <= w.q_last; ++q)
                    if (pane_err[q % ring]) { wit_copy(&res.wwit[2 * w.idx], &res.pwit[q % ring]); break; }
        }
        return;
    }
    const uint32_t K = p.key_col >= 0 ? p.num_keys : 1u;
    Part<NVC> s{};
    bool present = false;
    if (key < K) {
        for (int64_t q = w.q_first; q <= w.q_last; ++q) {
            const int64_t e = (q % ring) * ds.K + key;
            const int64_t c = ds.cnt[e];
            if (c == 0) continue;
            int64_t vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = p.vc_flags[v];
                vc[v] = (f & NEED_CNT) ? ds.vcnt[v][e] : c;
                is[v] = (!p.vc_is_float[v] && (f & NEED_SUM)) ? ds.sum[v][e] : 0;
                fs[v] = p.vc_is_float[v] ? ((f & NEED_SUM) ? __longlong_as_double(ds.sum[v][e]) : 0.0)
                                         : ((f & NEED_FSUM) ? ds.fsum[v][e] : 0.0);
                m2[v] = (f & NEED_M2) ? ds.m2[v][e] : 0.0;
                mn[v] = (f & NEED_MIN) ? (uint64_t)ds.mn[v][e] : 0ull;
                mx[v] = (f & NEED_MAX) ? (uint64_t)ds.mx[v][e] : 0ull;
            }
            part_merge(p, s, c, vc, is, fs, m2, mn, mx);
        }
        present = s.cnt > 0 && having_keep(p, s, res, w.idx, (uint32_t)key);
    }
    __shared__ uint32_t esh[20];
    emit_rows(p, present, s, key, w.out_base, w.idx, res, esh);
}

// Hopping finalize with a register ring (one value column whose fields are count / sum / min / max; VC: its non-nil
// count): one thread per key walks the launch's consecutive windows [c0, c1) pane by pane. Each pane's partial is
// loaded once — coalesced over the block's keys — into a ring of R register slots that shifts by one per pane, so
// every slot index is static (no scratch). When a window's last pane arrives it is merged from the ring's last
// panes in pane order (the same merge order as k_finalize: the same f64 sums). k_finalize re-reads a pane once per
// window that spans it (ppw times); here a block chunk of cw windows reads cw + ppw - 1 panes.
#ifndef EK_RING_WPE
#define EK_RING_WPE 1
#endif
#ifndef EK_RING_AHEAD
#define EK_RING_AHEAD 3
#endif
constexpr int kRingAhead = EK_RING_AHEAD;   // k_finalize_ring: panes loaded ahead of the one being merged
// PART 0: every aggregate in one walk. The split walk (no HAVING) halves the ring's registers: PART 1 carries count /
// non-nil count / sum and stores the row's key and its count / sum / avg slots, reserving the block's rows with the
// atomic and recording each (window, block) base in gbase; PART 2 carries count / non-nil count / min / max and stores
// the min / max slots of the same rows — same presence (count > 0), same ballots, the base read back from gbase.
template <int R, bool VC, bool HV, int PART>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(EK_RING_WPE))) void k_finalize_ring(DPlan* __restrict__ pp, const WinDesc* __restrict__ wins,
                                                          int32_t nwin, int32_t cw, DState ds, int32_t ring,
                                                          const int32_t* __restrict__ pane_err, Results res,
                                                          uint32_t* __restrict__ gbase) {
    static_assert(PART == 0 || !HV, "the split walk decides presence by the row count alone");
    constexpr bool kSum = PART != 2, kMinMax = PART != 1;
    const DPlan& p = *pp;
    const int c0 = (int)blockIdx.y * cw, c1 = min(nwin, c0 + cw);
    if (c0 >= c1) return;   // uniform over the block
    const int64_t key = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t K = p.key_col >= 0 ? p.num_keys : 1u;
    const bool live = key < (int64_t)K;
    const int f = p.vc_flags[0];
    const bool isf = p.vc_is_float[0] != 0;
    const bool fsum_out = isf || p.inc;   // sum / avg as float64 (funcs_agg.go; inc_* aggregates)
    // the ring, newest pane in slot R - 1 (a shift per pane keeps every index static): a pane's count (< 2^31 rows of
    // a key), non-nil count, sum bits, ordered min / max
    int32_t rc[R], rv[R], re[R];   // re: the pane's WHERE error flag (uniform)
    int64_t rs[R];
    uint64_t rmn[R], rmx[R];
#pragma unroll
    for (int t = 0; t < R; ++t) { rc[t] = rv[t] = re[t] = 0; rs[t] = 0; rmn[t] = rmx[t] = 0; }
    // block-compacted emission, one window behind: window w's rows are stored while window w + 1 is merged, so the
    // returning atomic on w's row counter is off the critical path. esh[8 par + wave]: row counts -> offsets of the
    // two windows in flight, esh[16 + par]: the block's base in the window's region
    __shared__ uint32_t esh[20];
    int par = 0;
    bool pd_has = false, pd_present = false;
    int64_t pd_out = 0;
    unsigned long long pd_mask = 0;
    int64_t pd_cnt = 0, pd_vcn = 0, pd_isum = 0;
    double pd_fsum = 0.0;
    uint64_t pd_omn = 0, pd_omx = 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    auto store_pending = [&]() {   // window pd's rows: esh[8 (1 - par) + wave] + esh[16 + (1 - par)] are final
        if (!pd_has || !pd_present) return;
        const int pp_ = par ^ 1;
        const int64_t pos = pd_out + (int64_t)esh[16 + pp_] + esh[8 * pp_ + wv] + __popcll(pd_mask & ((1ull << lane) - 1ull));
        if (PART != 2) res.key[pos] = (uint32_t)key;
        for (int k = 0; k < p.n_aggs; ++k) {
            const int fn = p.agg_fn[k];
            int64_t v = 0;
            uint8_t tg = EK_TAG_I64;
            if (PART == 1 && (fn == EK_AGG_MIN || fn == EK_AGG_MAX)) continue;
            if (PART == 2 && fn != EK_AGG_MIN && fn != EK_AGG_MAX) continue;
            if (fn == EK_AGG_COUNT_STAR) v = pd_cnt;
            else if (fn == EK_AGG_COUNT) v = pd_vcn;
            else if (pd_vcn == 0) tg = EK_TAG_NULL;
            else if (fn == EK_AGG_SUM) { if (fsum_out) { tg = EK_TAG_F64; v = __double_as_longlong(pd_fsum); } else v = pd_isum; }
            else if (fn == EK_AGG_AVG) {
                if (fsum_out) { tg = EK_TAG_F64; v = __double_as_longlong(__ddiv_rn(pd_fsum, (double)pd_vcn)); }
                else v = pd_isum / pd_vcn;
            } else {
                const uint64_t o = fn == EK_AGG_MIN ? pd_omn : pd_omx;
                if (isf) { tg = EK_TAG_F64; v = __double_as_longlong(ord_to_f64(o)); }
                else v = ord_to_i64(o);
            }
            res.tag[k][pos] = tg;
            res.val[k][pos] = v;
        }
    };
    const int64_t P0 = wins[c0].q_first, P1 = wins[c1 - 1].q_last;
    int w = c0;
    int64_t wl = wins[c0].q_last;   // the last pane of window w
    int32_t sq = (int32_t)(P0 % ring);
    // pane loads run kRingAhead panes ahead (a queue shifted like the ring): enough bytes in flight per wave to
    // cover the HBM latency at the two waves per SIMD the ring's registers leave
    constexpr int D = kRingAhead;
    int32_t pc[D], pv[D], pe[D];
    int64_t ps[D];
    uint64_t pmn[D], pmx[D];
    auto load = [&](int d, int32_t slot, bool ok) {
        const int64_t e = (int64_t)slot * ds.K + key;
        const bool l = live && ok;
        pe[d] = ok ? pane_err[slot] : 0;
        pc[d] = l ? (int32_t)ds.cnt[e] : 0;
        pv[d] = (VC && l) ? (int32_t)ds.vcnt[0][e] : 0;
        ps[d] = (kSum && l && (f & NEED_SUM)) ? ds.sum[0][e] : 0;
        pmn[d] = (kMinMax && l && (f & NEED_MIN)) ? (uint64_t)ds.mn[0][e] : 0ull;
        pmx[d] = (kMinMax && l && (f & NEED_MAX)) ? (uint64_t)ds.mx[0][e] : 0ull;
    };
#pragma unroll
    for (int d = 0; d < D; ++d) {
        load(d, sq, P0 + d <= P1);
        sq = sq + 1 == ring ? 0 : sq + 1;
    }
    for (int64_t q = P0; q <= P1; ++q) {
#pragma unroll
        for (int t = 0; t + 1 < R; ++t) {
            rc[t] = rc[t + 1]; rv[t] = rv[t + 1]; re[t] = re[t + 1]; rs[t] = rs[t + 1]; rmn[t] = rmn[t + 1]; rmx[t] = rmx[t + 1];
        }
        rc[R - 1] = pc[0]; rv[R - 1] = pv[0]; re[R - 1] = pe[0]; rs[R - 1] = ps[0]; rmn[R - 1] = pmn[0]; rmx[R - 1] = pmx[0];
#pragma unroll
        for (int d = 0; d + 1 < D; ++d) { pc[d] = pc[d + 1]; pv[d] = pv[d + 1]; pe[d] = pe[d + 1]; ps[d] = ps[d + 1]; pmn[d] = pmn[d + 1]; pmx[d] = pmx[d + 1]; }
        load(D - 1, sq, q + D <= P1);
        sq = sq + 1 == ring ? 0 : sq + 1;
        while (w < c1 && wl == q) {   // window w closes with pane q (uniform): its panes are the ring's last `span`
            const WinDesc wd = wins[w];
            const int span = (int)(q - wd.q_first + 1);   // <= R (host-checked)
            int32_t werr = 0;
#pragma unroll
            for (int t = 0; t < R; ++t) werr |= t >= R - span ? re[t] : 0;
            if (werr) {
                if (PART != 2 && blockIdx.x == 0 && threadIdx.x == 0) {
                    atomicOr(&res.win_err[wd.idx], werr);
                    if (res.wwit)   // the first pane with an error holds the window's first failed row
                        for (int64_t qq = wd.q_first; qq <= q; ++qq)
                            if (pane_err[qq % ring]) { wit_copy(&res.wwit[2 * wd.idx], &res.pwit[qq % ring]); break; }
                }
            } else {
                // part_merge restricted to count / sum / min / max, the same operations in the same pane order
                int64_t cnt = 0, vcn = 0, isum = 0;
                double fsum = 0.0;
                uint64_t omn = 0, omx = 0;
#pragma unroll
                for (int t = 0; t < R; ++t) {   // the window's panes in pane order
                    if (t < R - span || rc[t] == 0) continue;
                    cnt += rc[t];
                    const int64_t nb = VC ? (int64_t)rv[t] : (int64_t)rc[t];
                    if (nb == 0) continue;
                    const bool first = vcn == 0;
                    vcn += nb;
                    if (kSum) {
                        isum = (int64_t)((uint64_t)isum + (uint64_t)(isf ? 0 : rs[t]));
                        const double fs = isf ? __longlong_as_double(rs[t]) : 0.0;
                        fsum = first ? fs : __dadd_rn(fsum, fs);
                    }
                    if (kMinMax) {
                        omn = (first || rmn[t] < omn) ? rmn[t] : omn;
                        omx = (first || rmx[t] > omx) ? rmx[t] : omx;
                    }
                }
                bool present = live && cnt > 0;
                if (HV && present) {
                    Part<1> s{};
                    s.cnt = cnt; s.vcnt[0] = vcn; s.isum[0] = isum; s.fsum[0] = fsum; s.omn[0] = omn; s.omx[0] = omx;
                    present = having_keep(p, s, res, wd.idx, (uint32_t)key);
                }
                // rows of count / sum / avg / min / max (funcs_agg.go:56-113): counted now, stored one window later
                const unsigned long long mask = __ballot(present);
                if (lane == 0) esh[8 * par + wv] = (uint32_t)__popcll(mask);
                __syncthreads();   // this window's counts are in; the previous window's base (thread 0) too
                store_pending();
                if (threadIdx.x == 0) {
                    uint32_t run = 0;
                    for (int x = 0; x < kBlock / 64; ++x) { const uint32_t c = esh[8 * par + x]; esh[8 * par + x] = run; run += c; }
                    if (PART == 2) {
                        esh[16 + par] = run ? gbase[(int64_t)w * gridDim.x + blockIdx.x] : 0u;
                    } else {
                        esh[16 + par] = run ? (uint32_t)atomicAdd((unsigned long long*)&res.win_cnt[wd.idx], (unsigned long long)run) : 0u;
                        if (PART == 1) gbase[(int64_t)w * gridDim.x + blockIdx.x] = esh[16 + par];
                    }
                }
                pd_has = true;
                pd_present = present;
                pd_out = wd.out_base;
                pd_mask = mask;
                pd_cnt = cnt; pd_vcn = vcn; pd_isum = isum; pd_fsum = fsum; pd_omn = omn; pd_omx = omx;
                par ^= 1;
            }
            ++w;
            wl = w < c1 ? wins[w].q_last : INT64_MAX;
        }
    }
    __syncthreads();   // the last window's base
    store_pending();
}

// Un-grouped rule (pseudo keys): one workgroup per window merges every (pane, partial slot) entry of the window into
// ONE group (Chan merge for M2, a fixed tree order for the sums), then HAVING and the single row (key 0).
template <int NVC>
__global__ __launch_bounds__(kBlock) void k_finalize_merge(DPlan* __restrict__ pp, const WinDesc* __restrict__ wins,
                                                           DState ds, int32_t ring, const int32_t* __restrict__ pane_err,
                                                           Results res) {
    const DPlan& p = *pp;
    const WinDesc w = wins[blockIdx.x];
    int32_t werr = 0;
    for (int64_t q = w.q_first; q <= w.q_last; ++q) werr |= pane_err[q % ring];
    if (werr) {
        if (threadIdx.x == 0) {
            atomicOr(&res.win_err[w.idx], werr);
            if (res.wwit)   // the first pane with an error holds the window's first failed row
                for (int64_t q = w.q_first; q <= w.q_last; ++q)
                    if (pane_err[q % ring]) { wit_copy(&res.wwit[2 * w.idx], &res.pwit[q % ring]); break; }
        }
        return;
    }
    Part<NVC> s{};
    for (int64_t q = w.q_first; q <= w.q_last; ++q) {
        for (int64_t key = threadIdx.x; key < (int64_t)kPseudoKeys; key += kBlock) {
            const int64_t e = (q % ring) * ds.K + key;
            const int64_t c = ds.cnt[e];
            if (c == 0) continue;
            int64_t vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = p.vc_flags[v];
                vc[v] = (f & NEED_CNT) ? ds.vcnt[v][e] : c;
                is[v] = (!p.vc_is_float[v] && (f & NEED_SUM)) ? ds.sum[v][e] : 0;
                fs[v] = p.vc_is_float[v] ? ((f & NEED_SUM) ? __longlong_as_double(ds.sum[v][e]) : 0.0)
                                         : ((f & NEED_FSUM) ? ds.fsum[v][e] : 0.0);
                m2[v] = (f & NEED_M2) ? ds.m2[v][e] : 0.0;
                mn[v] = (f & NEED_MIN) ? (uint64_t)ds.mn[v][e] : 0ull;
                mx[v] = (f & NEED_MAX) ? (uint64_t)ds.mx[v][e] : 0ull;
            }
            part_merge(p, s, c, vc, is, fs, m2, mn, mx);
        }
    }
    // block tree merge of the per-thread partials through LDS
    __shared__ int64_t t_cnt[kBlock], t_vc[NVC][kBlock], t_is[NVC][kBlock];
    __shared__ double t_fs[NVC][kBlock], t_m2[NVC][kBlock];
    __shared__ uint64_t t_mn[NVC][kBlock], t_mx[NVC][kBlock];
    const int t = threadIdx.x;
    for (int stride = kBlock / 2; stride > 0; stride >>= 1) {
        if (t >= stride && t < 2 * stride) {
            t_cnt[t] = s.cnt;
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                t_vc[v][t] = s.vcnt[v]; t_is[v][t] = s.isum[v]; t_fs[v][t] = s.fsum[v]; t_m2[v][t] = s.m2[v];
                t_mn[v][t] = s.omn[v]; t_mx[v][t] = s.omx[v];
            }
        }
        __syncthreads();
        if (t < stride && t_cnt[t + stride] > 0) {
            const int o = t + stride;
            int64_t vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
#pragma unroll
            for (int v = 0; v < NVC; ++v) { vc[v] = t_vc[v][o]; is[v] = t_is[v][o]; fs[v] = t_fs[v][o]; m2[v] = t_m2[v][o]; mn[v] = t_mn[v][o]; mx[v] = t_mx[v][o]; }
            part_merge(p, s, t_cnt[o], vc, is, fs, m2, mn, mx);
        }
        __syncthreads();
    }
    bool present = false;
    if (t == 0) present = s.cnt > 0 && having_keep(p, s, res, w.idx, 0u);
    __shared__ uint32_t esh[20];
    emit_rows(p, present, s, 0, w.out_base, w.idx, res, esh);
}

// ---------------------------------------------------------------- un-grouped rules over ts-sorted groups: one pass
// Block tree merge of the per-thread partials through LDS (fixed order); thread 0 ends with the block's partial.
template <int NVC, int B>
__device__ __forceinline__ void block_merge_part(const DPlan& p, Part<NVC>& s) {
    __shared__ int64_t t_cnt[B], t_vc[NVC][B], t_is[NVC][B];
    __shared__ double t_fs[NVC][B], t_m2[NVC][B];
    __shared__ uint64_t t_mn[NVC][B], t_mx[NVC][B];
    const int t = threadIdx.x;
    for (int stride = B / 2; stride > 0; stride >>= 1) {
        if (t >= stride && t < 2 * stride) {
            t_cnt[t] = s.cnt;
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                t_vc[v][t] = s.vcnt[v]; t_is[v][t] = s.isum[v]; t_fs[v][t] = s.fsum[v]; t_m2[v][t] = s.m2[v];
                t_mn[v][t] = s.omn[v]; t_mx[v][t] = s.omx[v];
            }
        }
        __syncthreads();
        if (t < stride && t_cnt[t + stride] > 0) {
            const int o = t + stride;
            int64_t vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
#pragma unroll
            for (int v = 0; v < NVC; ++v) { vc[v] = t_vc[v][o]; is[v] = t_is[v][o]; fs[v] = t_fs[v][o]; m2[v] = t_m2[v][o]; mn[v] = t_mn[v][o]; mx[v] = t_mx[v][o]; }
            part_merge(p, s, t_cnt[o], vc, is, fs, m2, mn, mx);
        }
        __syncthreads();
    }
}

// An un-grouped rule (pseudo keys) over a ts-sorted group: every pane is a contiguous row range, so one workgroup
// per tile of rows folds each pane segment of its tile into ONE partial (accept mask, WHERE, a thread-local
// two-pass M2 about the thread's own mean, then the block's Chan tree merge) and merges it into partial slot
// (tile mod kPseudoKeys) of the pane — no staging round trip, every referenced column read once (count(*) alone
// reads nothing). The host sizes the tiles so a launch has at most kPseudoKeys of them (distinct slots per pane)
// and zeroes the slot counts of fresh panes first; k_finalize_merge folds a window's slots as before.
constexpr int kUngBlock = 256;
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_ung_zero(GroupDesc gd, DState ds) {
    const int r = blockIdx.y;
    if (!gd.fresh[r]) return;
    int64_t* c = ds.cnt + ((gd.q_lo + r) % gd.ring) * ds.K;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < (int64_t)kPseudoKeys; k += (int64_t)gridDim.x * blockDim.x) c[k] = 0;
}
#endif

template <int NVC, bool WHERE>
__global__ __launch_bounds__(kUngBlock) __attribute__((amdgpu_waves_per_eu(NVC <= 2 ? 4 : 3))) void k_ung_tile(DPlan* __restrict__ pp, DBatch b, GroupDesc gd,
                                                        const uint8_t* __restrict__ acc, DState ds, int64_t tile,
                                                        int32_t* __restrict__ pane_err) {
    const DPlan& p = *pp;
    const int64_t t0 = gd.lo + (int64_t)blockIdx.x * tile, t1 = min(gd.hi, t0 + tile);
    int r = 0;
    {   // first pane of the tile: the last r with pbnd[r] <= t0
        int lo = 0, hi = gd.n_panes - 1;
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (gd.pbnd[mid] <= t0) lo = mid; else hi = mid - 1; }
        r = lo;
    }
    const bool raw_count = p.n_vc == 0 && !WHERE && !gd.has_accept;
    int col[NVC], fl[NVC];
    bool isf[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) { col[v] = v < p.n_vc ? p.vc_col[v] : 0; fl[v] = v < p.n_vc ? p.vc_flags[v] : 0; isf[v] = p.vc_is_float[v] != 0; }
    for (; r < gd.n_panes && gd.pbnd[r] < t1; ++r) {
        const int64_t s0 = max(t0, gd.pbnd[r]), s1 = min(t1, gd.pbnd[r + 1]);
        if (s1 <= s0) continue;
        Part<NVC> s{};
        if (raw_count) {
            if (threadIdx.x == 0) s.cnt = s1 - s0;
        } else {
            int64_t c = 0, vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
#pragma unroll
            for (int v = 0; v < NVC; ++v) { vc[v] = 0; is[v] = 0; fs[v] = 0.0; m2[v] = 0.0; mn[v] = ~0ull; mx[v] = 0ull; }
            bool werr = false;
            for (int64_t i = s0 + threadIdx.x; i < s1; i += kUngBlock) {
                if (gd.has_accept && !acc[i]) continue;
                if (WHERE) {
                    const int w = where_decide_slow(p, b, i);
                    werr |= w < 0;
                    if (w <= 0) continue;
                }
                c++;
#pragma unroll
                for (int v = 0; v < NVC; ++v) {
                    if (!fl[v] || !col_valid(b, col[v], i)) continue;
                    const int64_t raw = ((const int64_t*)b.col[col[v]])[i];
                    const double x = isf[v] ? __longlong_as_double(raw) : (double)raw;
                    const uint64_t o = isf[v] ? f64_to_ord(x) : i64_to_ord(raw);
                    vc[v]++;
                    is[v] = (int64_t)((uint64_t)is[v] + (uint64_t)raw);
                    fs[v] = __dadd_rn(fs[v], x);
                    mn[v] = o < mn[v] ? o : mn[v];
                    mx[v] = o > mx[v] ? o : mx[v];
                }
            }
            if (werr) {
                const int64_t slot = (gd.q_lo + r) % gd.ring;
                atomicOr(&pane_err[slot], EK_WIN_WHERE_ERROR);
                if (gd.pwit)   // this thread's first failed row (found again: no register holds it in the loop)
                    for (int64_t i = s0 + threadIdx.x; i < s1; i += kUngBlock) {
                        if ((gd.has_accept && !acc[i]) || where_decide_slow(p, b, i) >= 0) continue;
                        wit_where_row(&gd.pwit[slot], gd.wit_ts ? i64_to_ord(((const int64_t*)b.col[gd.ts_col])[i]) : 0ull,
                                      (unsigned long long)(gd.wit_o2 + i), p, b, i);
                        break;
                    }
            }
#pragma unroll
            for (int v = 0; v < NVC; ++v) {   // centred second pass over the thread's own rows (L1/L2-warm)
                if (!(fl[v] & NEED_M2) || vc[v] == 0) continue;
                const double mean = __ddiv_rn(fs[v], (double)vc[v]);
                for (int64_t i = s0 + threadIdx.x; i < s1; i += kUngBlock) {
                    if (gd.has_accept && !acc[i]) continue;
                    if (WHERE && where_decide_slow(p, b, i) <= 0) continue;
                    if (!col_valid(b, col[v], i)) continue;
                    const int64_t raw = ((const int64_t*)b.col[col[v]])[i];
                    const double d = __dsub_rn(isf[v] ? __longlong_as_double(raw) : (double)raw, mean);
                    m2[v] = __dadd_rn(m2[v], __dmul_rn(d, d));
                }
            }
            if (c > 0) part_merge(p, s, c, vc, is, fs, m2, mn, mx);
        }
        if (!raw_count) block_merge_part<NVC, kUngBlock>(p, s);
        if (threadIdx.x == 0 && s.cnt > 0) {
            const int64_t e = ((gd.q_lo + r) % gd.ring) * ds.K + (int64_t)(blockIdx.x % kPseudoKeys);
            Part<NVC> a{};
            const int64_t ac = ds.cnt[e];
            if (ac) {
                int64_t avc[NVC], ais[NVC];
                double afs[NVC], am2[NVC];
                uint64_t amn[NVC], amx[NVC];
#pragma unroll
                for (int v = 0; v < NVC; ++v) {
                    const int f = fl[v];
                    avc[v] = (f & NEED_CNT) ? ds.vcnt[v][e] : ac;
                    ais[v] = (!isf[v] && (f & NEED_SUM)) ? ds.sum[v][e] : 0;
                    afs[v] = isf[v] ? ((f & NEED_SUM) ? __longlong_as_double(ds.sum[v][e]) : 0.0) : ((f & NEED_FSUM) ? ds.fsum[v][e] : 0.0);
                    am2[v] = (f & NEED_M2) ? ds.m2[v][e] : 0.0;
                    amn[v] = (f & NEED_MIN) ? (uint64_t)ds.mn[v][e] : 0ull;
                    amx[v] = (f & NEED_MAX) ? (uint64_t)ds.mx[v][e] : 0ull;
                }
                part_merge(p, a, ac, avc, ais, afs, am2, amn, amx);
            }
            part_merge(p, a, s.cnt, s.vcnt, s.isum, s.fsum, s.m2, s.omn, s.omx);
            ds.cnt[e] = a.cnt;
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = fl[v];
                if (f & NEED_CNT) ds.vcnt[v][e] = a.vcnt[v];
                if (f & NEED_SUM) ds.sum[v][e] = isf[v] ? __double_as_longlong(a.fsum[v]) : a.isum[v];
                if (f & NEED_FSUM) ds.fsum[v][e] = a.fsum[v];
                if (f & NEED_M2) ds.m2[v][e] = a.m2[v];
                if (f & NEED_MIN) ds.mn[v][e] = (int64_t)a.omn[v];
                if (f & NEED_MAX) ds.mx[v][e] = (int64_t)a.omx[v];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- debug: window membership fingerprint
// Per pane: number of accepted events (before WHERE) and Σ ek_mix64(arrival index); a window's
// fingerprint is the sum over its panes (order-independent, exact in u64 arithmetic).
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_members(DPlan* __restrict__ pp, DBatch b, PaneGrid g, const uint8_t* acc,
                                                    int has_acc, int64_t lo, int64_t hi, int64_t arrival_base,
                                                    const int64_t* __restrict__ arrival, int64_t qa, int64_t qb,
                                                    int32_t ring, int64_t* pane_mcnt, unsigned long long* pane_mhash) {
    const DPlan& p = *pp;
    for (int64_t i = lo + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < hi; i += (int64_t)gridDim.x * kBlock) {
        if (has_acc && !acc[i]) continue;
        int64_t q = pane_of(g, ((const int64_t*)b.col[p.ts_col])[i]);
        if (q < qa || q > qb) continue;
        int64_t a = arrival ? arrival[i] : arrival_base + i;
        atomicAdd((unsigned long long*)&pane_mcnt[q % ring], 1ull);
        atomicAdd(&pane_mhash[q % ring], (unsigned long long)d_mix64((uint64_t)a));
    }
}
#endif

#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_win_members(const WinDesc* __restrict__ wins, int32_t ring, const int64_t* __restrict__ pane_mcnt,
                              const unsigned long long* __restrict__ pane_mhash, int64_t* wmc, unsigned long long* wmh) {
    if (threadIdx.x != 0) return;
    const WinDesc w = wins[blockIdx.x];
    int64_t c = 0;
    unsigned long long h = 0;
    for (int64_t q = w.q_first; q <= w.q_last; ++q) { c += pane_mcnt[q % ring]; h += pane_mhash[q % ring]; }
    wmc[w.idx] = c;
    wmh[w.idx] = h;
}
#endif

}  // namespace ek
