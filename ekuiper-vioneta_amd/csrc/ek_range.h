// ek_range.h — gfx950 kernels of the engine's RANGE mode.
//
// Range mode keeps the accepted events of the stream in a device-resident event buffer, ordered the way
// the reference's WindowOperator sees them (its `inputs` slice, window_op.go:576-739):
//   event time:  release order of WatermarkOp = stable ts order (ties in arrival order)  watermark_op.go:157-214
//   count window: arrival order                                                         window_op.go:390-418
// Every triggered window is then an index range [a, b) of that buffer, so windows of any type
// (sliding, session, count, and tumbling/hopping when an aggregate needs the raw values) are
// aggregated by the same partition/aggregate kernels as "virtual panes" (k_part MODE 2 + k_agg).
#pragma once
#include <algorithm>

#include "ek_kernels.h"

namespace ek {

#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_iota64(int64_t* __restrict__ out, int64_t base, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = base + i;
}
#endif

// The event-buffer append of a batch's columns in one launch (blockIdx.y = segment): 16-byte vector copies when source
// and destination share their alignment mod 16 (a head / tail of single elements around the vector body), element-sized
// copies otherwise; 4 vectors in flight per thread. Replaces one runtime copy per column (rocclr copyBuffer).
struct CopySeg {
    const unsigned char* src;
    unsigned char* dst;
    int64_t bytes;
    int32_t es;       // element size (1, 4 or 8): the granularity both ends are aligned to
    int32_t pad;
};
struct CopySegs {
    CopySeg s[2 * EK_MAX_COLUMNS + 1];
};
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(256) void k_eb_copy(CopySegs cs) {
    const CopySeg g = cs.s[blockIdx.y];
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nthr = (int64_t)gridDim.x * 256;
    const uintptr_t sa = (uintptr_t)g.src, da = (uintptr_t)g.dst;
    if (((sa ^ da) & 15) == 0) {
        int64_t head = (int64_t)((16 - (da & 15)) & 15);
        if (head > g.bytes) head = g.bytes;
        const int64_t nv = (g.bytes - head) >> 4;
        const int64_t tail0 = head + (nv << 4);
        for (int64_t i = tid; i < head; i += nthr) g.dst[i] = g.src[i];
        const uint4* vs = (const uint4*)(g.src + head);
        uint4* vd = (uint4*)(g.dst + head);
        int64_t v = tid;
        for (; v + 3 * nthr < nv; v += 4 * nthr) {
            const uint4 a = vs[v], b = vs[v + nthr], c = vs[v + 2 * nthr], d = vs[v + 3 * nthr];
            vd[v] = a;
            vd[v + nthr] = b;
            vd[v + 2 * nthr] = c;
            vd[v + 3 * nthr] = d;
        }
        for (; v < nv; v += nthr) vd[v] = vs[v];
        for (int64_t i = tail0 + tid; i < g.bytes; i += nthr) g.dst[i] = g.src[i];
        return;
    }
    if (g.es == 8) {
        const int64_t n = g.bytes >> 3;
        for (int64_t i = tid; i < n; i += nthr) ((int64_t*)g.dst)[i] = ((const int64_t*)g.src)[i];
    } else if (g.es == 4) {
        const int64_t n = g.bytes >> 2;
        for (int64_t i = tid; i < n; i += nthr) ((uint32_t*)g.dst)[i] = ((const uint32_t*)g.src)[i];
    } else {
        for (int64_t i = tid; i < g.bytes; i += nthr) g.dst[i] = g.src[i];
    }
}
#endif

// Inclusive running max of ts in arrival order (the stream max M_j of watermark_op.go:217-225 after
// event j), seeded per kAccChunk chunk with the exclusive prefix max from k_chunk_max + k_scan_max.
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_runmax(const int64_t* __restrict__ ts, int64_t n, const int64_t* excl,
                                                   int64_t* __restrict__ out) {
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
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) {
        const int64_t i = base + k;
        run = max(run, v[k]);
        if (i < n) out[i] = run;
    }
}
#endif

// first j in [lo, hi) with a[j] >= x (hi if none); a non-decreasing
__device__ __forceinline__ int64_t lb_i64(const int64_t* a, int64_t lo, int64_t hi, int64_t x) {
    while (lo < hi) { int64_t m = (lo + hi) >> 1; if (a[m] < x) lo = m + 1; else hi = m; }
    return lo;
}
// first j in [lo, hi) with a[j] > x
__device__ __forceinline__ int64_t ub_i64(const int64_t* a, int64_t lo, int64_t hi, int64_t x) {
    while (lo < hi) { int64_t m = (lo + hi) >> 1; if (a[m] <= x) lo = m + 1; else hi = m; }
    return lo;
}

// Searches over a buffer's arrival column; barr == nullptr: the column is implicit, arrival(i) = arr0 + i (a buffer
// filled only by in-order appends keeps no arrival column at all)
__device__ __forceinline__ int64_t arr_at(const int64_t* barr, int64_t arr0, int64_t i) { return barr ? barr[i] : arr0 + i; }
__device__ __forceinline__ int64_t arr_lb(const int64_t* barr, int64_t arr0, int64_t lo, int64_t hi, int64_t x) {
    if (barr) return lb_i64(barr, lo, hi, x);
    return lo < hi ? min(hi, max(lo, x - arr0)) : lo;
}
__device__ __forceinline__ int64_t arr_ub(const int64_t* barr, int64_t arr0, int64_t lo, int64_t hi, int64_t x) {
    if (barr) return ub_i64(barr, lo, hi, x);
    return lo < hi ? min(hi, max(lo, x - arr0 + 1)) : lo;
}

// Galloping searches from lo (the answer is usually a few rows away: a ts-sorted batch releases an event at its own
// arrival or at the end of its equal-ts run): O(log distance) probes near lo instead of a binary search over the
// whole remaining batch (whose first probes miss every cache). Same results as lb_i64 / ub_i64.
__device__ __forceinline__ int64_t gallop_lb(const int64_t* a, int64_t lo, int64_t hi, int64_t x) {
    if (lo >= hi || a[lo] >= x) return lo;
    int64_t prev = lo, step = 1;
    while (lo + step < hi && a[lo + step] < x) { prev = lo + step; step <<= 1; }
    return lb_i64(a, prev + 1, min(hi, lo + step), x);
}
__device__ __forceinline__ int64_t gallop_ub(const int64_t* a, int64_t lo, int64_t hi, int64_t x) {
    if (lo >= hi || a[lo] > x) return lo;
    int64_t prev = lo, step = 1;
    while (lo + step < hi && a[lo + step] <= x) { prev = lo + step; step <<= 1; }
    return ub_i64(a, prev + 1, min(hi, lo + step), x);
}

// Release step of buffered events [i0, i1): the arrival index of the watermark advance that released the
// event (watermark_op.go:157-214: released at the first advance W_j > W_{j-1} at or after its arrival with
// W_j >= ts). runmax[0..nb) = batch running max (arrival arr_base + j), prevmax = stream max before the
// batch (INT64_MIN if none), W_j = runmax[j] - late_tol. Events not released in this batch get INT64_MAX.
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_release_step(const int64_t* __restrict__ bts, const int64_t* __restrict__ barr, int64_t arr0, int64_t i0,
                               int64_t i1, const int64_t* __restrict__ runmax, int64_t nb, int64_t arr_base,
                               int64_t prevmax, int64_t late_tol, int64_t* __restrict__ brel) {
    for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = bts[i] + late_tol;
        const int64_t ls = max((int64_t)0, arr_at(barr, arr0, i) - arr_base);
        int64_t r = INT64_MAX;
        if (ls < nb) {
            const int64_t j0 = gallop_lb(runmax, ls, nb, x);
            if (j0 < nb) {
                const int64_t prev = j0 > 0 ? runmax[j0 - 1] : prevmax;
                if (runmax[j0] > prev) r = arr_base + j0;
                else {
                    const int64_t j1 = gallop_ub(runmax, j0 + 1, nb, runmax[j0]);
                    if (j1 < nb) r = arr_base + j1;
                }
            }
        }
        brel[i] = r;
    }
}
#endif

// Released prefix of the buffer after a batch (single thread): events with ts < W, plus those with
// ts == W that arrived no later than the step sW at which the watermark reached W.
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_rel_end(const int64_t* __restrict__ bts, const int64_t* __restrict__ barr, int64_t arr0, int64_t n,
                          int64_t W, int64_t sW, int64_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int64_t p = lb_i64(bts, 0, n, W);
    const int64_t q = ub_i64(bts, p, n, W);
    out[0] = arr_ub(barr, arr0, p, q, sW);   // arrivals are increasing inside one ts run
}
#endif

// k_first_ge (when the batch moved the max: sW = arrival of that step) and k_rel_end at (W, sW) in one launch, one
// host round trip: out[0] = sW, out[1] = the released end of the buffer (n_buf == 0: not computed)
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_rel_bounds(const int64_t* __restrict__ runmax, int64_t nb, int64_t max_ts, int first, int64_t arr_base,
                             int64_t sW, const int64_t* __restrict__ bts, const int64_t* __restrict__ barr, int64_t arr0,
                             int64_t n_buf, int64_t W, int64_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (first) sW = arr_base + lb_i64(runmax, 0, nb, max_ts);
    out[0] = sW;
    if (n_buf > 0) {
        const int64_t p = lb_i64(bts, 0, n_buf, W);
        const int64_t q = ub_i64(bts, p, n_buf, W);
        out[1] = arr_ub(barr, arr0, p, q, sW);
    }
}
#endif

// first j in [0, n) with runmax[j] >= x (n if none) — the step at which the stream max reached x
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_first_ge(const int64_t* __restrict__ a, int64_t n, int64_t x, int64_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    out[0] = lb_i64(a, 0, n, x);
}
#endif

// Released prefix of the buffer at the WatermarkTuple that fires each window end (hopping windows): the first step j
// of the batch whose watermark runmax[j] - late_tol reaches the end, then the k_rel_end bound at (W_j, arrival j).
// handleInputs (window_op.go:605-655) drops every input present at that tuple when the window finds no member.
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_fire_prefix(const int64_t* __restrict__ runmax, int64_t nb, int64_t arr_base, int64_t late_tol,
                              const int64_t* __restrict__ bts, const int64_t* __restrict__ barr, int64_t arr0, int64_t n,
                              const int64_t* __restrict__ ends, int nq, int64_t* __restrict__ out) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nq) return;
    const int64_t j = lb_i64(runmax, 0, nb, ends[w] + late_tol);
    if (j >= nb) { out[w] = n; return; }   // not reached inside this batch (cannot happen for a fired window)
    const int64_t W = runmax[j] - late_tol;
    const int64_t p = lb_i64(bts, 0, n, W);
    const int64_t q = ub_i64(bts, p, n, W);
    out[w] = arr_ub(barr, arr0, p, q, arr_base + j);
}
#endif

// Derived columns (expression arguments of aggregates, GroupedTuples.AggregateEval row.go:712-718): per row the
// valuer's arithmetic over the batch's own columns (eval_prog); nil -> validity 0. The programs cannot error (host
// lowering: / and % only by non-zero constants).
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_derive(DPlan* __restrict__ pp, DBatch b, int64_t n, int64_t* __restrict__ out0, int64_t* __restrict__ out1,
                         int64_t* __restrict__ out2, int64_t* __restrict__ out3, uint8_t* __restrict__ v0, uint8_t* __restrict__ v1,
                         uint8_t* __restrict__ v2, uint8_t* __restrict__ v3) {
    const DPlan& p = *pp;
    int64_t* outs[4] = {out0, out1, out2, out3};
    uint8_t* vals[4] = {v0, v1, v2, v3};
    const int nd = p.n_columns - p.n_user_cols;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int d = 0; d < EK_MAX_DERIVED; ++d) {
            if (d >= nd) break;
            const Val v = eval_prog(p.derived_prog[d], p.n_derived_prog[d], p, &b, i, NoAggs{});
            const bool ok = v.tag == V_I64 || v.tag == V_F64;
            outs[d][i] = !ok ? 0 : (v.tag == V_F64 ? __double_as_longlong(v.f) : v.i);
            if (vals[d]) vals[d][i] = ok ? 1 : 0;
        }
    }
}
#endif

// SLIDINGWINDOW trigger flags over buffer rows [i0, i1): 1 when OVER (WHEN cond) holds
// (window_op.go:741-768: nil, error or non-bool -> no trigger); every row triggers without OVER.
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_trigger_flags(DPlan* __restrict__ pp, DBatch b, int64_t i0, int64_t i1, uint8_t* __restrict__ flags) {
    const DPlan& p = *pp;
    for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += (int64_t)gridDim.x * blockDim.x) {
        uint8_t f = 1;
        if (p.n_trigger > 0) {
            Val v = eval_prog(p.trigger_prog, p.n_trigger, p, &b, i, NoAggs{});
            f = (v.tag == V_BOOL && v.i) ? 1 : 0;
        }
        flags[i - i0] = f;
    }
}
#endif

// STATEWINDOW conditions of rows [i0, i1) of the buffer (isMatchCondition, window_v2_op.go:212-238: nil, an
// error or a non-bool is false): bit 0 = begin condition true, bit 1 = emit condition true
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_state_flags(DPlan* __restrict__ pp, DBatch b, int64_t i0, int64_t i1, uint8_t* __restrict__ flags) {
    const DPlan& p = *pp;
    for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += (int64_t)gridDim.x * blockDim.x) {
        uint8_t f = 0;
        if (p.n_begin > 0) {
            const Val v = eval_prog(p.begin_prog, p.n_begin, p, &b, i, NoAggs{});
            f |= (v.tag == V_BOOL && v.i) ? 1 : 0;
        } else {
            f |= 1;
        }
        if (p.n_emit > 0) {
            const Val v = eval_prog(p.emit_prog, p.n_emit, p, &b, i, NoAggs{});
            f |= (v.tag == V_BOOL && v.i) ? 2 : 0;
        } else {
            f |= 2;
        }
        flags[i - i0] = f;
    }
}
#endif

// Watermarks around the release step r of each listed row (incremental event-time windows): w_step = the
// watermark whose WatermarkTuple follows the row (emission), w_prev = the one before its step (the last gc).
// runmax[0..nb) = batch running max (arrival arr_base + j); prevmax = stream max before the batch.
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_step_wm(const int64_t* __restrict__ rel, int64_t n, const int64_t* __restrict__ runmax, int64_t nb,
                          int64_t arr_base, int64_t prevmax, int64_t late_tol, int64_t* __restrict__ w_step,
                          int64_t* __restrict__ w_prev) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = rel[k] - arr_base;
        w_step[k] = (j >= 0 && j < nb) ? runmax[j] - late_tol : INT64_MIN;
        const int64_t pm = (j - 1 >= 0 && j - 1 < nb) ? runmax[j - 1] : prevmax;
        w_prev[k] = pm == INT64_MIN ? INT64_MIN : pm - late_tol;
    }
}
#endif

// gather of the flag bytes at compacted positions (positions are absolute: base_idx + i)
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_gather_flags(const int64_t* __restrict__ pos, int64_t n, int64_t base_idx, const uint8_t* __restrict__ flags,
                               uint8_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = flags[pos[k] - base_idx];
}
#endif

// FilterOp over a window-less batch (filter_operator.go:36-90): 1 keep; nil/false drop; error drop + count
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_filter_flags(DPlan* __restrict__ pp, DBatch b, uint8_t* __restrict__ flags, unsigned long long* n_err) {
    const DPlan& p = *pp;
    unsigned long long e = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += (int64_t)gridDim.x * blockDim.x) {
        const int w = p.n_where > 0 ? where_decide_slow(p, b, i) : 1;
        flags[i] = w > 0 ? 1 : 0;
        e += w < 0;
    }
    for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
    if ((threadIdx.x & 63) == 0 && e) atomicAdd(n_err, e);
}
#endif

// rows sel[0..ns) of one column (4- or 8-byte elements) and of its validity bytes, compacted (pushed-down WHERE)
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_compact_col(const int64_t* __restrict__ sel, int64_t ns, const void* __restrict__ src, int es,
                              const uint8_t* __restrict__ vsrc, void* __restrict__ dst, uint8_t* __restrict__ vdst) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ns; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = sel[k];
        if (es == 4) ((uint32_t*)dst)[k] = ((const uint32_t*)src)[i];
        else ((int64_t*)dst)[k] = ((const int64_t*)src)[i];
        if (vdst) vdst[k] = vsrc[i];
    }
}
#endif
// out[k] = base + idx[k]
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_offset_idx(const int64_t* __restrict__ idx, int64_t n, int64_t base, int64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) out[k] = base + idx[k];
}
#endif

// SELECT * rows of the selected events: key = batch row, value c = column c (tag by type / validity)
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_filter_emit(DPlan* __restrict__ pp, DBatch b, const int64_t* __restrict__ sel, int64_t ns, int64_t out_base,
                              int32_t widx, Results res) {
    const DPlan& p = *pp;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ns; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = sel[k], o = out_base + k;
        res.key[o] = (uint32_t)i;
        for (int c = 0; c < p.n_columns; ++c) {
            const bool ok = col_valid(b, c, i);
            const int t = p.col_type[c];
            res.val[c][o] = !ok ? 0 : (t == EK_COL_U32 ? (int64_t)((const uint32_t*)b.col[c])[i] : ((const int64_t*)b.col[c])[i]);
            res.tag[c][o] = !ok ? EK_TAG_NULL : (t == EK_COL_F64 ? EK_TAG_F64 : t == EK_COL_BOOL ? EK_TAG_BOOL : EK_TAG_I64);
        }
        if (k == 0) res.win_cnt[widx] = ns;
    }
}
#endif

// The window's FILTER (WHERE ...) op between WatermarkOp and the window (planner.go:388-392), event time: acc_out[i] =
// the row was accepted (acc_in[i], or i >= start when acc_in is null) and its condition (the pre plan's where_prog) is
// true; nil / false drop it, an error drops it and is counted (filter_operator.go:41-57). st: n_accepted and
// min_accepted of the kept rows, n_dropped = the evaluation errors (all three reset by the caller).
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_filter_mask(DPlan* __restrict__ pp, DBatch b, const uint8_t* __restrict__ acc_in,
                                                        int64_t start, uint8_t* __restrict__ acc_out, BatchStats* st) {
    const DPlan& p = *pp;
    const int64_t* ts = (const int64_t*)b.col[p.ts_col];
    unsigned long long c = 0, e = 0;
    int64_t m = INT64_MAX;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += (int64_t)gridDim.x * blockDim.x) {
        bool keep = acc_in ? acc_in[i] != 0 : i >= start;
        if (keep) {
            const int w = where_decide_slow(p, b, i);
            e += w < 0;
            keep = w > 0;
        }
        acc_out[i] = keep ? 1 : 0;
        if (keep) { c++; m = min(m, ts[i]); }
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, 64);
        e += __shfl_xor(e, o, 64);
        m = min(m, (int64_t)__shfl_xor(m, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        if (c) { atomicAdd((unsigned long long*)&st->n_accepted, c); atomicMin((long long*)&st->min_accepted, (long long)m); }
        if (e) atomicAdd((unsigned long long*)&st->n_dropped, e);
    }
}
#endif

// Per-block counts of set flags (stable compaction, pass 1)
constexpr int kCompactTile = 4096;
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_flag_count(const uint8_t* __restrict__ flags, int64_t n, int64_t* cnt) {
    const int64_t base = (int64_t)blockIdx.x * kCompactTile;
    int64_t c = 0;
    for (int k = threadIdx.x; k < kCompactTile; k += kBlock) {
        const int64_t i = base + k;
        if (i < n && flags[i]) c++;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ int64_t s[kBlock / 64];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
#endif

// exclusive scan of nb block counts (single workgroup); cnt[nb] = total
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(1024) void k_scan_counts(int64_t* cnt, int nb) {
    __shared__ int64_t part[1024];
    const int per = (nb + 1023) / 1024;
    const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    int64_t s = 0;
    for (int k = b0; k < b1; ++k) s += cnt[k];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = 0;
        for (int t = 0; t < 1024; ++t) { int64_t x = part[t]; part[t] = run; run += x; }
        cnt[nb] = run;
    }
    __syncthreads();
    int64_t run = part[threadIdx.x];
    for (int k = b0; k < b1; ++k) { int64_t x = cnt[k]; cnt[k] = run; run += x; }
}
#endif

// pass 2: write base + i of every set flag, in order (one wave-ordered sweep per block)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_flag_write(const uint8_t* __restrict__ flags, int64_t n, const int64_t* cnt,
                                                       int64_t base_idx, int64_t* __restrict__ out) {
    const int64_t base = (int64_t)blockIdx.x * kCompactTile;
    __shared__ uint32_t wsum[kBlock / 64];
    int64_t run = cnt[blockIdx.x];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k0 = 0; k0 < kCompactTile; k0 += kBlock) {
        const int64_t i = base + k0 + threadIdx.x;
        const bool f = i < n && flags[i];
        const unsigned long long m = __ballot(f);
        if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t wb = 0, tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) { if (w < wv) wb += wsum[w]; tot += wsum[w]; }
        if (f) out[run + wb + __popcll(m & ((1ull << lane) - 1ull))] = base_idx + i;
        run += tot;
        __syncthreads();
    }
}
#endif

// Window range descriptor (host -> device): content = [max(floor, lo(lo_ts)), hi(...)) of the buffer.
enum : int32_t { RB_LB = 0, RB_SLIDE = 1, RB_FIXED = 2, RB_UPTO = 3, RB_CAP = 4, RB_ARR = 5 };
struct RangeQ {
    int64_t lo_ts;      // lower bound ts: content starts at the first row with ts >= lo_ts (INT64_MIN: from floor)
    int64_t hi_ts;      // RB_LB: first row with ts >= hi_ts; RB_SLIDE: ts <= hi_ts and release step <= rstep
                        // RB_ARR (shard count windows): rows with global arrival in [lo_ts, hi_ts)
    int64_t pos;        // RB_SLIDE: buffer index of the trigger event; RB_FIXED: a (index)
    int64_t rstep;      // RB_SLIDE: release step of the trigger event; RB_FIXED: b (index)
    int64_t floor;      // smallest buffer index a window may start at
    int32_t kind;
    int32_t pad;
};

#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_window_ranges(const int64_t* __restrict__ bts, const int64_t* __restrict__ brel,
                                const int64_t* __restrict__ barr, int64_t arr0, int64_t n_rel, const RangeQ* __restrict__ q,
                                int nq, int64_t* __restrict__ ab) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nq) return;
    const RangeQ d = q[w];
    int64_t a, b;
    if (d.kind == RB_ARR) {
        a = max(d.floor, arr_lb(barr, arr0, d.floor, n_rel, d.lo_ts));
        b = arr_lb(barr, arr0, a, n_rel, d.hi_ts);
    } else if (d.kind == RB_FIXED) {
        a = d.pos;
        b = d.rstep;
    } else if (d.kind == RB_CAP) {
        // [pos, min(rstep, first row with ts >= hi_ts)): an incremental window's rows from its opening row
        a = d.pos;
        b = min(d.rstep, lb_i64(bts, a, max(a, d.rstep), d.hi_ts));
    } else {
        a = d.lo_ts == INT64_MIN ? d.floor : max(d.floor, lb_i64(bts, d.floor, n_rel, d.lo_ts));
        if (d.kind == RB_LB) {
            b = lb_i64(bts, a, n_rel, d.hi_ts);
        } else if (d.kind == RB_UPTO) {
            b = d.pos + 1;   // v2 sliding: the rows the scanner holds when the trigger row is added (window_v2_event_op.go:78-96)
        } else {
            // sliding (window_op.go:605-655 with ts <= t): rows after the trigger with the same ts that were
            // released at the same watermark step belong to the window; later ones do not
            int64_t lo = d.pos + 1, hi = n_rel;
            while (lo < hi) {
                int64_t m = (lo + hi) >> 1;
                if (bts[m] > d.hi_ts || brel[m] > d.rstep) hi = m; else lo = m + 1;
            }
            b = lo;
        }
        if (b < a) b = a;
    }
    ab[2 * w] = a;
    ab[2 * w + 1] = b;
}
#endif

// debug_membership for range windows: count and Σ ek_mix64(arrival) over [a, b) (one block per window)
// (barr == nullptr: row i's arrival is arr_base + i — windows read straight from a batch in arrival order)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_range_members(const int64_t* __restrict__ barr, const int64_t* __restrict__ ab,
                                                          const int32_t* __restrict__ slot, int64_t* wmc,
                                                          unsigned long long* wmh, int64_t arr_base) {
    const int64_t a = ab[2 * blockIdx.x], b = ab[2 * blockIdx.x + 1];
    unsigned long long h = 0;
    for (int64_t i = a + threadIdx.x; i < b; i += kBlock) h += d_mix64(barr ? (uint64_t)barr[i] : (uint64_t)(arr_base + i));
    for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
    __shared__ unsigned long long s[kBlock / 64];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0 && slot[blockIdx.x] >= 0) {   // slot -1: window not reported
        wmc[slot[blockIdx.x]] = b - a;
        wmh[slot[blockIdx.x]] = s[0] + s[1] + s[2] + s[3];
    }
}
#endif

// Gather rows of the merge input (sources: [0, ntail) = saved buffer tail, [ntail, ..) = batch rows
// listed in bidx) into the destination column in sorted order (perm from the radix sort).
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_gather8(const int64_t* __restrict__ perm, int64_t n, int64_t ntail, const int64_t* __restrict__ tail,
                          const int64_t* __restrict__ batch, const int64_t* __restrict__ bidx, int64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = perm[k];
        out[k] = s < ntail ? tail[s] : batch[bidx[s - ntail]];
    }
}
#endif
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_gather4(const int64_t* __restrict__ perm, int64_t n, int64_t ntail, const uint32_t* __restrict__ tail,
                          const uint32_t* __restrict__ batch, const int64_t* __restrict__ bidx, uint32_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = perm[k];
        out[k] = s < ntail ? tail[s] : batch[bidx[s - ntail]];
    }
}
#endif
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_gather1(const int64_t* __restrict__ perm, int64_t n, int64_t ntail, const uint8_t* __restrict__ tail,
                          const uint8_t* __restrict__ batch, const int64_t* __restrict__ bidx, uint8_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = perm[k];
        out[k] = s < ntail ? (tail ? tail[s] : (uint8_t)1) : (batch ? batch[bidx[s - ntail]] : (uint8_t)1);
    }
}
#endif
// merge keys: ts of the saved tail rows and of the batch rows listed in bidx, and source ids 0..n-1
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_merge_keys(const int64_t* __restrict__ tail_ts, int64_t ntail, const int64_t* __restrict__ bts,
                             const int64_t* __restrict__ bidx, int64_t nb, int64_t tmin, uint64_t* __restrict__ keys,
                             int64_t* __restrict__ src) {
    const int64_t n = ntail + nb;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = k < ntail ? tail_ts[k] : bts[bidx[k - ntail]];
        keys[k] = (uint64_t)(t - tmin);
        src[k] = k;
    }
}
#endif
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_arrivals_of(const int64_t* __restrict__ bidx, int64_t nb, int64_t arr_base, int64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nb; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = arr_base + bidx[k];
}
#endif

// ---------------------------------------------------------------- first-row select fields
// A non-aggregate select field takes the column's value in the group's FIRST row (row.go:720-726: GroupedTuples
// .Content[0]; the group keeps its rows in window order). Every aggregation path folds the hidden position column
// (value = the row's event-buffer index, i.e. the window order) with MIN, so an emitted EK_AGG_FIRST slot holds the
// first row's position; one block per window fired by this push then swaps in the source column's value there
// (nil when that value is null).
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_first_fetch(DPlan* __restrict__ pp, DBatch b, const int32_t* __restrict__ wslot,
                              const int64_t* __restrict__ wbase, Results res) {
    const DPlan& p = *pp;
    const int32_t slot = wslot[blockIdx.x];
    const int64_t base = wbase[blockIdx.x], cnt = res.win_cnt[slot];
    for (int64_t r = base + threadIdx.x; r < base + cnt; r += blockDim.x) {
        for (int q = 0; q < p.n_aggs; ++q) {
            if (p.agg_fn[q] != EK_AGG_FIRST || res.tag[q][r] != EK_TAG_I64) continue;
            const int64_t pos = res.val[q][r];
            const int c = p.first_col[q];
            if (!col_valid(b, c, pos)) {
                res.tag[q][r] = EK_TAG_NULL;
                res.val[q][r] = 0;
            } else if (p.col_type[c] == EK_COL_F64) {
                res.tag[q][r] = EK_TAG_F64;
                res.val[q][r] = ((const int64_t*)b.col[c])[pos];
            } else {
                res.val[q][r] = col_i64(p, b, c, pos);
            }
        }
        // median over a nullable f64 column whose group starts with a nil (arg0[0] is not a number): the window's
        // aggregate error, at the smallest failing order-statistic slot; a WHERE error already replaced the window
        for (int q = 0; q < p.n_aggs; ++q) {
            const int h = p.med_first[q];
            if (h < 0 || res.tag[h][r] != EK_TAG_NULL || (res.win_err[slot] & EK_WIN_WHERE_ERROR)) continue;
            atomicOr(&res.win_err[slot], EK_WIN_AGG_ERROR);
            if (res.aslot) atomicMax(&res.aslot[slot], kMaxSortAggs - p.agg_sidx[q]);
        }
    }
}
#endif

// ---------------------------------------------------------------- WHERE above an incremental window
// FilterPlan stays above IncWindowPlan (planner.go:702-708; IncWindowPlan.PushDownPredicate keeps the predicate,
// incAggPlan.go:76-78): FilterOp.Apply runs over the emitted collection (filter_operator.go:59-90), whose rows are the
// groups' LAST rows with the inc_* fields set (window_inc_agg_op.go:443-457), then HavingOp over what is left. The
// aggregation folds a hidden MAX over the event-buffer position column into result slot `hidden` (the last row), with
// neither WHERE nor HAVING; one block per fired window then evaluates WHERE at each row's last row: an error or a
// non-bool replaces the window (its witness: the failing row with the smallest key, as the host's text re-evaluation
// expects), nil / false drops the row; HAVING (over the result values) decides the rest, and the kept rows are
// compacted in place, tile by tile (a tile is read whole before any of it is written, and its writes land at or
// below its own start).
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(256) void k_inc_where(DPlan* __restrict__ pp, DBatch b, const int32_t* __restrict__ wslot,
                                                   const int64_t* __restrict__ wbase, int hidden, int n_res, Results res) {
    const DPlan& p = *pp;
    const int32_t slot = wslot[blockIdx.x];
    const int64_t base = wbase[blockIdx.x], cnt = res.win_cnt[slot];
    __shared__ int s_err;
    __shared__ uint32_t wsum[4];
    __shared__ int64_t s_out;
    if (threadIdx.x == 0) { s_err = 0; s_out = 0; }
    __syncthreads();
    // WHERE errors first: any one replaces the whole window (FilterOp returns the error, no HAVING runs)
    for (int64_t r = base + threadIdx.x; r < base + cnt; r += blockDim.x) {
        const int64_t pos = res.val[hidden][r];
        if (where_decide_slow(p, b, pos) < 0) {
            s_err = 1;
            if (res.wwit) wit_where_row(&res.wwit[2 * slot], (unsigned long long)res.key[r], 0ull, p, b, pos);
        }
    }
    __syncthreads();
    if (s_err) {
        if (threadIdx.x == 0) { atomicOr(&res.win_err[slot], EK_WIN_WHERE_ERROR); res.win_cnt[slot] = 0; }
        return;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int64_t t0 = base; t0 < base + cnt; t0 += blockDim.x) {
        const int64_t r = t0 + threadIdx.x;
        const bool in = r < base + cnt;
        uint32_t key = 0;
        int64_t v[EK_MAX_AGGS];
        uint8_t tg[EK_MAX_AGGS];
#pragma unroll
        for (int q = 0; q < EK_MAX_AGGS; ++q) { v[q] = 0; tg[q] = EK_TAG_NULL; }
        bool keep = false;
        if (in) {
            key = res.key[r];
#pragma unroll
            for (int q = 0; q < EK_MAX_AGGS; ++q)
                if (q < n_res) { v[q] = res.val[q][r]; tg[q] = res.tag[q][r]; }
            keep = where_decide_slow(p, b, v[hidden]) > 0;
            if (keep && p.n_having > 0) {
                auto aggf = [&](int k) {
                    const uint8_t t = sel(tg, k);
                    const int64_t x = sel(v, k);
                    return t == EK_TAG_NULL ? Val{V_NULL, 0, 0.0} : t == EK_TAG_I64 ? Val{V_I64, x, 0.0} : Val{V_F64, 0, __longlong_as_double(x)};
                };
                const Val h = eval_prog(p.having_prog, p.n_having, p, nullptr, 0, aggf);
                if (h.tag != V_BOOL) {
                    atomicOr(&res.win_err[slot], EK_WIN_HAVING_ERROR);
                    if (res.wwit) wit_having(&res.wwit[2 * slot + 1], key, p, aggf);
                    keep = false;
                } else {
                    keep = h.i != 0;
                }
            }
        }
        const unsigned long long m = __ballot(keep);
        if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { if (w < wv) before += wsum[w]; total += wsum[w]; }
        const int64_t out = s_out;
        if (keep) {
            const int64_t o = base + out + before + __popcll(m & ((1ull << lane) - 1ull));
            res.key[o] = key;
#pragma unroll
            for (int q = 0; q < EK_MAX_AGGS; ++q)
                if (q < n_res) { res.val[q][o] = v[q]; res.tag[q][o] = tg[q]; }
        }
        __syncthreads();
        if (threadIdx.x == 0) s_out = out + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) res.win_cnt[slot] = s_out;
}
#endif

// ---------------------------------------------------------------- small range windows: one wave64 per window
// For a window of at most kSmallWin rows (COUNTWINDOW(1000), state windows, short sliding windows) the pane/bucket
// partition of k_part + k_agg costs a workgroup per (window, key bucket) that finds a handful of rows. Here ONE WAVE
// owns a whole window at a time (a 64-thread workgroup: its barriers are the wave's own LDS waits) and persistent
// waves walk the launch's windows, loading the next window's keys while grouping the current one. Per window:
//   WHERE (an error replaces the window's output, filter_operator.go:63-77);
//   a duplicate filter: every row sets its key's hash bit in an LDS bitmap of >= 32 bits per row and marks the bit
//     in a second map when it was already set — a row whose bit no other row set is a group of its own (count 1),
//     emitted straight from its lane (HAVING count(*) > 1 drops it without a fold);
//   the other rows (candidates: real duplicates plus the few hash collisions) are grouped exactly through an LDS hash
//     table sized by their count, with a slot scan (groups HAVING over count(*) drops are never placed) and one
//     lane per group;
//   every group folds its rows in window order (aggregate_operator.go:34-82; exact two-pass M2), applies HAVING and
//   is emitted by wave ballot compaction; the window's row count is stored once (no atomics on the counter).
// LDS per wave: the larger of the two bitmaps (8 KB for n = 1000) and the candidates' hash table (6 B per slot,
// 2n..4n slots, + 2 B per row + 4 B per group), sized by the launch's largest window.
constexpr int kSmallWin = 2048;
constexpr int kSwLanes = 64;                    // threads per k_small_win workgroup (one wave)
constexpr int kSwRows = kSmallWin / kSwLanes;   // rows per lane, at most (RM: 16 for windows up to 1024 rows, else 32)
__host__ __device__ inline int sw_slots(int n) { int h = 128; while (h < 2 * n) h <<= 1; return h; }
__host__ __device__ inline int sw_bits(int n) { int b = 2048; while (b < 32 * n) b <<= 1; return b; }
inline size_t sw_lds_bytes(int max_n) {
    const size_t tab = (size_t)sw_slots(max_n) * 6 + (((size_t)max_n * 2 + 3) & ~(size_t)3) + (size_t)max_n * 4;
    return std::max(tab, (size_t)sw_bits(max_n) / 4);
}
// A launch whose candidate tables are capped at kSwCandCap rows: the LDS is about the bitmaps alone (8 KB at 1 000
// rows), so 4 waves share a SIMD; a window with more candidate rows is left to a second launch with the full tables
// (its index in the redo list). Typical windows over a large key space hold a handful of candidates.
constexpr int kSwCandCap = 256;
inline size_t sw_lds_bytes_capped(int max_n) {
    const int c = std::min(max_n, kSwCandCap);
    const size_t tab = (size_t)sw_slots(c) * 6 + (((size_t)c * 2 + 3) & ~(size_t)3) + (size_t)c * 4;
    return std::max(tab, (size_t)sw_bits(max_n) / 4);
}
static_assert(kSmallWin + 1 <= kHStarTab, "the count-decision table covers every small window");

// a window group's rows (indices into the window, distinct) into ascending order, so the group folds its values in
// the window's row order: the f64 sums are the reference's sequential ones, whatever order the LDS atomics of the
// scatter placed them in. Insertion sort for short groups, heap sort (in place, O(n log n)) for long ones.
__device__ inline void sw_sort_rows(uint16_t* a, int n) {
    if (n <= 24) {
        for (int i = 1; i < n; ++i) {
            const uint16_t x = a[i];
            int j = i - 1;
            while (j >= 0 && a[j] > x) { a[j + 1] = a[j]; --j; }
            a[j + 1] = x;
        }
        return;
    }
    auto sift = [&](int r, int end) {
        const uint16_t x = a[r];
        while (2 * r + 1 < end) {
            int c = 2 * r + 1;
            if (c + 1 < end && a[c + 1] > a[c]) ++c;
            if (a[c] <= x) break;
            a[r] = a[c];
            r = c;
        }
        a[r] = x;
    };
    for (int r = n / 2 - 1; r >= 0; --r) sift(r, n);
    for (int end = n - 1; end > 0; --end) {
        const uint16_t x = a[0];
        a[0] = a[end];
        a[end] = x;
        sift(0, end);
    }
}

__device__ __forceinline__ uint32_t sw_hash(uint32_t k) {
    k ^= k >> 16; k *= 0x7feb352du; k ^= k >> 15; k *= 0x846ca68bu; k ^= k >> 16;
    return k;
}

// Windows laid out arithmetically (consecutive COUNTWINDOW blocks of one batch): window w = rows [a0 + w len, + len),
// result slot slot0 + w, result region ob0 + w rowcap — no per-window lists to upload.
constexpr int kSwFoldRegs = 4;   // k_small_win: groups of up to this many rows fold from registers
struct SwArith {
    int64_t a0, ob0, rowcap;
    int32_t len, slot0;
};
// k_small_win's redo list: cap > 0 (the capped launch) appends the work items with more candidate rows to out[] via
// *cnt; in != nullptr (the redo launch) runs in[0 .. *cnt)
struct SwRedo {
    int32_t cap;
    int32_t* out;
    int32_t* cnt;
    const int32_t* in;
};

// HAVING decision (1 keep, 0 drop, -1 non-bool: a window error) of a group's partial, without side effects
template <int NVC>
__device__ __forceinline__ int having_decide(const DPlan& p, const Part<NVC>& s) {
    if (p.n_having <= 0) return 1;
    const Val h = eval_prog(p.having_prog, p.n_having, p, nullptr, 0, [&](int k) { return agg_value(p, s, k); });
    if (h.tag != V_BOOL) return -1;
    return h.i != 0 ? 1 : 0;
}
// HAVING over count(*) alone, decided from a group's row count c (the decisions for 1 and 2 rows are cached; HS: all
// of them, from the plan's table)
template <int NVC, bool HS>
__device__ __forceinline__ int having_star_decide(const DPlan& p, int c, int h1, int h2) {
    if (c == 1) return h1;
    if (c == 2) return h2;
    if constexpr (HS) {
        return p.hstar_tab[c < kHStarTab ? c : kHStarTab - 1];
    } else {
        Part<NVC> cp{};
        cp.cnt = c;
        return having_decide(p, cp);
    }
}
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_hstar_tab(DPlan* __restrict__ pp) {
    for (int c = threadIdx.x; c < kHStarTab; c += blockDim.x) {
        Part<1> cp{};
        cp.cnt = c;
        pp->hstar_tab[c] = (int8_t)having_decide(*pp, cp);
    }
}
#endif

// One small window per call: rows [a, a + n) of b, keys already in key[] (lane + 64 j), result region out, slot widx.
// Returns the rows emitted (-1: a WHERE error replaced the window's output; -2: more than cand_cap candidate rows —
// nothing was written, the window goes to the redo launch). HS: HAVING is absent or reads count(*) alone (decided
// from the plan's table; no interpreter in the kernel).
template <int NVC, bool WHERE, int RM, bool HS>
__device__ __forceinline__ int64_t sw_window(const DPlan& p, const DBatch& b, const uint32_t* kcol, int64_t a, int n,
                                             int32_t widx, int64_t out, const uint32_t (&key)[RM], Results& res,
                                             uint32_t* s_dyn, int h1, int h2, int cand_cap) {
    const int lane = threadIdx.x;
    uint32_t live = 0;   // bit j: row lane + 64 j is in the window (and its WHERE is true)
#pragma unroll
    for (int j = 0; j < RM; ++j)
        if (lane + j * kSwLanes < n) live |= 1u << j;
    if (WHERE) {
        bool err = false;
        int64_t erow = INT64_MAX;   // this lane's first failed row
#pragma unroll
        for (int j = 0; j < RM; ++j) {
            if (!((live >> j) & 1u)) continue;
            const int wd = where_decide_slow(p, b, a + lane + j * kSwLanes);
            if (wd < 0 && !err) erow = a + lane + j * kSwLanes;
            err |= wd < 0;
            if (wd <= 0) live &= ~(1u << j);
        }
        if (__any(err)) {   // a WHERE error replaces the window's output (filter_operator.go:63-77)
            if (res.wwit) {   // the window's first failed row (buffer order = the window's order)
                for (int o = 32; o > 0; o >>= 1) erow = min(erow, (int64_t)__shfl_xor(erow, o, kSwLanes));
                if (lane == 0) wit_where_row(&res.wwit[2 * widx], 0ull, (unsigned long long)erow, p, b, erow);
            }
            if (lane == 0) atomicOr(&res.win_err[widx], EK_WIN_WHERE_ERROR);
            return -1;
        }
    }
    // ---- duplicate filter: two bitmaps over HB hash bits. A row whose bit no other row of the window set is a
    // group of its own (no other row shares its hash, so none shares its key); the others are candidates.
    const int HB = sw_bits(n);
    uint32_t* s_seen = s_dyn;
    uint32_t* s_dupb = s_dyn + HB / 32;
    for (int k = lane; k < HB / 64; k += kSwLanes) ((uint4*)s_dyn)[k] = make_uint4(0u, 0u, 0u, 0u);   // both maps
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RM; ++j) {
        if (!((live >> j) & 1u)) continue;
        const uint32_t h = sw_hash(key[j]) & (uint32_t)(HB - 1), bit = 1u << (h & 31u);
        if (atomicOr(&s_seen[h >> 5], bit) & bit) atomicOr(&s_dupb[h >> 5], bit);
    }
    __syncthreads();
    uint32_t cand = 0;
#pragma unroll
    for (int j = 0; j < RM; ++j) {
        if (!((live >> j) & 1u)) continue;
        const uint32_t h = sw_hash(key[j]) & (uint32_t)(HB - 1);
        if ((s_dupb[h >> 5] >> (h & 31u)) & 1u) cand |= 1u << j;
    }
    __syncthreads();   // the bitmaps are dead: their LDS is reused below
    int nc = __popc(cand);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nc += __shfl_xor(nc, o, kSwLanes);
    if (cand_cap > 0 && nc > cand_cap) return -2;   // the capped launch's tables cannot hold them: redo launch
    const uint32_t single = live & ~cand;
    int fl[NVC], col[NVC];
    bool isf[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) { fl[v] = v < p.n_vc ? p.vc_flags[v] : 0; col[v] = v < p.n_vc ? p.vc_col[v] : 0; isf[v] = p.vc_is_float[v] != 0; }
    int64_t emitted = 0;
    bool herr = false;
    auto emit = [&](bool present, const Part<NVC>& s, uint32_t k) {
        const unsigned long long m = __ballot(present);
        if (present) {
            const int64_t pos = out + emitted + __popcll(m & ((1ull << lane) - 1ull));
            res.key[pos] = k;
#pragma unroll
            for (int q = 0; q < EK_MAX_AGGS; ++q) {
                if (q >= p.n_aggs) break;
                const Val v = agg_value(p, s, q);
                res.tag[q][pos] = v.tag == V_NULL ? EK_TAG_NULL : (v.tag == V_I64 ? EK_TAG_I64 : EK_TAG_F64);
                res.val[q][pos] = v.tag == V_F64 ? __double_as_longlong(v.f) : v.i;
            }
        }
        emitted += __popcll(m);
    };
    // fold of a group given its rows in window order (row(u) for u in [0, c)): count, sums, min / max, centred M2
    auto fold = [&](Part<NVC>& s, int c, auto row) {
        int64_t vc[NVC], is[NVC];
        double fs[NVC], m2[NVC];
        uint64_t mn[NVC], mx[NVC];
#pragma unroll
        for (int v = 0; v < NVC; ++v) { vc[v] = 0; is[v] = 0; fs[v] = 0.0; m2[v] = 0.0; mn[v] = ~0ull; mx[v] = 0ull; }
        if constexpr (NVC == 1) {
            if (c <= kSwFoldRegs) {
                // a short group: its values are loaded together (one memory latency instead of one per row and pass)
                // and both passes run from registers, in the same row order as below (the same f64 operations)
                int64_t rv[kSwFoldRegs];
                bool ok[kSwFoldRegs];
#pragma unroll
                for (int u = 0; u < kSwFoldRegs; ++u) {
                    const int64_t r = a + row(u < c ? u : 0);
                    ok[u] = u < c && fl[0] && col_valid(b, col[0], r);
                    rv[u] = ok[u] ? ((const int64_t*)b.col[col[0]])[r] : 0;
                }
#pragma unroll
                for (int u = 0; u < kSwFoldRegs; ++u) {
                    if (!ok[u]) continue;
                    const double xv = isf[0] ? __longlong_as_double(rv[u]) : (double)rv[u];
                    const uint64_t o = isf[0] ? f64_to_ord(xv) : i64_to_ord(rv[u]);
                    vc[0]++;
                    is[0] = (int64_t)((uint64_t)is[0] + (uint64_t)rv[u]);
                    fs[0] = __dadd_rn(fs[0], xv);
                    mn[0] = o < mn[0] ? o : mn[0];
                    mx[0] = o > mx[0] ? o : mx[0];
                }
                if ((fl[0] & NEED_M2) && vc[0] > 0) {
                    const double mean = __ddiv_rn(fs[0], (double)vc[0]);
#pragma unroll
                    for (int u = 0; u < kSwFoldRegs; ++u) {
                        if (!ok[u]) continue;
                        const double d = __dsub_rn(isf[0] ? __longlong_as_double(rv[u]) : (double)rv[u], mean);
                        m2[0] = __dadd_rn(m2[0], __dmul_rn(d, d));
                    }
                }
                part_merge(p, s, c, vc, is, fs, m2, mn, mx);
                return;
            }
        }
        for (int u = 0; u < c; ++u) {
            const int64_t r = a + row(u);
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                if (!fl[v] || !col_valid(b, col[v], r)) continue;
                const int64_t raw = ((const int64_t*)b.col[col[v]])[r];
                const double xv = isf[v] ? __longlong_as_double(raw) : (double)raw;
                const uint64_t o = isf[v] ? f64_to_ord(xv) : i64_to_ord(raw);
                vc[v]++;
                is[v] = (int64_t)((uint64_t)is[v] + (uint64_t)raw);
                fs[v] = __dadd_rn(fs[v], xv);
                mn[v] = o < mn[v] ? o : mn[v];
                mx[v] = o > mx[v] ? o : mx[v];
            }
        }
#pragma unroll
        for (int v = 0; v < NVC; ++v) {   // centred second pass (stats._variance shape)
            if (!(fl[v] & NEED_M2) || vc[v] == 0) continue;
            const double mean = __ddiv_rn(fs[v], (double)vc[v]);
            for (int u = 0; u < c; ++u) {
                const int64_t r = a + row(u);
                if (!col_valid(b, col[v], r)) continue;
                const int64_t raw = ((const int64_t*)b.col[col[v]])[r];
                const double d = __dsub_rn(isf[v] ? __longlong_as_double(raw) : (double)raw, mean);
                m2[v] = __dadd_rn(m2[v], __dmul_rn(d, d));
            }
        }
        part_merge(p, s, c, vc, is, fs, m2, mn, mx);
    };
    // keep decision of a folded group: HAVING over count(*) alone from its row count, any other HAVING on the partial
    // a group HAVING over count(*) alone failed on: its witness (the count is its only aggregate input)
    auto star_wit = [&](int c, uint32_t k) {
        if (!res.wwit) return;
        Part<NVC> cp{};
        cp.cnt = c;
        wit_having(&res.wwit[2 * widx + 1], k, p, [&](int q) { return agg_value(p, cp, q); });
    };
    auto keep = [&](const Part<NVC>& s, int c, uint32_t k) -> bool {
        if (p.having_star) {
            const int d = having_star_decide<NVC, HS>(p, c, h1, h2);
            if (d < 0) { herr = true; star_wit(c, k); }
            return d > 0;
        }
        if constexpr (HS) return true;   // no HAVING
        else return having_keep(p, s, res, widx, k);
    };
    // ---- one-row groups, straight from their lanes (coalesced value loads; a rolled loop: one copy of the fold)
    if (__any(single != 0u) && !(p.having_star && h1 == 0)) {
        for (int j = 0; j < RM; ++j) {
            const bool mine = (single >> j) & 1u;
            if (!__any(mine)) continue;
            Part<NVC> s{};
            bool present = false;
            if (mine) {
                fold(s, 1, [&](int) { return lane + j * kSwLanes; });
                present = keep(s, 1, sel(key, j));
            }
            emit(present, s, sel(key, j));
        }
    }
    if (nc > 0) {
        // ---- the candidates (real duplicates + hash collisions): an LDS hash table over them sized by their count
        // (linear probing, 16-bit counts packed two per word), a slot scan into group offsets (groups HAVING over
        // count(*) drops get cursor 0x8000: their rows are never placed), the rows placed by slot, one lane per group
        const int H = sw_slots(nc);
        uint32_t* s_key = s_dyn;                        // [H] slot -> key; then group g -> off << 16 | rows
        uint32_t* s_cnt = s_key + H;                    // [H / 2] slot rows, then slot cursors
        uint16_t* s_row = (uint16_t*)(s_cnt + H / 2);   // [nc] candidate rows grouped by slot
        for (int k = lane; k < H; k += kSwLanes) s_key[k] = ~0u;
        for (int k = lane; k < H / 2; k += kSwLanes) s_cnt[k] = 0u;
        __syncthreads();
        for (int j = 0; j < RM; ++j) {
            bool pend = (cand >> j) & 1u;
            if (!__any(pend)) continue;
            const uint32_t kj = sel(key, j);
            int h = (int)(sw_hash(kj) & (uint32_t)(H - 1));
            while (__any(pend)) {
                if (pend) {
                    const uint32_t old = atomicCAS(&s_key[h], ~0u, kj);
                    if (old == ~0u || old == kj) pend = false;
                    else h = (h + 1) & (H - 1);
                }
            }
            if ((cand >> j) & 1u) atomicAdd(&s_cnt[h >> 1], 1u << ((h & 1) * 16));
        }
        __syncthreads();
        const int per = H / kSwLanes;   // slots per lane (even)
        const int s0 = lane * per;
        uint32_t x = 0;                 // kept groups << 16 | kept rows of this lane's slots
        for (int q = 0; q < per; q += 2) {
            const uint32_t wd = s_cnt[(s0 + q) >> 1];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int c = (int)((wd >> (16 * hh)) & 0xFFFFu);
                if (c == 0) continue;
                int d = 1;
                if (p.having_star) {
                    d = having_star_decide<NVC, HS>(p, c, h1, h2);
                    if (d < 0) { herr = true; star_wit(c, s_key[s0 + q + hh]); }
                }
                if (d > 0) x += 0x10000u + (uint32_t)c;
            }
        }
        uint32_t inc = x;
#pragma unroll
        for (int o = 1; o < kSwLanes; o <<= 1) { const uint32_t y = __shfl_up(inc, o, kSwLanes); if (lane >= o) inc += y; }
        const int ng = (int)(__shfl(inc, kSwLanes - 1, kSwLanes) >> 16);
        if (ng > 0) {
            // the key table is still needed below to find each row's slot: the group table goes after the rows
            uint32_t* s_grp = (uint32_t*)(s_row + ((nc + 1) & ~1));
            uint32_t run = inc - x;
            for (int q = 0; q < per; q += 2) {
                const uint32_t wd = s_cnt[(s0 + q) >> 1];
                uint32_t cur = 0;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int c = (int)((wd >> (16 * hh)) & 0xFFFFu);
                    int d = c > 0 ? 1 : 0;
                    if (c > 0 && p.having_star) d = having_star_decide<NVC, HS>(p, c, h1, h2);
                    if (d > 0) {
                        s_grp[run >> 16] = ((run & 0xFFFFu) << 16) | (uint32_t)c;
                        cur |= (run & 0xFFFFu) << (16 * hh);
                        run += 0x10000u + (uint32_t)c;
                    } else {
                        cur |= 0x8000u << (16 * hh);
                    }
                }
                s_cnt[(s0 + q) >> 1] = cur;
            }
            __syncthreads();
            for (int j = 0; j < RM; ++j) {
                const bool mine = (cand >> j) & 1u;
                if (!__any(mine)) continue;
                if (mine) {
                    const uint32_t kj = sel(key, j);
                    int h = (int)(sw_hash(kj) & (uint32_t)(H - 1));
                    while (s_key[h] != kj) h = (h + 1) & (H - 1);   // the row's slot (its key is in the table)
                    const uint32_t sh = (uint32_t)(h & 1) * 16;
                    const uint32_t pos = (atomicAdd(&s_cnt[h >> 1], 1u << sh) >> sh) & 0xFFFFu;
                    if (pos < 0x8000u) s_row[pos] = (uint16_t)(lane + j * kSwLanes);
                }
            }
            __syncthreads();
            for (int gbase = 0; gbase < ng; gbase += kSwLanes) {
                const int gi = gbase + lane;
                Part<NVC> s{};
                bool present = false;
                uint32_t k = 0;
                if (gi < ng) {
                    const uint32_t gw = s_grp[gi];
                    const int g0 = (int)(gw >> 16), c = (int)(gw & 0xFFFFu);
                    sw_sort_rows(s_row + g0, c);   // the placement's atomics put them in no fixed order
                    k = kcol ? kcol[a + s_row[g0]] : 0u;
                    fold(s, c, [&](int u) { return (int)s_row[g0 + u]; });
                    // HAVING over count(*) alone was decided by the slot scan
                    if constexpr (HS) present = true;
                    else present = p.having_star ? true : having_keep(p, s, res, widx, k);
                }
                emit(present, s, k);
            }
        }
    }
    if (__any(herr) && lane == 0) atomicOr(&res.win_err[widx], EK_WIN_HAVING_ERROR);
    __syncthreads();   // the next window reuses the LDS
    return emitted;
}

// Persistent waves over the launch's windows (grid-stride): the next window's keys are loaded while this one is
// grouped, so a wave never waits for its keys after the first window. Redo: cand_cap > 0 sends a window with more
// candidate rows to redo_out (work-item indices, counter redo_cnt); a launch with redo_in runs those items alone
// (their count read from redo_cnt) with cand_cap 0 and the full tables.
template <int NVC, bool WHERE, int RM, bool HS>
__global__ __launch_bounds__(kSwLanes) void k_small_win(DPlan* __restrict__ pp, DBatch b, const int64_t* __restrict__ ab,
                                                       const int32_t* __restrict__ wlist, const int32_t* __restrict__ slots,
                                                       const int64_t* __restrict__ obase, Results res, int nwin, SwArith ar,
                                                       SwRedo rd) {
    const DPlan& p = *pp;
    const int lane = threadIdx.x;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    const uint32_t* kcol = p.key_col >= 0 ? (const uint32_t*)b.col[p.key_col] : nullptr;
    if (rd.in) nwin = *rd.cnt;   // the redo launch: the items the capped launch left
    auto item = [&](int t) { return rd.in ? rd.in[t] : t; };
    // HAVING over count(*) alone: the decisions for one- and two-row groups, once per wave
    int h1 = 1, h2 = 1;
    if (p.having_star) {
        if constexpr (HS) {
            h1 = p.hstar_tab[1];
            h2 = p.hstar_tab[2];
        } else {
            Part<NVC> cp{};
            cp.cnt = 1;
            h1 = having_decide(p, cp);
            cp.cnt = 2;
            h2 = having_decide(p, cp);
        }
    }
    auto window_a = [&](int i) { return wlist ? ab[2 * wlist[i]] : ar.a0 + (int64_t)i * ar.len; };
    auto window_n = [&](int i) { return wlist ? (int)(ab[2 * wlist[i] + 1] - ab[2 * wlist[i]]) : ar.len; };   // 1..kSmallWin
    uint32_t key[RM];
    auto load_keys = [&](int i, uint32_t (&k)[RM]) {
        const int64_t a = window_a(i);
        const int n = window_n(i);
#pragma unroll
        for (int j = 0; j < RM; ++j) k[j] = (kcol && lane + j * kSwLanes < n) ? kcol[a + lane + j * kSwLanes] : 0u;
    };
    int t = blockIdx.x;
    if (t < nwin) load_keys(item(t), key);
    for (; t < nwin; t += gridDim.x) {
        const int i = item(t);
        const int w = wlist ? wlist[i] : i;
        const int64_t a = window_a(i);
        const int n = window_n(i);
        const int32_t widx = wlist ? slots[w] : ar.slot0 + i;
        const int64_t out = wlist ? obase[w] : ar.ob0 + (int64_t)i * ar.rowcap;
        uint32_t nkey[RM] = {};
        if (t + (int)gridDim.x < nwin) load_keys(item(t + gridDim.x), nkey);
        const int64_t e = sw_window<NVC, WHERE, RM, HS>(p, b, kcol, a, n, widx, out, key, res, s_dyn, h1, h2, rd.cap);
        if (e >= 0 && lane == 0) res.win_cnt[widx] = e;
        if (e == -2 && lane == 0) rd.out[atomicAdd(rd.cnt, 1)] = i;
#pragma unroll
        for (int j = 0; j < RM; ++j) key[j] = nkey[j];
    }
}

}  // namespace ek
