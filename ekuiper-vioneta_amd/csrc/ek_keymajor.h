// ek_keymajor.h — key-major aggregation of range windows (ek_engine.hip: Engine::km_run).
//
// A range window is an index range [a_k, b_k) of the event buffer (release order). The window-major path
// (k_part MODE 2 + k_agg) partitions every window's members by (window, key bucket), so a sliding window that
// overlaps its neighbours re-partitions each event once per window it belongs to, and a window over a huge key
// space (C5: 12.5 M keys) spreads a handful of rows over thousands of partitions. Here the span of the fired
// windows is sorted ONCE by key (stable, so each key's rows keep their buffer order), and one thread per key walks
// the windows that hold any of its rows with two cursors over its sorted positions: window k's members of key g are
// the contiguous sub-run of g's rows with a_k <= pos < b_k (aggregate_operator.go:34-82 groups a window's rows by
// key; window_op.go:576-739 decides the members). The windows must be monotone (a_k and b_k non-decreasing in
// trigger order), which holds for every window type the engine fires in order.
//
// Per (key, window) the thread folds the sub-run (count, sum, min, max, centred two-pass M2; median /
// percentile_* over at most kKmSegMax values sorted in LDS), finalises (funcs_agg.go), applies HAVING and
// emits. Result rows of window k land in its region [obase_k, obase_k + kept_k): a counting pass keeps a
// per-(window, block) histogram in LDS, one workgroup per window scans it over the blocks, and the write pass
// recomputes and stores at the block's offset + an LDS cursor (groups come in unspecified order, like the
// reference's Go map iteration).
#pragma once
#include "ek_kernels.h"

namespace ek {

constexpr int kKmBlock = 256;
constexpr int kKmMaxWin = 4096;    // windows per launch: the per-block LDS histogram
constexpr int kKmSegMax = 32;      // order statistics: longest (key, window) sub-run, sorted in the thread's LDS lane

struct KmDesc {
    int64_t n;                     // rows of the span (relative positions [0, n))
    int32_t nw, nblk;
    uint32_t nkeys;                // dense key ids < nkeys
    int32_t pad;
    const int64_t* ab;             // [2 * nw] window ranges relative to the span start
    const int64_t* obase;          // [nw] first result row of each window's region
    const int32_t* widx;           // [nw] result window slot
    const uint32_t* kstart;        // [nkeys + 1] first sorted row of each key
    const uint32_t* spos;          // relative positions in key order
    const int64_t* sval[kMaxVC];   // value columns gathered in key order
    const uint8_t* sok[kMaxVC];    // their validity (nullptr: all valid)
    uint32_t* bcnt;                // [nw][nblk + 1] kept rows per (window, block) -> exclusive offsets after k_km_scan
                                   // (the window's total at [nblk])
    int32_t* flags;                // [0] a (key, window) sub-run longer than kKmSegMax (order statistics), [1] scratch
    // packed emission (write pass of multi-window launches, n_aggs <= kKmRecAggs): rows go out as one 32-byte record
    // each, window k's at rec[rbase[k] + i] for its row obase[k] + i, and k_km_unpack transposes them to the result
    // columns with coalesced stores (the walk's threads emit into ~30 windows each: per-column scattered stores
    // left 5-7 partial lines per row, 10.9x write amplification on C4a)
    const int64_t* rbase;          // [nw + 1] exclusive prefix of the windows' kept rows
    uint4* rec;                    // nullptr: store the result columns directly
    // state emission (skend != nullptr): a kept membership state [k, kend) is counted and stored ONCE, in bucket k
    // (its first window), with skend = kend; k_km_expand copies it into every window of its run. rbase / bcnt then
    // count states per bucket instead of rows per window.
    uint16_t* skend;
    // single-pass state emission (sk != nullptr, !SORT write pass, no count pass): the walk stores its kept states
    // unsorted in its block's region [2 kstart[b * kKmBlock], ...) (a key of r rows has at most 2r membership states),
    // with their bucket in sk, counts them per (bucket, block) into bcnt and per block into scount; k_km_sscatter then
    // moves them into bucket order
    uint16_t* sk;
    uint32_t* scount;
    const uint16_t* sE;            // multi-window launches: KmCols::E / X of the sorted rows (SORT launches: when set,
    const uint16_t* sX;            // the walk merges them too; else it binary-searches the window bounds)
    int32_t* dbg;                  // EK_KM_CHECK builds: the first violated bound [code, values...] (km_bad)
    int32_t dbg_mode;              // EK_KM_CHECK builds: 1 = the walk skips the fold (states only)
    int32_t pad2;
};

// EK_KM_CHECK (debug builds, make EXTRA=-DEK_KM_CHECK): the walk and the gather test their index bounds and record the
// first violation (a code and four values) instead of touching memory out of range; the host reports it.
__device__ __forceinline__ void km_bad(int32_t* dbg, int code, int64_t a, int64_t b, int64_t c, int64_t e) {
    if (dbg && atomicCAS(dbg, 0, code) == 0) {
        dbg[1] = (int32_t)a; dbg[2] = (int32_t)b; dbg[3] = (int32_t)c; dbg[4] = (int32_t)e;
        dbg[5] = (int32_t)blockIdx.x; dbg[6] = (int32_t)threadIdx.x;
    }
}
#ifdef EK_KM_CHECK
#define KM_CHECK(dbg, cond, code, a, b, c, e) if (!(cond)) { km_bad(dbg, code, a, b, c, e); break; }
#else
#define KM_CHECK(dbg, cond, code, a, b, c, e)
#endif
constexpr int kKmRecAggs = 3;      // record: key u32 | 4 tag bytes | 3 x 8-byte values

// (key, relative position) of every row of the span; rows that fail WHERE (or carry an out-of-range key) get the
// sentinel key nkeys and sort last. WHERE errors are counted: the caller falls back to the window-major path,
// which attributes them per window (filter_operator.go:63-77).
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_km_keys(DPlan* __restrict__ pp, DBatch b, int64_t lo, int64_t n,
                                                    uint32_t* __restrict__ kout, uint32_t* __restrict__ pout,
                                                    unsigned int* __restrict__ nerr) {
    const DPlan& p = *pp;
    const uint32_t* kcol = (const uint32_t*)b.col[p.key_col];
    const uint32_t K = p.num_keys;
    unsigned int e = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int64_t r = lo + i;
        const int wd = p.n_where > 0 ? where_decide_slow(p, b, r) : 1;
        uint32_t k = kcol[r];
        if (wd <= 0 || k >= K) k = K;
        e += wd < 0;
        kout[i] = k;
        if (pout) pout[i] = (uint32_t)i;
    }
    if (e) atomicAdd(nerr, e);
}
#endif

// kstart[g] = first sorted row with key >= g, for g in [0, K] (kstart[K] = rows that passed WHERE).
#ifndef EK_NO_PLAIN_KERNELS
__global__ void k_km_starts(const uint32_t* __restrict__ sk, int64_t n, uint32_t K, uint32_t* __restrict__ kstart) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        // row i starts every key in (sk[i - 1], sk[i]] (keys <= K; the span's end closes (sk[n - 1], K])
        const uint32_t g0 = i == 0 ? 0u : sk[i - 1] + 1u;
        const uint32_t g1 = i == n ? K : min(sk[i], K);
        for (uint32_t g = g0; g <= g1; ++g) kstart[g] = (uint32_t)i;
    }
}
#endif

// longest key run (rows of one key over the whole span) -> atomicMax(*out)
// (one atomic per workgroup on a grid of at most 256: per-wave atomics on the one word serialised, 0.18 ms on C4a)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_km_maxrun(const uint32_t* __restrict__ kstart, uint32_t K, unsigned int* out) {
    __shared__ unsigned int s_m[kBlock / 64];
    unsigned int m = 0;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < K; g += (int64_t)gridDim.x * kBlock)
        m = max(m, kstart[g + 1] - kstart[g]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) m = max(m, s_m[w]);
        if (m) atomicMax(out, m);
    }
}
#endif

// first window k in [k0, nw) with e[k] > x (e non-decreasing: window starts or ends in LDS), nw if none
__device__ __forceinline__ int km_first_gt(const int32_t* e, int k0, int nw, int64_t x) {
    int lo = k0, hi = nw;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)e[mid] > x) hi = mid; else lo = mid + 1;
    }
    return lo;
}

struct KmCols {
    int64_t* val[kMaxVC];
    uint8_t* ok[kMaxVC];
    // multi-window launches: per row in key order, the first window that holds it (E: first k with b_k > pos) and the
    // first window past it (X: first k with a_k > pos); row i is a member of window k iff E_i <= k < X_i
    uint16_t* E;
    uint16_t* X;
    const int64_t* ab;   // [2 * nw] window ranges relative to the span start
    int32_t nw;
    int64_t n;           // rows of the span
    int32_t* dbg;        // EK_KM_CHECK
    int32_t no_vals;     // the value columns are already in key order (km_msd): E / X only
};

// value columns (and validity) of the rows that passed WHERE, in key order
template <int NVC>
__global__ __launch_bounds__(kBlock) void k_km_gather(DPlan* __restrict__ pp, DBatch b, int64_t lo,
                                                      const uint32_t* __restrict__ spos, const uint32_t* __restrict__ kstart,
                                                      KmCols out) {
    const DPlan& p = *pp;
    extern __shared__ int32_t s_ab[];   // E / X: window starts [nw], ends [nw]
    if (out.E) {
        for (int k = threadIdx.x; k < out.nw; k += kBlock) { s_ab[k] = (int32_t)out.ab[2 * k]; s_ab[out.nw + k] = (int32_t)out.ab[2 * k + 1]; }
        __syncthreads();
    }
    const int64_t m = kstart[p.num_keys];
#ifdef EK_KM_CHECK
    if (m > out.n) { if (threadIdx.x == 0) km_bad(out.dbg, 1, m, out.n, p.num_keys, 0); return; }
#endif
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBlock) {
        KM_CHECK(out.dbg, (int64_t)spos[i] < out.n, 2, i, spos[i], out.n, m)
        const int64_t r = lo + spos[i];
        KM_CHECK(out.dbg, r >= 0 && r < b.n, 3, i, r, b.n, lo)
        if (out.E) {
            out.E[i] = (uint16_t)km_first_gt(s_ab + out.nw, 0, out.nw, (int64_t)spos[i]);
            out.X[i] = (uint16_t)km_first_gt(s_ab, 0, out.nw, (int64_t)spos[i]);
        }
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            if (v >= p.n_vc || out.no_vals) break;
            const int c = p.vc_col[v];
            out.val[v][i] = ((const int64_t*)b.col[c])[r];
            if (out.ok[v]) out.ok[v][i] = b.valid[c] ? b.valid[c][r] : (uint8_t)1;
        }
    }
}


// HAVING (having_operator.go:41-56): 1 keeps the group, 0 drops it, -1 = a non-bool result (window error)
template <int NVC>
__device__ __forceinline__ int km_having(const DPlan& p, const Part<NVC>& s, const SortRes* sr) {
    if (p.n_having <= 0) return 1;
    const Val h = eval_prog(p.having_prog, p.n_having, p, nullptr, 0, [&](int k) { return agg_value(p, s, k, sr); });
    if (h.tag != V_BOOL) return -1;
    return h.i != 0 ? 1 : 0;
}

// Fold one (key, window run) membership state: rows [j0, j1) of the key's sorted rows. First pass (count, sums,
// min, max), centred second pass (M2), then the order statistics. Returns true on an aggregate error.
template <int NVC, bool SORT>
__device__ __forceinline__ bool km_fold(const DPlan& p, const KmDesc& d, int64_t j0, int64_t j1, const int (&fl)[NVC],
                                        const bool (&isf)[NVC], uint64_t* s_seg, Part<NVC>& part,
                                        uint64_t (&sres)[kMaxSortAggs], uint8_t (&stag)[kMaxSortAggs]) {
    // ---- order statistics: a sub-run of more than kKmSegMax values is not folded here at all (the launch falls back to
    // the window-major radix select): its in-memory rank counting faulted on MI355X
    if constexpr (SORT) {
        for (int sc = 0; sc < p.n_scol; ++sc) {
            const uint8_t* __restrict__ ok = d.sok[p.scol_vc[sc]];
            int64_t n = j1 - j0;
            if (ok && n > kKmSegMax) { n = 0; for (int64_t j = j0; j < j1; ++j) n += ok[j] ? 1 : 0; }
            if (n > kKmSegMax) { d.flags[0] = 1; return true; }
        }
    }
    // ---- fold the sub-run [j0, j1): first pass (count, sums, min, max), centred second pass (M2)
#ifdef EK_KM_CHECK
    if (!(j0 >= 0 && j0 < j1 && j1 <= d.n)) { km_bad(d.dbg, 20, j0, j1, d.n, 0); return true; }
    for (int v = 0; v < NVC; ++v)
        if (fl[v] && !d.sval[v]) { km_bad(d.dbg, 21, v, fl[v], 0, 0); return true; }
    for (int sc = 0; SORT && sc < p.n_scol; ++sc)
        if (p.scol_vc[sc] < 0 || p.scol_vc[sc] >= NVC || !d.sval[p.scol_vc[sc]]) { km_bad(d.dbg, 22, sc, p.scol_vc[sc], NVC, 0); return true; }
#endif
    int64_t vc[NVC], is[NVC];
    double fs[NVC], m2[NVC];
    uint64_t mn[NVC], mx[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) {
        vc[v] = 0; is[v] = 0; fs[v] = 0.0; m2[v] = 0.0; mn[v] = ~0ull; mx[v] = 0ull;
        if (!fl[v]) continue;
        const int64_t* __restrict__ val = d.sval[v];
        const uint8_t* __restrict__ ok = d.sok[v];
        for (int64_t j = j0; j < j1; ++j) {
            if (ok && !ok[j]) continue;
            const int64_t raw = val[j];
            const double x = isf[v] ? __longlong_as_double(raw) : (double)raw;
            const uint64_t o = isf[v] ? f64_to_ord(x) : i64_to_ord(raw);
            vc[v]++;
            is[v] = (int64_t)((uint64_t)is[v] + (uint64_t)raw);
            fs[v] = __dadd_rn(fs[v], x);
            mn[v] = o < mn[v] ? o : mn[v];
            mx[v] = o > mx[v] ? o : mx[v];
        }
        if ((fl[v] & NEED_M2) && vc[v] > 0) {   // stats._variance shape
            const double mean = __ddiv_rn(fs[v], (double)vc[v]);
            for (int64_t j = j0; j < j1; ++j) {
                if (ok && !ok[j]) continue;
                const int64_t raw = val[j];
                const double dd = __dsub_rn(isf[v] ? __longlong_as_double(raw) : (double)raw, mean);
                m2[v] = __dadd_rn(m2[v], __dmul_rn(dd, dd));
            }
        }
    }
    part_merge(p, part, j1 - j0, vc, is, fs, m2, mn, mx);
    bool agg_err = false;
#pragma unroll
    for (int a = 0; a < kMaxSortAggs; ++a) { sres[a] = 0; stag[a] = EK_TAG_NULL; }
    if constexpr (SORT) {
        // per sort column: the sub-run's valid values (ordered bits, at most kKmSegMax: checked above), insertion-sorted
        // in this thread's LDS lane (interleaved, conflict-free)
        for (int sc = 0; sc < p.n_scol; ++sc) {
            const int v = p.scol_vc[sc];
            const int64_t* __restrict__ val = d.sval[v];
            const uint8_t* __restrict__ ok = d.sok[v];
            const bool fv = p.vc_is_float[v] != 0;
            int m = 0;
            for (int64_t j = j0; j < j1; ++j) {
                if (ok && !ok[j]) continue;
                const uint64_t x = fv ? f64_to_ord(__longlong_as_double(val[j])) : i64_to_ord(val[j]);
                int q = m;
                while (q > 0 && s_seg[(q - 1) * kKmBlock + threadIdx.x] > x) {
                    s_seg[q * kKmBlock + threadIdx.x] = s_seg[(q - 1) * kKmBlock + threadIdx.x];
                    --q;
                }
                s_seg[q * kKmBlock + threadIdx.x] = x;
                ++m;
            }
            const int64_t n = m;
#pragma unroll
            for (int a = 0; a < kMaxSortAggs; ++a) {
                if (a >= p.n_sagg || p.sagg_scol[a] != sc) continue;
                const int ka = p.sagg_agg[a];
                order_stat(p.agg_fn[ka], fv, p.agg_p[ka], n,
                           [&](int64_t r) { return s_seg[(r < 0 ? 0 : r >= kKmSegMax ? kKmSegMax - 1 : r) * kKmBlock + threadIdx.x]; },
                           &sres[a], &stag[a]);
                agg_err |= stag[a] == kTagErr;
            }
        }
    }
    return agg_err;
}

// the emitted values of a kept group
template <int NVC>
__device__ __forceinline__ void km_row(const DPlan& p, const Part<NVC>& part, const SortRes* sr, int64_t (&ov)[EK_MAX_AGGS],
                                       uint8_t (&ot)[EK_MAX_AGGS]) {
#pragma unroll
    for (int q = 0; q < EK_MAX_AGGS; ++q) {
        ov[q] = 0;
        ot[q] = EK_TAG_NULL;
        if (q >= p.n_aggs) continue;
        const Val av = agg_value(p, part, q, sr);
        ot[q] = av.tag == V_NULL ? EK_TAG_NULL : (av.tag == V_I64 ? EK_TAG_I64 : EK_TAG_F64);
        ov[q] = av.tag == V_F64 ? __double_as_longlong(av.f) : av.i;
    }
}

// WRITE = false: count the rows each (window, block) keeps; true: emit them (and raise window errors).
// ONE (a launch of ONE window spanning the whole sorted span, WRITE = true): every row of a key is a member, so the
// walk needs no positions, each key yields at most one row, and the rows are block-compacted with one atomic per
// workgroup on the window's row counter — a single pass, no count pass / scan.
// A key's membership [j0, j1) of its sorted rows only changes where a window start passes row j0 or a window end
// passes row j1, so the thread folds, finalises and tests HAVING once per membership state and emits that row into
// every window of the state's run [k, kend) — about two states per row instead of one fold per (key, window).
// HS (no order statistics): HAVING is absent, or reads count(*) alone and every key run of the span is shorter than
// kHStarTab rows: each state is decided from DPlan.hstar_tab (k_hstar_tab, create time) and the walk carries no
// expression interpreter (C4a: fewer VGPRs, more waves per SIMD).
template <int NVC, bool SORT, bool WRITE, bool ONE = false, bool HS = false>
__global__ __launch_bounds__(kKmBlock) void k_km_walk(DPlan* __restrict__ pp, KmDesc d, Results res) {
    extern __shared__ uint32_t s_dyn[];
    __shared__ uint32_t s_wc[kKmBlock / 64 + 1];
    __shared__ uint32_t s_n;   // single-pass state emission: states stored by this block
    if (threadIdx.x == 0) s_n = 0;
    bool one_present = false;
    int64_t one_v[EK_MAX_AGGS];
    uint8_t one_t[EK_MAX_AGGS];
    const int nw = d.nw;
    uint32_t* s_h = s_dyn;                          // [nw] kept rows (count pass) / cursors (write pass)
    // SORT launches walk by binary search over the window starts / ends in LDS; the others merge E / X (k_km_gather)
    int32_t* s_a = (int32_t*)(s_dyn + nw);          // SORT: [nw] window starts (relative rows)
    int32_t* s_b = s_a + nw;                        // SORT: [nw] window ends
    uint64_t* s_seg = (uint64_t*)(s_dyn + ((3 * nw + 1) & ~1));   // SORT: [kKmSegMax][kKmBlock] ordered values
    const DPlan& p = *pp;
    __shared__ int s_hc[2];   // HAVING over count(*) alone: the decisions for 1 and 2 rows (most states), once per block
    if constexpr (!SORT && !HS) {
        if (threadIdx.x == 0 && p.having_star) {
            Part<NVC> cp{};
            cp.cnt = 1;
            s_hc[0] = km_having(p, cp, nullptr);
            cp.cnt = 2;
            s_hc[1] = km_having(p, cp, nullptr);
        }
    }
    for (int k = threadIdx.x; k < nw; k += kKmBlock) {
        // write pass: the cursor starts at this block's offset in the window's region (no per-row bcnt read)
        s_h[k] = (WRITE && !ONE && !d.sk) ? d.bcnt[(int64_t)k * (d.nblk + 1) + blockIdx.x] : 0u;
        if (SORT && !ONE) {
            s_a[k] = (int32_t)d.ab[2 * k];
            s_b[k] = (int32_t)d.ab[2 * k + 1];
        }
    }
    __syncthreads();
    const int64_t g = (int64_t)blockIdx.x * kKmBlock + threadIdx.x;
    if (g < d.nkeys) {
        const int64_t s = d.kstart[g], e = d.kstart[g + 1];
        int fl[NVC];
        bool isf[NVC];
#pragma unroll
        for (int v = 0; v < NVC; ++v) { fl[v] = v < p.n_vc ? p.vc_flags[v] : 0; isf[v] = p.vc_is_float[v] != 0; }
        int64_t j0 = s, j1 = s;
        const bool merge = !SORT || d.sE != nullptr;   // uniform
#ifdef EK_KM_CHECK
        if (!(s <= e && e <= d.n)) { km_bad(d.dbg, 10, g, s, e, d.n); return; }
#endif
        int k = s < e ? (ONE ? 0 : !merge ? km_first_gt(s_b, 0, nw, (int64_t)d.spos[s]) : min((int)d.sE[s], (int)d.sX[s])) : nw;
        while (k < nw) {
            int kend = 1;
            KM_CHECK(d.dbg, k >= 0, 11, g, k, nw, 0)
            if constexpr (ONE) {
                j0 = s;
                j1 = e;
            } else if (!merge) {
                const int64_t wa = s_a[k], wb = s_b[k];
                while (j0 < e && (int64_t)d.spos[j0] < wa) ++j0;
                if (j0 == e) break;
                if (j1 < j0) j1 = j0;
                while (j1 < e && (int64_t)d.spos[j1] < wb) ++j1;
                const int64_t p0 = d.spos[j0];
                if (j1 == j0) { k = km_first_gt(s_b, k + 1, nw, p0); continue; }
                // windows [k, kend) hold exactly rows [j0, j1) of this key
                kend = km_first_gt(s_a, k + 1, nw, p0);
                if (j1 < e) kend = min(kend, km_first_gt(s_b, k + 1, nw, (int64_t)d.spos[j1]));
            } else {
                // window k's members: rows with E <= k (a prefix, up to j1) and X > k (a suffix, from j0); the set
                // changes at the next row's E or the first member's X: a merge of the two non-decreasing lists
                while (j1 < e && (int)d.sE[j1] <= k) ++j1;
                while (j0 < e && (int)d.sX[j0] <= k) ++j0;
                if (j0 == e) break;
                kend = min(j1 < e ? (int)d.sE[j1] : nw, (int)d.sX[j0]);
                KM_CHECK(d.dbg, kend > k && kend <= nw, 12, g, k, kend, j0)
                if (j1 <= j0) { k = kend; continue; }
                // windows [k, kend) hold exactly rows [j0, j1) of this key
            }
            KM_CHECK(d.dbg, s <= j0 && j0 < j1 && j1 <= e && kend > k && kend <= nw, 13, j0 - s, j1 - s, k, kend)
            if (!SORT && p.having_star) {
                // HAVING over count(*) alone (C4a: count(*) > 1): decided from the state's row count before any fold;
                // a state it drops (most (key, window) states hold one row) reads no value at all
                Part<NVC> cp{};
                cp.cnt = j1 - j0;
                int hc;
                if constexpr (HS) hc = p.hstar_tab[cp.cnt < kHStarTab ? cp.cnt : kHStarTab - 1];
                else hc = cp.cnt <= 2 ? s_hc[cp.cnt - 1] : km_having(p, cp, nullptr);
                if (hc <= 0) {
                    if (WRITE && hc < 0)
                        for (int kk = k; kk < kend; ++kk) {
                            atomicOr(&res.win_err[d.widx[kk]], EK_WIN_HAVING_ERROR);
                            if (res.wwit) wit_having(&res.wwit[2 * d.widx[kk] + 1], (uint32_t)g, p, [&](int q) { return agg_value(p, cp, q); });
                        }
                    k = kend;
                    continue;
                }
                if (!WRITE && !ONE) {   // the count pass needs only the decision
                    if (d.skend) atomicAdd(&s_h[k], 1u);
                    else for (int kk = k; kk < kend; ++kk) atomicAdd(&s_h[kk], 1u);
                    k = kend;
                    continue;
                }
            }
            uint64_t sres[kMaxSortAggs];
            uint8_t stag[kMaxSortAggs];
            Part<NVC> part{};
#ifdef EK_KM_CHECK
            if (d.dbg_mode == 1) { k = kend; continue; }
#endif
            const bool agg_err = km_fold<NVC, SORT>(p, d, j0, j1, fl, isf, s_seg, part, sres, stag);
            const SortRes sr{sres, stag, 0, 1};
            if (agg_err) {   // "run Select error" replaces each of these windows' output
                int ea = 0;   // the first order statistic that failed
                for (int a = p.n_sagg - 1; a >= 0; --a) if (sel(stag, a) == kTagErr) ea = a;
                if (WRITE)
                    for (int kk = k; kk < kend; ++kk) {
                        atomicOr(&res.win_err[d.widx[kk]], EK_WIN_AGG_ERROR);
                        if (res.aslot) atomicMax(&res.aslot[d.widx[kk]], kMaxSortAggs - ea);
                    }
            } else {
                // (HAVING over count(*) alone already kept this state above)
                int hv = 1;
                if constexpr (!HS) hv = (!SORT && p.having_star) ? 1 : km_having(p, part, SORT ? &sr : nullptr);
                if (WRITE && hv < 0)
                    for (int kk = k; kk < kend; ++kk) {
                        atomicOr(&res.win_err[d.widx[kk]], EK_WIN_HAVING_ERROR);
                        if (res.wwit)
                            wit_having(&res.wwit[2 * d.widx[kk] + 1], (uint32_t)g, p,
                                       [&](int q) { return agg_value(p, part, q, SORT ? &sr : nullptr); });
                    }
                if (hv > 0) {
                    if constexpr (ONE) {
                        one_present = true;
                        km_row(p, part, SORT ? &sr : nullptr, one_v, one_t);
                    } else if constexpr (!WRITE) {
                        if (d.skend) atomicAdd(&s_h[k], 1u);
                        else for (int kk = k; kk < kend; ++kk) atomicAdd(&s_h[kk], 1u);
                    } else {
                        int64_t ov[EK_MAX_AGGS];
                        uint8_t ot[EK_MAX_AGGS];
                        km_row(p, part, SORT ? &sr : nullptr, ov, ot);
                        if (d.rec) {   // one 32-byte record per row (two 16-byte stores), unpacked by k_km_unpack
                            const uint32_t tg = (uint32_t)ot[0] | ((uint32_t)ot[1] << 8) | ((uint32_t)ot[2] << 16);
                            const uint4 r0 = make_uint4((uint32_t)g, tg, (uint32_t)ov[0], (uint32_t)((uint64_t)ov[0] >> 32));
                            const uint4 r1 = make_uint4((uint32_t)ov[1], (uint32_t)((uint64_t)ov[1] >> 32), (uint32_t)ov[2],
                                                        (uint32_t)((uint64_t)ov[2] >> 32));
                            if (d.sk) {   // single pass: unsorted in the block's region, counted per bucket
                                const int64_t ri = 2 * (int64_t)d.kstart[(int64_t)blockIdx.x * kKmBlock] + (int64_t)atomicAdd(&s_n, 1u);
                                atomicAdd(&s_h[k], 1u);
                                d.rec[2 * ri] = r0;
                                d.rec[2 * ri + 1] = r1;
                                d.skend[ri] = (uint16_t)kend;
                                d.sk[ri] = (uint16_t)k;
                            } else if (d.skend) {   // the state once, in bucket k (k_km_expand fans it out)
                                const int64_t ri = d.rbase[k] + (int64_t)atomicAdd(&s_h[k], 1u);
                                d.rec[2 * ri] = r0;
                                d.rec[2 * ri + 1] = r1;
                                d.skend[ri] = (uint16_t)kend;
                            } else
                                for (int kk = k; kk < kend; ++kk) {
                                    const int64_t ri = d.rbase[kk] + (int64_t)atomicAdd(&s_h[kk], 1u);
                                    d.rec[2 * ri] = r0;
                                    d.rec[2 * ri + 1] = r1;
                                }
                        } else {
                            for (int kk = k; kk < kend; ++kk) {
                                const int64_t pos = d.obase[kk] + (int64_t)atomicAdd(&s_h[kk], 1u);
                                res.key[pos] = (uint32_t)g;
#pragma unroll
                                for (int q = 0; q < EK_MAX_AGGS; ++q) {
                                    if (q >= p.n_aggs) break;
                                    res.tag[q][pos] = ot[q];
                                    res.val[q][pos] = ov[q];
                                }
                            }
                        }
                    }
                }
            }
            k = kend;
        }
    }
    if constexpr (ONE) {
        const unsigned long long mask = __ballot(one_present);
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        if (lane == 0) s_wc[wv] = (uint32_t)__popcll(mask);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int w = 0; w < kKmBlock / 64; ++w) { const uint32_t c = s_wc[w]; s_wc[w] = run; run += c; }
            s_wc[kKmBlock / 64] = run ? (uint32_t)atomicAdd((unsigned long long*)&res.win_cnt[d.widx[0]], (unsigned long long)run) : 0u;
        }
        __syncthreads();
        if (one_present) {
            const int64_t pos = d.obase[0] + (int64_t)s_wc[kKmBlock / 64] + s_wc[wv] + __popcll(mask & ((1ull << lane) - 1ull));
            res.key[pos] = (uint32_t)g;
#pragma unroll
            for (int q = 0; q < EK_MAX_AGGS; ++q) {
                if (q >= p.n_aggs) break;
                res.tag[q][pos] = one_t[q];
                res.val[q][pos] = one_v[q];
            }
        }
    }
    if (!WRITE || (!ONE && d.sk)) {
        __syncthreads();
        for (int k = threadIdx.x; k < nw; k += kKmBlock) d.bcnt[(int64_t)k * (d.nblk + 1) + blockIdx.x] = s_h[k];
        if (WRITE && threadIdx.x == 0) d.scount[blockIdx.x] = s_n;
    }
}

// single-pass state emission: block b's unsorted states (k_km_walk) -> bucket order. State q of the block lands at
// rbase[k] + bcnt[k][b] (the block's exclusive offset in bucket k after k_km_scan) + an LDS cursor per bucket.
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kKmBlock) void k_km_sscatter(KmDesc d, const uint4* __restrict__ urec,
                                                         const uint16_t* __restrict__ ukend, const uint16_t* __restrict__ uk) {
    extern __shared__ uint32_t s_c[];   // [nw] cursors
    for (int k = threadIdx.x; k < d.nw; k += kKmBlock) s_c[k] = 0;
    __syncthreads();
    const int b = blockIdx.x;
    const int64_t base = 2 * (int64_t)d.kstart[(int64_t)b * kKmBlock];
    const uint32_t cnt = d.scount[b];
    for (uint32_t q = threadIdx.x; q < cnt; q += kKmBlock) {
        const int64_t i = base + q;
        const int k = uk[i];
        const int64_t ri = d.rbase[k] + (int64_t)d.bcnt[(int64_t)k * (d.nblk + 1) + b] + (int64_t)atomicAdd(&s_c[k], 1u);
        const uint4 r0 = urec[2 * i], r1 = urec[2 * i + 1];
        d.rec[2 * ri] = r0;
        d.rec[2 * ri + 1] = r1;
        d.skend[ri] = ukend[i];
    }
}
#endif

// rbase[k] = exclusive prefix over the launch's windows of their kept rows (bcnt[k][nblk] after k_km_scan);
// rbase[nw] = the total (one workgroup)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(1024) void k_km_rbase(KmDesc d, int64_t* __restrict__ rbase) {
    __shared__ int64_t s_w[16];
    __shared__ int64_t s_carry;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base < d.nw; base += 1024) {
        const int k = base + threadIdx.x;
        const int64_t x0 = k < d.nw ? (int64_t)d.bcnt[(int64_t)k * (d.nblk + 1) + d.nblk] : 0;
        int64_t x = x0;
        for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        int64_t wb = 0;
        for (int w = 0; w < wv; ++w) wb += s_w[w];
        const int64_t carry = s_carry;
        if (k < d.nw) rbase[k] = carry + wb + x - x0;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = carry + wb + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) rbase[d.nw] = s_carry;
}
#endif

// records -> result columns: window blockIdx.y's rows i = 0 .. kept - 1 land at obase + i (coalesced stores)
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kBlock) void k_km_unpack(KmDesc d, int n_aggs, Results res) {
    const int k = blockIdx.y;
    const int64_t cnt = d.rbase[k + 1] - d.rbase[k];
    const int64_t ob = d.obase[k];
    const uint4* __restrict__ rec = d.rec + 2 * d.rbase[k];
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * kBlock) {
        const uint4 r0 = rec[2 * i];
        const int64_t pos = ob + i;
        res.key[pos] = r0.x;
        res.tag[0][pos] = (uint8_t)r0.y;
        res.val[0][pos] = (int64_t)(((uint64_t)r0.w << 32) | r0.z);
        if (n_aggs > 1) {
            const uint4 r1 = rec[2 * i + 1];
            res.tag[1][pos] = (uint8_t)(r0.y >> 8);
            res.val[1][pos] = (int64_t)(((uint64_t)r1.y << 32) | r1.x);
            if (n_aggs > 2) {
                res.tag[2][pos] = (uint8_t)(r0.y >> 16);
                res.val[2][pos] = (int64_t)(((uint64_t)r1.w << 32) | r1.z);
            }
        }
    }
}
#endif

// states -> result rows. Window w's rows are the states of buckets k in [w - R + 1, w] whose run reaches it
// (kend > w; R = the most windows any one buffer position belongs to bounds every run). kKmExpChunks workgroups per
// window each take every kKmExpChunks-th tile of kKmExpTile candidates (4 per thread: independent loads in flight);
// a tile's rows are compacted per (candidate slot, wave) with ballots, reserved with one atomic on the window's row
// counter and stored on consecutive rows (each wave's store instructions cover consecutive addresses). Grid layout:
// XCD x (workgroup b runs on XCD b % 8) takes a contiguous range of windows, all chunks of each: neighbouring windows
// share most of their candidate states, which then come from that XCD's L2.
constexpr int kKmExpBlock = 256, kKmExpU = 4, kKmExpTile = kKmExpBlock * kKmExpU, kKmExpChunks = 8;
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kKmExpBlock) void k_km_expand(KmDesc d, int n_aggs, int R, Results res) {
    const int per = (d.nw + 7) >> 3;   // windows per XCD
    const int xcd = (int)(blockIdx.x & 7u), idx = (int)(blockIdx.x >> 3);
    const int w = xcd * per + idx / kKmExpChunks, chunk = idx % kKmExpChunks;
    if (w >= d.nw) return;   // uniform per workgroup
    constexpr int NW = kKmExpBlock / 64;
    __shared__ uint32_t s_off[kKmExpU * NW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t c0 = d.rbase[max(0, w - R + 1)], c1 = d.rbase[w + 1];
    const int64_t ob = d.obase[w];
    unsigned long long* cnt = (unsigned long long*)&res.win_cnt[d.widx[w]];
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int64_t t = c0 + (int64_t)chunk * kKmExpTile; t < c1; t += (int64_t)kKmExpChunks * kKmExpTile) {
        bool sel[kKmExpU];
        unsigned long long m[kKmExpU];
#pragma unroll
        for (int u = 0; u < kKmExpU; ++u) {
            const int64_t i = t + u * kKmExpBlock + threadIdx.x;
            sel[u] = i < c1 && (int)d.skend[i] > w;
        }
#pragma unroll
        for (int u = 0; u < kKmExpU; ++u) {
            m[u] = __ballot(sel[u]);
            if (lane == 0) s_off[u * NW + wv] = (uint32_t)__popcll(m[u]);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
#pragma unroll
            for (int e = 0; e < kKmExpU * NW; ++e) { const uint32_t c = s_off[e]; s_off[e] = run; run += c; }
            const uint32_t base = run ? (uint32_t)atomicAdd(cnt, (unsigned long long)run) : 0u;
#pragma unroll
            for (int e = 0; e < kKmExpU * NW; ++e) s_off[e] += base;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kKmExpU; ++u) {
            if (!sel[u]) continue;
            const int64_t i = t + u * kKmExpBlock + threadIdx.x;
            const int64_t pos = ob + (int64_t)s_off[u * NW + wv] + __popcll(m[u] & lt);
            const uint4 r0 = d.rec[2 * i];
            res.key[pos] = r0.x;
            res.tag[0][pos] = (uint8_t)r0.y;
            res.val[0][pos] = (int64_t)(((uint64_t)r0.w << 32) | r0.z);
            if (n_aggs > 1) {
                const uint4 r1 = d.rec[2 * i + 1];
                res.tag[1][pos] = (uint8_t)(r0.y >> 8);
                res.val[1][pos] = (int64_t)(((uint64_t)r1.y << 32) | r1.x);
                if (n_aggs > 2) {
                    res.tag[2][pos] = (uint8_t)(r0.y >> 16);
                    res.val[2][pos] = (int64_t)(((uint64_t)r1.w << 32) | r1.z);
                }
            }
        }
        __syncthreads();   // s_off is rewritten by the next tile
    }
}
#endif

// ---------------------------------------------------------------- one window over a huge key space (C5 shape)
// A window whose every row is a member and whose single value column is read without validity needs the rows
// grouped by key, in no particular order inside a key (count / min / max / order statistics are order-free; the f64
// sums stay within the north-star tolerance). Two MSD partition passes on 8-bit digits of the dense key
// (k_grp_hist + k_grp_scatter: per 4096-row tile an LDS counting sort, one global reservation per (tile, digit),
// runs written with consecutive lanes on consecutive addresses) cut the span into sub-buckets of 2^s2 keys; then
// one workgroup per sub-bucket (k_grp_walk) loads its rows into LDS, counting-sorts them by key, and one thread per
// key folds its LDS segment, sorts it in place for the order statistics, tests HAVING and emits (block-compacted).
// 4 + 24 + 4 + 24 + 12 B per row instead of the radix sort's 3 passes + a random gather + a strided per-key walk.
constexpr int kGrpTile = 4096;
constexpr int kGrpBlock = 256;
constexpr int kGrpCap = 4096;         // rows of one sub-bucket held in LDS by k_grp_walk (host-checked)
constexpr int kGrpWalkBlock = 256;    // k_grp_walk workgroup (256 threads; R rows each)

struct GrpTile {
    int64_t start;                    // first row of the tile in the pass's input
    int32_t len;                      // rows (<= kGrpTile)
    int32_t pre;                      // digit index offset (level 2: bucket * 256)
};

// totals per (replica, pre + digit) of the tile's rows with key < K. A tile counts into replica blockIdx.x % rep
// (stride 256): the first pass's tiles all share one set of 256 digits, and 64 replicas keep every counter's global
// atomics (here and in k_grp_scatter's reservations) from serialising on one address; the host lays the replicas'
// regions out consecutively inside each digit's region.
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(kGrpBlock) void k_grp_hist(const uint32_t* __restrict__ keys, const GrpTile* __restrict__ tiles,
                                                        int shift, uint32_t dmask, uint32_t K, int rep, unsigned int* __restrict__ tot) {
    __shared__ unsigned int h[256];
    const GrpTile t = tiles[blockIdx.x];
    h[threadIdx.x] = 0;
    __syncthreads();
    constexpr int R = kGrpTile / kGrpBlock;
    uint32_t k[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {                 // all of the tile's loads in flight before the first atomic
        const int i = threadIdx.x + j * kGrpBlock;
        k[j] = i < t.len ? keys[t.start + i] : K;
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (k[j] < K) atomicAdd(&h[(k[j] >> shift) & dmask], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&tot[(blockIdx.x % rep) * 256 + t.pre + threadIdx.x], h[threadIdx.x]);
}
#endif

// rows of a tile -> their (replica, pre + digit) region: base[] exclusive region starts, cur[] reservation cursors.
// 512 threads (8 rows each): the 52 KB of LDS staging allow two workgroups per CU, so 16 waves keep loads in flight
// (256 threads left 8 waves per CU and ran the pass at 2.7 TB/s). The digit is re-derived from the staged key.
// POS: the rows also carry their span position (pass 1: the row index itself; pass 2: the pass-1 output), for the
// key-major path of range windows (km_msd), whose walk needs the rows of a key in position order.
constexpr int kGrpScatBlock = 512;
template <bool POS>
__global__ __launch_bounds__(kGrpScatBlock) void k_grp_scatter(const uint32_t* __restrict__ keys, const int64_t* __restrict__ vals,
                                                               const GrpTile* __restrict__ tiles, int shift, uint32_t dmask,
                                                               uint32_t K, int rep,
                                                               const int64_t* __restrict__ base, unsigned int* __restrict__ cur,
                                                               uint32_t* __restrict__ okeys, int64_t* __restrict__ ovals,
                                                               const uint32_t* __restrict__ pos, uint32_t* __restrict__ opos) {
    __shared__ unsigned int h[256], lofs[257];
    __shared__ int64_t gb[256];
    __shared__ uint32_t s_key[kGrpTile];
    __shared__ int64_t s_val[kGrpTile];
    __shared__ uint32_t s_pos[POS ? kGrpTile : 1];
    __shared__ unsigned int wsum[kGrpScatBlock / 64];
    const GrpTile t = tiles[blockIdx.x];
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    __syncthreads();
    constexpr int R = kGrpTile / kGrpScatBlock;
    uint32_t k[R], ps[R];
    int64_t v[R];
    int rk[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int i = threadIdx.x + j * kGrpScatBlock;
        rk[j] = -1;
        if (i >= t.len) continue;
        k[j] = keys[t.start + i];
        v[j] = vals[t.start + i];
        if (POS) ps[j] = pos ? pos[t.start + i] : (uint32_t)(t.start + i);
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (threadIdx.x + j * kGrpScatBlock < t.len && k[j] < K) rk[j] = (int)atomicAdd(&h[(k[j] >> shift) & dmask], 1u);
    __syncthreads();
    if (threadIdx.x < 256) {
        const unsigned int c = h[threadIdx.x];
        const int ci = (int)(blockIdx.x % rep) * 256 + t.pre + threadIdx.x;
        if (c) gb[threadIdx.x] = base[ci] + (int64_t)atomicAdd(&cur[ci], c);
        lofs[threadIdx.x] = c;
    }
    __syncthreads();
    block_excl_scan<kGrpScatBlock>(lofs, 256, wsum);   // lofs[256] = rows kept
#pragma unroll
    for (int j = 0; j < R; ++j) {
        if (rk[j] < 0) continue;
        const unsigned int p = lofs[(k[j] >> shift) & dmask] + (unsigned int)rk[j];
        s_key[p] = k[j];
        s_val[p] = v[j];
        if (POS) s_pos[p] = ps[j];
    }
    __syncthreads();
    const unsigned int m = lofs[256];
    for (unsigned int p = threadIdx.x; p < m; p += kGrpScatBlock) {
        const uint32_t kk = s_key[p];
        const unsigned int d = (kk >> shift) & dmask;
        const int64_t dst = gb[d] + (int64_t)(p - lofs[d]);
        okeys[dst] = kk;
        ovals[dst] = s_val[p];
        if (POS) opos[dst] = s_pos[p];
    }
}

// km_msd's last step, one workgroup per sub-bucket of 2^s2 keys (the two k_grp_scatter<true> passes grouped the rows
// by key >> s2, in no order inside): the sub-bucket's rows are counted by key and placed in LDS in key order, each
// key's segment is insertion-sorted by span position (one thread per key), and the rows go back to the same range
// sorted by (key, position) — the order the radix sort gave — with kstart[key] for every key of the sub-bucket and
// the longest key run (maxrun). Dynamic LDS: (nk + 1) counters + cursors, then m positions and m values (m <=
// kKmFixCap). The sorted keys are not written back: kstart is all the walk reads of them.
constexpr int kKmFixBlock = 256;
constexpr int kKmFixCap = 2048;   // rows of one sub-bucket k_kmsd_fix holds in LDS (more: the radix-sort fallback)
#ifndef EK_NO_PLAIN_KERNELS
// km_msd's offsets on the device (no host round trip): pass 1's per-(replica, digit) counts -> region starts in digit-major,
// replica-minor order, and pass 2's tiles (each digit's rows cut into kGrpTile pieces, digit << w2 as their sub-bucket
// base; the tiles past the last are empty). One workgroup of 1024 threads; ntc = the tile list's capacity.
// 256-wide exclusive scan of s[0..255] into s (s[256] = total) by the first 4 waves (all 1024 threads call it)
__device__ __forceinline__ void scan256(int64_t* s) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    __shared__ int64_t wsum[4];
    int64_t x = t < 256 ? s[t] : 0, v = x;
    for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(v, o, 64); if (lane >= o) v += y; }
    if (t < 256 && lane == 63) wsum[w] = v;
    __syncthreads();
    if (t < 256) {
        int64_t base = 0;
        for (int k = 0; k < w; ++k) base += wsum[k];
        s[t] = base + v - x;
        if (t == 255) s[256] = base + v;
    }
    __syncthreads();
}
__global__ __launch_bounds__(1024) void k_msd_plan1(const unsigned int* __restrict__ tot1, int rep, int w2, int ntc,
                                                    int64_t* __restrict__ base1, GrpTile* __restrict__ tiles2) {
    __shared__ int64_t s_cnt[257], s_nt[257];
    __shared__ unsigned int s_rep[64][256];   // replica counts, then their exclusive prefixes inside each digit
    const int t = threadIdx.x;
    for (int i = t; i < rep * 256; i += 1024) s_rep[i >> 8][i & 255] = tot1[i];
    __syncthreads();
    if (t < 256) {
        unsigned int c = 0;
        for (int q = 0; q < rep; ++q) { const unsigned int x = s_rep[q][t]; s_rep[q][t] = c; c += x; }
        s_cnt[t] = c;
        s_nt[t] = ((int64_t)c + kGrpTile - 1) / kGrpTile;
    }
    __syncthreads();
    scan256(s_cnt);
    scan256(s_nt);
    for (int i = t; i < rep * 256; i += 1024) base1[i] = s_cnt[i & 255] + s_rep[i >> 8][i & 255];
    if (t < 256) {
        const int64_t c_end = s_cnt[t + 1];
        int64_t k = s_nt[t];
        for (int64_t x = s_cnt[t]; x < c_end; x += kGrpTile, ++k)
            tiles2[k] = GrpTile{x, (int32_t)min<int64_t>(kGrpTile, c_end - x), t << w2};
    }
    for (int64_t k = s_nt[256] + t; k < ntc; k += 1024) tiles2[k] = GrpTile{0, 0, 0};
}
// pass 2's sub-bucket counts -> exclusive starts base2[nsub + 1]; a sub-bucket above cap rows sets over[0], and
// over[1] gets the largest sub-bucket (atomicMax)
__global__ __launch_bounds__(1024) void k_msd_plan2(const unsigned int* __restrict__ tot2, int nsub, int64_t* __restrict__ base2,
                                                    unsigned int cap, unsigned int* __restrict__ over) {
    // rounds of 8192 counts staged through LDS with coalesced loads / stores (one thread's 8 consecutive counts summed
    // from LDS, a block scan, the exclusive starts written back coalesced): no strided global access
    constexpr int kR = 8192, kPer = kR / 1024;
    __shared__ unsigned int s[kR];
    __shared__ int64_t wsum[16];
    __shared__ int64_t s_run;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_run = 0;
    unsigned int mx = 0;
    for (int c0 = 0; c0 < nsub; c0 += kR) {
        const int n = min(kR, nsub - c0);
        for (int i = t; i < kR; i += 1024) s[i] = i < n ? tot2[c0 + i] : 0u;
        __syncthreads();
        int64_t sm = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) { const unsigned int x = s[t * kPer + k]; sm += x; mx = max(mx, x); }
        int64_t v = sm;
        for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(v, o, 64); if (lane >= o) v += y; }
        if (lane == 63) wsum[w] = v;
        __syncthreads();
        int64_t r = v - sm;
        for (int k = 0; k < w; ++k) r += wsum[k];
        const int64_t run0 = s_run;
        // exclusive starts inside the round (< 2^32: a round holds at most 8192 sub-buckets of < 2^32 rows in all,
        // host-checked batch bound 2^31) back into LDS, then out with the round's base
        uint32_t rr = (uint32_t)r;
#pragma unroll
        for (int k = 0; k < kPer; ++k) { const unsigned int x = s[t * kPer + k]; s[t * kPer + k] = rr; rr += x; }
        __syncthreads();
        for (int i = t; i < n; i += 1024) base2[c0 + i] = run0 + (int64_t)s[i];
        if (t == 1023) s_run = run0 + r + sm;
        __syncthreads();
    }
    if (t == 0) base2[nsub] = s_run;
    unsigned int m = mx;
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
    if (lane == 0 && m) {
        if (m > cap) atomicOr(over, 1u);
        atomicMax(over + 1, m);
    }
}

__global__ __launch_bounds__(kKmFixBlock) void k_kmsd_fix(const int64_t* __restrict__ base2, int nsub, int s2, uint32_t K,
                                                          const uint32_t* __restrict__ keys, uint32_t* __restrict__ pos,
                                                          int64_t* __restrict__ vals, uint32_t* __restrict__ kstart,
                                                          unsigned int* __restrict__ maxrun, int cap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int sb = blockIdx.x;
    const int64_t b0 = base2[sb], b1 = base2[sb + 1];
    const int m = (int)(b1 - b0);
    if (m > cap) return;   // k_msd_plan2 flagged it: the caller falls back
    const int nk = 1 << s2;
    uint32_t* cnt = (uint32_t*)smem;                      // [nk + 1] -> exclusive starts
    uint32_t* cur = cnt + nk + 1;                         // [nk]
    int64_t* s_val = (int64_t*)(smem + (((size_t)(2 * nk + 1) * 4 + 15) & ~(size_t)15));   // [m]
    uint32_t* s_pos = (uint32_t*)(s_val + cap);           // [m <= cap]
    __shared__ unsigned int wsum[kKmFixBlock / 64];
    (void)cur;
    for (int k = threadIdx.x; k <= nk; k += kKmFixBlock) cnt[k] = 0;
    __syncthreads();
    // one read of the sub-bucket: every row's (local key, position, value) in registers, its rank within its key from
    // the LDS count, then its slot = the key's start + rank
    constexpr int RR = kKmFixCap / kKmFixBlock;
    uint32_t kl[RR], pp[RR], rk[RR];
    int64_t vv[RR];
#pragma unroll
    for (int j = 0; j < RR; ++j) {
        const int i = threadIdx.x + j * kKmFixBlock;
        if (i < m) { kl[j] = keys[b0 + i] & (uint32_t)(nk - 1); pp[j] = pos[b0 + i]; vv[j] = vals[b0 + i]; }
    }
#pragma unroll
    for (int j = 0; j < RR; ++j)
        if (threadIdx.x + j * kKmFixBlock < m) rk[j] = atomicAdd(&cnt[kl[j]], 1u);
    __syncthreads();
    block_excl_scan<kKmFixBlock>(cnt, nk, wsum);
#pragma unroll
    for (int j = 0; j < RR; ++j) {
        if (threadIdx.x + j * kKmFixBlock >= m) continue;
        const uint32_t d = cnt[kl[j]] + rk[j];
        s_pos[d] = pp[j];
        s_val[d] = vv[j];
    }
    __syncthreads();
    unsigned int mr = 0;
    for (int k = threadIdx.x; k < nk; k += kKmFixBlock) {
        const int a = (int)cnt[k], e = (int)cnt[k + 1];
        for (int i = a + 1; i < e; ++i) {   // insertion sort by position (a key holds ~n / K rows)
            const uint32_t pp = s_pos[i];
            const int64_t vv = s_val[i];
            int j = i - 1;
            while (j >= a && s_pos[j] > pp) { s_pos[j + 1] = s_pos[j]; s_val[j + 1] = s_val[j]; --j; }
            s_pos[j + 1] = pp;
            s_val[j + 1] = vv;
        }
        mr = max(mr, (unsigned int)(e - a));
        const int64_t g = ((int64_t)sb << s2) + k;
        if (g < (int64_t)K) kstart[g] = (uint32_t)(b0 + a);
    }
    if (sb == nsub - 1 && threadIdx.x == 0) kstart[K] = (uint32_t)base2[nsub];
    for (int o = 32; o > 0; o >>= 1) mr = max(mr, (unsigned int)__shfl_xor((int)mr, o, 64));
    if ((threadIdx.x & 63) == 0 && mr) atomicMax(maxrun, mr);
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += kKmFixBlock) {   // (the sorted keys themselves: kstart holds them)
        pos[b0 + i] = s_pos[i];
        vals[b0 + i] = s_val[i];
    }
}
#endif

struct GrpDesc {
    const int64_t* base2;             // [nsub + 1] sub-bucket row ranges in the level-2 output
    const uint32_t* keys;
    const int64_t* vals;
    int s1, s2;                       // key = (bucket << s1) | (digit2 << s2) | local key
    int64_t obase;                    // the window's result region
    int32_t widx;
    int32_t pad;
};

// R: rows per thread held in registers (R * kGrpWalkBlock >= the launch's largest sub-bucket, host-chosen). With
// SORT, every row's rank inside its key's segment (values below it, ties broken by position) is counted from the
// grouped LDS copy with independent reads, then the row is stored at its rank: the segments come out sorted with no
// dependent per-key insertion chain (the time of a wave is its longest segment, not that segment squared).
// HV: the plan has a HAVING (without one the kernel carries no interpreter: 123 -> 85 VGPRs, 5 waves/SIMD).
template <bool SORT, bool ISF, int R, bool HV>
__global__ __launch_bounds__(kGrpWalkBlock) void k_grp_walk(DPlan* __restrict__ pp, GrpDesc g, Results res) {
    extern __shared__ __attribute__((aligned(16))) unsigned char g_lds[];
    const DPlan& p = *pp;
    const int nloc = 1 << g.s2;                                   // keys of a sub-bucket (<= 2048)
    int64_t* s_b = (int64_t*)g_lds;                               // [R * kGrpWalkBlock] values grouped by key
    unsigned int* s_off = (unsigned int*)(s_b + R * kGrpWalkBlock);   // [nloc + 1] per-key counts -> offsets
    __shared__ unsigned int wsum[kGrpWalkBlock / 64];
    __shared__ uint32_t esh[20];
    const int sb = blockIdx.x;
    const int64_t r0 = g.base2[sb], r1 = g.base2[sb + 1];
    const int m = (int)(r1 - r0);                                 // <= R * kGrpWalkBlock (host-checked)
    if (m <= 0) return;                                           // uniform: no row, no emission
    const uint32_t kbase = ((uint32_t)(sb >> 8) << g.s1) | ((uint32_t)(sb & 255) << g.s2);
    const uint32_t mask = (uint32_t)nloc - 1u;
    for (int i = threadIdx.x; i < nloc; i += kGrpWalkBlock) s_off[i] = 0;
    __syncthreads();
    // counting sort by local key: every row's key and value are loaded into registers up front (all loads in flight
    // at once instead of one latency per strided iteration), ranked by one LDS atomic, then placed after the scan
    static_assert(R * kGrpWalkBlock <= kGrpCap, "sub-bucket rows beyond the LDS slab");
    uint32_t rkey[R];
    int64_t rval[R];
    unsigned int rrk[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int i = threadIdx.x + j * kGrpWalkBlock;
        if (i < m) { rkey[j] = g.keys[r0 + i] & mask; rval[j] = g.vals[r0 + i]; }
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (threadIdx.x + j * kGrpWalkBlock < m) rrk[j] = atomicAdd(&s_off[rkey[j]], 1u);
    __syncthreads();
    block_excl_scan<kGrpWalkBlock>(s_off, nloc, wsum);
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (threadIdx.x + j * kGrpWalkBlock < m) s_b[s_off[rkey[j]] + rrk[j]] = rval[j];
    __syncthreads();
    constexpr bool isf = ISF;     // the value column's type (host-dispatched)
    if constexpr (SORT) {
        // rank of each row inside its segment by ordered bits; equal ordered bits are equal values, so the tie
        // order only has to make the ranks a permutation
#pragma unroll
        for (int j = 0; j < R; ++j) {
            if (threadIdx.x + j * kGrpWalkBlock >= m) continue;
            const int a = (int)s_off[rkey[j]], b = (int)s_off[rkey[j] + 1];
            const int me = a + (int)rrk[j];
            const uint64_t ox = isf ? f64_to_ord(__longlong_as_double(rval[j])) : i64_to_ord(rval[j]);
            unsigned int r = 0;
            for (int q = a; q < b; ++q) {
                const int64_t y = s_b[q];
                const uint64_t oy = isf ? f64_to_ord(__longlong_as_double(y)) : i64_to_ord(y);
                r += (oy < ox || (oy == ox && q < me)) ? 1u : 0u;
            }
            rrk[j] = (unsigned int)a + r;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (threadIdx.x + j * kGrpWalkBlock < m) s_b[rrk[j]] = rval[j];
        __syncthreads();
    }
    const int fl[1] = {p.vc_flags[0]};
    for (int kb = 0; kb < nloc; kb += kGrpWalkBlock) {
        const int lk = kb + threadIdx.x;
        bool present = false;
        Part<1> part{};
        uint64_t sres[kMaxSortAggs];
        uint8_t stag[kMaxSortAggs];
#pragma unroll
        for (int a = 0; a < kMaxSortAggs; ++a) { sres[a] = 0; stag[a] = EK_TAG_NULL; }
        if (lk < nloc) {
            const int j0 = (int)s_off[lk], j1 = (int)s_off[lk + 1];
            if (j1 > j0) {
                int64_t vc[1] = {0}, is[1] = {0};
                double fs[1] = {0.0}, m2[1] = {0.0};
                uint64_t mn[1] = {~0ull}, mx[1] = {0ull};
                for (int j = j0; j < j1; ++j) {
                    const int64_t raw = s_b[j];
                    const double x = isf ? __longlong_as_double(raw) : (double)raw;
                    const uint64_t o = isf ? f64_to_ord(x) : i64_to_ord(raw);
                    vc[0]++;
                    is[0] = (int64_t)((uint64_t)is[0] + (uint64_t)raw);
                    fs[0] = __dadd_rn(fs[0], x);
                    mn[0] = o < mn[0] ? o : mn[0];
                    mx[0] = o > mx[0] ? o : mx[0];
                }
                if ((fl[0] & NEED_M2) && vc[0] > 0) {
                    const double mean = __ddiv_rn(fs[0], (double)vc[0]);
                    for (int j = j0; j < j1; ++j) {
                        const double dd = __dsub_rn(isf ? __longlong_as_double(s_b[j]) : (double)s_b[j], mean);
                        m2[0] = __dadd_rn(m2[0], __dmul_rn(dd, dd));
                    }
                }
                part_merge(p, part, j1 - j0, vc, is, fs, m2, mn, mx);
                bool agg_err = false;
                if constexpr (SORT) {   // the segment is sorted ascending by ordered bits (rank placement above)
#pragma unroll
                    for (int a = 0; a < kMaxSortAggs; ++a) {
                        if (a >= p.n_sagg) continue;
                        const int ka = p.sagg_agg[a];
                        order_stat(p.agg_fn[ka], isf, p.agg_p[ka], (int64_t)(j1 - j0),
                                   [&](int64_t r) {
                                       const int64_t x = s_b[j0 + (int)r];
                                       return isf ? f64_to_ord(__longlong_as_double(x)) : i64_to_ord(x);
                                   },
                                   &sres[a], &stag[a]);
                        agg_err |= stag[a] == kTagErr;
                    }
                }
                const SortRes sr{sres, stag, 0, 1};
                if (agg_err) {
                    atomicOr(&res.win_err[g.widx], EK_WIN_AGG_ERROR);
                    int ea = 0;   // the first order statistic that failed
                    for (int a = p.n_sagg - 1; a >= 0; --a) if (sel(stag, a) == kTagErr) ea = a;
                    if (res.aslot) atomicMax(&res.aslot[g.widx], kMaxSortAggs - ea);
                } else {
                    int hv = 1;
                    if constexpr (HV) hv = km_having(p, part, SORT ? &sr : nullptr);
                    if (hv < 0) {
                        atomicOr(&res.win_err[g.widx], EK_WIN_HAVING_ERROR);
                        if (res.wwit)
                            wit_having(&res.wwit[2 * g.widx + 1], kbase | (uint32_t)lk, p,
                                       [&](int q) { return agg_value(p, part, q, SORT ? &sr : nullptr); });
                    }
                    present = hv > 0;
                }
            }
        }
        // block-compacted emission of this round's kept keys
        const unsigned long long msk = __ballot(present);
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        if (!__syncthreads_or(present)) continue;
        if (lane == 0) esh[wv] = (uint32_t)__popcll(msk);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int w = 0; w < kGrpWalkBlock / 64; ++w) { const uint32_t c = esh[w]; esh[w] = run; run += c; }
            esh[16] = (uint32_t)atomicAdd((unsigned long long*)&res.win_cnt[g.widx], (unsigned long long)run);
        }
        __syncthreads();
        if (present) {   // the row's values are computed only now: nothing of them lives across the barriers
            int64_t ov[EK_MAX_AGGS];
            uint8_t ot[EK_MAX_AGGS];
            const SortRes sr{sres, stag, 0, 1};
            km_row(p, part, SORT ? &sr : nullptr, ov, ot);
            const int64_t pos = g.obase + (int64_t)esh[16] + esh[wv] + __popcll(msk & ((1ull << lane) - 1ull));
            res.key[pos] = kbase | (uint32_t)lk;
#pragma unroll
            for (int q = 0; q < EK_MAX_AGGS; ++q) {
                if (q >= p.n_aggs) break;
                res.tag[q][pos] = ot[q];
                res.val[q][pos] = ov[q];
            }
        }
        __syncthreads();
    }
}
// dynamic LDS of k_grp_walk<.., R>: the R * kGrpWalkBlock value slab, then the nloc + 1 offsets
inline size_t grp_walk_lds(int s2, int R) { return (size_t)R * kGrpWalkBlock * 8 + ((size_t)(1 << s2) + 1) * 4 + 16; }


// one workgroup per window: exclusive scan of its per-block counts in place; the total is the window's row count
#ifndef EK_NO_PLAIN_KERNELS
__global__ __launch_bounds__(1024) void k_km_scan(KmDesc d, Results res) {
    const int k = blockIdx.x;
    uint32_t* c = d.bcnt + (int64_t)k * (d.nblk + 1);
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base < d.nblk; base += 1024) {
        const int i = base + threadIdx.x;
        const uint32_t x0 = i < d.nblk ? c[i] : 0u;
        uint32_t x = x0;
        for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        uint32_t wb = 0;
        for (int w = 0; w < wv; ++w) wb += s_w[w];
        const uint32_t carry = s_carry;
        if (i < d.nblk) c[i] = carry + wb + x - x0;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = carry + wb + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        c[d.nblk] = s_carry;
        if (s_carry && !d.skend) atomicAdd((unsigned long long*)&res.win_cnt[d.widx[k]], (unsigned long long)s_carry);
    }
}
#endif

}  // namespace ek
