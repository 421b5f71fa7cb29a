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

namespace ek {

struct BatchStats {
    int64_t min_ts;
    int64_t max_ts;
    int64_t n_accepted;
    int64_t min_accepted;
    int32_t unsorted;
    int32_t pad;
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
__global__ __launch_bounds__(kBlock) void k_stats(const int64_t* __restrict__ ts, int64_t n, BatchStats* st) {
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    int uns = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock * 2;
    for (int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 2; i < n; i += stride) {
        int64_t a = ts[i];
        int64_t b = (i + 1 < n) ? ts[i + 1] : a;
        int64_t p = (i > 0) ? ts[i - 1] : a;
        uns |= (a < p) | (b < a);
        mn = min(mn, min(a, b));
        mx = max(mx, max(a, b));
    }
    mn = wave_min64(mn);
    mx = wave_max64(mx);
    uns = __any(uns);
    if ((threadIdx.x & 63) == 0) {
        atomicMin((long long*)&st->min_ts, (long long)mn);
        atomicMax((long long*)&st->max_ts, (long long)mx);
        if (uns) atomicOr(&st->unsorted, 1);
    }
}

// ---------------------------------------------------------------- late-event drop (out-of-order batches)
constexpr int kAccPerThread = 16;
constexpr int kAccChunk = kBlock * kAccPerThread;  // 4096 events per block

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

// exclusive prefix max over chunk maxima, seeded with the carried stream max (single workgroup)
__global__ __launch_bounds__(1024) void k_scan_max(int64_t* cmax, int nch, int64_t seed) {
    __shared__ int64_t part[1024];
    int per = (nch + 1023) / 1024;
    int b = threadIdx.x * per, e = min(nch, b + per);
    int64_t m = INT64_MIN;
    for (int i = b; i < e; ++i) m = max(m, cmax[i]);
    part[threadIdx.x] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = seed;
        for (int t = 0; t < 1024; ++t) { int64_t v = part[t]; part[t] = run; run = max(run, v); }
    }
    __syncthreads();
    int64_t run = part[threadIdx.x];
    for (int i = b; i < e; ++i) { int64_t v = cmax[i]; cmax[i] = run; run = max(run, v); }
}

__global__ __launch_bounds__(kBlock) void k_accept(const int64_t* __restrict__ ts, int64_t n, const int64_t* excl,
                                                   int64_t late_tol, uint8_t* acc, BatchStats* st) {
    __shared__ int64_t tmax[kBlock];
    int64_t base = (int64_t)blockIdx.x * kAccChunk + (int64_t)threadIdx.x * kAccPerThread;
    int64_t v[kAccPerThread];
    int64_t lm = INT64_MIN;
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) {
        int64_t i = base + k;
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
    int64_t cnt = 0, mn = INT64_MAX;
#pragma unroll
    for (int k = 0; k < kAccPerThread; ++k) {
        int64_t i = base + k;
        if (i < n) {
            // W_{i-1} = M_{i-1} - lateTol; no watermark yet (run == INT64_MIN) accepts everything
            bool ok = (run == INT64_MIN) || (v[k] >= run - late_tol);
            acc[i] = ok ? 1 : 0;
            if (ok) { cnt++; mn = min(mn, v[k]); }
            run = max(run, v[k]);
        }
    }
    mn = wave_min64(mn);
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd((unsigned long long*)&st->n_accepted, (unsigned long long)cnt);
        atomicMin((long long*)&st->min_accepted, (long long)mn);
    }
}

// first index in [lo, hi) with ts >= bound[k] (sorted batches)
__global__ void k_lower_bound(const int64_t* __restrict__ ts, int64_t lo, int64_t hi, const int64_t* bound, int nb,
                              int64_t* out) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nb) return;
    int64_t x = bound[k], a = lo, b = hi;
    while (a < b) { int64_t m = (a + b) >> 1; if (ts[m] < x) a = m + 1; else b = m; }
    out[k] = a;
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
};

__device__ __forceinline__ int part_of(const DPlan& p, const DBatch& b, const PaneGrid& g, const GroupDesc& gd,
                                       const uint8_t* acc, int64_t i, int64_t* q_out) {
    if (gd.has_accept && !acc[i]) return -1;
    int64_t q = pane_of(g, ((const int64_t*)b.col[p.ts_col])[i]);
    int64_t rel = q - gd.q_lo;
    if (q < 0 || rel < 0 || rel >= gd.n_panes) return -1;
    uint32_t key = p.key_col >= 0 ? ((const uint32_t*)b.col[p.key_col])[i] : 0u;
    if (key >= p.num_keys && p.key_col >= 0) return -1;
    *q_out = q;
    return (int)rel * gd.nb + (int)(key >> gd.kbits);
}

__global__ __launch_bounds__(kBlock) void k_hist(DPlan* __restrict__ pp, DBatch b, PaneGrid g, GroupDesc gd,
                                                 const uint8_t* __restrict__ acc, uint32_t* __restrict__ hist,
                                                 int32_t* __restrict__ pane_err) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lh[];
    const DPlan& p = *pp;
    for (int k = threadIdx.x; k < gd.np; k += kBlock) lh[k] = 0;
    __syncthreads();
    int64_t c0 = gd.lo + (int64_t)blockIdx.x * gd.chunk;
    int64_t c1 = min(gd.hi, c0 + gd.chunk);
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock) {
        int64_t q;
        int pid = part_of(p, b, g, gd, acc, i, &q);
        if (pid < 0) continue;
        int w = where_decide(p, b, i);
        if (w < 0) { atomicOr(&pane_err[q % gd.ring], EK_WIN_WHERE_ERROR); continue; }
        if (w == 0) continue;
        atomicAdd(&lh[pid], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < gd.np; k += kBlock) hist[(int64_t)k * gd.nch + blockIdx.x] = lh[k];
}

// ---- exclusive scan (3 phase) over u32 counts -> u32 offsets
constexpr int kScanTile = 4096;
__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t* __restrict__ in, int64_t n, uint32_t* tile_sum) {
    int64_t base = (int64_t)blockIdx.x * kScanTile;
    uint32_t s = 0;
    for (int k = threadIdx.x; k < kScanTile; k += kBlock) {
        int64_t i = base + k;
        if (i < n) s += in[i];
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ uint32_t w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

__global__ __launch_bounds__(1024) void k_scan_tiles(uint32_t* tile_sum, int nt) {
    __shared__ uint32_t part[1024];
    int per = (nt + 1023) / 1024;
    int b = threadIdx.x * per, e = min(nt, b + per);
    uint32_t s = 0;
    for (int i = b; i < e; ++i) s += tile_sum[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int i = b; i < e; ++i) { uint32_t v = tile_sum[i]; tile_sum[i] = run; run += v; }
}

__global__ __launch_bounds__(kBlock) void k_scan_down(const uint32_t* __restrict__ in, int64_t n,
                                                      const uint32_t* __restrict__ tile_off, uint32_t* __restrict__ out) {
    // each thread owns 16 consecutive elements of the 4096-element tile
    __shared__ uint32_t ts[kBlock];
    int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * 16;
    uint32_t v[16];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) { int64_t i = base + k; v[k] = i < n ? in[i] : 0; s += v[k]; }
    ts[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < kBlock; o <<= 1) {
        uint32_t t = threadIdx.x >= o ? ts[threadIdx.x - o] : 0;
        __syncthreads();
        ts[threadIdx.x] += t;
        __syncthreads();
    }
    uint32_t run = tile_off[blockIdx.x] + (threadIdx.x ? ts[threadIdx.x - 1] : 0);
#pragma unroll
    for (int k = 0; k < 16; ++k) { int64_t i = base + k; if (i < n) out[i] = run; run += v[k]; }
}

struct Staging {
    uint16_t* klo;
    int64_t* val[kMaxVC];
    uint8_t* valid[kMaxVC];
    uint32_t nullable_mask;   // bit v: staging carries validity for value column v
};

__global__ __launch_bounds__(kBlock) void k_scatter(DPlan* __restrict__ pp, DBatch b, PaneGrid g, GroupDesc gd,
                                                    const uint8_t* __restrict__ acc, const uint32_t* __restrict__ off,
                                                    Staging st) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    const DPlan& p = *pp;
    for (int k = threadIdx.x; k < gd.np; k += kBlock) cur[k] = off[(int64_t)k * gd.nch + blockIdx.x];
    __syncthreads();
    const uint32_t kmask = (1u << gd.kbits) - 1u;
    int64_t c0 = gd.lo + (int64_t)blockIdx.x * gd.chunk;
    int64_t c1 = min(gd.hi, c0 + gd.chunk);
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock) {
        int64_t q;
        int pid = part_of(p, b, g, gd, acc, i, &q);
        if (pid < 0) continue;
        if (where_decide(p, b, i) != 1) continue;
        uint32_t pos = atomicAdd(&cur[pid], 1u);
        uint32_t key = p.key_col >= 0 ? ((const uint32_t*)b.col[p.key_col])[i] : 0u;
        st.klo[pos] = (uint16_t)(key & kmask);
        for (int v = 0; v < p.n_vc; ++v) {
            int c = p.vc_col[v];
            st.val[v][pos] = ((const int64_t*)b.col[c])[i];
            if (st.nullable_mask & (1u << v)) st.valid[v][pos] = col_valid(b, c, i) ? 1 : 0;
        }
    }
}

// ---------------------------------------------------------------- per-partition aggregation
// LDS layout per partition (kk = 1 << kbits keys): cnt u32[kk], then per value column the fields it needs.
struct LdsLayout {
    int32_t off_cnt;
    int32_t off_vcnt[kMaxVC];
    int32_t off_sum[kMaxVC];
    int32_t off_min[kMaxVC];
    int32_t off_max[kMaxVC];
    int32_t off_m2[kMaxVC];
    int32_t off_fsum[kMaxVC];
    int32_t bytes;
};

__global__ __launch_bounds__(kBlock) void k_agg(DPlan* __restrict__ pp, GroupDesc gd, LdsLayout lay,
                                                const uint32_t* __restrict__ off, Staging st, DState ds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const DPlan& p = *pp;
    const int pid = blockIdx.x;
    const int kk = 1 << gd.kbits;
    const int rel = pid / gd.nb, bucket = pid % gd.nb;
    const int64_t q = gd.q_lo + rel;
    const int64_t slot = q % gd.ring;
    const uint32_t s0 = off[(int64_t)pid * gd.nch];
    const uint32_t s1 = off[(int64_t)(pid + 1) * gd.nch];   // off has np*nch+1 entries (last = total)
    if (s1 == s0) return;   // nothing to merge

    uint32_t* lcnt = (uint32_t*)(lds + lay.off_cnt);
    for (int k = threadIdx.x; k < lay.bytes / 4; k += kBlock) ((uint32_t*)lds)[k] = 0;
    __syncthreads();
    for (uint32_t i = s0 + threadIdx.x; i < s1; i += kBlock) {
        int kl = st.klo[i];
        atomicAdd(&lcnt[kl], 1u);
        for (int v = 0; v < p.n_vc; ++v) {
            if ((st.nullable_mask & (1u << v)) && !st.valid[v][i]) continue;
            const int f = p.vc_flags[v];
            int64_t raw = st.val[v][i];
            if (f & NEED_CNT) atomicAdd(&((uint32_t*)(lds + lay.off_vcnt[v]))[kl], 1u);
            if (p.vc_is_float[v]) {
                double x = __longlong_as_double(raw);
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
    __syncthreads();
    bool need_m2 = false;
    for (int v = 0; v < p.n_vc; ++v) need_m2 |= (p.vc_flags[v] & NEED_M2) != 0;
    if (need_m2) {
        // second pass over the (L2-resident) run: Σ (x - mean)^2 with this partial's mean (stats._variance shape)
        for (uint32_t i = s0 + threadIdx.x; i < s1; i += kBlock) {
            int kl = st.klo[i];
            for (int v = 0; v < p.n_vc; ++v) {
                if (!(p.vc_flags[v] & NEED_M2)) continue;
                if ((st.nullable_mask & (1u << v)) && !st.valid[v][i]) continue;
                int64_t raw = st.val[v][i];
                double x = p.vc_is_float[v] ? __longlong_as_double(raw) : (double)raw;
                double n = (p.vc_flags[v] & NEED_CNT) ? (double)((uint32_t*)(lds + lay.off_vcnt[v]))[kl] : (double)lcnt[kl];
                double s = p.vc_is_float[v] ? ((double*)(lds + lay.off_sum[v]))[kl] : ((double*)(lds + lay.off_fsum[v]))[kl];
                double d = __dsub_rn(x, __ddiv_rn(s, n));
                atomicAdd(&((double*)(lds + lay.off_m2[v]))[kl], __dmul_rn(d, d));
            }
        }
        __syncthreads();
    }
    // merge this partial into the pane state (the workgroup owns these (pane, key) entries)
    for (int kl = threadIdx.x; kl < kk; kl += kBlock) {
        uint32_t c = lcnt[kl];
        if (c == 0) continue;
        int64_t key = (int64_t)bucket * kk + kl;
        int64_t e = slot * ds.K + key;
        int64_t cprev = ds.cnt[e];
        ds.cnt[e] = cprev + c;
        for (int v = 0; v < p.n_vc; ++v) {
            const int f = p.vc_flags[v];
            int64_t nb_ = (f & NEED_CNT) ? (int64_t)((uint32_t*)(lds + lay.off_vcnt[v]))[kl] : (int64_t)c;
            if (nb_ == 0) continue;
            int64_t na = (f & NEED_CNT) ? ds.vcnt[v][e] : cprev;
            if (f & NEED_CNT) ds.vcnt[v][e] = na + nb_;
            if (p.vc_is_float[v]) {
                double sb = (f & (NEED_SUM | NEED_M2)) ? ((double*)(lds + lay.off_sum[v]))[kl] : 0.0;
                double sa = (f & (NEED_SUM | NEED_M2)) && na ? __longlong_as_double(ds.sum[v][e]) : 0.0;
                if (f & NEED_M2) {
                    double m2b = ((double*)(lds + lay.off_m2[v]))[kl];
                    if (na == 0) ds.m2[v][e] = m2b;
                    else {
                        double dlt = __dsub_rn(__ddiv_rn(sb, (double)nb_), __ddiv_rn(sa, (double)na));
                        ds.m2[v][e] = ds.m2[v][e] + m2b + dlt * dlt * ((double)na * (double)nb_ / (double)(na + nb_));
                    }
                }
                if (f & NEED_SUM) ds.sum[v][e] = __double_as_longlong(na ? __dadd_rn(sa, sb) : sb);
                if (f & NEED_MIN) {
                    uint64_t ob = ~((unsigned long long*)(lds + lay.off_min[v]))[kl];
                    uint64_t oa = (uint64_t)ds.mn[v][e];
                    ds.mn[v][e] = (int64_t)(na == 0 ? ob : (ob < oa ? ob : oa));
                }
                if (f & NEED_MAX) {
                    uint64_t ob = ((unsigned long long*)(lds + lay.off_max[v]))[kl];
                    uint64_t oa = (uint64_t)ds.mx[v][e];
                    ds.mx[v][e] = (int64_t)(na == 0 ? ob : (ob > oa ? ob : oa));
                }
            } else {
                if (f & NEED_SUM) {
                    int64_t sb = (int64_t)((unsigned long long*)(lds + lay.off_sum[v]))[kl];
                    ds.sum[v][e] = (int64_t)((uint64_t)(na ? ds.sum[v][e] : 0) + (uint64_t)sb);
                }
                double fb = (f & NEED_FSUM) ? ((double*)(lds + lay.off_fsum[v]))[kl] : 0.0;
                double fa = (f & NEED_FSUM) && na ? ds.fsum[v][e] : 0.0;
                if (f & NEED_M2) {
                    double m2b = ((double*)(lds + lay.off_m2[v]))[kl];
                    if (na == 0) ds.m2[v][e] = m2b;
                    else {
                        double dlt = __dsub_rn(__ddiv_rn(fb, (double)nb_), __ddiv_rn(fa, (double)na));
                        ds.m2[v][e] = ds.m2[v][e] + m2b + dlt * dlt * ((double)na * (double)nb_ / (double)(na + nb_));
                    }
                }
                if (f & NEED_FSUM) ds.fsum[v][e] = na ? fa + fb : fb;
                if (f & NEED_MIN) {
                    uint64_t ob = ~((unsigned long long*)(lds + lay.off_min[v]))[kl];
                    uint64_t oa = (uint64_t)ds.mn[v][e];
                    ds.mn[v][e] = (int64_t)(na == 0 ? ob : (ob < oa ? ob : oa));
                }
                if (f & NEED_MAX) {
                    uint64_t ob = ((unsigned long long*)(lds + lay.off_max[v]))[kl];
                    uint64_t oa = (uint64_t)ds.mx[v][e];
                    ds.mx[v][e] = (int64_t)(na == 0 ? ob : (ob > oa ? ob : oa));
                }
            }
        }
    }
}

// ---------------------------------------------------------------- finalize closed windows
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
};

__global__ __launch_bounds__(kBlock) void k_finalize(DPlan* __restrict__ pp, const WinDesc* __restrict__ wins,
                                                     DState ds, int32_t ring, const int32_t* __restrict__ pane_err,
                                                     Results res) {
    const DPlan& p = *pp;
    const WinDesc w = wins[blockIdx.y];
    int64_t key = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    int32_t werr = 0;
    for (int64_t q = w.q_first; q <= w.q_last; ++q) werr |= pane_err[q % ring];
    if (werr) {
        if (key == 0) atomicOr(&res.win_err[w.idx], werr);
        return;
    }
    const uint32_t K = p.key_col >= 0 ? p.num_keys : 1u;
    if (key >= K) return;
    // merge panes in time order
    int64_t cnt = 0;
    int64_t vcnt[kMaxVC], isum[kMaxVC];
    double fsum[kMaxVC], m2[kMaxVC];
    uint64_t omn[kMaxVC], omx[kMaxVC];
    for (int v = 0; v < p.n_vc; ++v) { vcnt[v] = 0; isum[v] = 0; fsum[v] = 0; m2[v] = 0; omn[v] = ~0ull; omx[v] = 0; }
    for (int64_t q = w.q_first; q <= w.q_last; ++q) {
        int64_t e = (q % ring) * ds.K + key;
        int64_t c = ds.cnt[e];
        if (c == 0) continue;
        int64_t cprev = cnt;
        cnt += c;
        for (int v = 0; v < p.n_vc; ++v) {
            const int f = p.vc_flags[v];
            int64_t nb_ = (f & NEED_CNT) ? ds.vcnt[v][e] : c;
            if (nb_ == 0) continue;
            int64_t na = (f & NEED_CNT) ? vcnt[v] : cprev;
            vcnt[v] = na + nb_;
            double sb = 0;
            if (p.vc_is_float[v]) {
                if (f & (NEED_SUM | NEED_M2)) sb = __longlong_as_double(ds.sum[v][e]);
            } else {
                if (f & NEED_SUM) isum[v] = (int64_t)((uint64_t)isum[v] + (uint64_t)ds.sum[v][e]);
                if (f & NEED_FSUM) sb = ds.fsum[v][e];
            }
            if (f & NEED_M2) {
                double m2b = ds.m2[v][e];
                if (na == 0) m2[v] = m2b;
                else {
                    double dlt = __dsub_rn(__ddiv_rn(sb, (double)nb_), __ddiv_rn(fsum[v], (double)na));
                    m2[v] = m2[v] + m2b + dlt * dlt * ((double)na * (double)nb_ / (double)(na + nb_));
                }
            }
            fsum[v] = na ? __dadd_rn(fsum[v], sb) : sb;
            if (f & NEED_MIN) { uint64_t o = (uint64_t)ds.mn[v][e]; omn[v] = o < omn[v] ? o : omn[v]; }
            if (f & NEED_MAX) { uint64_t o = (uint64_t)ds.mx[v][e]; omx[v] = o > omx[v] ? o : omx[v]; }
        }
    }
    if (cnt == 0) return;  // group absent from this window
    Val a[EK_MAX_AGGS];
    for (int k = 0; k < p.n_aggs; ++k) {
        const int fn = p.agg_fn[k];
        const int v = p.agg_vc[k];
        Val r{V_NULL, 0, 0.0};
        if (fn == EK_AGG_COUNT_STAR) r = Val{V_I64, cnt, 0.0};
        else if (fn == EK_AGG_COUNT) r = Val{V_I64, vcnt[v], 0.0};
        else if (vcnt[v] > 0) {
            const bool fl = p.vc_is_float[v];
            switch (fn) {
            case EK_AGG_SUM: r = fl ? Val{V_F64, 0, fsum[v]} : Val{V_I64, isum[v], 0.0}; break;
            case EK_AGG_AVG:   // funcs_agg.go:56-86: int -> int64 truncating division
                r = fl ? Val{V_F64, 0, __ddiv_rn(fsum[v], (double)vcnt[v])}
                       : Val{V_I64, (isum[v] == INT64_MIN && vcnt[v] == -1) ? isum[v] : isum[v] / vcnt[v], 0.0};
                break;
            case EK_AGG_MIN: r = fl ? Val{V_F64, 0, ord_to_f64(omn[v])} : Val{V_I64, ord_to_i64(omn[v]), 0.0}; break;
            case EK_AGG_MAX: r = fl ? Val{V_F64, 0, ord_to_f64(omx[v])} : Val{V_I64, ord_to_i64(omx[v]), 0.0}; break;
            case EK_AGG_VAR: r = Val{V_F64, 0, __ddiv_rn(m2[v], (double)vcnt[v])}; break;
            case EK_AGG_VARS: r = Val{V_F64, 0, __ddiv_rn(m2[v], (double)(vcnt[v] - 1))}; break;
            case EK_AGG_STDDEV: r = Val{V_F64, 0, __dsqrt_rn(__ddiv_rn(m2[v], (double)vcnt[v]))}; break;
            case EK_AGG_STDDEVS: r = Val{V_F64, 0, __dsqrt_rn(__ddiv_rn(m2[v], (double)(vcnt[v] - 1)))}; break;
            default: break;
            }
        }
        a[k] = r;
    }
    if (p.n_having > 0) {
        Val h = eval_prog(p.having_prog, p.n_having, p, nullptr, 0, a);
        if (h.tag != V_BOOL) { atomicOr(&res.win_err[w.idx], EK_WIN_HAVING_ERROR); return; }
        if (!h.i) return;
    }
    int64_t pos = w.out_base + atomicAdd((unsigned long long*)&res.win_cnt[w.idx], 1ull);
    res.key[pos] = (uint32_t)key;
    for (int k = 0; k < p.n_aggs; ++k) {
        res.tag[k][pos] = a[k].tag == V_NULL ? EK_TAG_NULL : (a[k].tag == V_I64 ? EK_TAG_I64 : EK_TAG_F64);
        res.val[k][pos] = a[k].tag == V_F64 ? __double_as_longlong(a[k].f) : a[k].i;
    }
}

// ---------------------------------------------------------------- debug: window membership fingerprint
// Per pane: number of accepted events (before WHERE) and Σ ek_mix64(arrival index); a window's
// fingerprint is the sum over its panes (order-independent, exact in u64 arithmetic).
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

}  // namespace ek
