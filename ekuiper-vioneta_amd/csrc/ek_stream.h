// ek_stream.h — XCD-resident streaming partition + aggregation (pane mode, ts-sorted batches).
//
// The two-kernel path (k_part writes every chunk's (key, values) runs to an HBM staging area, k_agg reads them
// back per (pane, key bucket)) moves 18 B/event of staging through HBM twice on top of the 20 B/event of input.
// Here one persistent launch keeps that staging on chip:
//   * each XCD (read from HW_REG_XCC_ID) owns every 8th pane of the batch; its workgroups take the chunks of
//     those panes from the XCD's own queue (an atomic head), so a chunk is produced and consumed inside one XCD;
//   * every workgroup is a PRODUCER (load a 4096-event chunk once: 16-byte key / value loads, LDS counting sort by
//     owner, coalesced run writes into a small per-XCD staging ring that stays in the XCD's L2 / the Infinity Cache)
//     and a CONSUMER: it owns a fixed key range (key >> obits == owner) and keeps that range's partial table of the
//     current pane in LDS for the whole pane, folding in its run of every produced chunk in chunk order;
//   * when a workgroup has folded in the last chunk of a pane it finalises its key range exactly as k_agg does:
//     direct emission of a tumbling window closing at this batch's watermark (HAVING, block-compacted rows) or a
//     write / Chan merge into the pane-state ring.
// Hand-off inside the XCD: a producer's plain stores reach the XCD's shared L2 (s_waitcnt vmcnt(0) in every storing
// wave, then a workgroup barrier), then one lane publishes the chunk with an agent-scope atomic store; a consumer
// polls that word and reads the payload with sc1 (L1-bypassing, L2-served) loads only, so a stale L1 line of an
// earlier lap of the ring is never read. Producer and consumer of a ring slot are on the same XCD by construction
// (the ring is indexed by the executing XCD), and a slot is rewritten only after every owner of the XCD has counted
// it consumed. Every spin is bounded; a grid that is not fully resident is detected by an arrival count before any
// side effect (sync->err = 1: the host takes the two-kernel path).
#pragma once
#include "ek_kernels.h"

namespace ek {

constexpr int kSBlock = 512;          // threads per workgroup (2 per CU)
constexpr int kSTile = 4096;          // events per chunk
constexpr int kSTileE = kSTile / kSBlock;
constexpr int kSRing = 160;           // staging slots per XCD
constexpr int kSXcd = 8;
constexpr int kSMaxOwners = 128;      // workgroups per XCD
constexpr int kSBatch = 32;           // chunks folded in per consume step (<= 64: one wave polls them)
constexpr int kSU = 4;                // staged rows in flight per thread while folding in
constexpr int kSMaxXPanes = 512;      // panes per XCD per launch

struct StreamDesc {
    int64_t nbatch;
    int64_t q_lo;
    int32_t n_panes;       // panes [q_lo, q_lo + n_panes) of the batch
    int32_t ring;          // pane-state ring
    int32_t key_col, n_where;
    uint32_t num_keys;
    int32_t owners;        // workgroups (= key ranges) per XCD
    int32_t obits;         // key range of an owner = [o << obits, (o + 1) << obits)
    int32_t max_chunks;    // per-XCD capacity of the chunk flags
    int32_t nvc;
    int32_t pad;
    int64_t timeout;       // s_memrealtime ticks (100 MHz) a spin may last
    const int64_t* pbnd;   // [n_panes + 1] first event of each pane
    const int32_t* xpane;  // panes of each XCD (group-relative), x-major, [n_panes]
    const int32_t* xoff;   // [kSXcd + 1] offsets into xpane
    const int32_t* xcpre;  // per XCD x: chunk prefix over its panes at xcpre[xoff[x] + x + k], k = 0..count
    const int64_t* dbase;  // per pane: direct-emission row base or -1
    const int32_t* didx;   // per pane: window index (direct emission)
    const uint8_t* fresh;  // per pane: 1 = write, 0 = merge into the pane state
    uint32_t* sync;        // [0] arrived, [1] err, [2..10) members, [10..18) head, then flags[8][max_chunks], cons[8][kSRing]
    uint16_t* klo;         // [kSXcd][kSRing][kSTile]
    int64_t* val[kMaxVC];  // [kSXcd][kSRing][kSTile]
    uint32_t* ctab;        // [kSXcd][kSRing][owners + 1]
    unsigned long long* prof;   // optional [grid][8] per-workgroup time split (EKGPU_STREAM_PROF)
};

__device__ __forceinline__ int xcc_id() {
    // HW_REG_XCC_ID (hwreg 20), bits [3:0]
    return (int)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 15);
}
__device__ __forceinline__ uint32_t ld_acq32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t ld_sc1_64(const int64_t* p) {
    return (int64_t)__hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u16(const uint16_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t w = __hip_atomic_load((const uint32_t*)(a & ~(uintptr_t)3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (a & 2) ? (w >> 16) : (w & 0xFFFFu);
}

// LDS: [table: per key of the owner range, 8-byte fields then u32 counts][producer: s_val kSTile x 8, s_klo kSTile x 2]
template <int NVC, bool WHERE>
__global__ __launch_bounds__(kSBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_stream(
    DPlan* __restrict__ pp, DBatch b, StreamDesc sd, LdsLayout lay, DState ds, Results res, int32_t* __restrict__ pane_err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const DPlan& p = *pp;
    const int tid = threadIdx.x;
    __shared__ int s_i[8];
    __shared__ uint32_t s_tcnt[kSMaxOwners + 4];
    __shared__ uint32_t s_wsum[kSBlock / 64];
    __shared__ uint32_t r_start[kSBatch], r_pre[kSBatch + 1];
    static_assert(kSBatch <= 63, "one wave polls a consume batch");
    __shared__ uint32_t esh[20];
    uint32_t* g_arrived = sd.sync;
    uint32_t* g_err = sd.sync + 1;
    uint32_t* g_members = sd.sync + 2;
    uint32_t* g_head = sd.sync + 10;
    uint32_t* g_flags = sd.sync + 18;
    uint32_t* g_cons = g_flags + (size_t)kSXcd * sd.max_chunks;
    const int x = xcc_id();
    const int kpo = 1 << sd.obits;
    const uint32_t omask = (uint32_t)kpo - 1u;

    // ---- residency: every workgroup of the grid must be running, each XCD with exactly `owners` of them
    if (tid == 0) {
        s_i[0] = (int)atomicAdd(&g_members[x], 1u);
        atomicAdd(g_arrived, 1u);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (ld_acq32(g_arrived) < gridDim.x) {
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > sd.timeout / 8) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        if (ok && ld_acq32(&g_members[x]) != (uint32_t)sd.owners) ok = 0;
        if (!ok) atomicOr(g_err, 1u);
        s_i[1] = ok;
    }
    __syncthreads();
    if (!s_i[1]) return;
    const int owner = s_i[0];

    const int xo = sd.xoff[x], nxp = sd.xoff[x + 1] - xo;
    const int32_t* cpre = sd.xcpre + xo + x;     // [nxp + 1]
    const int c_total = nxp > 0 ? cpre[nxp] : 0;
    uint32_t* flags = g_flags + (size_t)x * sd.max_chunks;
    uint32_t* cons = g_cons + (size_t)x * kSRing;

    unsigned char* prod = lds + lay.bytes;
    int64_t* s_val = (int64_t*)prod;
    uint16_t* s_klo = (uint16_t*)(prod + (size_t)kSTile * 8);
    uint32_t* lcnt = (uint32_t*)(lds + lay.off_cnt);
    int fl[NVC], vcol[NVC];
    bool isf[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) { fl[v] = v < p.n_vc ? p.vc_flags[v] : 0; vcol[v] = v < p.n_vc ? p.vc_col[v] : 0; isf[v] = p.vc_is_float[v] != 0; }
    const uint32_t* kcol = sd.key_col >= 0 ? (const uint32_t*)b.col[sd.key_col] : nullptr;

    auto zero_table = [&]() {
        for (int k = tid; k < lay.bytes / 4; k += kSBlock) ((uint32_t*)lds)[k] = 0;
    };
    auto timed_out = [&](uint64_t t0) {
        return (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > sd.timeout;
    };
    auto pane_of_chunk = [&](int j, int* k_out) {
        int k = 0;
        while (k + 1 < nxp && cpre[k + 1] <= j) ++k;
        *k_out = k;
        return sd.xpane[xo + k];
    };

    // ---- finalise this owner's key range of pane r (k_agg's emission / merge for one key range)
    auto finish_pane = [&](int r) {
        const int64_t q = sd.q_lo + r;
        const int64_t slot = q % sd.ring;
        const int64_t dbase = sd.dbase[r];
        const int64_t key0 = (int64_t)owner << sd.obits;
        auto lds_part = [&](int kl, int64_t& c, int64_t (&vc)[NVC], int64_t (&is)[NVC], double (&fs)[NVC], double (&m2)[NVC],
                            uint64_t (&mn)[NVC], uint64_t (&mx)[NVC]) {
            c = lcnt[kl];
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = fl[v];
                vc[v] = c;
                is[v] = (!isf[v] && (f & NEED_SUM)) ? ((int64_t*)(lds + lay.off_sum[v]))[kl] : 0;
                fs[v] = isf[v] ? ((f & NEED_SUM) ? ((double*)(lds + lay.off_sum[v]))[kl] : 0.0) : 0.0;
                m2[v] = 0.0;
                mn[v] = (f & NEED_MIN) ? ~((unsigned long long*)(lds + lay.off_min[v]))[kl] : 0ull;
                mx[v] = (f & NEED_MAX) ? ((unsigned long long*)(lds + lay.off_max[v]))[kl] : 0ull;
            }
        };
        if (dbase >= 0) {
            const int32_t widx = sd.didx[r];
            const int32_t perr = (int32_t)__hip_atomic_load((const uint32_t*)&pane_err[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (perr) {   // a WHERE error replaces the window's output (filter_operator.go:63-77)
                if (tid == 0 && owner == 0) atomicOr(&res.win_err[widx], perr);
                return;
            }
            const uint32_t K = sd.key_col >= 0 ? sd.num_keys : 1u;
            for (int kb = 0; kb < kpo; kb += kSBlock) {
                const int kl = kb + tid;
                const int64_t key = key0 + kl;
                Part<NVC> s{};
                bool present = false;
                if (kl < kpo && key < K) {
                    int64_t c, vc[NVC], is[NVC];
                    double fs[NVC], m2[NVC];
                    uint64_t mn[NVC], mx[NVC];
                    lds_part(kl, c, vc, is, fs, m2, mn, mx);
                    if (c > 0) {
                        part_merge(p, s, c, vc, is, fs, m2, mn, mx);
                        present = having_keep(p, s, &res.win_err[widx]);
                    }
                }
                emit_rows(p, present, s, key, dbase, widx, res, esh);
            }
            return;
        }
        const bool fresh = sd.fresh[r] != 0;
        for (int kl = tid; kl < kpo; kl += kSBlock) {
            const int64_t key = key0 + kl;
            if (key >= ds.K) break;
            const int64_t e = slot * ds.K + key;
            int64_t c, vc[NVC], is[NVC];
            double fs[NVC], m2[NVC];
            uint64_t mn[NVC], mx[NVC];
            lds_part(kl, c, vc, is, fs, m2, mn, mx);
            if (fresh) {
                ds.cnt[e] = c;
#pragma unroll
                for (int v = 0; v < NVC; ++v) {
                    const int f = fl[v];
                    if (f & NEED_SUM) ds.sum[v][e] = isf[v] ? __double_as_longlong(fs[v]) : is[v];
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
                const int f = fl[v];
                avc[v] = ac;
                ais[v] = (!isf[v] && (f & NEED_SUM)) ? ds.sum[v][e] : 0;
                afs[v] = isf[v] && (f & NEED_SUM) ? __longlong_as_double(ds.sum[v][e]) : 0.0;
                am2[v] = 0.0;
                amn[v] = (f & NEED_MIN) ? (uint64_t)ds.mn[v][e] : 0ull;
                amx[v] = (f & NEED_MAX) ? (uint64_t)ds.mx[v][e] : 0ull;
            }
            if (ac) part_merge(p, a, ac, avc, ais, afs, am2, amn, amx);
            part_merge(p, a, c, vc, is, fs, m2, mn, mx);
            ds.cnt[e] = a.cnt;
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int f = fl[v];
                if (f & NEED_SUM) ds.sum[v][e] = isf[v] ? __double_as_longlong(a.fsum[v]) : a.isum[v];
                if (f & NEED_MIN) ds.mn[v][e] = (int64_t)a.omn[v];
                if (f & NEED_MAX) ds.mx[v][e] = (int64_t)a.omx[v];
            }
        }
    };

    // ---- consumer: fold in up to kSBatch published chunks of the current pane (chunk order); false if none
    int next_c = 0, cur_k = 0;
    uint64_t pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // produce, slot wait, consume, finish, idle, n_produce, n_consume, -
    auto consume = [&]() -> bool {
        if (next_c >= c_total) return false;
        const uint64_t tc0 = __builtin_amdgcn_s_memrealtime();
        if (tid < 64) {   // wave 0: lane t polls chunk next_c + t; g = the leading run of published chunks
            const int want = min(cpre[cur_k + 1], next_c + kSBatch) - next_c;
            const bool set = tid < want && ld_acq32(&flags[next_c + tid]) != 0u;
            const unsigned long long m = __ballot(set);
            if (tid == 0) s_i[2] = (int)__builtin_ctzll(~m);
        }
        __syncthreads();
        const int g = s_i[2];
        if (g == 0) { __syncthreads(); return false; }
        if (tid < g) {
            const int slot = (next_c + tid) % kSRing;
            const uint32_t* ct = sd.ctab + ((size_t)x * kSRing + slot) * (sd.owners + 1);
            const uint32_t o0 = ld_acq32(ct + owner), o1 = ld_acq32(ct + owner + 1);
            r_start[tid] = (uint32_t)(((size_t)x * kSRing + slot) * kSTile) + o0;
            r_pre[tid + 1] = o1 - o0;
        }
        __syncthreads();
        if (tid == 0) {
            r_pre[0] = 0;
            for (int t = 0; t < g; ++t) r_pre[t + 1] += r_pre[t];
        }
        __syncthreads();
        const uint32_t total = r_pre[g];
        for (uint32_t v0 = 0; v0 < total; v0 += kSBlock * kSU) {
            int kl[kSU];
            int64_t raw[NVC][kSU];
#pragma unroll
            for (int u = 0; u < kSU; ++u) {
                const uint32_t v = v0 + u * kSBlock + tid;
                kl[u] = -1;
                if (v < total) {
                    int lo = 0, hi = g - 1;   // run of row v: last j with r_pre[j] <= v
                    while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (r_pre[mid] <= v) lo = mid; else hi = mid - 1; }
                    const size_t pos = (size_t)r_start[lo] + (v - r_pre[lo]);
                    kl[u] = (int)ld_sc1_u16(sd.klo + pos);
#pragma unroll
                    for (int w = 0; w < NVC; ++w) raw[w][u] = fl[w] ? ld_sc1_64(sd.val[w] + pos) : 0;
                }
            }
#pragma unroll
            for (int u = 0; u < kSU; ++u) {
                if (kl[u] < 0) break;
                atomicAdd(&lcnt[kl[u]], 1u);
#pragma unroll
                for (int w = 0; w < NVC; ++w) {
                    const int f = fl[w];
                    if (f == 0) continue;
                    if (isf[w]) {
                        const double xv = __longlong_as_double(raw[w][u]);
                        if (f & NEED_SUM) atomicAdd(&((double*)(lds + lay.off_sum[w]))[kl[u]], xv);
                        if (f & NEED_MIN) atomicMax(&((unsigned long long*)(lds + lay.off_min[w]))[kl[u]], (unsigned long long)~f64_to_ord(xv));
                        if (f & NEED_MAX) atomicMax(&((unsigned long long*)(lds + lay.off_max[w]))[kl[u]], (unsigned long long)f64_to_ord(xv));
                    } else {
                        if (f & NEED_SUM) atomicAdd(&((unsigned long long*)(lds + lay.off_sum[w]))[kl[u]], (unsigned long long)raw[w][u]);
                        if (f & NEED_MIN) atomicMax(&((unsigned long long*)(lds + lay.off_min[w]))[kl[u]], (unsigned long long)~i64_to_ord(raw[w][u]));
                        if (f & NEED_MAX) atomicMax(&((unsigned long long*)(lds + lay.off_max[w]))[kl[u]], (unsigned long long)i64_to_ord(raw[w][u]));
                    }
                }
            }
        }
        __syncthreads();   // every run of these slots has been read (loads returned into the LDS atomics)
        if (tid < g) atomicAdd(&cons[(next_c + tid) % kSRing], 1u);
        next_c += g;
        const uint64_t tc1 = __builtin_amdgcn_s_memrealtime();
        pt[2] += tc1 - tc0;
        pt[6]++;
        if (next_c == cpre[cur_k + 1]) {
            finish_pane(sd.xpane[xo + cur_k]);
            __syncthreads();
            zero_table();
            cur_k++;
            __syncthreads();
            pt[3] += __builtin_amdgcn_s_memrealtime() - tc1;
        }
        return true;
    };

    // ---- producer: partition chunk j of this XCD by owner into its ring slot and publish it
    auto produce = [&](int j) {
        int k;
        const int r = pane_of_chunk(j, &k);
        // per-pane chunk grid aligned to kSTile rows, so every thread's row pair is 16-byte aligned in the columns
        const int64_t c0 = (sd.pbnd[r] & ~(int64_t)(kSTile - 1)) + (int64_t)(j - cpre[k]) * kSTile;
        const int64_t e0 = max(sd.pbnd[r], c0), e1 = min(sd.pbnd[r + 1], c0 + kSTile);
        const int slot = j % kSRing;
        const uint32_t need = (uint32_t)sd.owners * (uint32_t)(j / kSRing);
        // the slot's previous chunk must have been folded in by every owner of the XCD (consume meanwhile)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            if (tid == 0) s_i[3] = ld_acq32(&cons[slot]) >= need ? 1 : (ld_acq32(g_err) ? 2 : 0);
            __syncthreads();
            const int st = s_i[3];
            __syncthreads();
            if (st == 1) break;
            if (st == 2 || timed_out(t0)) { if (tid == 0) atomicOr(g_err, 2u); return false; }
            if (!consume()) __builtin_amdgcn_s_sleep(2);
        }
        const uint64_t tp1 = __builtin_amdgcn_s_memrealtime();
        pt[1] += tp1 - t0;
        const int64_t q = sd.q_lo + r;
        uint32_t key[kSTileE];
        int64_t val[NVC][kSTileE];
#pragma unroll
        for (int m = 0; m < kSTileE / 2; ++m) {
            const int64_t i = c0 + (int64_t)m * 2 * kSBlock + 2 * tid;   // even, inside the batch's row space
            const bool pair = i + 1 < sd.nbatch;
            if (kcol && pair && (((uintptr_t)(kcol + i)) & 7) == 0) {
                const uint2 kp = *(const uint2*)(kcol + i);
                key[2 * m] = kp.x;
                key[2 * m + 1] = kp.y;
            } else {
                key[2 * m] = (kcol && i < sd.nbatch) ? kcol[i] : 0u;
                key[2 * m + 1] = (kcol && pair) ? kcol[i + 1] : 0u;
            }
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                const int64_t* col = (const int64_t*)b.col[vcol[v]];
                if (fl[v] && pair && (((uintptr_t)(col + i)) & 15) == 0) {
                    const longlong2 vp = *(const longlong2*)(col + i);
                    val[v][2 * m] = vp.x;
                    val[v][2 * m + 1] = vp.y;
                } else {
                    val[v][2 * m] = (fl[v] && i < sd.nbatch) ? col[i] : 0;
                    val[v][2 * m + 1] = (fl[v] && pair) ? col[i + 1] : 0;
                }
            }
        }
        for (int t = tid; t <= sd.owners; t += kSBlock) s_tcnt[t] = 0;
        __syncthreads();
        int lp[kSTileE];
        uint32_t rank[kSTileE];
#pragma unroll
        for (int jj = 0; jj < kSTileE; ++jj) {
            const int64_t i = c0 + (int64_t)(jj >> 1) * 2 * kSBlock + 2 * tid + (jj & 1);
            lp[jj] = -1;
            if (i >= e0 && i < e1 && (sd.key_col < 0 || key[jj] < sd.num_keys)) {
                int w = 1;
                if (WHERE) {
                    w = where_decide_slow(p, b, i);
                    if (w < 0) atomicOr(&pane_err[q % sd.ring], EK_WIN_WHERE_ERROR);
                }
                if (w > 0) lp[jj] = (int)(key[jj] >> sd.obits);
            }
            if (lp[jj] >= 0) rank[jj] = atomicAdd(&s_tcnt[lp[jj]], 1u);
        }
        __syncthreads();
        block_excl_scan<kSBlock>(s_tcnt, sd.owners, s_wsum);
        uint32_t* ct = sd.ctab + ((size_t)x * kSRing + slot) * (sd.owners + 1);
        for (int t = tid; t <= sd.owners; t += kSBlock) ct[t] = s_tcnt[t];
        uint32_t spos[kSTileE];
#pragma unroll
        for (int jj = 0; jj < kSTileE; ++jj) {
            if (lp[jj] < 0) continue;
            spos[jj] = s_tcnt[lp[jj]] + rank[jj];
            s_klo[spos[jj]] = (uint16_t)(key[jj] & omask);
        }
        __syncthreads();
        const uint32_t total = s_tcnt[sd.owners];
        const size_t region = ((size_t)x * kSRing + slot) * kSTile;
        for (uint32_t s = tid; s < total; s += kSBlock) sd.klo[region + s] = s_klo[s];
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            if (!fl[v]) continue;
            __syncthreads();
#pragma unroll
            for (int jj = 0; jj < kSTileE; ++jj)
                if (lp[jj] >= 0) s_val[spos[jj]] = val[v][jj];
            __syncthreads();
            for (uint32_t s = tid; s < total; s += kSBlock) sd.val[v][region + s] = s_val[s];
        }
        // publish: every storing wave drains, then one lane flags the chunk (agent-scope atomic)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(&flags[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pt[0] += __builtin_amdgcn_s_memrealtime() - tp1;
        pt[5]++;
        return true;
    };

    zero_table();
    __syncthreads();
    bool exhausted = false;
    uint64_t idle_since = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        bool did = false;
        if (!exhausted) {
            if (tid == 0) s_i[4] = (int)atomicAdd(&g_head[x], 1u);
            __syncthreads();
            const int j = s_i[4];
            __syncthreads();
            if (j < c_total) {
                if (!produce(j)) return;
                did = true;
            } else {
                exhausted = true;
            }
        }
        const uint64_t ti0 = __builtin_amdgcn_s_memrealtime();
        const bool dc = consume();
        did |= dc;
        if (!dc) pt[4] += __builtin_amdgcn_s_memrealtime() - ti0;
        if (next_c >= c_total) break;
        if (did) {
            idle_since = __builtin_amdgcn_s_memrealtime();
        } else {
            if (tid == 0) s_i[5] = (int)ld_acq32(g_err);
            __syncthreads();
            const int e = s_i[5];
            __syncthreads();
            if (e || timed_out(idle_since)) { if (tid == 0) atomicOr(g_err, 2u); return; }
            const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_s_sleep(4);
            pt[4] += __builtin_amdgcn_s_memrealtime() - ts0;
        }
    }
    if (sd.prof && tid == 0)
        for (int k = 0; k < 8; ++k) sd.prof[(size_t)blockIdx.x * 8 + k] = pt[k];
}

}  // namespace ek
