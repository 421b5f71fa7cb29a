// ek_stream.h — XCD-resident streaming partition + aggregation (pane mode, ts-sorted batches).
//
// The two-kernel path (k_part writes every chunk's (key, values) runs to an HBM staging area, k_agg reads them
// back per (pane, key bucket)) moves 18 B/event of staging through HBM twice on top of the 20 B/event of input;
// the Infinity Cache does not absorb that round trip (a just-written buffer reads back at the HBM rate,
// tools/mb_mall.hip). Here one persistent launch keeps the staging inside each XCD's 4 MiB L2:
//   * every XCD (HW_REG_XCC_ID) owns a contiguous range of the batch's panes, balanced by events; its panes are
//     cut into 2048-row chunks on a per-pane grid, numbered j = 0, 1, ... in event order;
//   * half of the XCD's workgroups are PRODUCERS: producer i takes chunks i, i + P, i + 2P, ...; it loads a chunk
//     once (16-byte key / value loads, the next chunk's loads issued before this one is partitioned), counting-
//     sorts it in LDS by owner and writes the owner runs into ring slot j mod kSRing (kSRing x 36 KiB stays in L2);
//   * the other half are CONSUMERS: consumer o owns the key range [o << obits, (o + 1) << obits) and keeps its
//     partial table of the current pane in LDS; it folds in its run of every chunk of the XCD in chunk order and
//     finalises its key range of a pane after the pane's last chunk, exactly as k_agg does (direct emission of a
//     tumbling window closing at this batch's watermark, with HAVING, or a write / Chan merge into the pane state).
// Hand-off inside the XCD (MI355X_MICROARCH.md, inter-workgroup visibility): a producer's plain stores reach the
// XCD's shared L2 (s_waitcnt vmcnt(0) in every storing wave, then a workgroup barrier), then one lane publishes
// the chunk with an agent-scope atomic store; a consumer polls that word and reads the payload with non-temporal
// (L1-bypassing, L2-served) loads only, so no stale L1 line of an earlier lap of the ring is read. Producer and
// consumer of a slot share an XCD by construction (the ring is indexed by the executing XCD); a slot is
// rewritten only after every consumer of the XCD has counted it folded in. Every spin is bounded; a grid that is
// not co-resident (P producers + P consumers on each XCD) is detected before any side effect (sync->err = 1).
#pragma once
// constants, StreamDesc, xcc_id / ld_acq32 and the launcher declaration
#include "ek_stream_desc.h"

namespace ek {

// LDS: consumer = [table: per key of the owner range, 8-byte fields then u32 counts];
//      producer = [s_val: NVC x kSTile x 8][s_klo: kSTile x 2]
template <int NVC, bool WHERE>
__global__ __launch_bounds__(kSBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_stream(
    DPlan* __restrict__ pp, DBatch b, StreamDesc sd, LdsLayout lay, DState ds, Results res, int32_t* __restrict__ pane_err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const DPlan& p = *pp;
    const int tid = threadIdx.x;
    __shared__ int s_i[8];
    __shared__ uint32_t s_tcnt[kSMaxOwners + 4];
    __shared__ uint32_t s_wsum[kSBlock / 64];
    static_assert(kSWaveBatch < 64, "one wave polls its batch");
    __shared__ uint32_t esh[20];
    uint32_t* g_arrived = sd.sync;
    uint32_t* g_err = sd.sync + 1;
    uint32_t* g_members = sd.sync + 2;
    uint32_t* g_cons = sd.sync + 10;
    const int x = xcc_id();
    const int P = sd.owners;

    // ---- residency: every workgroup of the grid must be running, each XCD with exactly 2 P of them
    if (tid == 0) {
        s_i[0] = (int)atomicAdd(&g_members[x], 1u);
        atomicAdd(g_arrived, 1u);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (ld_acq32(g_arrived) < gridDim.x) {
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > sd.timeout / 8) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        if (ok && ld_acq32(&g_members[x]) != (uint32_t)(2 * P)) ok = 0;
        if (!ok) atomicOr(g_err, 1u);
        s_i[1] = ok;
    }
    __syncthreads();
    if (!s_i[1]) return;
    const bool producer = (s_i[0] & 1) == 0;
    const int me = s_i[0] >> 1;          // producer index / owner (consumer) index inside the XCD

    const int xo = sd.xoff[x], nxp = sd.xoff[x + 1] - xo;
    const int32_t* cpre = sd.xcpre + xo + x;     // [nxp + 1]
    const int c_total = nxp > 0 ? cpre[nxp] : 0;
    uint32_t* cons = g_cons + (size_t)x * kSRing;
    int fl[NVC], vcol[NVC];
    bool isf[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) { fl[v] = v < p.n_vc ? p.vc_flags[v] : 0; vcol[v] = v < p.n_vc ? p.vc_col[v] : 0; isf[v] = p.vc_is_float[v] != 0; }
    auto timed_out = [&](uint64_t t0) {
        return (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > sd.timeout;
    };
    uint64_t pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // producer: -, slot-wait, sort+store | consumer: poll, fold, -, n, finish

    if (producer) {
        // ======================================================== producer
        const uint32_t* kcol = sd.key_col >= 0 ? (const uint32_t*)b.col[sd.key_col] : nullptr;
        int64_t* s_val = (int64_t*)lds;                                   // [NVC][kSTile]
        uint16_t* s_klo = (uint16_t*)(lds + (size_t)NVC * kSTile * 8);    // [kSTile]
        const uint32_t omask = (1u << sd.obits) - 1u;
        int pk = 0;   // pane (index into this XCD's list) of the latest chunk located: chunks come in rising order
        // chunk j: rows [c0, c0 + kSTile) of its pane's kSTile-aligned grid, masked to the pane's rows [e0, e1)
        auto chunk_rows = [&](int j, int64_t* c0, int64_t* e0, int64_t* e1, int* r) {
            while (pk + 1 < nxp && cpre[pk + 1] <= j) ++pk;
            *r = sd.xpane[xo + pk];
            *c0 = (sd.pbnd[*r] & ~(int64_t)(kSTile - 1)) + (int64_t)(j - cpre[pk]) * kSTile;
            *e0 = max(sd.pbnd[*r], *c0);
            *e1 = min(sd.pbnd[*r + 1], *c0 + kSTile);
        };
        // thread t holds rows c0 + 4 t + {0..3} and c0 + 2048 + 4 t + {0..3}: one 16-byte key load per group of 4
        constexpr int G = kSTileE / 4;   // row groups of 4 per thread
        struct Regs { uint32_t key[kSTileE]; int64_t val[NVC][kSTileE]; };
        auto load = [&](int64_t c0, Regs& rg) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int64_t i = c0 + (int64_t)g * (kSTile / G) + 4 * tid;
                const bool full = i + 3 < sd.nbatch;
                if (kcol && full && (((uintptr_t)(kcol + i)) & 15) == 0) {
                    const uint4 k4 = *(const uint4*)(kcol + i);
                    rg.key[4 * g] = k4.x; rg.key[4 * g + 1] = k4.y; rg.key[4 * g + 2] = k4.z; rg.key[4 * g + 3] = k4.w;
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) rg.key[4 * g + c] = (kcol && i + c < sd.nbatch) ? kcol[i + c] : 0u;
                }
#pragma unroll
                for (int v = 0; v < NVC; ++v) {
                    const int64_t* col = (const int64_t*)b.col[vcol[v]];
                    if (fl[v] && full && (((uintptr_t)(col + i)) & 15) == 0) {
                        const longlong2 a0 = *(const longlong2*)(col + i), a1 = *(const longlong2*)(col + i + 2);
                        rg.val[v][4 * g] = a0.x; rg.val[v][4 * g + 1] = a0.y; rg.val[v][4 * g + 2] = a1.x; rg.val[v][4 * g + 3] = a1.y;
                    } else {
#pragma unroll
                        for (int c = 0; c < 4; ++c) rg.val[v][4 * g + c] = (fl[v] && i + c < sd.nbatch) ? col[i + c] : 0;
                    }
                }
            }
        };
        Regs cur, nxt;
        int j = me;
        int64_t c0 = 0, e0 = 0, e1 = 0;
        int r = 0;
        if (j < c_total) { chunk_rows(j, &c0, &e0, &e1, &r); load(c0, cur); }
        while (j < c_total) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            const int jn = j + P;
            int64_t n0 = 0, n_e0 = 0, n_e1 = 0;
            int nr = 0;
            // the next chunk's loads go out before this chunk is partitioned (they land during the sort / stores)
            if (jn < c_total) {
                chunk_rows(jn, &n0, &n_e0, &n_e1, &nr);
                load(n0, nxt);
            }
            // slot j mod kSRing: its previous chunk (j - kSRing) must have been folded in by every consumer
            const int slot = j % kSRing;
            const uint32_t need = (uint32_t)P * (uint32_t)(j / kSRing);
            if (tid == 0) {
                int st = 1;
                while (ld_acq32(&cons[slot]) < need) {
                    if (ld_acq32(g_err) || timed_out(t0)) { st = 0; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                s_i[3] = st;
            }
            __syncthreads();
            if (!s_i[3]) { if (tid == 0) atomicOr(g_err, 2u); return; }
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            pt[1] += t1 - t0;
            const int64_t q = sd.q_lo + r;
            for (int t = tid; t <= P; t += kSBlock) s_tcnt[t] = 0;
            __syncthreads();
            int lp[kSTileE];
            uint32_t rank[kSTileE];
#pragma unroll
            for (int jj = 0; jj < kSTileE; ++jj) {
                const int64_t i = c0 + (int64_t)(jj >> 2) * (kSTile / G) + 4 * tid + (jj & 3);
                lp[jj] = -1;
                if (i >= e0 && i < e1 && (sd.key_col < 0 || cur.key[jj] < sd.num_keys)) {
                    int w = 1;
                    if (WHERE) {
                        w = where_decide_slow(p, b, i);
                        if (w < 0) atomicOr(&pane_err[q % sd.ring], EK_WIN_WHERE_ERROR);
                    }
                    if (w > 0) lp[jj] = (int)(cur.key[jj] >> sd.obits);
                }
                if (lp[jj] >= 0) rank[jj] = atomicAdd(&s_tcnt[lp[jj]], 1u);
            }
            __syncthreads();
            block_excl_scan<kSBlock>(s_tcnt, P, s_wsum);
#pragma unroll
            for (int jj = 0; jj < kSTileE; ++jj) {
                if (lp[jj] < 0) continue;
                const uint32_t sp = s_tcnt[lp[jj]] + rank[jj];
                s_klo[sp] = (uint16_t)(cur.key[jj] & omask);
#pragma unroll
                for (int v = 0; v < NVC; ++v) if (fl[v]) s_val[(size_t)v * kSTile + sp] = cur.val[v][jj];
            }
            __syncthreads();
            const uint32_t total = s_tcnt[P];
            const size_t region = ((size_t)x * kSRing + slot) * kSTile;
            // coalesced stores of the owner-sorted chunk: 8 key-lows / 2 values per lane and store
            for (uint32_t s = 8 * tid; s < total; s += 8 * kSBlock) {
                if (s + 8 <= total) {
                    *(uint4*)(sd.klo + region + s) = *(const uint4*)(s_klo + s);
                } else {
                    for (uint32_t u = s; u < total; ++u) sd.klo[region + u] = s_klo[u];
                }
            }
#pragma unroll
            for (int v = 0; v < NVC; ++v) {
                if (!fl[v]) continue;
                for (uint32_t s = 2 * tid; s < total; s += 2 * kSBlock) {
                    if (s + 2 <= total) *(longlong2*)(sd.val[v] + region + s) = *(const longlong2*)(s_val + (size_t)v * kSTile + s);
                    else sd.val[v][region + s] = s_val[(size_t)v * kSTile + s];
                }
            }
            // publish: every storing wave drains (this also waits for the next chunk's loads), then each consumer's
            // run descriptor goes out tagged with the chunk: (j + 1) << 32 | offset << 16 | length, one 8-byte
            // agent-scope atomic store per owner, so a consumer learns readiness and its run in one load
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid < P) {
                const uint64_t d = ((uint64_t)(uint32_t)(j + 1) << 32) | ((uint64_t)s_tcnt[tid] << 16) |
                                   (uint64_t)(s_tcnt[tid + 1] - s_tcnt[tid]);
                __hip_atomic_store(sd.ctab + ((size_t)x * kSRing + slot) * P + tid, (unsigned long long)d, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            pt[2] += __builtin_amdgcn_s_memrealtime() - t1;
            pt[5]++;
            cur = nxt;
            j = jn;
            c0 = n0; e0 = n_e0; e1 = n_e1; r = nr;
        }
    } else {
        // ======================================================== consumer
        const int owner = me;
        const int kpo = 1 << sd.obits;
        uint32_t* lcnt = (uint32_t*)(lds + lay.off_cnt);
        auto zero_table = [&]() {
            for (int k = tid; k < lay.bytes / 4; k += kSBlock) ((uint32_t*)lds)[k] = 0;
        };
        // finalise this owner's key range of pane r (k_agg's emission / merge for one key range)
        auto finish_pane = [&](int rr) {
            const int64_t q = sd.q_lo + rr;
            const int64_t slot = q % sd.ring;
            const int64_t dbase = sd.dbase[rr];
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
                const int32_t widx = sd.didx[rr];
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
            const bool fresh = sd.fresh[rr] != 0;
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

        zero_table();
        __syncthreads();
        // Every wave folds in its own chunks independently (no workgroup barrier inside a pane): wave w takes chunks
        // c0 + w, c0 + w + kSWaves, ... of the pane, polls up to kSWaveBatch of them at once (one tagged descriptor
        // per lane), folds the ready ones' runs with all its lanes (LDS atomics on the shared table) and counts
        // them consumed. The workgroup meets only at a pane's end, to finalise the pane.
        constexpr int kSWaves = kSBlock / 64;
        const int lane = tid & 63, wv = tid >> 6;
        __shared__ uint32_t w_start[kSWaves][kSWaveBatch], w_pre[kSWaves][kSWaveBatch + 1];
        for (int k = 0; k < nxp; ++k) {
            const int c1 = cpre[k + 1];
            int j = cpre[k] + wv;
            uint64_t idle_since = __builtin_amdgcn_s_memrealtime();
            bool failed = false;
            while (j < c1) {
                const uint64_t tc0 = __builtin_amdgcn_s_memrealtime();
                const int jj = j + kSWaves * lane;
                uint64_t d = 0;
                if (lane < kSWaveBatch && jj < c1)
                    d = __hip_atomic_load(sd.ctab + ((size_t)x * kSRing + jj % kSRing) * P + owner, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                const bool set = lane < kSWaveBatch && jj < c1 && (uint32_t)(d >> 32) == (uint32_t)(jj + 1);
                const unsigned long long m = __ballot(set);
                const int g = (int)__builtin_ctzll(~m);   // kSWaveBatch < 64: ~m is never 0
                if (g == 0) {
                    if (ld_acq32(g_err) || timed_out(idle_since)) { failed = true; break; }
                    __builtin_amdgcn_s_sleep(1);
                    pt[3] += __builtin_amdgcn_s_memrealtime() - tc0;
                    continue;
                }
                const uint32_t len = lane < g ? (uint32_t)(d & 0xFFFFu) : 0u;
                uint32_t incl = len;
                for (int o = 1; o < kSWaveBatch; o <<= 1) { const uint32_t y = __shfl_up(incl, o, 64); if (lane >= o) incl += y; }
                if (lane < g) {
                    w_start[wv][lane] = (uint32_t)(((size_t)x * kSRing + jj % kSRing) * kSTile) + (uint32_t)((d >> 16) & 0xFFFFu);
                    w_pre[wv][lane] = incl - len;
                }
                const uint32_t total = __shfl(incl, g - 1, 64);
                for (uint32_t v0 = 0; v0 < total; v0 += 64 * kSU) {
                    int kl[kSU];
                    int64_t raw[NVC][kSU];
#pragma unroll
                    for (int u = 0; u < kSU; ++u) {
                        const uint32_t v = v0 + u * 64 + lane;
                        kl[u] = -1;
                        if (v < total) {
                            int r = 0;   // run of row v: last r with w_pre[r] <= v
                            while (r + 1 < g && w_pre[wv][r + 1] <= v) ++r;
                            const size_t pos = (size_t)w_start[wv][r] + (v - w_pre[wv][r]);
                            kl[u] = (int)__builtin_nontemporal_load(sd.klo + pos);
#pragma unroll
                            for (int w = 0; w < NVC; ++w) raw[w][u] = fl[w] ? __builtin_nontemporal_load(sd.val[w] + pos) : 0;
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
                // the wave's loads of these slots have returned (their values went into the LDS atomics): free them
                if (lane < g) atomicAdd(&cons[jj % kSRing], 1u);
                j += kSWaves * g;
                idle_since = __builtin_amdgcn_s_memrealtime();
                pt[4] += idle_since - tc0;
                pt[6]++;
            }
            if (failed) atomicOr(g_err, 2u);
            __syncthreads();   // every wave has folded in its chunks of the pane
            if (tid == 0) s_i[6] = (int)ld_acq32(g_err);
            __syncthreads();
            if (s_i[6]) return;   // (uniform: one read for the whole workgroup)
            const uint64_t tc1 = __builtin_amdgcn_s_memrealtime();
            finish_pane(sd.xpane[xo + k]);
            __syncthreads();
            zero_table();
            __syncthreads();
            pt[7] += __builtin_amdgcn_s_memrealtime() - tc1;
        }
    }
    if (sd.prof && tid == 0)
        for (int k = 0; k < 8; ++k) sd.prof[(size_t)blockIdx.x * 8 + k] = pt[k];
}

}  // namespace ek
