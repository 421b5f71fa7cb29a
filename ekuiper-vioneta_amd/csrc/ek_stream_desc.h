// ek_stream_desc.h — shared between the engine (host side) and ek_stream.hip (the kernel): the streaming path's
// constants, its launch descriptor and the launcher. See ek_stream.h for the design.
#pragma once
#include "ek_kernels.h"

namespace ek {

constexpr int kSBlock = 512;          // threads per workgroup (two per CU: one producer, one consumer)
constexpr int kSTile = 2048;          // events per chunk (4 per producer thread: two chunks in registers fit 128 VGPRs)
constexpr int kSTileE = kSTile / kSBlock;
#ifndef EK_SRING
#define EK_SRING 64
#endif
constexpr int kSRing = EK_SRING;      // staging slots per XCD (64 x 36 KiB for two f64 columns: L2-resident)
constexpr int kSXcd = 8;
constexpr int kSMaxOwners = 64;       // consumers (= producers) per XCD
constexpr int kSBatch = 64;           // chunks folded in per consume step (<= 64: one wave polls them)
constexpr int kSU = 4;                // staged rows in flight per lane while folding in
constexpr int kSWaveBatch = 8;        // chunks a consumer wave polls at once
constexpr int kSMaxXPanes = 512;      // panes per XCD per launch

struct StreamDesc {
    int64_t nbatch;
    int64_t q_lo;
    int32_t n_panes;       // panes [q_lo, q_lo + n_panes) of the batch
    int32_t ring;          // pane-state ring
    int32_t key_col, n_where;
    uint32_t num_keys;
    int32_t owners;        // consumers (= producers) per XCD
    int32_t obits;         // key range of a consumer = [o << obits, (o + 1) << obits)
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
    uint32_t* sync;        // [0] arrived, [1] err, [2..10) members, then cons[8][kSRing]
    uint16_t* klo;         // [kSXcd][kSRing][kSTile]
    int64_t* val[kMaxVC];  // [kSXcd][kSRing][kSTile]
    unsigned long long* ctab;   // [kSXcd][kSRing][owners]: tagged run descriptor (chunk + 1) << 32 | offset << 16 | length
    unsigned long long* prof;   // optional [grid][8] per-workgroup time split (EKGPU_STREAM_PROF)
};

__device__ __forceinline__ int xcc_id() {
    // HW_REG_XCC_ID (hwreg 20), bits [3:0]
    return (int)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 15);
}
__device__ __forceinline__ uint32_t ld_acq32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ek_stream.hip: k_stream<nvc (1..2), where> on `grid` workgroups of kSBlock threads with `lds` dynamic bytes
void launch_stream_kernel(int nvc, bool where, int grid, size_t lds, hipStream_t s, DPlan* p, const DBatch& db,
                          const StreamDesc& sd, const LdsLayout& lay, const DState& ds, const Results& rv, int32_t* perr);

}  // namespace ek
