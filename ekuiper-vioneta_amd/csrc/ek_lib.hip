// ek_lib.hip — hipCUB radix sorts (separate translation unit: hipCUB headers are heavy). Two users:
//   * range mode, when an out-of-order batch is merged into the ts-ordered event buffer (the release order of
//     WatermarkOp, watermark_op.go:157-168: stable in arrival order for equal ts) — off the in-order hot path;
//   * the key-major span sort of range windows (ek_engine.hip km_run(): (key, position) or (key, value) pairs) — only
//     as the fallback of the MSD partition (km_msd / grp_run: skewed keys, validity, K outside [2^16, 2^27]); no
//     BASELINE config runs it since round 5 (no rocPRIM kernel in profiles/r05_kernels_*.csv or r06).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "ek_lib.h"

int ekl_sort_pairs_u64(void* tmp, size_t* tmp_bytes, const uint64_t* kin, uint64_t* kout, const int64_t* vin,
                       int64_t* vout, int64_t n, int end_bit, hipStream_t s) {
    // LSD radix sort: stable, so equal timestamps keep their input order (buffer tail first, then arrival)
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kin, kout, vin, vout, (int)n, 0, end_bit, s);
    return e == hipSuccess ? 0 : -1;
}

int ekl_sort_pairs_u32(void* tmp, size_t* tmp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                       uint32_t* vout, int64_t n, int end_bit, hipStream_t s) {
    // stable: each key's rows keep their buffer order
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kin, kout, vin, vout, (int)n, 0, end_bit, s);
    return e == hipSuccess ? 0 : -1;
}

int ekl_sort_pairs_u32_i64(void* tmp, size_t* tmp_bytes, const uint32_t* kin, uint32_t* kout, const int64_t* vin,
                           int64_t* vout, int64_t n, int end_bit, hipStream_t s) {
    // stable: each key's values keep their buffer order (one-window key-major aggregation sorts the values directly)
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kin, kout, vin, vout, (int)n, 0, end_bit, s);
    return e == hipSuccess ? 0 : -1;
}
