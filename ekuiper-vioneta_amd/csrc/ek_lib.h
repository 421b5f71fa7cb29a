// ek_lib.h — host wrappers implemented in ek_lib.hip (hipCUB radix sorts; see that file for where they run).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Stable ascending sort of (key, value) pairs on the low end_bit bits of the keys. With tmp == nullptr
// only *tmp_bytes is computed. Returns 0 on success.
int ekl_sort_pairs_u64(void* tmp, size_t* tmp_bytes, const uint64_t* kin, uint64_t* kout, const int64_t* vin,
                       int64_t* vout, int64_t n, int end_bit, hipStream_t s);
// Same for u32 keys with u32 values (key-major aggregation: (key, relative position) pairs).
int ekl_sort_pairs_u32(void* tmp, size_t* tmp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                       uint32_t* vout, int64_t n, int end_bit, hipStream_t s);
// u32 keys with 8-byte values (one-window key-major aggregation: the value column sorted by key, no gather).
int ekl_sort_pairs_u32_i64(void* tmp, size_t* tmp_bytes, const uint32_t* kin, uint32_t* kout, const int64_t* vin,
                           int64_t* vout, int64_t n, int end_bit, hipStream_t s);
