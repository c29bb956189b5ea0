// radix_sort.hpp — the hand-written stable key/value sort and integer scan
// behind the row-sparse scatter-adds (rs_embedding_sgd, rs_fm_train_step) and
// the dedup route's large-batch path (rs_shard_dedup_route).  Replaces the
// library radix sort / scan those call sites used; see radix_sort.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rs {

// Workspace bytes of sort_pairs_u32 for n pairs (256-B aligned pieces).
int64_t sort_pairs_ws_bytes(int64_t n);
// Stable ascending sort of (key, val) pairs by the low `bits` bits of key
// (1 <= bits <= 32): LSD passes of 8 bits; pairs with equal keys keep their
// input order.  key_in / val_in are not modified.  Every launch goes on `st`.
hipError_t sort_pairs_u32(const uint32_t* key_in, const uint32_t* val_in, uint32_t* key_out, uint32_t* val_out,
                          int64_t n, int bits, void* ws, hipStream_t st);

// Workspace bytes of inclusive_sum_i32 for n values.
int64_t scan_ws_bytes(int64_t n);
// out[i] = in[0] + ... + in[i] (in and out may alias).
hipError_t inclusive_sum_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, hipStream_t st);

}  // namespace rs
