// shard_route.hpp — field route of the sharded FM's partial protocol, shared
// by the standalone kernel (shard.hip, rs_shard_field_route) and the fused
// pipelined step (embed_fm.hip, rs_shard_fm_pipe).
//
// A block split of the concatenated table (global row of (b,c) =
// field_offsets[c] + id) gives owner o a contiguous FIELD range
// [field_lo(o), field_lo(o) + n_owned(o)) — the fields its row block
// intersects.  Message to owner o: batch records of rec_stride int32 words;
// word j < stride of record b = the local row of lookup (b, field_lo(o) + j)
// if o owns it, else -1 (words past `stride` are left alone: the pipelined
// exchange keeps FM partials there).  Pure index arithmetic: no scan, no
// capacity, no overflow; every row-id word is written every step.
#pragma once
#include "rs_common.hpp"

namespace rs {

struct RouteArgs {
  const void* ids;
  int id_kind;
  int64_t id_stride;
  const int64_t* offs;
  const int64_t* vocab;
  int64_t rpr;         // rows per rank
  const int32_t* ofl;  // [world][2] = (field_lo, n_owned)
  int stride;          // row-id words per record (>= every n_owned)
  int batch;
  int64_t rec_stride;  // words per record
  int32_t* send;
  int* err;
  int64_t total;       // world * batch * stride (< 2^31)
  // row protocol (rs_shard_row_route) only, else null: slot_of[b*n_fields+c]
  // = the record word of lookup (b, c) = its row's index in the owner's reply
  int32_t* slot_of;
  int n_fields;
};

template <int NTH>
__device__ __forceinline__ void field_route_part(const RouteArgs& a, int blk, int nblk) {
  const int total = (int)a.total;
  for (int idx = blk * NTH + threadIdx.x; idx < total; idx += nblk * NTH) {
    const int ob = idx / a.stride;
    const int j = idx - ob * a.stride;
    const int o = ob / a.batch;
    const int b = ob - o * a.batch;
    const int c0 = a.ofl[2 * o], nf = a.ofl[2 * o + 1];
    int32_t out = -1;
    if (j < nf) {
      const int c = c0 + j;
      const int64_t off = (int64_t)b * a.id_stride + c;
      int64_t id;
      bool ok;
      if (a.id_kind == RS_ID_F32) {
        const float f = static_cast<const float*>(a.ids)[off];
        ok = f > -1.0f && static_cast<double>(f) < static_cast<double>(a.vocab[c]);
        id = ok ? static_cast<int64_t>(f) : 0;
      } else {
        id = (a.id_kind == RS_ID_I64) ? static_cast<const int64_t*>(a.ids)[off]
                                      : static_cast<const int32_t*>(a.ids)[off];
        ok = id >= 0 && id < a.vocab[c];
      }
      if (!ok) {
        flag_error(a.err);
      } else {
        const int64_t local = a.offs[c] + id - (int64_t)o * a.rpr;
        if (local >= 0 && local < a.rpr) out = (int32_t)local;
      }
      // exactly one owner holds a valid lookup; a bad id is -1 (every owner
      // of its field writes the same value)
      if (a.slot_of != nullptr && (out >= 0 || !ok)) a.slot_of[(int64_t)b * a.n_fields + c] = out >= 0 ? idx : -1;
    }
    a.send[(int64_t)ob * a.rec_stride + j] = out;
  }
}

}  // namespace rs
