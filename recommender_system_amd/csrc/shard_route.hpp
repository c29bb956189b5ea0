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
  int world;
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

// The same route, one thread per LOOKUP (b, c) instead of one per record
// word (RS_OPT_SHARD_ROUTE 0, the default): the thread's id is requested
// first, the field metadata (offsets, vocab, the owners whose field range
// holds each field) is staged in LDS meanwhile, so the launch makes one
// dependent memory trip (ids) instead of three (owner ranges -> ids and
// field metadata).  Lookup (b, c) writes its word in the record of every
// owner whose range holds field c (its local row at the row's owner, -1 at
// the others); the thread of an owner's last field also writes that owner's
// padding words (j in [n_owned, stride)).  Needs n_fields <= RT_MAXF and a
// field range per owner as the host computes it (the fields its row block
// intersects).
constexpr int RT_MAXF = 256;
constexpr int RT_MAXW = 64;
struct RouteLds {
  int64_t off[RT_MAXF], voc[RT_MAXF];
  int olo[RT_MAXF], ohi[RT_MAXF];  // owners whose field range holds field c (olo > ohi: none)
  int c0[RT_MAXW], nf[RT_MAXW];
  int empty_owner;                 // some owner holds no field (its words: -1, written by the c == 0 threads)
};

template <int NTH>
__device__ __forceinline__ void lookup_route_part(const RouteArgs& a, int blk, int nblk, RouteLds& L) {
  const int F = a.n_fields, W = a.world, B = a.batch;
  const int n = B * F;
  int idx = blk * NTH + (int)threadIdx.x;
  auto load_id = [&](int i, int64_t& iv, float& fv) {
    const int b = i / F;
    const int64_t off = (int64_t)b * a.id_stride + (i - b * F);
    if (a.id_kind == RS_ID_F32) fv = static_cast<const float*>(a.ids)[off];
    else if (a.id_kind == RS_ID_I64) iv = static_cast<const int64_t*>(a.ids)[off];
    else iv = static_cast<const int32_t*>(a.ids)[off];
  };
  int64_t iv = 0;
  float fv = 0.f;
  if (idx < n) load_id(idx, iv, fv);  // in flight while the metadata is staged
  if (threadIdx.x == 0) L.empty_owner = 0;
  for (int t = threadIdx.x; t < W; t += NTH) {
    L.c0[t] = a.ofl[2 * t];
    L.nf[t] = a.ofl[2 * t + 1];
  }
  for (int t = threadIdx.x; t < F; t += NTH) {
    L.off[t] = a.offs[t];
    L.voc[t] = a.vocab[t];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < F; t += NTH) {
    int lo = W, hi = -1;
    for (int o = 0; o < W; ++o) {
      if (t >= L.c0[o] && t < L.c0[o] + L.nf[o]) {
        lo = min(lo, o);
        hi = max(hi, o);
      }
    }
    L.olo[t] = lo;
    L.ohi[t] = hi;
  }
  for (int t = threadIdx.x; t < W; t += NTH)
    if (L.nf[t] == 0) L.empty_owner = 1;
  __syncthreads();
  for (bool first = true; idx < n; idx += nblk * NTH, first = false) {
    if (!first) load_id(idx, iv, fv);
    const int b = idx / F, c = idx - b * F;
    bool ok;
    int64_t id;
    if (a.id_kind == RS_ID_F32) {
      ok = fv > -1.0f && static_cast<double>(fv) < static_cast<double>(L.voc[c]);
      id = ok ? static_cast<int64_t>(fv) : 0;
    } else {
      ok = iv >= 0 && iv < L.voc[c];
      id = ok ? iv : 0;
    }
    const int olo = L.olo[c], ohi = L.ohi[c];
    int own = -1;
    int64_t local = 0;
    if (!ok) {
      flag_error(a.err);
    } else {
      const int64_t row = L.off[c] + id;
      own = olo;
      while (own < ohi && row >= (int64_t)(own + 1) * a.rpr) ++own;
      local = row - (int64_t)own * a.rpr;
      if (local < 0 || local >= a.rpr) own = -1;  // not a layout the host routes (the word stays -1)
    }
    int32_t slot = -1;
    for (int o = olo; o <= ohi; ++o) {
      const int64_t rec = (int64_t)o * B + b;
      const int j = c - L.c0[o];
      a.send[rec * a.rec_stride + j] = o == own ? (int32_t)local : -1;
      if (o == own) slot = (int32_t)(rec * a.stride + j);
      if (c == L.c0[o] + L.nf[o] - 1)
        for (int jj = L.nf[o]; jj < a.stride; ++jj) a.send[rec * a.rec_stride + jj] = -1;
    }
    if (c == 0 && L.empty_owner) {
      for (int o = 0; o < W; ++o)
        if (L.nf[o] == 0)
          for (int jj = 0; jj < a.stride; ++jj) a.send[((int64_t)o * B + b) * a.rec_stride + jj] = -1;
    }
    if (a.slot_of != nullptr) a.slot_of[(int64_t)b * F + c] = slot;
  }
}

}  // namespace rs
