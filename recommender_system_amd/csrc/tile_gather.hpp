// tile_gather.hpp — the headline kernel's front end (embed_fm.hip, kernarg
// path) for the kernels that assemble a 16-sample tile of embedding rows in
// LDS before their interaction phase: embed_cross / dcn_fused (cross.hip,
// CrossLayer / DCN, layer/interaction.py:75-83, model/dcn.py:24-27) and
// inner_fast (inner.hip, InnerProductLayer / PNN, layer/interaction.py:170-183).
//
//   * field metadata (offset, vocab) as kernel arguments (FieldMeta by value):
//     every wave owns whole fields, so they are wave-uniform scalar loads —
//     no cooperative id tile, no barrier before the first row request, and
//     no per-wave metadata loads that would hit one hot L2 line;
//   * wave w owns fields w (pass 0) and w + NW (pass 1); lane = 4 sample +
//     chunk (k = 16: four adjacent lanes read one whole 64-B row, 16 samples
//     per wave-instruction);
//   * both passes' ids are requested first; the second pass's rows after
//     the first pass's have arrived (two row bursts, as the headline kernel).
// k = 16 and at most 2 NW fields only (the configs' shapes); the kernels keep
// their cooperative-tile front end for every other shape.
#pragma once
#include "embed_fm.hpp"
#include "rs_common.hpp"

namespace rs {

// store(s, c, q, x): float4 x = chunk q of sample s's row of field c (zeros
// for a bad id or a padded sample s >= rows).  Returns whether this lane saw
// an out-of-range id of a valid sample.
template <int NW, int KIND, class Store>
__device__ __forceinline__ bool gather_tile_k16(const void* ids, int64_t id_stride, const float* __restrict__ table,
                                                const FieldMeta* m, int F, int64_t b0, int rows, Store&& store) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane >> 2, q = lane & 3;
  const int64_t bb = b0 + (s < rows ? s : rows - 1);
  const int c0 = w, c1 = w + NW;
  typename I::raw_t r0{}, r1{};
  if (c0 < F) r0 = I::load(ids, bb * id_stride + c0);
  if (c1 < F) r1 = I::load(ids, bb * id_stride + c1);
  bool bad = false;
  auto pass = [&](int c, typename I::raw_t r) {
    int64_t id;
    const bool ok = I::decode(r, m->voc[c], id);
    bad |= !ok && s < rows;
    floatx4 x = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(table + (m->off[c] + id) * 16) + q);
    if (!ok || s >= rows) x = floatx4{0.f, 0.f, 0.f, 0.f};
    store(s, c, q, x);
  };
  if (c0 < F) pass(c0, r0);
  if (c1 < F) pass(c1, r1);
  return bad;
}

}  // namespace rs
