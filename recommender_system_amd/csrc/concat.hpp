// concat.hpp — the per-feature pieces of a model's concat (DIN.call,
// model/din.py:64-69,84-85: one Embedding lookup per non-behaviour sparse
// feature plus the raw dense features): their description (kernel
// arguments), the host-side validation and the device-side value of one
// piece column.  Used by rs_concat_pieces (concat.hip: the pieces written
// into the caller's buffer) and by the DIN tower (mlp.hip,
// rs_mlp_affine_pieces_fwd: the pieces read straight into the tower's input
// tile, no buffer, no launch of their own).
#pragma once
#include "rs_common.hpp"

namespace rs {

constexpr int CC_MAXP = 16;  // pieces (sparse fields + dense features) per launch

struct ConcatArgs {
  int np;                      // pieces
  int ncol;                    // output columns written (sum of widths)
  int col0[CC_MAXP + 1];       // first piece-local column of piece p (prefix sums of widths)
  int out_col[CC_MAXP];        // output column of the piece's first column
  int kind[CC_MAXP];           // RS_ID_* for a sparse piece, -1 for a dense one
  const void* src[CC_MAXP];    // ids (sparse) or values (dense, fp32)
  int64_t src_stride[CC_MAXP]; // elements between samples
  const float* table[CC_MAXP];
  int64_t vocab[CC_MAXP];
  float* out;
  int64_t out_stride;
  int64_t batch;
  int* err;
};

template <int KIND>
__device__ __forceinline__ bool cc_id(const void* p, int64_t off, int64_t vocab, int64_t& id) {
  typedef Ids<KIND> I;
  return I::decode(I::load(p, off), vocab, id);
}

// value of column j of piece p for sample b (an out-of-range id: 0, bad = true)
__device__ __forceinline__ float concat_value(const ConcatArgs& a, int p, int j, int64_t b, bool& bad) {
  if (a.kind[p] < 0) return static_cast<const float*>(a.src[p])[b * a.src_stride[p] + j];
  int64_t id = 0;
  bool ok;
  const int64_t off = b * a.src_stride[p];
  switch (a.kind[p]) {
    case RS_ID_I32: ok = cc_id<0>(a.src[p], off, a.vocab[p], id); break;
    case RS_ID_I64: ok = cc_id<1>(a.src[p], off, a.vocab[p], id); break;
    default: ok = cc_id<2>(a.src[p], off, a.vocab[p], id); break;
  }
  bad |= !ok;
  const int k = a.col0[p + 1] - a.col0[p];
  return ok ? a.table[p][id * k + j] : 0.f;
}

// Host: validate and fill the pieces (RS_OK or RS_ERR_ARG with the message set)
inline int concat_fill(int n_pieces, const int* widths, const int* out_cols, const int* kinds,
                       const void* const* srcs, const int64_t* src_strides, const float* const* tables,
                       const int64_t* vocabs, int64_t out_stride, const char* what, ConcatArgs& a) {
  RS_REQUIRE(n_pieces > 0 && n_pieces <= CC_MAXP, "%s: 1..%d pieces", what, CC_MAXP);
  RS_REQUIRE(widths && out_cols && kinds && srcs && src_strides, "%s: null pointer", what);
  a.np = n_pieces;
  int cols = 0;
  for (int p = 0; p < n_pieces; ++p) {
    const bool sparse = kinds[p] >= 0;
    RS_REQUIRE(widths[p] >= 1 && out_cols[p] >= 0 && (int64_t)out_cols[p] + widths[p] <= out_stride && srcs[p],
               "%s: piece %d: bad width / column / source", what, p);
    RS_REQUIRE(kinds[p] == -1 || (kinds[p] >= RS_ID_I32 && kinds[p] <= RS_ID_F32), "%s: bad kind", what);
    RS_REQUIRE(!sparse || (tables && tables[p] && vocabs && vocabs[p] >= 1),
               "%s: sparse piece %d needs a table and a vocab", what, p);
    RS_REQUIRE(src_strides[p] >= (sparse ? 1 : widths[p]), "%s: piece %d: bad source stride", what, p);
    a.col0[p] = cols;
    cols += widths[p];
    a.out_col[p] = out_cols[p];
    a.kind[p] = kinds[p];
    a.src[p] = srcs[p];
    a.src_stride[p] = src_strides[p];
    a.table[p] = sparse ? tables[p] : nullptr;
    a.vocab[p] = sparse ? vocabs[p] : 0;
  }
  a.col0[n_pieces] = cols;
  a.ncol = cols;
  return RS_OK;
}

}  // namespace rs
