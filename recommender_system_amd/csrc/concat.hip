// concat.hip — one launch for the per-feature pieces of a model's concat that
// live in DIFFERENT tables: DIN.call (model/din.py:64-69,84-85) concatenates the
// embeddings of every non-behaviour sparse feature (one EmbedLayer, i.e. one
// table, each) and the raw dense features beside the pooled attention; the
// reference runs one Embedding lookup per feature and a concat.  Here every
// piece is written straight into its columns of the caller's [B, width]
// buffer by one kernel: thread = (sample, output column of a piece), the
// column's piece found in a small table in the kernel arguments.
// Out-of-range ids (Keras Embedding raises) write a zero row and set the
// error flag (rs_embed_gather's rule).
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

__global__ __launch_bounds__(256) void concat_pieces_kernel(ConcatArgs a) {
  const int64_t total = a.batch * a.ncol;
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / a.ncol;
    const int c = (int)(i - b * a.ncol);
    int p = 0;
    while (p + 1 < a.np && c >= a.col0[p + 1]) ++p;
    const int j = c - a.col0[p];
    float v;
    if (a.kind[p] < 0) {
      v = static_cast<const float*>(a.src[p])[b * a.src_stride[p] + j];
    } else {
      int64_t id = 0;
      bool ok;
      const int64_t off = b * a.src_stride[p];
      switch (a.kind[p]) {
        case RS_ID_I32: ok = cc_id<0>(a.src[p], off, a.vocab[p], id); break;
        case RS_ID_I64: ok = cc_id<1>(a.src[p], off, a.vocab[p], id); break;
        default: ok = cc_id<2>(a.src[p], off, a.vocab[p], id); break;
      }
      const int k = a.col0[p + 1] - a.col0[p];
      v = ok ? a.table[p][id * k + j] : 0.f;
      bad |= !ok;
    }
    a.out[b * a.out_stride + a.out_col[p] + j] = v;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) flag_error(a.err);
}

}  // namespace rs

using namespace rs;

extern "C" int rs_concat_pieces(int n_pieces, const int* widths, const int* out_cols, const int* kinds,
                                const void* const* srcs, const int64_t* src_strides, const float* const* tables,
                                const int64_t* vocabs, float* out, int64_t out_stride, int64_t batch, int* err_flag,
                                rs_stream_t stream) {
  if (batch == 0 || n_pieces == 0) return RS_OK;  // nothing to launch (null data pointers allowed)
  RS_REQUIRE(n_pieces > 0 && n_pieces <= CC_MAXP, "rs_concat_pieces: 1..%d pieces", CC_MAXP);
  RS_REQUIRE(widths && out_cols && kinds && srcs && src_strides && out && batch > 0, "rs_concat_pieces: null pointer");
  ConcatArgs a{};
  a.np = n_pieces;
  int cols = 0;
  for (int p = 0; p < n_pieces; ++p) {
    const bool sparse = kinds[p] >= 0;
    RS_REQUIRE(widths[p] >= 1 && out_cols[p] >= 0 && (int64_t)out_cols[p] + widths[p] <= out_stride && srcs[p],
               "rs_concat_pieces: piece %d: bad width / column / source", p);
    RS_REQUIRE(kinds[p] == -1 || (kinds[p] >= RS_ID_I32 && kinds[p] <= RS_ID_F32), "rs_concat_pieces: bad kind");
    RS_REQUIRE(!sparse || (tables && tables[p] && vocabs && vocabs[p] >= 1),
               "rs_concat_pieces: sparse piece %d needs a table and a vocab", p);
    RS_REQUIRE(src_strides[p] >= (sparse ? 1 : widths[p]), "rs_concat_pieces: piece %d: bad source stride", p);
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
  a.out = out;
  a.out_stride = out_stride;
  a.batch = batch;
  a.err = err_flag;
  RS_REQUIRE(batch * cols < ((int64_t)1 << 40), "rs_concat_pieces: too large");
  int64_t g = (batch * cols + 255) / 256;
  if (g > 4096) g = 4096;
  concat_pieces_kernel<<<(unsigned)g, 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_concat_pieces");
}
