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
#include "concat.hpp"

namespace rs {

__global__ __launch_bounds__(256) void concat_pieces_kernel(ConcatArgs a) {
  const int64_t total = a.batch * a.ncol;
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / a.ncol;
    const int c = (int)(i - b * a.ncol);
    int p = 0;
    while (p + 1 < a.np && c >= a.col0[p + 1]) ++p;
    const int j = c - a.col0[p];
    const float v = concat_value(a, p, j, b, bad);
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
  RS_REQUIRE(out && batch > 0, "rs_concat_pieces: null pointer");
  ConcatArgs a{};
  const int st = concat_fill(n_pieces, widths, out_cols, kinds, srcs, src_strides, tables, vocabs, out_stride,
                             "rs_concat_pieces", a);
  if (st != RS_OK) return st;
  const int cols = a.ncol;
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
