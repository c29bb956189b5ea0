// mlp.hip — the whole DNN tower of a CTR model in one launch: DNNLayer
// (layer/interaction.py:30-46: Dense(h_i, act) per hidden unit count, then a
// linear Dense(output_dim)), optionally closed by the model head
// sigmoid(c0*z + c1*extra) (DeepFM model/deepFM.py:30 with extra = FM logit).
//
// Layout and schedule (gfx950):
//   * A workgroup owns 16 samples (one v_mfma_f32_16x16x4_f32 row tile) and
//     16 waves.  The 16 x K0 input tile is staged in LDS once; every layer
//     reads its input tile from LDS and writes its activations back to LDS
//     (ping-pong buffers), so hidden activations never touch HBM.
//   * Weights are pre-packed (rs_mlp_prepare) into MFMA B-fragment order:
//     for output tile t (16 units) and k-group g (16 inputs) a contiguous
//     1 KB block in which lane l holds float4 W[16g + 4(l>>4) + j][16t + (l&15)],
//     j = 0..3.  One coalesced global_load_dwordx4 per lane feeds 4 MFMAs; the
//     A operand is the matching ds_read_b128 of the LDS tile (the k order
//     inside a group is permuted identically on both sides).
//   * Waves split a layer into (output tile, k-slice) items; k-slices are
//     summed through LDS in a fixed order (deterministic).  Bias and
//     activation are fused into the epilogue.
//   * The packed weights (0.6 MB for 429-256-128-64-1) are shared by every
//     workgroup and stay L2-resident; per 4 MFMAs a wave reads 1 KB of
//     weights from L2 and 1 KB of activations from LDS, both under the
//     per-CU rates at MFMA peak.
#include "concat.hpp"
#include "mlp_tower.hpp"

namespace rs {

struct MlpPrepArgs {
  const float* W[MLP_MAXL];
  const float* bias[MLP_MAXL];
  const float* alpha[MLP_MAXL];
  const int32_t* in_rows;
  MlpGeom g;
  float* out;
};

__global__ void mlp_prepare_kernel(MlpPrepArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.g.total) return;
  float v = 0.f;
  if (i < a.g.wtot) {
    int l = 0;
    while (l + 1 < a.g.L && i >= a.g.off[l + 1]) ++l;
    const int64_t r = i - a.g.off[l];
    const int Kp = a.g.Kp[l], K = a.g.K[l], N = a.g.N[l];
    const int G = Kp / 16;
    const int j = (int)(r & 3), lane = (int)((r >> 2) & 63);
    const int64_t blk = r >> 8;
    const int gg = (int)(blk % G), t = (int)(blk / G);
    const int k = 16 * gg + 4 * (lane >> 4) + j, n = 16 * t + (lane & 15);
    const int kr = (l == 0 && a.in_rows) ? a.in_rows[k] : k;
    if (kr >= 0 && kr < K && n < N) v = a.W[l][(int64_t)kr * N + n];
  } else {
    const int p = (int)(i - a.g.wtot);
    int l = 0;
    while (l + 1 < a.g.L && p >= a.g.poff[l + 1]) ++l;
    const int q = p - a.g.poff[l], Np = a.g.Np[l], N = a.g.N[l];
    const int n = q < Np ? q : q - Np;
    const float* src = q < Np ? a.bias[l] : a.alpha[l];
    v = (n < N && src) ? src[n] : 0.f;
  }
  a.out[i] = v;
}

// PC: some input columns are concat pieces (rs_mlp_affine_pieces_fwd: DIN's
// other sparse embeddings + dense features, model/din.py:64-69,84-85) read
// straight into the input tile — id, then table row — instead of from x;
// at most 64 input columns (one per lane)
template <int NW, bool TAIL, bool PC>
__device__ __forceinline__ void mlp_tower_body(const MlpArgs& a, const ConcatArgs* pc) {
  extern __shared__ float smem[];
  const int RS = a.rs;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * 16;
  MLP_STAMP(0);

  // layer-0 weights first (independent of everything), then the input tile
  // (one row per wave, coalesced; rows past M re-read row M-1 and are never
  // stored) and the bias/alpha block into LDS
  floatx4 ring[MLP_R];
  mlp_first_fill<NW>(a, ring);
  for (int r = w; r < 16; r += NW) {
    const int64_t m = m0 + r < a.M ? m0 + r : a.M - 1;
    const float* xr = a.x + m * a.xs;
    constexpr int XU = PC ? 1 : MLP_MAXD / 64;
    float xv[XU];
    if constexpr (PC) {
      // the lane's column: a piece column (its piece found in the kernarg
      // table) or a column of x
      int p = -1;
      for (int q = 0; q < pc->np; ++q)
        if (lane >= pc->out_col[q] && lane < pc->out_col[q] + (pc->col0[q + 1] - pc->col0[q])) p = q;
      bool bad = false;
      xv[0] = lane >= a.K0 ? 0.f : (p >= 0 ? concat_value(*pc, p, lane - pc->out_col[p], m, bad) : xr[lane]);
      if (__any(bad && m0 + r < a.M) && lane == 0) flag_error(pc->err);
    } else {
#pragma unroll
      for (int i = 0; i < XU; ++i) {
        const int c = lane + 64 * i;
        xv[i] = c < a.K0 ? xr[c] : 0.f;
      }
    }
    if (a.in_scale) {  // the BatchNormalization affine, as rs_affine_act computes it
#pragma unroll
      for (int i = 0; i < XU; ++i) {
        const int c = lane + 64 * i;
        if (c < a.K0) {
#pragma clang fp contract(off)  // two roundings, as rs_affine_act (no fma)
          xv[i] = xv[i] * a.in_scale[c] + a.in_shift[c];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < XU; ++i) {
      const int c = lane + 64 * i;
      if (c < a.Kp[0]) smem[r * RS + c] = xv[i];
    }
  }
  float* par = smem + 32 * RS + NW * 256;
  for (int i = threadIdx.x; i < a.ptot; i += NW * 64) par[i] = a.prep[a.wtot + i];
  MLP_STAMP(1);
  if constexpr (TAIL) {
    // a 256 -> 128 -> 64 -> 1 tail (the reference's DNN widths): layer 0 as
    // usual, the rest as the split-K tail on all 16 waves (mlp_tail_splitk)
    if (a.Np[0] == NW * 16) mlp_layer0_tiles<NW>(a, smem, ring);
    else mlp_tower_tile<NW>(a, smem, m0, ring, nullptr, 0, 1);
    mlp_tail_run<NW>(a, smem, m0, nullptr);
  } else {
    mlp_tower_tile<NW>(a, smem, m0, ring);
  }
}

template <int NW, bool TAIL = false>
__global__ __launch_bounds__(NW * 64) void mlp_tower(MlpArgs a) {
  mlp_tower_body<NW, TAIL, false>(a, nullptr);
}
template <int NW, bool TAIL = false>
__global__ __launch_bounds__(NW * 64) void mlp_tower_pc(MlpArgs a, ConcatArgs pc) {
  mlp_tower_body<NW, TAIL, true>(a, &pc);
}

}  // namespace rs

using namespace rs;

static unsigned long long* g_mlp_dbg = nullptr;
extern "C" void rs_diag_mlp_set_dbg(unsigned long long* p) { g_mlp_dbg = p; }
namespace rs {
unsigned long long* mlp_diag_dbg() { return g_mlp_dbg; }  // the fused towers' stamps too (deepfm_run)
}  // namespace rs

extern "C" int64_t rs_mlp_prepared_size(int n_layers, const int* dims) {
  MlpGeom g;
  if (!mlp_geom(n_layers, dims, g)) {
    set_error("rs_mlp_prepared_size: need 1..%d layers with widths 1..%d (and <= 160 KB LDS)",
              MLP_MAXL, MLP_MAXD);
    return -1;
  }
  return g.total;
}

extern "C" int rs_mlp_prepare(int n_layers, const int* dims, const float* const* W, const float* const* bias,
                              const float* const* alpha, const int32_t* in_rows, float* prepared,
                              rs_stream_t stream) {
  MlpGeom g;
  RS_REQUIRE(mlp_geom(n_layers, dims, g), "rs_mlp_prepare: need 1..%d layers with widths 1..%d", MLP_MAXL,
             MLP_MAXD);
  RS_REQUIRE(W && prepared, "rs_mlp_prepare: null pointer");
  MlpPrepArgs a{};
  for (int l = 0; l < n_layers; ++l) {
    RS_REQUIRE(W[l], "rs_mlp_prepare: layer %d has no kernel", l);
    a.W[l] = W[l];
    a.bias[l] = bias ? bias[l] : nullptr;
    a.alpha[l] = alpha ? alpha[l] : nullptr;
  }
  a.in_rows = in_rows;
  a.g = g;
  a.out = prepared;
  mlp_prepare_kernel<<<(unsigned)((g.total + 255) / 256), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_mlp_prepare");
}

static int mlp_run(const float* x, int64_t x_stride, const float* in_scale, const float* in_shift, int n_layers,
                   const int* dims, const int* acts, const float* prepared, float* y, int64_t y_stride, int head,
                   const float* extra, float c0, float c1, int64_t batch, rs_stream_t stream,
                   const ConcatArgs* pc = nullptr) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  MlpGeom g;
  RS_REQUIRE(mlp_geom(n_layers, dims, g), "rs_mlp_fwd: need 1..%d layers with widths 1..%d", MLP_MAXL, MLP_MAXD);
  RS_REQUIRE(x && prepared && y && acts, "rs_mlp_fwd: null pointer");
  RS_REQUIRE(batch >= 0 && x_stride >= dims[0], "rs_mlp_fwd: bad batch/stride");
  RS_REQUIRE(head == 0 || head == 1, "rs_mlp_fwd: head must be 0 (raw) or 1 (sigmoid)");
  RS_REQUIRE(head == 0 ? y_stride >= dims[n_layers] : (dims[n_layers] == 1 && y_stride >= 1),
             "rs_mlp_fwd: bad output shape (head=1 needs output width 1)");
  MlpArgs a{};
  RS_REQUIRE(mlp_fill_args(g, acts, prepared, a), "rs_mlp_fwd: bad activation");
  if (batch == 0) return RS_OK;
  a.x = x;
  a.xs = x_stride;
  a.y = y;
  a.ys = y_stride;
  a.head = head;
  a.extra = extra;
  a.c0 = c0;
  a.c1 = c1;
  a.M = batch;
  a.dbg = g_mlp_dbg;
  a.in_scale = in_scale;
  a.in_shift = in_shift;
  const size_t lds = g.lds;
  const int64_t grid = (batch + 15) / 16;
  RS_REQUIRE(grid < (1ll << 31), "rs_mlp_fwd: batch too large");
  int gwa = 0, gwb = 0;
  const bool tail = MLP_NW == 16 && mlp_tail_ok(a.Np, a.Kp, a.N, a.L, 1, gwa, gwb) && gwa == 8 && gwb == 2;
  if (pc) {
    if (tail) {
      static LdsAttr lds_pt;
      lds_attr(lds_pt, (const void*)mlp_tower_pc<MLP_NW, true>, lds);
      mlp_tower_pc<MLP_NW, true><<<(unsigned)grid, MLP_NW * 64, lds, as_stream(stream)>>>(a, *pc);
    } else {
      static LdsAttr lds_p;
      lds_attr(lds_p, (const void*)mlp_tower_pc<MLP_NW>, lds);
      mlp_tower_pc<MLP_NW><<<(unsigned)grid, MLP_NW * 64, lds, as_stream(stream)>>>(a, *pc);
    }
    return launch_status("rs_mlp_affine_pieces_fwd");
  }
  if (tail) {
    static LdsAttr lds_tail;
    lds_attr(lds_tail, (const void*)mlp_tower<MLP_NW, true>, lds);
    mlp_tower<MLP_NW, true><<<(unsigned)grid, MLP_NW * 64, lds, as_stream(stream)>>>(a);
    return launch_status("rs_mlp_fwd");
  }
  static LdsAttr lds_set;  // opt in to exactly what is needed beyond the default
  lds_attr(lds_set, (const void*)mlp_tower<MLP_NW>, lds);
  mlp_tower<MLP_NW><<<(unsigned)grid, MLP_NW * 64, lds, as_stream(stream)>>>(a);
  return launch_status("rs_mlp_fwd");
}

extern "C" int rs_mlp_fwd(const float* x, int64_t x_stride, int n_layers, const int* dims, const int* acts,
                          const float* prepared, float* y, int64_t y_stride, int head, const float* extra, float c0,
                          float c1, int64_t batch, rs_stream_t stream) {
  return mlp_run(x, x_stride, nullptr, nullptr, n_layers, dims, acts, prepared, y, y_stride, head, extra, c0, c1,
                 batch, stream);
}

extern "C" int rs_mlp_affine_fwd(const float* x, int64_t x_stride, const float* in_scale, const float* in_shift,
                                 int n_layers, const int* dims, const int* acts, const float* prepared, float* y,
                                 int64_t y_stride, int head, const float* extra, float c0, float c1, int64_t batch,
                                 rs_stream_t stream) {
  RS_REQUIRE(batch == 0 || (in_scale && in_shift), "rs_mlp_affine_fwd: null in_scale / in_shift");
  return mlp_run(x, x_stride, in_scale, in_shift, n_layers, dims, acts, prepared, y, y_stride, head, extra, c0, c1,
                 batch, stream);
}

extern "C" int rs_mlp_affine_pieces_fwd(const float* x, int64_t x_stride, const float* in_scale,
                                        const float* in_shift, int n_layers, const int* dims, const int* acts,
                                        const float* prepared, float* y, int64_t y_stride, int head, const float* extra,
                                        float c0, float c1, int64_t batch, int n_pieces, const int* widths,
                                        const int* in_cols, const int* kinds, const void* const* srcs,
                                        const int64_t* src_strides, const float* const* tables,
                                        const int64_t* vocabs, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(in_scale && in_shift, "rs_mlp_affine_pieces_fwd: null in_scale / in_shift");
  RS_REQUIRE(n_layers >= 1 && dims && dims[0] >= 1 && dims[0] <= 64,
             "rs_mlp_affine_pieces_fwd: at most 64 input columns");
  RS_REQUIRE(err_flag, "rs_mlp_affine_pieces_fwd: null error flag");
  ConcatArgs pc{};
  const int st = concat_fill(n_pieces, widths, in_cols, kinds, srcs, src_strides, tables, vocabs, dims[0],
                             "rs_mlp_affine_pieces_fwd", pc);
  if (st != RS_OK) return st;
  pc.err = err_flag;
  // x provides every column no piece covers (rows x_stride apart)
  RS_REQUIRE(x || pc.ncol == dims[0], "rs_mlp_affine_pieces_fwd: x is null");
  return mlp_run(x ? x : in_scale, x ? x_stride : dims[0], in_scale, in_shift, n_layers, dims, acts, prepared, y,
                 y_stride, head, extra, c0, c1, batch, stream, &pc);
}
