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
#include "rs_common.hpp"

namespace rs {

constexpr int MLP_MAXL = 8;
constexpr int MLP_MAXD = 1024;
constexpr int MLP_NW = 16;

struct MlpGeom {
  int L;
  int K[MLP_MAXL], N[MLP_MAXL], Kp[MLP_MAXL], Np[MLP_MAXL];
  int64_t off[MLP_MAXL];  // floats: packed W of layer l
  int poff[MLP_MAXL];     // floats from `wtot`: bias[Np] then alpha[Np] of layer l
  int64_t wtot, total;    // prepared = [W_0 .. W_{L-1} | params (ptot)]
  int ptot;
  int rs;                 // LDS row stride (floats) of the activation buffers
  size_t lds;             // dynamic LDS bytes of mlp_tower
};

static inline int rup(int v, int m) { return (v + m - 1) / m * m; }

static bool mlp_geom(int L, const int* dims, MlpGeom& g) {
  if (L < 1 || L > MLP_MAXL || !dims) return false;
  g.L = L;
  int64_t off = 0;
  int maxw = 0, poff = 0;
  for (int l = 0; l < L; ++l) {
    if (dims[l] < 1 || dims[l + 1] < 1) return false;
    g.K[l] = dims[l];
    g.N[l] = dims[l + 1];
    g.Kp[l] = rup(dims[l], 16);
    g.Np[l] = rup(dims[l + 1], 16);
    if (g.Kp[l] > MLP_MAXD || g.Np[l] > MLP_MAXD) return false;
    g.off[l] = off;
    off += (int64_t)g.Kp[l] * g.Np[l];
    g.poff[l] = poff;
    poff += 2 * g.Np[l];
    maxw = std::max(maxw, std::max(g.Kp[l], g.Np[l]));
  }
  g.wtot = off;
  g.ptot = poff;
  g.total = off + poff;
  // Row stride = 8 (mod 64) dwords: the four 16-lane groups of each
  // ds_read_b128 (rows l&15, k-slot l>>4) then hit 16 distinct bank slots.
  g.rs = rup(maxw, 64) + 8;
  g.lds = (size_t)(32 * g.rs + MLP_NW * 256 + g.ptot) * sizeof(float);
  return g.lds <= 160 * 1024;
}

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

struct MlpArgs {
  const float* x;
  int64_t xs;
  const float* prep;
  int L, K0, rs, ptot;
  int64_t wtot;
  int Kp[MLP_MAXL], Np[MLP_MAXL], N[MLP_MAXL], act[MLP_MAXL], poff[MLP_MAXL];
  int64_t off[MLP_MAXL];
  float* y;
  int64_t ys;
  int head;
  const float* extra;
  float c0, c1;
  int64_t M;
  unsigned long long* dbg;  // diagnostics only: per-wave phase stamps (rs_diag_mlp_set_dbg)
};
#define MLP_STAMP(i)                                                                              \
  do {                                                                                            \
    if (a.dbg && (threadIdx.x & 63) == 0)                                                         \
      a.dbg[((int64_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

__device__ __forceinline__ float mlp_act(float v, int act, float alpha) {
  switch (act) {
    case RS_ACT_RELU: return fmaxf(v, 0.f);
    case RS_ACT_PRELU: return fmaxf(v, 0.f) + alpha * fminf(v, 0.f);
    case RS_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}

// Work split of layer l: T output tiles x S k-slices; item = part*T + t.
struct MlpItem {
  int t, g0, g1;
};
__device__ __forceinline__ int mlp_slices(int T, int G, int NW) {
  int S = NW / T;
  return S < 1 ? 1 : (S > G ? G : S);
}
__device__ __forceinline__ MlpItem mlp_item(int item, int T, int G, int S) {
  const int t = item % T, part = item / T;
  return MlpItem{t, part * G / S, (part + 1) * G / S};
}

// B fragments (1 KB per k-group per output tile) stream through a ring of 4
// registers.  mlp_ring_fill issues the first 4 groups of an item (it can run
// before the barrier that publishes the item's A tile); mlp_mac<D> consumes
// the ring D deep, refilling the slot it just consumed with group g + D, so
// every MFMA's weights were requested D groups (4D MFMAs) earlier.  D | (g1-g0)
// keeps it branch-free; refills past g1 are clamped in-bounds re-reads.
__device__ __forceinline__ void mlp_ring_fill(floatx4 (&ring)[4], const floatx4* bp, int g0, int g1) {
#pragma unroll
  for (int u = 0; u < 4; ++u) ring[u] = bp[(int64_t)min(g0 + u, g1 - 1) * 64];
}

template <int D>
__device__ __forceinline__ void mlp_mac_d(floatx4 (&ring)[4], const float* __restrict__ ap,
                                          const floatx4* __restrict__ bp, int g0, int g1, floatx4& acc) {
  for (int g = g0; g < g1; g += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const floatx4 av = *reinterpret_cast<const floatx4*>(ap + 16 * (g + u));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma16x16x4(av[j], ring[u][j], acc);
      // refill the slot in place right after its MFMAs and pin it there: left
      // alone the scheduler sinks every refill to the end of the iteration
      // (or copies in-flight registers), which drains the ring each pass
      ring[u] = bp[(int64_t)min(g + u + D, g1 - 1) * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

__device__ __forceinline__ void mlp_mac(floatx4 (&ring)[4], const float* ap, const floatx4* bp, int g0, int g1,
                                        floatx4& acc) {
  const int n = g1 - g0;  // wave-uniform
  // (a 4-deep ring gets a full vmcnt(0) at its loop head from the compiler)
  if (n % 3 == 0) mlp_mac_d<3>(ring, ap, bp, g0, g1, acc);
  else if (n % 2 == 0) mlp_mac_d<2>(ring, ap, bp, g0, g1, acc);
  else mlp_mac_d<1>(ring, ap, bp, g0, g1, acc);
}

// The tower on a 16-row tile whose input is already in LDS buf0 (barrier not
// yet taken) and whose layer-0 ring was filled by the caller.  smem layout:
// buf0 [16][rs] | buf1 [16][rs] | red [NW][256] | par [ptot] (loaded here).
template <int NW>
__device__ __forceinline__ void mlp_tower_tile(const MlpArgs& a, float* smem, int64_t m0, floatx4 (&ring)[4]) {
  const int RS = a.rs;
  float* red = smem + 32 * RS;
  float* par = red + NW * 256;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  float* in = smem;
  float* out = smem + 16 * RS;
  for (int l = 0; l < a.L; ++l) {
    __syncthreads();
    MLP_STAMP(2 + 2 * l);
    const int T = a.Np[l] >> 4, G = a.Kp[l] >> 4;
    const int S = mlp_slices(T, G, NW);
    const floatx4* W = reinterpret_cast<const floatx4*>(a.prep + a.off[l]) + lane;
    const float* bias = par + a.poff[l];
    const float* alpha = bias + a.Np[l];
    const int act = a.act[l];
    const bool last = l == a.L - 1;
    const int Nl = a.N[l];

    auto finish = [&](int row, int col, float v) {
      v = mlp_act(v + bias[col], act, alpha[col]);
      if (!last) {
        out[row * RS + col] = v;
      } else {
        const int64_t m = m0 + row;
        if (m < a.M && col < Nl) {
          if (a.head == 0) {
            a.y[m * a.ys + col] = v;
          } else if (col == 0) {
            float z = a.c0 * v;
            if (a.extra) z = z + a.c1 * a.extra[m];
            a.y[m * a.ys] = 1.0f / (1.0f + expf(-z));
          }
        }
      }
    };

    const float* ap = in + (lane & 15) * RS + 4 * (lane >> 4);
    for (int item = w; item < T * S; item += NW) {
      const MlpItem it = mlp_item(item, T, G, S);
      const floatx4* bp = W + (int64_t)it.t * G * 64;
      if (item != w) mlp_ring_fill(ring, bp, it.g0, it.g1);
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      mlp_mac(ring, ap, bp, it.g0, it.g1, acc);
      if (S == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) finish(4 * (lane >> 4) + r, 16 * it.t + (lane & 15), acc[r]);
      } else {
        *reinterpret_cast<floatx4*>(red + item * 256 + lane * 4) = acc;
      }
    }
    MLP_STAMP(3 + 2 * l);
    // next layer's first weights do not depend on this layer: request them
    // now, so they arrive during the barrier / reduction below
    if (l + 1 < a.L) {
      const int T2 = a.Np[l + 1] >> 4, G2 = a.Kp[l + 1] >> 4;
      const int S2 = mlp_slices(T2, G2, NW);
      if (w < T2 * S2) {
        const MlpItem it = mlp_item(w, T2, G2, S2);
        mlp_ring_fill(ring, reinterpret_cast<const floatx4*>(a.prep + a.off[l + 1]) + lane + (int64_t)it.t * G2 * 64,
                      it.g0, it.g1);
      }
    }
    if (S > 1) {
      __syncthreads();
      for (int e = threadIdx.x; e < T * 256; e += NW * 64) {
        const int t = e >> 8, q = e & 255, ln = q >> 2, r = q & 3;
        float v = 0.f;
        for (int p = 0; p < S; ++p) v += red[(p * T + t) * 256 + q];
        finish(4 * (ln >> 4) + r, 16 * t + (ln & 15), v);
      }
    }
    float* tmp = in;
    in = out;
    out = tmp;
  }
  MLP_STAMP(15);
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void mlp_tower(MlpArgs a) {
  extern __shared__ float smem[];
  const int RS = a.rs;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * 16;
  MLP_STAMP(0);

  // layer-0 weights first (independent of everything), then the input tile
  // (one row per wave, coalesced; rows past M re-read row M-1 and are never
  // stored) and the bias/alpha block into LDS
  floatx4 ring[4];
  {
    const int T = a.Np[0] >> 4, G = a.Kp[0] >> 4;
    const int S = mlp_slices(T, G, NW);
    if (w < T * S) {
      const MlpItem it = mlp_item(w, T, G, S);
      mlp_ring_fill(ring, reinterpret_cast<const floatx4*>(a.prep + a.off[0]) + lane + (int64_t)it.t * G * 64,
                    it.g0, it.g1);
    }
  }
  // All of a row's loads are issued before any LDS store: a load->store loop
  // would pay one HBM round trip per 64 columns.
  for (int r = w; r < 16; r += NW) {
    const int64_t m = m0 + r < a.M ? m0 + r : a.M - 1;
    const float* xr = a.x + m * a.xs;
    constexpr int XU = MLP_MAXD / 64;
    float xv[XU];
#pragma unroll
    for (int i = 0; i < XU; ++i) {
      const int c = lane + 64 * i;
      xv[i] = c < a.K0 ? xr[c] : 0.f;
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
  mlp_tower_tile<NW>(a, smem, m0, ring);
}

}  // namespace rs

using namespace rs;

static unsigned long long* g_mlp_dbg = nullptr;
extern "C" void rs_diag_mlp_set_dbg(unsigned long long* p) { g_mlp_dbg = p; }

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

extern "C" int rs_mlp_fwd(const float* x, int64_t x_stride, int n_layers, const int* dims, const int* acts,
                          const float* prepared, float* y, int64_t y_stride, int head, const float* extra, float c0,
                          float c1, int64_t batch, rs_stream_t stream) {
  MlpGeom g;
  RS_REQUIRE(mlp_geom(n_layers, dims, g), "rs_mlp_fwd: need 1..%d layers with widths 1..%d", MLP_MAXL, MLP_MAXD);
  RS_REQUIRE(x && prepared && y && acts, "rs_mlp_fwd: null pointer");
  RS_REQUIRE(batch >= 0 && x_stride >= dims[0], "rs_mlp_fwd: bad batch/stride");
  RS_REQUIRE(head == 0 || head == 1, "rs_mlp_fwd: head must be 0 (raw) or 1 (sigmoid)");
  RS_REQUIRE(head == 0 ? y_stride >= dims[n_layers] : (dims[n_layers] == 1 && y_stride >= 1),
             "rs_mlp_fwd: bad output shape (head=1 needs output width 1)");
  MlpArgs a{};
  for (int l = 0; l < n_layers; ++l) {
    RS_REQUIRE(acts[l] >= RS_ACT_NONE && acts[l] <= RS_ACT_SIGMOID, "rs_mlp_fwd: bad activation");
    a.Kp[l] = g.Kp[l];
    a.Np[l] = g.Np[l];
    a.N[l] = g.N[l];
    a.act[l] = acts[l];
    a.off[l] = g.off[l];
    a.poff[l] = g.poff[l];
  }
  a.wtot = g.wtot;
  a.ptot = g.ptot;
  if (batch == 0) return RS_OK;
  a.x = x;
  a.xs = x_stride;
  a.prep = prepared;
  a.L = n_layers;
  a.K0 = dims[0];
  a.rs = g.rs;
  a.y = y;
  a.ys = y_stride;
  a.head = head;
  a.extra = extra;
  a.c0 = c0;
  a.c1 = c1;
  a.M = batch;
  a.dbg = g_mlp_dbg;
  const size_t lds = g.lds;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)mlp_tower<MLP_NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  const int64_t grid = (batch + 15) / 16;
  RS_REQUIRE(grid < (1ll << 31), "rs_mlp_fwd: batch too large");
  mlp_tower<MLP_NW><<<(unsigned)grid, MLP_NW * 64, lds, as_stream(stream)>>>(a);
  return launch_status("rs_mlp_fwd");
}
