// mlp_tower.hpp — device side of the fused MLP tower (mlp.hip), shared with
// the fused DeepFM kernel (embed_fm.hip).  See mlp.hip for the design.
#pragma once
#include <algorithm>
#include <type_traits>

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
  int unroll;               // RS_OPT_MLP_UNROLL at launch
  const float* in_scale;    // rs_mlp_affine_fwd: input column c staged as x * in_scale[c] + in_shift[c]
  const float* in_shift;    //   (an inference BatchNormalization folded into the staging; null = none)
};
// Per-wave phase stamps (rs_diag_mlp_set_dbg) exist only in the diagnostic
// build (scripts/build_diag.sh, -DRS_DIAG_STAMPS): the product's runtime
// check of a.dbg at every stamp cost 2.5 % of the fused DeepFM and 1.5 % of
// the fused DCN (instruction fetch; profiles/r4_ab_stamps_compiled_out.jsonl).
#ifdef RS_DIAG_STAMPS
#define MLP_STAMP(i)                                                                              \
  do {                                                                                            \
    if (a.dbg && (threadIdx.x & 63) == 0)                                                         \
      a.dbg[((int64_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define MLP_STAMP(i) \
  do {               \
  } while (0)
#endif

template <int ACT>
__device__ __forceinline__ float mlp_act_c(float v, float alpha) {
  if constexpr (ACT == RS_ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == RS_ACT_PRELU) return fmaxf(v, 0.f) + alpha * fminf(v, 0.f);
  else if constexpr (ACT == RS_ACT_SIGMOID) return 1.0f / (1.0f + expf(-v));
  else return v;
}
__device__ __forceinline__ float mlp_act(float v, int act, float alpha) {
  switch (act) {
    case RS_ACT_RELU: return mlp_act_c<RS_ACT_RELU>(v, alpha);
    case RS_ACT_PRELU: return mlp_act_c<RS_ACT_PRELU>(v, alpha);
    case RS_ACT_SIGMOID: return mlp_act_c<RS_ACT_SIGMOID>(v, alpha);
    default: return v;
  }
}
// f(std::integral_constant<int, act>): the activation switch taken once
// around an epilogue, not per element inside it
template <class Fn>
__device__ __forceinline__ void with_act(int act, Fn&& f) {
  switch (act) {
    case RS_ACT_RELU: f(std::integral_constant<int, RS_ACT_RELU>()); break;
    case RS_ACT_PRELU: f(std::integral_constant<int, RS_ACT_PRELU>()); break;
    case RS_ACT_SIGMOID: f(std::integral_constant<int, RS_ACT_SIGMOID>()); break;
    default: f(std::integral_constant<int, RS_ACT_NONE>()); break;
  }
}

// Work split of layer l: T output tiles x S k-slices; item = part*T + t.
struct MlpItem {
  int t, g0, g1;
};
// k-slices per output tile: layers with >= 4 tiles keep whole columns per
// wave (no partial-sum exchange: measured faster than filling all 16 waves);
// narrow layers (the 64->1 head) split K over the idle waves.
constexpr int MLP_SPLIT_T = 4;  // layers with fewer output tiles than this split K over the idle waves
__device__ __forceinline__ int mlp_slices(int T, int G, int NW) {
  if (T >= MLP_SPLIT_T) return 1;
  const int S = NW / T;
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
constexpr int MLP_R = 4;  // B-fragment ring slots (the deepest D; a 9-slot ring measured slower)
__device__ __forceinline__ void mlp_ring_fill(floatx4 (&ring)[MLP_R], const floatx4* bp, int g0, int g1) {
#pragma unroll
  for (int u = 0; u < MLP_R; ++u) ring[u] = bp[(int64_t)min(g0 + u, g1 - 1) * 64];
}

// CH = 4: MFMA j of every k-group accumulates into chain j (four independent
// dependency chains, summed (c0 + c1) + (c2 + c3) at the end): a dependent
// fp32 MFMA issues only ~100 cycles after its predecessor, so a single chain
// leaves the pipe idle on a SIMD with one or two busy waves.
template <int CH>
struct MacAcc {
  floatx4 c[CH];
  __device__ __forceinline__ MacAcc() {
#pragma unroll
    for (int i = 0; i < CH; ++i) c[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  __device__ __forceinline__ void mac4(const floatx4& a, const floatx4& b) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j % CH] = mfma16x16x4(a[j], b[j], c[j % CH]);
  }
  __device__ __forceinline__ floatx4 sum() const {
    if constexpr (CH == 1) {
      return c[0];
    } else {
      floatx4 r;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = (c[0][i] + c[1][i]) + (c[2][i] + c[3][i]);
      return r;
    }
  }
};

template <int D, int CH>
__device__ __forceinline__ void mlp_mac_d(floatx4 (&ring)[MLP_R], const float* __restrict__ ap,
                                          const floatx4* __restrict__ bp, int g0, int g1, floatx4& out) {
  MacAcc<CH> acc;
  // A fragments are read one group ahead so the LDS latency hides behind
  // the previous group's MFMAs
  floatx4 an = *reinterpret_cast<const floatx4*>(ap + 16 * g0);
  for (int g = g0; g < g1; g += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const floatx4 av = an;
      an = *reinterpret_cast<const floatx4*>(ap + 16 * min(g + u + 1, g1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      acc.mac4(av, ring[u]);
      // refill the slot in place right after its MFMAs and pin it there: left
      // alone the scheduler sinks every refill to the end of the iteration
      // (or copies in-flight registers), which drains the ring each pass
      ring[u] = bp[(int64_t)min(g + u + D, g1 - 1) * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  out = acc.sum();
}

// The same contraction over exactly N k-groups, fully unrolled: straight-line
// code, so the compiler waits on each ring slot's own load (vmcnt(D-1)-style)
// instead of draining the ring at a loop head (the looped form's back-edge
// gets a full vmcnt(0) every D groups).
// groups ahead in the 16 / 8 / 4-group layers: 2 (A/B of rs_mlp_fwd, B 4096:
// 20.66 us vs 20.75 at 1 and 20.89 at 4; profiles/r4_ab_mlp_small_d.json)
constexpr int MLP_SMALL_D = 2;
template <int N, int D, int CH>
__device__ __forceinline__ void mlp_mac_u(floatx4 (&ring)[MLP_R], const float* __restrict__ ap,
                                          const floatx4* __restrict__ bp, int g0, floatx4& out) {
  static_assert(N % D == 0 && D <= MLP_R, "unrolled contraction: D | N, D <= ring");
  MacAcc<CH> acc;
  const int g1 = g0 + N;
  floatx4 an = *reinterpret_cast<const floatx4*>(ap + 16 * g0);
#pragma unroll
  for (int i = 0; i < N; i += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int g = g0 + i;
      const floatx4 av = an;
      an = *reinterpret_cast<const floatx4*>(ap + 16 * min(g + u + 1, g1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      acc.mac4(av, ring[u]);
      ring[u] = bp[(int64_t)min(g + u + D, g1 - 1) * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  out = acc.sum();
}

template <int CH>
__device__ __forceinline__ void mlp_mac_ch(floatx4 (&ring)[MLP_R], const float* ap, const floatx4* bp, int g0,
                                           int g1, floatx4& acc, int unroll) {
  const int n = g1 - g0;  // wave-uniform
  if (unroll) {  // the DeepFM / DCN tower widths (429|432 -> 256 -> 128 -> 64 -> head)
    switch (n) {
      case 27: return mlp_mac_u<27, 3, CH>(ring, ap, bp, g0, acc);
      case 16: return mlp_mac_u<16, MLP_SMALL_D, CH>(ring, ap, bp, g0, acc);
      case 8: return mlp_mac_u<8, MLP_SMALL_D, CH>(ring, ap, bp, g0, acc);
      case 4: return mlp_mac_u<4, MLP_SMALL_D, CH>(ring, ap, bp, g0, acc);
      case 2: return mlp_mac_u<2, 2, CH>(ring, ap, bp, g0, acc);
      case 1: return mlp_mac_u<1, 1, CH>(ring, ap, bp, g0, acc);
      default: break;
    }
  }
  // (a 4-deep ring gets a full vmcnt(0) at its loop head from the compiler)
  if (n % 3 == 0) mlp_mac_d<3, CH>(ring, ap, bp, g0, g1, acc);
  else if (n % 2 == 0) mlp_mac_d<2, CH>(ring, ap, bp, g0, g1, acc);
  else mlp_mac_d<1, CH>(ring, ap, bp, g0, g1, acc);
}

// four accumulation chains (MFMA j of a k-group into chain j), compile-time
__device__ __forceinline__ void mlp_mac(floatx4 (&ring)[MLP_R], const float* ap, const floatx4* bp, int g0, int g1,
                                        floatx4& acc, int unroll = 0) {
  mlp_mac_ch<4>(ring, ap, bp, g0, g1, acc, unroll);
}

// The tower on a 16-row tile whose input is already in LDS buf0 (barrier not
// yet taken) and whose layer-0 ring was filled by the caller.  smem layout:
// buf0 [16][rs] | buf1 [16][rs] | red [NW][256] | par [ptot] (loaded here).
// l0 > 0: layers 0 .. l0-1 were computed by the caller (layer l0's input is
// in buf (l0 & 1), its ring filled).
template <int NW>
__device__ __forceinline__ void mlp_tower_tile(const MlpArgs& a, float* smem, int64_t m0, floatx4 (&ring)[MLP_R],
                                               const float* extra_lds = nullptr, int l0 = 0, int lstop = MLP_MAXL) {
  // layers l0 .. min(a.L, lstop) - 1 (lstop < a.L: a caller's split-K tail runs the rest)
  const int RS = a.rs;
  float* red = smem + 32 * RS;
  float* par = red + NW * 256;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  float* in = (l0 & 1) ? smem + 16 * RS : smem;
  float* out = (l0 & 1) ? smem : smem + 16 * RS;
  // A one-unit head after a layer that keeps whole columns per wave folds into
  // that layer's epilogue: each wave dots its 16 activation columns with the
  // head weights (a DPP row sum per sample) into red, and after one barrier
  // 16 threads add the tiles' partials in tile order — no head layer of its
  // own (ring fill, barrier, K-split reduction).
  const int LH = a.L - 1;
  const bool fhead = lstop >= a.L && LH - 1 >= l0 && a.N[LH] == 1 &&
                     mlp_slices(a.Np[LH - 1] >> 4, a.Kp[LH - 1] >> 4, NW) == 1;
  const int Lrun = fhead ? LH : (lstop < a.L ? lstop : a.L);
  for (int l = l0; l < Lrun; ++l) {
    const int T = a.Np[l] >> 4, G = a.Kp[l] >> 4;
    const int S = mlp_slices(T, G, NW);
    __syncthreads();
    MLP_STAMP(2 + 2 * l);
    const floatx4* W = reinterpret_cast<const floatx4*>(a.prep + a.off[l]) + lane;
    const float* bias = par + a.poff[l];
    const float* alpha = bias + a.Np[l];
    const int act = a.act[l];
    const bool last = l == a.L - 1;
    const int Nl = a.N[l];

    // bias / alpha come in as values: read between LDS stores they would be
    // re-read after every store (the compiler cannot prove out != par)
    auto finish = [&](auto A, int row, int col, float v, float bc, float ac) {
      v = mlp_act_c<decltype(A)::value>(v + bc, ac);
      if (!last) {
        out[row * RS + col] = v;
      } else {
        const int64_t m = m0 + row;
        if (m < a.M && col < Nl) {
          if (a.head == 0) {
            a.y[m * a.ys + col] = v;
          } else if (col == 0) {
            float z = a.c0 * v;
            if (extra_lds) z = z + a.c1 * extra_lds[row];
            else if (a.extra) z = z + a.c1 * a.extra[m];
            a.y[m * a.ys] = 1.0f / (1.0f + expf(-z));
          }
        }
      }
    };

    const float* ap = in + (lane & 15) * RS + 4 * (lane >> 4);
    const bool head_here = fhead && l == LH - 1;
    for (int item = w; item < T * S; item += NW) {
      const MlpItem it = mlp_item(item, T, G, S);
      const floatx4* bp = W + (int64_t)it.t * G * 64;
      if (item != w) mlp_ring_fill(ring, bp, it.g0, it.g1);
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      mlp_mac(ring, ap, bp, it.g0, it.g1, acc, a.unroll);
      if (head_here) {
        // head weight of this lane's column k: the packed head layer holds
        // W[k][0] at lane 16 ((k & 15) >> 2), element k & 3, of k-group k >> 4
        const int col = 16 * it.t + (lane & 15);
        const float hw = col < Nl ? a.prep[a.off[LH] + ((int64_t)(col >> 4) * 64 + 16 * ((col & 15) >> 2)) * 4 +
                                           (col & 3)]
                                  : 0.f;
        const float bc = bias[col], ac = alpha[col];
        with_act(act, [&](auto A) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float p = col < Nl ? mlp_act_c<decltype(A)::value>(acc[r] + bc, ac) * hw : 0.f;
            p = row16_sum(p);
            if ((lane & 15) == 0) red[it.t * 16 + 4 * (lane >> 4) + r] = p;
          }
        });
      } else if (S == 1) {
        const int col = 16 * it.t + (lane & 15);
        const float bc = bias[col], ac = alpha[col];
        with_act(act, [&](auto A) {
#pragma unroll
          for (int r = 0; r < 4; ++r) finish(A, 4 * (lane >> 4) + r, col, acc[r], bc, ac);
        });
      } else {
        *reinterpret_cast<floatx4*>(red + item * 256 + lane * 4) = acc;
      }
    }
    MLP_STAMP(3 + 2 * l);
    // next layer's first weights do not depend on this layer: request them
    // now, so they arrive during the barrier / reduction below
    if (l + 1 < Lrun || (fhead && l + 1 < a.L)) {
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
      with_act(act, [&](auto A) {
        for (int e = threadIdx.x; e < T * 256; e += NW * 64) {
          const int t = e >> 8, q = e & 255, ln = q >> 2, r = q & 3;
          float v = 0.f;
          for (int p = 0; p < S; ++p) v += red[(p * T + t) * 256 + q];
          const int col = 16 * t + (ln & 15);
          finish(A, 4 * (ln >> 4) + r, col, v, bias[col], alpha[col]);
        }
      });
    }
    float* tmp = in;
    in = out;
    out = tmp;
  }
  if (fhead) {
    __syncthreads();
    MLP_STAMP(2 + 2 * LH);
    if (threadIdx.x < 16) {
      const int row = threadIdx.x, T = a.Np[LH - 1] >> 4;
      float z = 0.f;
      for (int t = 0; t < T; ++t) z += red[t * 16 + row];
      const float* hb = par + a.poff[LH];
      float v = mlp_act(z + hb[0], a.act[LH], hb[a.Np[LH]]);
      const int64_t m = m0 + row;
      if (m < a.M) {
        if (a.head == 0) {
          a.y[m * a.ys] = v;
        } else {
          float zz = a.c0 * v;
          if (extra_lds) zz = zz + a.c1 * extra_lds[row];
          else if (a.extra) zz = zz + a.c1 * a.extra[m];
          a.y[m * a.ys] = 1.0f / (1.0f + expf(-zz));
        }
      }
    }
  }
  MLP_STAMP(15);
}

// ---- Split-K tail: the tower after its first layer at the DeepFM / DCN
// widths (256 -> 128 -> 64 -> 1), every layer on all 16 waves.  The one-role
// tail (mlp_tower_tile) runs the 8- and 4-tile layers on 8 / 4 waves with a
// 2-deep weight ring, and its narrow layers stall on the L2 latency of every
// weight refill (stamps: ~450 cycles per k-group per wave, layer 2 at ~110
// cycles per MFMA).  Here layer l (T output tiles, G k-groups) is cut into
// 16 items of one tile and G*T/16 <= 8 k-groups: a wave's whole weight slice
// (<= 8 KB) is requested at the end of the previous layer, so the MFMAs of a
// layer wait on nothing but the barrier; the 16 partial tiles meet in LDS and
// are reduced in part order (+ bias, activation) by all 1024 threads; the
// one-unit head is folded into the last reduction (wave = sample row, lane =
// column, a wave sum).  Host side: mlp_tail_ok.
inline bool mlp_tail_ok(const int* Np, const int* Kp, const int* N, int L, int l0, int& gwa, int& gwb) {
  // exactly two split layers after l0's caller-run layer, then a one-unit head
  // (+ at most one more 1 -> 1 layer: NFM's Dense(1) after its DNNLayer)
  const bool extra = L == l0 + 4 && N[L - 2] == 1 && N[L - 1] == 1 && Kp[L - 1] == 16;
  if ((L != l0 + 3 && !extra) || N[l0 + 2] != 1) return false;
  int gw[2];
  for (int q = 0; q < 2; ++q) {
    const int l = l0 + q, T = Np[l] >> 4, G = Kp[l] >> 4;
    if (T < 1 || T > 16 || 16 % T || G % (16 / T)) return false;
    gw[q] = G / (16 / T);
  }
  gwa = gw[0];
  gwb = gw[1];
  return (gwa == 8 && gwb == 2) || (gwa == 4 && gwb == 2) || (gwa == 8 && gwb == 4) || (gwa == 4 && gwb == 1);
}
// this wave's weight slice of layer l (item w: tile w % T, k-groups part w / T);
// TC > 0: the layer's tile count T known at compile time (no integer division)
template <int GW, int TC = 0>
__device__ __forceinline__ void mlp_tail_fetch(const MlpArgs& a, int l, floatx4 (&wr)[GW]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int T = TC > 0 ? TC : a.Np[l] >> 4, G = a.Kp[l] >> 4;
  const int t = w % T, g0 = (w / T) * GW;
  const floatx4* W = reinterpret_cast<const floatx4*>(a.prep + a.off[l]) + lane + ((int64_t)t * G + g0) * 64;
#pragma unroll
  for (int u = 0; u < GW; ++u) wr[u] = W[(int64_t)u * 64];
}
// layer l's contraction of this wave's slice (its partial tile)
template <int GW, int TC = 0>
__device__ __forceinline__ floatx4 mlp_tail_mac(const MlpArgs& a, int l, const floatx4 (&wr)[GW], const float* in) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int T = TC > 0 ? TC : a.Np[l] >> 4;
  const int g0 = (w / T) * GW;
  const float* ap = in + (lane & 15) * a.rs + 4 * (lane >> 4);
  floatx4 an[GW];
#pragma unroll
  for (int u = 0; u < GW; ++u) an[u] = *reinterpret_cast<const floatx4*>(ap + 16 * (g0 + u));
  MacAcc<4> acc;
#pragma unroll
  for (int u = 0; u < GW; ++u) acc.mac4(an[u], wr[u]);
  return acc.sum();
}
// Layers l0, l0+1 (split K over the 16 waves) and the one-unit head l0+2.
// On entry: layer l0's input is in buf (l0 & 1) (written, barrier not yet
// taken), wa holds this wave's slice of layer l0 (mlp_tail_fetch), the bias /
// alpha block is in LDS (par).  Wave w of a layer with T tiles owns tile
// w % T, k-part w / T; the waves of parts >= 1 leave their partial tile in
// LDS and the part-0 wave of each tile adds them in part order (one
// ds_read_b128 per partial, conflict-free) and runs the tile's epilogue —
// no all-thread reduction pass.
// TAC / TBC > 0: the two split layers' tile counts known at compile time
// (mlp_tail_dispatch: the DeepFM / DCN / DIN widths 256 -> 128 -> 64, T = 8 /
// 4): part counts, item indices and the partial / head loops fold to
// constants — the generic form spends its hand-offs in integer division and
// loop control (profiles/r6_tail_stamps.jsonl)
template <int NW, int GWA, int GWB, int TAC = 0, int TBC = 0>
__device__ __forceinline__ void mlp_tail_splitk(const MlpArgs& a, float* smem, int64_t m0, const floatx4 (&wa)[GWA],
                                                const float* extra_lds, int l0) {
  static_assert(NW == 16, "split-K tail: 16 waves");
  const int RS = a.rs;
  float* red = smem + 32 * RS;
  float* par = red + NW * 256;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  float* in = (l0 & 1) ? smem + 16 * RS : smem;
  float* out = (l0 & 1) ? smem : smem + 16 * RS;
  const int l1 = l0 + 1, LH = l0 + 2;
  // the part-0 wave of tile t: its accumulator + the other parts' partial tiles
  auto gather_parts = [&](floatx4 acc, int T) {
    const int S = 16 / T;
#pragma unroll
    for (int p = 1; p < S; ++p) {
      const floatx4 q = *reinterpret_cast<const floatx4*>(red + (w + p * T) * 256 + lane * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += q[r];
    }
    return acc;
  };
  // ---- layer l0
  const int TA = TAC > 0 ? TAC : a.Np[l0] >> 4;
  __syncthreads();  // its input complete
  MLP_STAMP(2 + 2 * l0);
  floatx4 acc = mlp_tail_mac<GWA, TAC>(a, l0, wa, in);
  MLP_STAMP(3 + 2 * l0);
  if (w >= TA) *reinterpret_cast<floatx4*>(red + w * 256 + lane * 4) = acc;
  floatx4 wb[GWB];
  mlp_tail_fetch<GWB, TBC>(a, l1, wb);  // the next layer's slice, in flight over the hand-off
  MLP_STAMP(10);                   // (diagnostic stamps 10..14: the layer hand-offs)
  __syncthreads();                 // the partial tiles in red
  MLP_STAMP(11);
  if (w < TA) {
    acc = gather_parts(acc, TA);
    const int col = 16 * w + s;
    // bias / alpha in registers first: read between the LDS stores below they
    // are re-read after every store (the compiler cannot prove out != par)
    const float bc = par[a.poff[l0] + col], ac = par[a.poff[l0] + a.Np[l0] + col];
    with_act(a.act[l0], [&](auto A) {
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(4 * kk + r) * RS + col] = mlp_act_c<decltype(A)::value>(acc[r] + bc, ac);
    });
  }
  // ---- layer l1, its epilogue folded with the head
  const int TB = TBC > 0 ? TBC : a.Np[l1] >> 4;
  // the head's weight of this lane's column (packed head layer: W[k][0] at
  // lane 16 ((k & 15) >> 2), element k & 3, of k-group k >> 4), requested
  // before the barrier (an L2 trip the part-0 epilogue would otherwise wait for)
  const int colh = 16 * (w % TB) + s;
  const float hw = a.prep[a.off[LH] + ((int64_t)(min(colh, a.Np[l1] - 1) >> 4) * 64 +
                                       16 * ((colh & 15) >> 2)) * 4 + (colh & 3)];
  MLP_STAMP(12);
  __syncthreads();  // its input complete; red free
  MLP_STAMP(2 + 2 * l1);
  acc = mlp_tail_mac<GWB, TBC>(a, l1, wb, out);
  MLP_STAMP(3 + 2 * l1);
  if (w >= TB) *reinterpret_cast<floatx4*>(red + w * 256 + lane * 4) = acc;
  MLP_STAMP(13);
  __syncthreads();  // the partial tiles in red
  MLP_STAMP(14);
  float* redh = red;  // [TB][16] head partials (red[0 .. 256 TB) is never a partial: parts >= 1 are waves >= TB)
  if (w < TB) {
    acc = gather_parts(acc, TB);
    const float bc = par[a.poff[l1] + colh], ac = par[a.poff[l1] + a.Np[l1] + colh];  // (registers: see l0)
    const bool live = colh < a.N[l1];
    with_act(a.act[l1], [&](auto A) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float h = live ? mlp_act_c<decltype(A)::value>(acc[r] + bc, ac) * hw : 0.f;  // (padded columns: 0)
        h = row16_sum(h);
        if (s == 0) redh[w * 16 + 4 * kk + r] = h;
      }
    });
  }
  __syncthreads();  // the tiles' head partials
  MLP_STAMP(2 + 2 * LH);
  if (threadIdx.x < 16) {
    const int row = threadIdx.x;
    float z = 0.f;
#pragma unroll
    for (int t = 0; t < TB; ++t) z += redh[t * 16 + row];  // tile order
    const float* hb = par + a.poff[LH];
    float v = mlp_act(z + hb[0], a.act[LH], hb[a.Np[LH]]);
    if (a.L == LH + 2) {  // a trailing 1 -> 1 layer: v * W[0][0] + b, then its activation
      const int L2 = LH + 1;
      const float* hb2 = par + a.poff[L2];
      float u;
      {
#pragma clang fp contract(off)  // product, then bias: as its MFMA epilogue would round
        u = v * a.prep[a.off[L2]] + hb2[0];
      }
      v = mlp_act(u, a.act[L2], hb2[a.Np[L2]]);
    }
    const int64_t m = m0 + row;
    if (m < a.M) {
      if (a.head == 0) {
        a.y[m * a.ys] = v;
      } else {
        float zz = a.c0 * v;
        if (extra_lds) zz = zz + a.c1 * extra_lds[row];
        else if (a.extra) zz = zz + a.c1 * a.extra[m];
        a.y[m * a.ys] = 1.0f / (1.0f + expf(-zz));
      }
    }
  }
  MLP_STAMP(15);
}

// Layer 0 of a tower whose first layer has NW 16-unit output tiles (256
// units: the DeepFM / DCN / DIN widths) before the split-K tail: wave w owns
// output tile w over every k-group (its ring filled by mlp_first_fill), the
// epilogue (bias, activation) writes buf1.  The generic mlp_tower_tile does
// the same work through run-time item / part arithmetic and a per-layer
// loop; here only G (the k-groups) is a run-time value.  Input in buf0
// (written, barrier not yet taken).
template <int NW>
__device__ __forceinline__ void mlp_layer0_tiles(const MlpArgs& a, float* smem, floatx4 (&ring)[MLP_R],
                                                 const float* extra_lds = nullptr) {
  const int RS = a.rs;
  float* par = smem + 32 * RS + NW * 256;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = a.Kp[0] >> 4;
  __syncthreads();
  MLP_STAMP(2);
  const floatx4* bp = reinterpret_cast<const floatx4*>(a.prep + a.off[0]) + lane + (int64_t)w * G * 64;
  const float* ap = smem + (lane & 15) * RS + 4 * (lane >> 4);
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  mlp_mac(ring, ap, bp, 0, G, acc, a.unroll);
  const int col = 16 * w + (lane & 15);
  const float bc = par[a.poff[0] + col], ac = par[a.poff[0] + a.Np[0] + col];
  float* out = smem + 16 * RS;
  with_act(a.act[0], [&](auto A) {
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(4 * (lane >> 4) + r) * RS + col] = mlp_act_c<decltype(A)::value>(acc[r] + bc, ac);
  });
  MLP_STAMP(3);
  (void)extra_lds;
}

// The split-K tail at GWA = 8 / GWB = 2 with its tile counts as constants
// when the widths are the DeepFM / DCN / DIN ones (a uniform branch on the
// kernel arguments), the generic form otherwise.  wa: layer l0's slice,
// fetched by the caller (mlp_tail_fetch<8> — the same values either way).
template <int NW>
__device__ __forceinline__ void mlp_tail_dispatch(const MlpArgs& a, float* smem, int64_t m0, const floatx4 (&wa)[8],
                                                  const float* extra_lds, int l0) {
  if (a.Np[l0] == 128 && a.Np[l0 + 1] == 64) mlp_tail_splitk<NW, 8, 2, 8, 4>(a, smem, m0, wa, extra_lds, l0);
  else mlp_tail_splitk<NW, 8, 2>(a, smem, m0, wa, extra_lds, l0);
}
// ... fetching layer 1's slice itself (wave w: tile w % T, part w / T — with T
// a constant in the specialised form)
template <int NW>
__device__ __forceinline__ void mlp_tail_run(const MlpArgs& a, float* smem, int64_t m0, const float* extra_lds) {
  floatx4 wa[8];
  if (a.Np[1] == 128 && a.Np[2] == 64) {
    mlp_tail_fetch<8, 8>(a, 1, wa);
    mlp_tail_splitk<NW, 8, 2, 8, 4>(a, smem, m0, wa, extra_lds, 1);
  } else {
    mlp_tail_fetch<8>(a, 1, wa);
    mlp_tail_splitk<NW, 8, 2>(a, smem, m0, wa, extra_lds, 1);
  }
}

// Layer-0 ring fill for the wave's first item (issue before anything else).
template <int NW>
__device__ __forceinline__ void mlp_first_fill(const MlpArgs& a, floatx4 (&ring)[MLP_R]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int T = a.Np[0] >> 4, G = a.Kp[0] >> 4;
  const int S = mlp_slices(T, G, NW);
  if (w < T * S) {
    const MlpItem it = mlp_item(w, T, G, S);
    mlp_ring_fill(ring, reinterpret_cast<const floatx4*>(a.prep + a.off[0]) + lane + (int64_t)it.t * G * 64, it.g0,
                  it.g1);
  }
}

// Diagnostics: the per-wave stamp buffer set by rs_diag_mlp_set_dbg (null = off).
unsigned long long* mlp_diag_dbg();

// Host: fill the tower part of MlpArgs from a validated geometry.
inline bool mlp_fill_args(const MlpGeom& g, const int* acts, const float* prepared, MlpArgs& a) {
  for (int l = 0; l < g.L; ++l) {
    if (acts[l] < RS_ACT_NONE || acts[l] > RS_ACT_SIGMOID) return false;
    a.Kp[l] = g.Kp[l];
    a.Np[l] = g.Np[l];
    a.N[l] = g.N[l];
    a.act[l] = acts[l];
    a.off[l] = g.off[l];
    a.poff[l] = g.poff[l];
  }
  a.wtot = g.wtot;
  a.ptot = g.ptot;
  a.prep = prepared;
  a.L = g.L;
  a.K0 = g.K[0];
  a.rs = g.rs;
  a.unroll = opt(RS_OPT_MLP_UNROLL);
  return true;
}

}  // namespace rs
