// din.hip — DIN attention unit straight from behaviour ids (model/din.py:
// 56-80 + Attention, layer/interaction.py:355-406, 'prelu' mode):
//   q   = E[cand]                    key_t = value_t = E[hist_t]
//   e_t = [q, key_t, q-key_t, q*key_t]                 (:381-391)
//   h1  = PReLU_{alpha1[t]}(e_t W1 + b1)               (:366,393-394)
//   h2  = PReLU_{alpha2[t]}(h1 W2 + b2)
//   s_t = h2 w3 + b3; s_t = -4294967296 where hist_t == 0 (:396-401, din.py mask)
//   out = softmax_t(s) @ value                          (:403-405)
//
// MI355X design (two launches, weight-reuse first):
//  * The behaviour table (63,001 x 8 fp32 = 2 MB in the config) is L2-resident:
//    keys/values are read through the ids, never materialised as [B,T,k].
//  * Layer 1 is regrouped per sample: with W1 = [Wq; Wk; Wd; Wp] (k rows each),
//    e_t W1 = q (Wq + Wd) + key_t (Wk - Wd + diag(q) Wp).  The per-sample
//    matrix W'_b = Wkd + diag(q) Wp is built in registers (one FMA per A
//    value), so layer 1 costs k + k MAC rows per position instead of 4k:
//    on v_mfma_f32_16x16x4_f32 (swapped orientation C^T = W^T e^T) the B
//    operand is key_t for the W'_b steps and q (the same for every position
//    column) for the Wqd steps — q(Wq+Wd) lands in every column for free.
//  * din_scores: one workgroup per (16-position tile, 16 samples).  PReLU
//    alphas depend on the position only, so the tile's alpha1/alpha2 slices
//    (16 x 120 floats) and the W2^T image are staged in LDS once per
//    workgroup and reused by all 16 samples; layer 1's accumulators are
//    layer 2's B operand in registers (k order permuted to match).
//  * din_pool: one wave per sample — masked softmax over the T scores and
//    the weighted sum of the value rows (gathered through the ids again).
#include "concat.hpp"
#include "mlp_tower.hpp"
#include "rs_common.hpp"

namespace rs {

struct DinGeom {
  int k, KS, H1, H2, HT1, HT2, T, NTT;
  int64_t wkd, wp, wqd, b1, a1, w2, b2, a2, w3, b3, size;
};

static inline DinGeom din_geom(int T, int k, int H1, int H2) {
  DinGeom g{};
  g.k = k;
  g.KS = k / 4;
  g.H1 = H1;
  g.H2 = H2;
  g.HT1 = (H1 + 15) / 16;
  g.HT2 = (H2 + 15) / 16;
  g.T = T;
  g.NTT = (T + 15) / 16;
  const int64_t img1 = (int64_t)g.HT1 * g.KS * 64;
  int64_t o = 0;
  g.wkd = o; o += img1;
  g.wp = o; o += img1;
  g.wqd = o; o += img1;
  g.b1 = o; o += g.HT1 * 16;
  g.a1 = o; o += (int64_t)g.NTT * 16 * g.HT1 * 16;  // [t (padded)][h1 (padded)]
  g.w2 = o; o += (int64_t)g.HT2 * g.HT1 * 64 * 4;
  g.b2 = o; o += g.HT2 * 16;
  g.a2 = o; o += (int64_t)g.NTT * 16 * g.HT2 * 16;
  g.w3 = o; o += g.HT2 * 16;
  g.b3 = o; o += 4;
  g.size = o;
  return g;
}

struct DinPrepArgs {
  const float *W1, *b1, *alpha1, *W2, *b2, *alpha2, *w3, *b3;
  DinGeom g;
  float* out;
};

// Packs every operand image; element i of the prepared buffer.
__global__ void din_prepare_kernel(DinPrepArgs a) {
  const DinGeom& g = a.g;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.size) return;
  const int k = g.k, H1 = g.H1, H2 = g.H2;
  float v = 0.f;
  if (i < g.b1) {
    // layer-1 A images [HT1][KS][64]: lane (h = 16ht + (l&15), kk = l>>4),
    // step s <-> input row j = kk*KS + s of each k-row block
    const int which = (int)(i / (g.wp - g.wkd));
    const int64_t r = i - which * (g.wp - g.wkd);
    const int lane = (int)(r & 63), st = (int)(r >> 6);
    const int s = st % g.KS, ht = st / g.KS;
    const int h = 16 * ht + (lane & 15), j = (lane >> 4) * g.KS + s;
    if (h < H1) {
      const float wq = a.W1[(int64_t)(0 * k + j) * H1 + h], wk = a.W1[(int64_t)(1 * k + j) * H1 + h];
      const float wd = a.W1[(int64_t)(2 * k + j) * H1 + h], wpp = a.W1[(int64_t)(3 * k + j) * H1 + h];
      v = which == 0 ? wk - wd : which == 1 ? wpp : wq + wd;
    }
  } else if (i < g.a1) {
    const int h = (int)(i - g.b1);
    v = h < H1 ? a.b1[h] : 0.f;
  } else if (i < g.w2) {
    const int64_t r = i - g.a1;
    const int t = (int)(r / (g.HT1 * 16)), h = (int)(r % (g.HT1 * 16));
    v = (t < g.T && h < H1) ? a.alpha1[(int64_t)t * H1 + h] : 0.f;
  } else if (i < g.b2) {
    // W2^T image [HT2][HT1][64][4]: lane (h2 = 16ht2 + (l&15), kk), r:
    // W2[h1 = 16ht + 4kk + r][h2]
    const int64_t r0 = i - g.w2;
    const int r = (int)(r0 & 3), lane = (int)((r0 >> 2) & 63);
    const int64_t st = r0 >> 8;
    const int ht = (int)(st % g.HT1), ht2 = (int)(st / g.HT1);
    const int h2 = 16 * ht2 + (lane & 15), h1 = 16 * ht + 4 * (lane >> 4) + r;
    v = (h1 < H1 && h2 < H2) ? a.W2[(int64_t)h1 * H2 + h2] : 0.f;
  } else if (i < g.a2) {
    const int h = (int)(i - g.b2);
    v = h < H2 ? a.b2[h] : 0.f;
  } else if (i < g.w3) {
    const int64_t r = i - g.a2;
    const int t = (int)(r / (g.HT2 * 16)), h = (int)(r % (g.HT2 * 16));
    v = (t < g.T && h < H2) ? a.alpha2[(int64_t)t * H2 + h] : 0.f;
  } else if (i < g.b3) {
    const int h = (int)(i - g.w3);
    v = h < H2 ? a.w3[h] : 0.f;
  } else {
    v = i == g.b3 ? a.b3[0] : 0.f;
  }
  a.out[i] = v;
}

struct DinArgs {
  const void* hist;
  int64_t hist_stride;
  const void* cand;
  int64_t cand_stride;
  const float* table;
  int64_t vocab;
  const float* prep;
  DinGeom g;
  int64_t spc;    // samples per workgroup (din_scores)
  float* scores;  // [B, T] workspace
  float* out;     // [B, k], rows ldo floats apart
  int64_t ldo;
  int64_t batch;
  int* err;
  unsigned long long* dbg;  // diagnostics only: per-wave phase stamps (rs_diag_din_set_dbg)
  float* cand_out;          // optional [B, k] copy of the candidate rows (table[cand]), rows ldc floats apart
  int64_t ldc;
};
// (phase stamps only in the diagnostic build, scripts/build_diag.sh)
#ifdef RS_DIAG_STAMPS
#define DIN_STAMP(i)                                                                                   \
  do {                                                                                                 \
    if (a.dbg && (threadIdx.x & 63) == 0)                                                              \
      a.dbg[(((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6)) * 8 + (i)] =     \
          __builtin_amdgcn_s_memtime();                                                                \
  } while (0)
#else
#define DIN_STAMP(i) \
  do {               \
  } while (0)
#endif


// Keras PReLU max(0,x) + alpha*min(0,x) == x * (x < 0 ? alpha : 1) (one
// rounding either way).  The slope is chosen with the sign bit as a mask
// (v_ashrrev + v_bfi), then one multiply: fmaxf/fminf would add a
// NaN-canonicalising v_max per element, and a compare+select adds VCC-hazard
// nops between the MFMAs.
__device__ __forceinline__ float prelu(float x, float alpha) {
  const int m = __float_as_int(x) >> 31;  // all ones when x < 0 (sign bit)
  const int slope = (m & __float_as_int(alpha)) | (~m & 0x3f800000);
  return x * __int_as_float(slope);
}
constexpr int ATT_POOL_TMAX = 1024;

template <int KS>
__device__ __forceinline__ void din_row(const float* table, int64_t row, int kk, float (&v)[KS]) {
  const float* p = table + row * (4 * KS) + kk * KS;
  if constexpr (KS == 4) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(p);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  } else if constexpr (KS == 2) {
    const floatx2 x = *reinterpret_cast<const floatx2*>(p);
    v[0] = x[0]; v[1] = x[1];
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) v[s] = p[s];
  }
}

// HT1M/HT2M are the EXACT tile counts when EXACT (the reference's (80, 40) is
// (5, 3)): every guard folds away and the body is one straight MFMA stream;
// otherwise they are upper bounds checked at run time.
template <int KS, int HT1M, int HT2M, int KIND, bool EXACT>
__global__ __launch_bounds__(256, 4) void din_scores(DinArgs a) {  // 4 waves/SIMD: all 896 workgroups resident
  typedef Ids<KIND> I;
  const DinGeom& g = a.g;
  const int HT1 = EXACT ? HT1M : g.HT1, HT2 = EXACT ? HT2M : g.HT2;
  __shared__ float a1s[16][HT1M * 16 + 4];
  __shared__ float a2s[16][HT2M * 16 + 4];
  __shared__ floatx4 w2s[HT2M * HT1M * 64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, kg = lane >> 4;
  const int t0 = blockIdx.x * 16;
  DIN_STAMP(0);
#ifdef RS_DIAG_STAMPS
  if (a.dbg && (threadIdx.x & 63) == 0)
    a.dbg[(((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6)) * 8 + 6] =
        __builtin_amdgcn_s_memrealtime();
#endif

  // ---- stage the tile's alphas and the W2^T image (shared by 16 samples)
  const float* pa1 = a.prep + g.a1 + (int64_t)t0 * (HT1 * 16);
  const float* pa2 = a.prep + g.a2 + (int64_t)t0 * (HT2 * 16);
  // all loads first, then the LDS stores (one L2 round trip, not one per
  // iteration of a load->store loop)
  const floatx4* pw2 = reinterpret_cast<const floatx4*>(a.prep + g.w2);
  {
    constexpr int N1 = (16 * HT1M * 16 + 255) / 256, N2 = (16 * HT2M * 16 + 255) / 256;
    constexpr int NW2 = (HT2M * HT1M * 64 + 255) / 256;
    float v1[N1], v2[N2];
    floatx4 vw[NW2];
#pragma unroll
    for (int u = 0; u < N1; ++u) {
      const int i = threadIdx.x + 256 * u;
      v1[u] = i < 16 * HT1 * 16 ? pa1[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int i = threadIdx.x + 256 * u;
      v2[u] = i < 16 * HT2 * 16 ? pa2[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NW2; ++u) {
      const int i = threadIdx.x + 256 * u;
      vw[u] = i < HT2 * HT1 * 64 ? pw2[i] : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < N1; ++u) {
      const int i = threadIdx.x + 256 * u;
      if (i < 16 * HT1 * 16) a1s[i / (HT1 * 16)][i % (HT1 * 16)] = v1[u];
    }
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int i = threadIdx.x + 256 * u;
      if (i < 16 * HT2 * 16) a2s[i / (HT2 * 16)][i % (HT2 * 16)] = v2[u];
    }
#pragma unroll
    for (int u = 0; u < NW2; ++u) {
      const int i = threadIdx.x + 256 * u;
      if (i < HT2 * HT1 * 64) w2s[i] = vw[u];
    }
  }

  // biases and w3 in LDS (float4 per lane and tile at use): registers go to
  // the per-lane layer-1 images instead, keeping 4 waves/SIMD
  __shared__ floatx4 b1s[HT1M * 4], b2s[HT2M * 4], w3s[HT2M * 4];
  if (threadIdx.x < HT1M * 16) reinterpret_cast<float*>(b1s)[threadIdx.x] = threadIdx.x < HT1 * 16 ? a.prep[g.b1 + threadIdx.x] : 0.f;
  if (threadIdx.x < HT2M * 16) {
    reinterpret_cast<float*>(b2s)[threadIdx.x] = threadIdx.x < HT2 * 16 ? a.prep[g.b2 + threadIdx.x] : 0.f;
    reinterpret_cast<float*>(w3s)[threadIdx.x] = threadIdx.x < HT2 * 16 ? a.prep[g.w3 + threadIdx.x] : 0.f;
  }
  // ---- per-lane constants: layer-1 images
  float wkd[HT1M][KS], wpv[HT1M][KS], wqd[HT1M][KS];
#pragma unroll
  for (int ht = 0; ht < HT1M; ++ht) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int64_t o = (int64_t)(ht * KS + s) * 64 + lane;
      const bool on = ht < HT1;
      wkd[ht][s] = on ? a.prep[g.wkd + o] : 0.f;
      wpv[ht][s] = on ? a.prep[g.wp + o] : 0.f;
      wqd[ht][s] = on ? a.prep[g.wqd + o] : 0.f;
    }
  }
  const float b3 = a.prep[g.b3];
  __syncthreads();
  DIN_STAMP(1);

  const int t = t0 + col;
  const bool tv = t < g.T;
  bool bad = false;
  // The workgroup owns samples [c0, c1) of its tile; its 4 waves pull them
  // from an LDS counter (the next index is claimed while the current sample
  // is computed), so a wave that runs ahead takes more and the SIMDs of the
  // CU finish together.
  __shared__ int wctr;
  const int64_t c0 = (int64_t)blockIdx.y * a.spc, c1 = min(c0 + a.spc, a.batch);
  if (threadIdx.x == 0) wctr = 4;
  __syncthreads();
  int64_t nb = c0 + w;
  int cnt = 0;
  for (;;) {
    const int64_t b = nb;  // wave-uniform
    if (b >= c1) break;
    int nxt = 0;
    if (lane == 0) nxt = atomicAdd(&wctr, 1);
    nb = c0 + __builtin_amdgcn_readfirstlane(nxt);
    // candidate (query) row and this lane's behaviour row
    int64_t cid, hid;
    const typename I::raw_t craw = I::load(a.cand, b * a.cand_stride);
    const bool cok = I::decode(craw, a.vocab, cid);
    const typename I::raw_t hraw = I::load(a.hist, b * a.hist_stride + (tv ? t : 0));
    const bool hok = I::decode(hraw, a.vocab, hid);
    bad |= !cok || (tv && !hok);
    float q[KS], kv[KS];
    din_row<KS>(a.table, cid, kg, q);
    din_row<KS>(a.table, hid, kg, kv);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      q[s] = cok ? q[s] : 0.f;
      kv[s] = hok ? kv[s] : 0.f;
    }
    const bool masked = static_cast<float>(hraw) == 0.f;  // din.py: mask = hist != 0

    // layer 1 (lane holds h = 16ht + 4kg + r of position t)
    float y1[HT1M][4];
#pragma unroll
    for (int ht = 0; ht < HT1M; ++ht) {
      if (ht < HT1) {
        floatx4 acc = b1s[ht * 4 + kg];  // bias as the C input
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = mfma16x16x4(fmaf(q[s], wpv[ht][s], wkd[ht][s]), kv[s], acc);
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = mfma16x16x4(wqd[ht][s], q[s], acc);
        const floatx4 al = *reinterpret_cast<const floatx4*>(&a1s[col][16 * ht + 4 * kg]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          y1[ht][r] = prelu(acc[r], al[r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) y1[ht][r] = 0.f;
      }
    }
    // layer 2 + score
    float part = 0.f;
#pragma unroll
    for (int ht2 = 0; ht2 < HT2M; ++ht2) {
      if (ht2 < HT2) {
        floatx4 acc = b2s[ht2 * 4 + kg];
        const floatx4 w3v = w3s[ht2 * 4 + kg];
#pragma unroll
        for (int ht = 0; ht < HT1M; ++ht) {
          if (ht < HT1) {
            const floatx4 wa = w2s[(ht2 * HT1 + ht) * 64 + lane];
#pragma unroll
            for (int r = 0; r < 4; ++r) acc = mfma16x16x4(wa[r], y1[ht][r], acc);
          }
        }
        const floatx4 al = *reinterpret_cast<const floatx4*>(&a2s[col][16 * ht2 + 4 * kg]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          part = fmaf(prelu(acc[r], al[r]), w3v[r], part);
        }
      }
    }
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    if (kg == 0 && tv) a.scores[b * g.T + t] = masked ? -4294967296.0f : part + b3;
    if (cnt < 4) DIN_STAMP(2 + cnt);
    ++cnt;
  }
  if (__any(bad) && lane == 0) flag_error(a.err);
#ifdef RS_DIAG_STAMPS
  if (a.dbg && (threadIdx.x & 63) == 0)
    a.dbg[(((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6)) * 8 + 7] =
        __builtin_amdgcn_s_memrealtime();
#endif
}

// masked softmax over the T scores and out[b] = sum_t a_t * E[hist_t].
// One wave per sample: (1) lanes take positions t = lane + 64i: score, id
// -> e_t = exp(s_t - max) and the row index into LDS; (2) lanes (position
// group tg, channel j) sum e_t * E[id_t][j] with independent (L2) loads.
template <int KIND>
__global__ __launch_bounds__(256) void din_pool(DinArgs a) {
  typedef Ids<KIND> I;
  __shared__ float es[4][ATT_POOL_TMAX];
  __shared__ int rs_[4][ATT_POOL_TMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * 4 + w;
  if (b >= a.batch) return;  // wave-uniform; no block barrier below
  const int T = a.g.T, k = a.g.k;
  const float* sc = a.scores + b * T;
  float mx = -INFINITY;
  for (int t = lane; t < T; t += 64) mx = fmaxf(mx, sc[t]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float sum = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float e = expf(sc[t] - mx);
    int64_t id;
    const bool ok = I::decode(I::load(a.hist, b * a.hist_stride + t), a.vocab, id);
    es[w][t] = ok ? e : 0.f;  // an OOR id (flagged by din_scores) contributes a zero row
    rs_[w][t] = ok ? (int)id : 0;
    sum += e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int ntg = 64 / k, j = lane % k, tg = lane / k;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int t = tg;
  for (; t + 3 * ntg < T; t += 4 * ntg) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = fmaf(es[w][t + u * ntg], a.table[(int64_t)rs_[w][t + u * ntg] * k + j], acc[u]);
  }
  for (; t < T; t += ntg) acc[0] = fmaf(es[w][t], a.table[(int64_t)rs_[w][t] * k + j], acc[0]);
  float v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  for (int o = k; o < 64; o <<= 1) v += __shfl_xor(v, o);
  if (lane < k) a.out[b * a.ldo + lane] = v / sum;
  if (a.cand_out && lane < k) {  // the candidate row (an OOR id: a zero row, flagged by din_scores)
    int64_t cid;
    const bool ok = I::decode(I::load(a.cand, b * a.cand_stride), a.vocab, cid);
    a.cand_out[b * a.ldc + lane] = ok ? a.table[cid * k + lane] : 0.f;
  }
}

// ---- One-launch DIN attention unit (din_fused; RS_OPT_DIN_KERNEL 0, the
// default at the reference's (80, 40) widths): scores, masked softmax and the
// pool in ONE kernel, no [B, T] score round trip through HBM and no second
// launch.  One 16-wave workgroup per CU owns DF_SPW samples, ALL their
// position tiles: the PReLU alphas of every position (a [NTT*16][HT*16]
// slice of each layer) and the W2^T image are staged in LDS once per
// workgroup; item (sample, tile) = one 16-position MFMA tile exactly as in
// din_scores (layer 1 regrouped per sample, layer 1's accumulators are layer
// 2's B operand), the wave's next item's rows requested while the current
// one computes (the ids are read once per workgroup into LDS).  Only LIVE
// tiles (>= 1 unmasked position) are items: a fully masked tile's scores
// are the mask value whatever the MLP gives, and its merge weight is exactly
// 0.  Each item ends with its tile's online-softmax partial {m_j = max s_t,
// l_j = sum e^(s_t - m_j), o_j = sum e^(s_t - m_j) key_t} in LDS; after one
// barrier a wave per sample merges its live tiles (m = max m_j, weights
// e^(m_j - m)) and writes out[b] = o / l.  Live items are dealt round-robin
// to the waves (w, w + 16, ..): with no masking, 8 samples x 7 tiles put 14
// items on every SIMD.  Masking as the reference (din.py: hist != 0 ->
// score -2^32 + 1 in fp32 = -4294967296): a fully masked row averages its
// keys; an out-of-range id reads a zero row and sets the flag (din_pool's
// rule).  Reference: layer/interaction.py:369-406, model/din.py:56-80.
#ifdef RS_DIAG_STAMPS
#define DF_STAMP(i)                                                                                            \
  do {                                                                                                         \
    if (a.dbg && (threadIdx.x & 63) == 0)                                                                      \
      a.dbg[((int64_t)blockIdx.x * DF_NW + (threadIdx.x >> 6)) * 16 + (i)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define DF_STAMP(i) \
  do {              \
  } while (0)
#endif
constexpr int DF_SPW = 8;     // samples per workgroup
constexpr int DF_NW = 16;     // waves per workgroup
constexpr int DF_MAXK = 16;   // embedding width (k) at most
constexpr int DF_TMAX = 128;  // history length at most (8 position tiles)

struct DfLayout {  // dynamic LDS (floats): a1s | a2s | w2s | w1s (layer-1 lane images) | part
  int a1, a2, w2, w1, part, total;
};
__host__ __device__ inline DfLayout df_layout(int NTT, int HT1, int HT2, int KS) {
  DfLayout L;
  L.a1 = 0;
  L.a2 = L.a1 + NTT * 16 * (HT1 * 16 + 4);
  L.w2 = L.a2 + NTT * 16 * (HT2 * 16 + 4);
  L.w1 = L.w2 + HT2 * HT1 * 64 * 4;
  L.part = L.w1 + 3 * HT1 * KS * 64;
  L.total = L.part + DF_SPW * NTT * (2 + DF_MAXK);
  return L;
}

// NTTC > 0: the position-tile count known at compile time (config 4: T =
// 100 -> 7 tiles): the (sample, tile) item codes, the live-tile scan and the
// merge loops fold to constants instead of run-time division / loop control
// TW (rs_din_forward_ids: DIN.call from the attention to the logit in ONE
// launch): after the merge the workgroup's tower input rows [pooled | cand |
// pieces] (model/din.py:84-85) are staged in LDS — BatchNormalization's affine
// applied as rs_mlp_affine_pieces_fwd stages it, the pieces' ids and rows
// requested at kernel start — over the dead alpha images, and the PReLU tower
// + Dense(1, sigmoid) runs on the 16-row MFMA tile (rows >= the workgroup's
// samples are zero and never stored) with the DIN tower's own code
// (mlp_layer0_tiles + mlp_tail_run): every valid row's arithmetic is the
// separate tower launch's, so the logits are bit-identical to
// rs_din_attention_ids_cand_fwd + rs_mlp_affine_pieces_fwd.
struct DinTower {
  MlpArgs t;       // the tower (y, head = 0, M = batch)
  ConcatArgs pc;   // the pieces at tower columns >= 2k
  int tbase;       // floats: the tower's LDS region in the dynamic LDS (0: over the alpha images)
};

template <int KS, int HT1, int HT2, int KIND, int NTTC, bool TW>
__device__ __forceinline__ void din_fused_body(const DinArgs& a, const DinTower* tw) {
  typedef Ids<KIND> I;
  constexpr int K = 4 * KS;
  const DinGeom& g = a.g;
  const int NTT = NTTC > 0 ? NTTC : g.NTT, T = g.T;
  const DfLayout L = df_layout(NTT, HT1, HT2, KS);
  extern __shared__ float dsm[];
  float* a1s = dsm + L.a1;  // [NTT*16][HT1*16 + 4]
  float* a2s = dsm + L.a2;  // [NTT*16][HT2*16 + 4]
  floatx4* w2s = reinterpret_cast<floatx4*>(dsm + L.w2);
  float* part = dsm + L.part;  // [DF_SPW * NTT][2 + DF_MAXK]
  __shared__ floatx4 b1s[HT1 * 4], b2s[HT2 * 4], w3s[HT2 * 4];
  constexpr int A1W = HT1 * 16 + 4, A2W = HT2 * 16 + 4;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, kg = lane >> 4;
  const int64_t s0 = (int64_t)blockIdx.x * DF_SPW;
  const int nsmp = (int)min<int64_t>(DF_SPW, a.batch - s0);
  DF_STAMP(0);

  // ---- the workgroup's ids: wave s < nsmp loads sample s's history ids
  // (positions lane, lane + 64) and its candidate id into LDS and marks its
  // LIVE tiles, the 16-position tiles holding at least one unmasked position.
  // A tile whose valid positions are all masked adds exactly nothing to its
  // sample's pool when the sample has a live tile: its scores are the mask
  // value -2^32 whatever the MLP computes, so its merge weight
  // e^(-2^32 - m) is 0 in fp32 and the merge adds l_j x 0 and o_j x 0.  So
  // only live tiles run the MLP (bit-identical output); a sample with no live
  // tile runs all its tiles (the fully-masked average of din.py's softmax).
  __shared__ typename I::raw_t hs[DF_SPW][DF_TMAX];
  __shared__ typename I::raw_t cs[DF_SPW];
  __shared__ unsigned tmask[DF_SPW];
  typename I::raw_t h0 = 0, h1 = 0, c0 = 0;
  float cq = 0.f;
  if (w < nsmp) {
    const int64_t b = s0 + w;
    if (lane < T) h0 = I::load(a.hist, b * a.hist_stride + lane);
    if (lane + 64 < T) h1 = I::load(a.hist, b * a.hist_stride + lane + 64);
    c0 = I::load(a.cand, b * a.cand_stride);
  }
  // TW: lane c of wave s < nsmp holds tower input column c of sample s; a
  // piece column's raw id (or dense value) is requested now, its row after
  // the ids reach LDS
  int tp = -1;
  int64_t traw = 0;
  float tval = 0.f, tpar = 0.f, tsc = 0.f, tsh = 0.f;
  if constexpr (TW) {
    const ConcatArgs& pc = tw->pc;
    // the BatchNormalization affine of this lane's tower column (read at the merge)
    if (lane < tw->t.K0) {
      tsc = tw->t.in_scale[lane];
      tsh = tw->t.in_shift[lane];
    }
    // the tower's bias / alpha block (its first 1024 floats; the DIN tower's
    // is 928): requested now, stored to LDS after the items — its trip stays
    // off the merge
    if (threadIdx.x < (unsigned)tw->t.ptot) tpar = tw->t.prep[tw->t.wtot + threadIdx.x];
    if (w < nsmp && lane >= 2 * K && lane < tw->t.K0) {
      for (int q = 0; q < pc.np; ++q)
        if (lane >= pc.out_col[q] && lane < pc.out_col[q] + (pc.col0[q + 1] - pc.col0[q])) tp = q;
      if (tp >= 0) {
        const int64_t off = (s0 + w) * pc.src_stride[tp];
        switch (pc.kind[tp]) {
          case RS_ID_I32: traw = static_cast<const int32_t*>(pc.src[tp])[off]; break;
          case RS_ID_I64: traw = static_cast<const int64_t*>(pc.src[tp])[off]; break;
          case RS_ID_F32: traw = (int64_t)__float_as_uint(static_cast<const float*>(pc.src[tp])[off]); break;
          default: tval = static_cast<const float*>(pc.src[tp])[off + (lane - pc.out_col[tp])]; break;
        }
      }
    }
  }
  bool tbad = false;
  auto ids_to_lds = [&]() {
    if (w < nsmp) {
      hs[w][lane] = h0;
      hs[w][lane + 64] = h1;
      if (lane == 0) cs[w] = c0;
      if (TW || a.cand_out) {  // the candidate row for the caller's concat, written at the merge
        int64_t cid;
        const bool ok = I::decode(c0, a.vocab, cid);
        const int cl = TW ? lane - K : lane;  // TW: lanes K..2K-1 hold the tower's cand columns
        cq = ok && cl >= 0 && cl < K ? a.table[cid * K + cl] : 0.f;
      }
      if constexpr (TW) {  // the piece's row (its id arrived with the history ids)
        const ConcatArgs& pc = tw->pc;
        if (tp >= 0 && pc.kind[tp] >= 0) {
          int64_t id = 0;
          bool ok;
          if (pc.kind[tp] == RS_ID_F32) {
            const float f = __uint_as_float((unsigned)traw);
            ok = f > -1.0f && static_cast<double>(f) < static_cast<double>(pc.vocab[tp]);
            id = ok ? static_cast<int64_t>(f) : 0;
          } else {
            id = traw;
            ok = id >= 0 && id < pc.vocab[tp];
          }
          tbad = !ok;
          const int kw = pc.col0[tp + 1] - pc.col0[tp];
          tval = ok ? pc.table[tp][id * kw + (lane - pc.out_col[tp])] : 0.f;
        }
      }
      const uint64_t l0 = __ballot(lane < T && static_cast<float>(h0) != 0.f);  // din.py: mask = hist != 0
      const uint64_t l1 = __ballot(lane + 64 < T && static_cast<float>(h1) != 0.f);
      unsigned m = 0;
      for (int j = 0; j < NTT; ++j) m |= (((j < 4 ? l0 >> (16 * j) : l1 >> (16 * (j - 4))) & 0xffffu) != 0) << j;
      if (lane == 0) tmask[w] = m ? m : (1u << NTT) - 1;
    }
  };
  auto item_rows = [&](int code, float (&q)[KS], float (&kv)[KS]) {  // code = sample * NTT + tile
    const int si = code / NTT, j = code - si * NTT;
    int64_t cid, hid;
    I::decode(cs[si], a.vocab, cid);
    I::decode(hs[si][16 * j + col], a.vocab, hid);
    din_row<KS>(a.table, cid, kg, q);
    din_row<KS>(a.table, hid, kg, kv);
  };
  float q[KS], kv[KS];
  __builtin_amdgcn_sched_barrier(0);

  // ---- stage every position's alphas and the W2^T image: every load of a
  // round is issued before its LDS stores (a load -> store loop pays one L2
  // round trip per iteration: 7.7k cycles of staging in the first version)
  {
    // 16-B loads and stores (round 5: 4-B ones issued 4x the vector memory
    // instructions — 51 per wave with the per-lane constants — and the
    // staging took 5.8k-7.7k cycles); rows of HT*16 floats never straddle a float4
    const floatx4* pa1 = reinterpret_cast<const floatx4*>(a.prep + g.a1);
    const floatx4* pa2 = reinterpret_cast<const floatx4*>(a.prep + g.a2);
    const floatx4* pw2 = reinterpret_cast<const floatx4*>(a.prep + g.w2);
    const int n1 = NTT * 16 * HT1 * 4, n2 = NTT * 16 * HT2 * 4, nw2 = HT2 * HT1 * 64;  // float4s
    constexpr int R1 = 3, R2 = 2, NTH = DF_NW * 64, W1 = HT1 * 4, W2 = HT2 * 4;
    for (int b1 = 0, b2 = 0, bw = 0; b1 < n1 || b2 < n2 || bw < nw2; b1 += R1 * NTH, b2 += R2 * NTH, bw += NTH) {
      floatx4 v1[R1], v2[R2], vw;
#pragma unroll
      for (int u = 0; u < R1; ++u) v1[u] = pa1[min(b1 + u * NTH + (int)threadIdx.x, n1 - 1)];  // clamped: unconditional
#pragma unroll
      for (int u = 0; u < R2; ++u) v2[u] = pa2[min(b2 + u * NTH + (int)threadIdx.x, n2 - 1)];
      vw = pw2[min(bw + (int)threadIdx.x, nw2 - 1)];
      if (b1 == 0) {
        __builtin_amdgcn_sched_barrier(0);
        ids_to_lds();
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < R1; ++u) {
        const int i = b1 + u * NTH + threadIdx.x;
        if (i < n1) *reinterpret_cast<floatx4*>(a1s + (i / W1) * A1W + 4 * (i % W1)) = v1[u];
      }
#pragma unroll
      for (int u = 0; u < R2; ++u) {
        const int i = b2 + u * NTH + threadIdx.x;
        if (i < n2) *reinterpret_cast<floatx4*>(a2s + (i / W2) * A2W + 4 * (i % W2)) = v2[u];
      }
      if (bw + (int)threadIdx.x < nw2) w2s[bw + threadIdx.x] = vw;
    }
    // the layer-1 lane images (wkd | wp | wqd, contiguous in prep) once per
    // workgroup: each wave reads its 3 x HT1 x KS values from LDS after the
    // barrier instead of 30 4-B global loads per wave
    {
      const int nl = 3 * HT1 * KS * 16;  // float4s
      const floatx4* pl = reinterpret_cast<const floatx4*>(a.prep + g.wkd);
      for (int i = threadIdx.x; i < nl; i += NTH) reinterpret_cast<floatx4*>(dsm + L.w1)[i] = pl[i];
    }
    if (threadIdx.x < HT1 * 16) reinterpret_cast<float*>(b1s)[threadIdx.x] = a.prep[g.b1 + threadIdx.x];
    if (threadIdx.x < HT2 * 16) {
      reinterpret_cast<float*>(b2s)[threadIdx.x] = a.prep[g.b2 + threadIdx.x];
      reinterpret_cast<float*>(w3s)[threadIdx.x] = a.prep[g.w3 + threadIdx.x];
    }
  }
  const float b3 = a.prep[g.b3];
  DF_STAMP(6);  // staging stores issued (before the barrier)
  __syncthreads();
  DF_STAMP(1);
  // the wave's live items, built once: lane L < nsmp * NTT stands for
  // (sample L / NTT, tile L % NTT); the live ones are numbered in lane order
  // (sample-major) and dealt round-robin (w, w + 16, ..): at most 4 per wave,
  // kept as 6-bit lane codes in one register
  unsigned items = 0;
  int nmine = 0;
  {
    const int si = lane / NTT, j = lane - si * NTT;
    const bool live = lane < nsmp * NTT && (tmask[si < DF_SPW ? si : 0] >> j & 1);
    const uint64_t lv = __ballot(live);
    const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(lv >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)lv, 0));
    for (int m = 0; m < 4; ++m) {
      const uint64_t hit = __ballot(live && rank == w + DF_NW * m);
      if (!hit) break;
      items |= (unsigned)__builtin_ctzll(hit) << (6 * m);
      ++nmine;
    }
  }
  // the first item's rows now: their trip overlaps the lane-image reads
  if (nmine > 0) item_rows(items & 63, q, kv);
  // layer 1's lane images in registers; at k = 16 the q image stays in LDS
  // and is read at its MFMA (all three in registers spill at 128 VGPRs)
  constexpr bool QREG = KS < 4;
  float wkd[HT1][KS], wpv[HT1][KS], wqd[HT1][QREG ? KS : 1];
  const float* w1q = dsm + L.w1 + 2 * HT1 * KS * 64 + lane;  // the q image, [HT1][KS][64]
  {
    const float* w1s = dsm + L.w1;  // [wkd | wp | wqd], each [HT1][KS][64]
    const int img = HT1 * KS * 64;
#pragma unroll
    for (int ht = 0; ht < HT1; ++ht) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int o = (ht * KS + s) * 64 + lane;
        wkd[ht][s] = w1s[o];
        wpv[ht][s] = w1s[img + o];
        if constexpr (QREG) wqd[ht][s] = w1s[2 * img + o];
      }
    }
  }

  bool bad = false;
  int cnt = 0;
  for (int m = 0; m < nmine; ++m) {
    const int code = __builtin_amdgcn_readfirstlane((items >> (6 * m)) & 63);
    const int si = code / NTT, j = code - si * NTT;
    const int t = 16 * j + col;
    const bool tv = t < T;
    const typename I::raw_t cr0 = cs[si], hr0 = hs[si][t];
    int64_t cid, hid;
    const bool cok = I::decode(cr0, a.vocab, cid);
    const bool hok = I::decode(hr0, a.vocab, hid);
    bad |= !cok || (tv && !hok);
    const bool masked = static_cast<float>(hr0) == 0.f;  // din.py: mask = hist != 0
    float qc[KS], kc[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qc[s] = cok ? q[s] : 0.f;
      kc[s] = hok ? kv[s] : 0.f;
    }
    // the next item's rows (ids in LDS), requested under this item's MFMAs
    if (m + 1 < nmine) item_rows((items >> (6 * (m + 1))) & 63, q, kv);
    // pinned here: left alone the scheduler sinks these loads to the end of
    // the item, and the next item's loop-head vmcnt(0) then pays their trip
    __builtin_amdgcn_sched_barrier(0);

    if (cnt == 0) DF_STAMP(8);  // item 0: its operands in registers, MFMAs start
    // layer 1 (lane holds h = 16ht + 4kg + r of position t)
    float y1[HT1][4];
#pragma unroll
    for (int ht = 0; ht < HT1; ++ht) {
      floatx4 acc = b1s[ht * 4 + kg];  // bias as the C input
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = mfma16x16x4(fmaf(qc[s], wpv[ht][s], wkd[ht][s]), kc[s], acc);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if constexpr (QREG) acc = mfma16x16x4(wqd[ht][s], qc[s], acc);
        else acc = mfma16x16x4(w1q[(ht * KS + s) * 64], qc[s], acc);
      }
      const floatx4 al = *reinterpret_cast<const floatx4*>(&a1s[t * A1W + 16 * ht + 4 * kg]);
#pragma unroll
      for (int r = 0; r < 4; ++r) y1[ht][r] = prelu(acc[r], al[r]);
    }
    if (cnt == 0) DF_STAMP(9);  // item 0: layer 1 done
    // layer 2 + score: the HT2 accumulators advance together (independent chains)
    floatx4 acc2[HT2];
#pragma unroll
    for (int h2 = 0; h2 < HT2; ++h2) acc2[h2] = b2s[h2 * 4 + kg];
#pragma unroll
    for (int ht = 0; ht < HT1; ++ht) {
      floatx4 wa[HT2];
#pragma unroll
      for (int h2 = 0; h2 < HT2; ++h2) wa[h2] = w2s[(h2 * HT1 + ht) * 64 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int h2 = 0; h2 < HT2; ++h2) acc2[h2] = mfma16x16x4(wa[h2][r], y1[ht][r], acc2[h2]);
    }
    if (cnt == 0) DF_STAMP(10);  // item 0: layer 2 issued
    float sc = 0.f;
#pragma unroll
    for (int h2 = 0; h2 < HT2; ++h2) {
      const floatx4 al = *reinterpret_cast<const floatx4*>(&a2s[t * A2W + 16 * h2 + 4 * kg]);
      const floatx4 w3v = w3s[h2 * 4 + kg];
#pragma unroll
      for (int r = 0; r < 4; ++r) sc = fmaf(prelu(acc2[h2][r], al[r]), w3v[r], sc);
    }
    sc += __shfl_xor(sc, 16);
    sc += __shfl_xor(sc, 32);
    sc = masked ? -4294967296.0f : sc + b3;
    // the tile's online-softmax partial (positions past T excluded)
    float mj = tv ? sc : -INFINITY;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mj = fmaxf(mj, __shfl_xor(mj, o));
    const float e = tv ? __expf(sc - mj) : 0.f;
    const float lj = row16_sum(e);
    float* pp = part + (size_t)code * (2 + DF_MAXK);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float os = row16_sum(e * kc[s]);
      if (col == 0) pp[2 + kg * KS + s] = os;
    }
    if (lane == 0) {
      pp[0] = mj;
      pp[1] = lj;
    }
    if (cnt < 4) DF_STAMP(2 + cnt);
    ++cnt;
  }
  if (__any(bad) && lane == 0) flag_error(a.err);
  __syncthreads();
  floatx4 ring[MLP_R];
  floatx4 wa[8];
  const bool tspec = TW && tw->t.Np[1] == 128 && tw->t.Np[2] == 64;  // mlp_tail_run's specialised widths
  // TW: the tower's buf0 | buf1 | red | par — over the alpha / weight images
  // (dead now) when they fit below the partials the merge reads, else past them
  float* tsm = TW ? dsm + tw->tbase : dsm;
  if constexpr (TW) {
    const MlpArgs& t = tw->t;
    if (__any(tbad) && lane == 0) flag_error(tw->pc.err);
    mlp_first_fill<DF_NW>(t, ring);  // layer 0's weights under the merge
    // ... and layer 1's slice of this wave (its 128 KB per workgroup through
    // the CU's L2 port would otherwise sit between layer 0 and layer 1)
    if (tspec) mlp_tail_fetch<8, 8>(t, 1, wa);
    else mlp_tail_fetch<8>(t, 1, wa);
    float* par = tsm + 32 * t.rs + DF_NW * 256;
    if (threadIdx.x < (unsigned)t.ptot) par[threadIdx.x] = tpar;
    for (int i = threadIdx.x + DF_NW * 64; i < t.ptot; i += DF_NW * 64) par[i] = t.prep[t.wtot + i];
  }
  // merge the tiles of sample w (one wave per sample, lane c < k = channel)
  if (TW && w < 16) {
    // tower input row w: [pooled (merge below) | cand | pieces | 0 padding];
    // rows >= nsmp are zero
    const MlpArgs& t = tw->t;
    float v = 0.f;
    if (w < nsmp && lane >= K && lane < t.K0) v = lane < 2 * K ? cq : tval;
    if (w < nsmp && lane >= K && lane < t.K0) {
#pragma clang fp contract(off)  // two roundings, as rs_affine_act (no fma)
      v = v * tsc + tsh;
    }
    if (lane >= K || w >= nsmp)
      if (lane < t.Kp[0]) tsm[w * t.rs + lane] = v;
  }
  if (w < nsmp && lane < K) {
    const float* pp = part + (size_t)w * NTT * (2 + DF_MAXK);
    const unsigned mk = tmask[w];  // live tiles only (the others would add exact zeros)
    float m = -INFINITY;
    for (int jj = 0; jj < NTT; ++jj)
      if (mk >> jj & 1) m = fmaxf(m, pp[jj * (2 + DF_MAXK)]);
    float l = 0.f, o = 0.f;
    for (int jj = 0; jj < NTT; ++jj) {
      if (!(mk >> jj & 1)) continue;
      const float sj = __expf(pp[jj * (2 + DF_MAXK)] - m);
      l = fmaf(pp[jj * (2 + DF_MAXK) + 1], sj, l);
      o = fmaf(pp[jj * (2 + DF_MAXK) + 2 + lane], sj, o);
    }
    const float pooled = o / l;
    if constexpr (TW) {
      const MlpArgs& t = tw->t;
      float v;
      {
#pragma clang fp contract(off)  // two roundings, as rs_affine_act (no fma)
        v = pooled * tsc + tsh;
      }
      tsm[w * t.rs + lane] = v;
      if (a.out) a.out[(s0 + w) * a.ldo + lane] = pooled;
    } else {
      a.out[(s0 + w) * a.ldo + lane] = pooled;
      if (a.cand_out) a.cand_out[(s0 + w) * a.ldc + lane] = cq;
    }
  }
  DF_STAMP(7);
  if constexpr (TW) {
    // rows s0 .. s0 + nsmp - 1 are this workgroup's (M: the others are never stored)
    MlpArgs t = tw->t;
    t.M = s0 + nsmp;
    mlp_layer0_tiles<DF_NW>(t, tsm, ring);
    if (tspec) mlp_tail_splitk<DF_NW, 8, 2, 8, 4>(t, tsm, s0, wa, nullptr, 1);  // = mlp_tail_run, slice fetched above
    else mlp_tail_splitk<DF_NW, 8, 2>(t, tsm, s0, wa, nullptr, 1);
  }
}

template <int KS, int HT1, int HT2, int KIND, int NTTC = 0>
__global__ __launch_bounds__(DF_NW * 64) void din_fused(DinArgs a) {
  din_fused_body<KS, HT1, HT2, KIND, NTTC, false>(a, nullptr);
}
template <int KS, int HT1, int HT2, int KIND, int NTTC = 0>
__global__ __launch_bounds__(DF_NW * 64) void din_fused_tower(DinArgs a, DinTower tw) {
  din_fused_body<KS, HT1, HT2, KIND, NTTC, true>(a, &tw);
}

template <int KS, int HT1M, int HT2M, int KIND, bool EXACT>
static void launch_din(const DinArgs& a, hipStream_t st) {
  // One resident round: 4 workgroups per CU (4 waves/SIMD), the batch split
  // evenly over (position tile, sample chunk).
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1) n_cu = 256;
  }
  DinArgs b = a;
  const int64_t per_tile = std::max<int64_t>(1, std::min<int64_t>((4 * n_cu) / a.g.NTT, (a.batch + 3) / 4));
  b.spc = (a.batch + per_tile - 1) / per_tile;
  const dim3 grid(a.g.NTT, (unsigned)((a.batch + b.spc - 1) / b.spc));
  din_scores<KS, HT1M, HT2M, KIND, EXACT><<<grid, 256, 0, st>>>(b);
  din_pool<KIND><<<(unsigned)((a.batch + 3) / 4), 256, 0, st>>>(b);
}

// din_fused's dynamic LDS for this shape, or 0 when it does not fit
static size_t df_lds(const DinGeom& g) {
  const size_t b = (size_t)df_layout(g.NTT, g.HT1, g.HT2, g.KS).total * sizeof(float);
  // (+ the static bias / w3 tiles and the id tile: <= 8 B per id)
  return g.NTT * 16 <= DF_TMAX && b + 1024 + DF_SPW * (DF_TMAX + 2) * 8 <= 160 * 1024 ? b : 0;
}

template <int KS, int KIND>
static void launch_din_h(const DinArgs& a, hipStream_t st) {
  if (a.g.HT1 == 5 && a.g.HT2 == 3) {  // reference (80, 40)
    const size_t lds = df_lds(a.g);
    if (opt(RS_OPT_DIN_KERNEL) == 0 && lds) {
      DinArgs b = a;
      const unsigned grid = (unsigned)((a.batch + DF_SPW - 1) / DF_SPW);
      if (KS == 2 && a.g.NTT == 7) {  // config 4 (k 8, T 97..112)
        static LdsAttr set7;
        lds_attr(set7, (const void*)din_fused<KS, 5, 3, KIND, 7>, lds);
        din_fused<KS, 5, 3, KIND, 7><<<grid, DF_NW * 64, lds, st>>>(b);
        return;
      }
      static LdsAttr set;
      lds_attr(set, (const void*)din_fused<KS, 5, 3, KIND>, lds);
      din_fused<KS, 5, 3, KIND><<<grid, DF_NW * 64, lds, st>>>(b);
      return;
    }
    launch_din<KS, 5, 3, KIND, true>(a, st);
  } else {
    launch_din<KS, 8, 4, KIND, false>(a, st);
  }
}

}  // namespace rs

using namespace rs;

static unsigned long long* g_din_dbg = nullptr;
extern "C" void rs_diag_din_set_dbg(unsigned long long* p) { g_din_dbg = p; }

extern "C" int64_t rs_din_prepared_size(int T, int k, int H1, int H2) {
  if (T < 1 || (k != 4 && k != 8 && k != 16) || H1 < 1 || H1 > 128 || H2 < 1 || H2 > 64) return -1;
  return din_geom(T, k, H1, H2).size;
}

extern "C" int rs_din_prepare(const float* W1, const float* b1, const float* alpha1, int H1, const float* W2,
                              const float* b2, const float* alpha2, int H2, const float* w3, const float* b3, int T,
                              int k, float* prepared, rs_stream_t stream) {
  RS_REQUIRE(rs_din_prepared_size(T, k, H1, H2) > 0, "rs_din_prepare: need k in {4,8,16}, H1 <= 128, H2 <= 64");
  RS_REQUIRE(W1 && b1 && alpha1 && W2 && b2 && alpha2 && w3 && b3 && prepared, "rs_din_prepare: null pointer");
  DinPrepArgs a{W1, b1, alpha1, W2, b2, alpha2, w3, b3, din_geom(T, k, H1, H2), prepared};
  din_prepare_kernel<<<(unsigned)((a.g.size + 255) / 256), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_din_prepare");
}

static int din_ids_run(const void* hist, int id_kind, int64_t hist_stride, const void* cand,
                                        int64_t cand_stride, int T, int k, const float* table, int64_t vocab,
                                        int H1, int H2, const float* prepared, float* scores, float* out,
                                        int64_t out_stride, float* cand_out, int64_t cand_out_stride, int64_t batch,
                      int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(rs_din_prepared_size(T, k, H1, H2) > 0,
             "rs_din_attention_ids_fwd: need k in {4,8,16}, H1 <= 128, H2 <= 64");
  RS_REQUIRE(hist && cand && table && prepared && scores && out, "rs_din_attention_ids_fwd: null pointer");
  RS_REQUIRE(T <= ATT_POOL_TMAX && vocab < (1ll << 31), "rs_din_attention_ids_fwd: T > %d or vocab >= 2^31", ATT_POOL_TMAX);
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32 && vocab >= 1 && batch >= 0 && hist_stride >= T,
             "rs_din_attention_ids_fwd: bad ids / shape");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_din_attention_ids_fwd: table must be 16-B aligned");
  RS_REQUIRE(out_stride >= k, "rs_din_attention_ids_fwd: out_stride < k");
  RS_REQUIRE(!cand_out || cand_out_stride >= k, "rs_din_attention_ids_cand_fwd: cand_out_stride < k");
  if (batch == 0) return RS_OK;
  DinArgs a{hist, hist_stride, cand, cand_stride, table, vocab, prepared, din_geom(T, k, H1, H2),
            0, scores, out, out_stride, batch, err_flag, g_din_dbg, cand_out, cand_out_stride};
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KIND = decltype(K)::value;
    if (k == 4) launch_din_h<1, KIND>(a, st);
    else if (k == 8) launch_din_h<2, KIND>(a, st);
    else launch_din_h<4, KIND>(a, st);
  });
  return launch_status(cand_out ? "rs_din_attention_ids_cand_fwd" : "rs_din_attention_ids_fwd");
}

extern "C" int rs_din_attention_ids_fwd(const void* hist, int id_kind, int64_t hist_stride, const void* cand,
                                        int64_t cand_stride, int T, int k, const float* table, int64_t vocab,
                                        int H1, int H2, const float* prepared, float* scores, float* out,
                                        int64_t out_stride, int64_t batch, int* err_flag, rs_stream_t stream) {
  return din_ids_run(hist, id_kind, hist_stride, cand, cand_stride, T, k, table, vocab, H1, H2, prepared, scores,
                     out, out_stride, nullptr, 0, batch, err_flag, stream);
}

extern "C" int rs_din_attention_ids_cand_fwd(const void* hist, int id_kind, int64_t hist_stride, const void* cand,
                                             int64_t cand_stride, int T, int k, const float* table, int64_t vocab,
                                             int H1, int H2, const float* prepared, float* scores, float* out,
                                             int64_t out_stride, float* cand_out, int64_t cand_out_stride,
                                             int64_t batch, int* err_flag, rs_stream_t stream) {
  RS_REQUIRE(batch == 0 || cand_out, "rs_din_attention_ids_cand_fwd: null cand_out");
  return din_ids_run(hist, id_kind, hist_stride, cand, cand_stride, T, k, table, vocab, H1, H2, prepared, scores,
                     out, out_stride, cand_out, cand_out_stride, batch, err_flag, stream);
}

// ---- DIN.call in ONE launch (din_fused_tower): the attention unit from the
// behaviour ids, then BatchNormalization + the PReLU tower + Dense(1,
// sigmoid) over [pooled | cand | pieces] (model/din.py:56-95) — the
// two-launch path is rs_din_attention_ids_cand_fwd + rs_mlp_affine_pieces_fwd.
namespace rs {
// the shapes the fused launch takes (else the caller keeps the two launches);
// tbase / lds: where the tower's LDS region starts (floats) and the launch's
// dynamic LDS bytes
static bool din_tower_ok(const DinGeom& g, int n_layers, const int* dims, MlpGeom& mg, int& tbase, size_t& lds) {
  if (opt(RS_OPT_DIN_KERNEL) != 0 || g.HT1 != 5 || g.HT2 != 3 || !df_lds(g)) return false;
  if (!mlp_geom(n_layers, dims, mg) || dims[0] > 64 || dims[0] < 2 * g.k || mg.Np[0] != DF_NW * 16) return false;
  int gwa = 0, gwb = 0;
  if (!mlp_tail_ok(mg.Np, mg.Kp, mg.N, mg.L, 1, gwa, gwb) || gwa != 8 || gwb != 2) return false;
  // the tower's LDS (buf0 | buf1 | red | par) lies over the alpha / weight
  // images when it fits below the online-softmax partials the merge still
  // reads (config 4), else after everything (short histories)
  const DfLayout L = df_layout(g.NTT, g.HT1, g.HT2, g.KS);
  const int tfl = 32 * mg.rs + DF_NW * 256 + mg.ptot;
  tbase = tfl <= L.part ? 0 : L.total;
  lds = std::max(df_lds(g), (size_t)(tbase + tfl) * sizeof(float));
  return lds + 1024 + DF_SPW * (DF_TMAX + 2) * 8 <= 160 * 1024;
}

template <int KS, int KIND>
static void launch_din_tower(const DinArgs& a, const DinTower& tw, size_t lds, hipStream_t st) {
  const unsigned grid = (unsigned)((a.batch + DF_SPW - 1) / DF_SPW);
  if (KS == 2 && a.g.NTT == 7) {  // config 4 (k 8, T 97..112)
    static LdsAttr set7;
    lds_attr(set7, (const void*)din_fused_tower<KS, 5, 3, KIND, 7>, lds);
    din_fused_tower<KS, 5, 3, KIND, 7><<<grid, DF_NW * 64, lds, st>>>(a, tw);
    return;
  }
  static LdsAttr set;
  lds_attr(set, (const void*)din_fused_tower<KS, 5, 3, KIND>, lds);
  din_fused_tower<KS, 5, 3, KIND><<<grid, DF_NW * 64, lds, st>>>(a, tw);
}
}  // namespace rs

extern "C" int rs_din_forward_ids_supported(int T, int k, int H1, int H2, int n_layers, const int* dims) {
  if (rs_din_prepared_size(T, k, H1, H2) <= 0 || T > ATT_POOL_TMAX || !dims) return 0;
  MlpGeom mg;
  int tbase = 0;
  size_t lds = 0;
  return din_tower_ok(din_geom(T, k, H1, H2), n_layers, dims, mg, tbase, lds) ? 1 : 0;
}

extern "C" int rs_din_forward_ids(const void* hist, int id_kind, int64_t hist_stride, const void* cand,
                                  int64_t cand_stride, int T, int k, const float* table, int64_t vocab, int H1,
                                  int H2, const float* att_prepared, float* pooled, int64_t pooled_stride,
                                  const float* in_scale, const float* in_shift, int n_layers, const int* dims,
                                  const int* acts, const float* tower_prepared, float* y, int64_t y_stride,
                                  int n_pieces, const int* widths, const int* in_cols, const int* kinds,
                                  const void* const* srcs, const int64_t* src_strides, const float* const* tables,
                                  const int64_t* vocabs, int64_t batch, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(rs_din_prepared_size(T, k, H1, H2) > 0, "rs_din_forward_ids: need k in {4,8,16}, H1 <= 128, H2 <= 64");
  RS_REQUIRE(hist && cand && table && att_prepared && tower_prepared && y && acts && in_scale && in_shift &&
                 err_flag,
             "rs_din_forward_ids: null pointer");
  RS_REQUIRE(T <= ATT_POOL_TMAX && vocab < (1ll << 31), "rs_din_forward_ids: T > %d or vocab >= 2^31", ATT_POOL_TMAX);
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32 && vocab >= 1 && batch >= 0 && hist_stride >= T,
             "rs_din_forward_ids: bad ids / shape");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_din_forward_ids: table must be 16-B aligned");
  RS_REQUIRE(!pooled || pooled_stride >= k, "rs_din_forward_ids: pooled_stride < k");
  const DinGeom g = din_geom(T, k, H1, H2);
  MlpGeom mg;
  int tbase = 0;
  size_t lds = 0;
  RS_REQUIRE(n_layers >= 1 && dims && din_tower_ok(g, n_layers, dims, mg, tbase, lds),
             "rs_din_forward_ids: shape not supported by the fused launch (rs_din_forward_ids_supported)");
  RS_REQUIRE(dims[n_layers] == 1 && y_stride >= 1, "rs_din_forward_ids: the tower must end in one unit");
  DinTower tw{};
  int st = concat_fill(n_pieces, widths, in_cols, kinds, srcs, src_strides, tables, vocabs, dims[0],
                       "rs_din_forward_ids", tw.pc);
  if (st != RS_OK) return st;
  for (int p = 0; p < n_pieces; ++p)
    RS_REQUIRE(in_cols[p] >= 2 * k, "rs_din_forward_ids: piece %d overlaps the pooled / candidate columns", p);
  RS_REQUIRE(tw.pc.ncol == dims[0] - 2 * k, "rs_din_forward_ids: the pieces must cover columns 2k .. %d", dims[0] - 1);
  tw.pc.err = err_flag;
  tw.tbase = tbase;
  RS_REQUIRE(mlp_fill_args(mg, acts, tower_prepared, tw.t), "rs_din_forward_ids: bad activation");
  tw.t.y = y;
  tw.t.ys = y_stride;
  tw.t.head = 0;  // the output Dense(1, sigmoid) is the tower's last layer
  tw.t.c0 = 1.f;
  tw.t.c1 = 1.f;
  tw.t.M = batch;
  tw.t.dbg = mlp_diag_dbg();
  tw.t.in_scale = in_scale;
  tw.t.in_shift = in_shift;
  DinArgs a{hist, hist_stride, cand, cand_stride, table, vocab, att_prepared, g,
            0, nullptr, pooled, pooled_stride, batch, err_flag, g_din_dbg, nullptr, 0};
  hipStream_t hs = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KIND = decltype(K)::value;
    if (k == 4) launch_din_tower<1, KIND>(a, tw, lds, hs);
    else if (k == 8) launch_din_tower<2, KIND>(a, tw, lds, hs);
    else launch_din_tower<4, KIND>(a, tw, lds, hs);
  });
  return launch_status("rs_din_forward_ids");
}
