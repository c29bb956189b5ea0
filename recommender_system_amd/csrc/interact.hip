// interact.hip — the other interaction ops on the same per-field gather
// (SURVEY §8(f) rank 3): pair pooling (NFM bi-interaction, AFM), the pairwise
// product tensor (InteractionLayer) and the field-aware FM (FFMLayer).
//
// Reference semantics:
//   NFM bi-interaction   algorithm/deep_learning/model/nfm.py:26-29
//                        0.5 * ((sum_c e_c)^2 - sum_c e_c^2)  per dim, [B,k]
//   InteractionLayer     layer/interaction.py:280-297  [B,F,k] -> [B,P,k],
//                        pairs (i<j) row-major
//   AttentionLayer       layer/interaction.py:300-319: softmax over a size-1
//                        axis is exactly 1, so the pooled output is the SUM
//                        of the pair products (== the bi-interaction)
//   AFMLayer / AFM       layer/interaction.py:322-351, model/afm.py:11-19:
//                        'avg' mean / 'max' max / 'att' sum over pairs ->
//                        Dense(1) -> sigmoid -> (AFM) sigmoid again
//   FFMLayer / FFM       layer/interaction.py:117-163, model/ffm.py:14-23:
//                        field_f = x @ v ([B, NF, k], x = [dense | one-hot]),
//                        logit = w0 + x@w + sum_{f<g} <field_f, field_g>
//
// All three are gather-bound (HBM roofline, per-sample bytes in DESIGN.md).
#include "rs_common.hpp"

namespace rs {

constexpr int PMAXF = 32;  // fields held in registers for the 'max' pair pool

struct PoolArgs {
  const void* ids;
  int64_t id_stride;
  const float* table;  // one concatenated [sum V_c, k] table
  const int64_t* offs;
  const int64_t* vocab;
  int F, k;
  int mode;  // 0 sum (bi-interaction / AFM 'att'), 1 mean over pairs, 2 max over pairs
  const float* dense;  // optional: copied to out[:, 0:nd]
  int64_t dense_stride;
  int nd;
  float* out;  // optional: pooled -> out[b*out_stride + out_col + j]
  int64_t out_stride;
  int out_col;
  const float* head_w;  // optional head: y = pooled @ head_w + head_b, then n_sig sigmoids
  const float* head_b;
  int n_sig;
  float* head_out;
  int64_t batch;
  int* err;
};

// VW = 4: G = k/4 lanes per sample, lane l holds dims [4l, 4l+4) as one
// float4 (a wave-instruction reads 64/G whole rows); VW = 1: G = power of two
// >= k lanes, lane j = dim j.  Every field's id (and metadata) is loaded
// before any row, and all rows of a chunk of CH fields are in flight at once.
// 'max' keeps the FM field values in registers (F <= FM).
template <int VW>
struct Vec;
template <>
struct Vec<1> {
  typedef float T;
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T ld(const float* p) { return *p; }
  static __device__ __forceinline__ float hsum(T v) { return v; }
};
template <>
struct Vec<4> {
  typedef floatx4 T;
  static __device__ __forceinline__ T zero() { return floatx4{0.f, 0.f, 0.f, 0.f}; }
  static __device__ __forceinline__ T ld(const float* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
  }
  static __device__ __forceinline__ float hsum(T v) { return (v[0] + v[1]) + (v[2] + v[3]); }
};

__device__ __forceinline__ float vmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ floatx4 vmax(floatx4 a, floatx4 b) {
  return floatx4{fmaxf(a[0], b[0]), fmaxf(a[1], b[1]), fmaxf(a[2], b[2]), fmaxf(a[3], b[3])};
}

template <int G, int VW, int KIND, int FM>
__global__ __launch_bounds__(256) void pair_pool_kernel(PoolArgs a) {
  typedef Ids<KIND> I;
  typedef Vec<VW> V;
  typedef typename V::T T;
  constexpr int CH = FM > 0 ? FM : 32;
  const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int l = threadIdx.x & (G - 1);
  const bool valid = b < a.batch;
  const int64_t bb = valid ? b : a.batch - 1;
  const bool lane_ok = VW * l < a.k;
  const int jj = lane_ok ? VW * l : 0;  // first dim of this lane
  T s = V::zero(), q = V::zero(), mx = V::zero();
  bool bad = false;
  T e[FM > 0 ? FM : 1];
  for (int c0 = 0; c0 < a.F; c0 += CH) {
    int64_t row[CH];
    bool okc[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int c = c0 + u < a.F ? c0 + u : a.F - 1;
      int64_t id;
      okc[u] = I::decode(I::load(a.ids, bb * a.id_stride + c), a.vocab[c], id) && c0 + u < a.F;
      bad |= c0 + u < a.F && !okc[u];
      row[u] = a.offs[c] + id;
    }
    T v[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) v[u] = V::ld(a.table + row[u] * a.k + jj);
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const T x = okc[u] ? v[u] : V::zero();
      if constexpr (FM > 0) {
        e[u] = x;
      } else {
        s += x;
        q += x * x;
      }
    }
  }
  if constexpr (FM > 0) {
    // max over the pairs (c < d < F) of e_c * e_d, per dim
    bool first = true;
#pragma unroll
    for (int c = 0; c < FM; ++c)
#pragma unroll
      for (int d = c + 1; d < FM; ++d)
        if (d < a.F) {
          const T p = e[c] * e[d];
          mx = first ? p : vmax(mx, p);
          first = false;
        }
  }
  if (bad && valid && lane_ok) flag_error(a.err);
  T pooled;
  if constexpr (FM > 0) {
    pooled = a.F >= 2 ? mx : V::zero();
  } else {
    pooled = 0.5f * (s * s - q);
    if (a.mode == 1) pooled = a.F >= 2 ? pooled * (1.0f / (0.5f * (float)a.F * (float)(a.F - 1))) : V::zero();
  }
  if (valid && a.out) {
    float* o = a.out + b * a.out_stride;
    if (lane_ok) {
      if constexpr (VW == 4) {
        if (((a.out_col | (int)a.out_stride) & 3) == 0) {
          *reinterpret_cast<floatx4*>(o + a.out_col + jj) = pooled;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) o[a.out_col + jj + t] = pooled[t];
        }
      } else {
        o[a.out_col + jj] = pooled;
      }
    }
    for (int d = l; d < a.nd; d += G) o[d] = a.dense[b * a.dense_stride + d];
  }
  if (a.head_w) {
    float y = 0.f;
    if (lane_ok) {
      if constexpr (VW == 4) {
        const floatx4 w = *reinterpret_cast<const floatx4*>(a.head_w + jj);
        y = V::hsum(pooled * w);
      } else {
        y = pooled * a.head_w[jj];
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) y += __shfl_xor(y, o, G);
    y += a.head_b ? a.head_b[0] : 0.f;
    for (int t = 0; t < a.n_sig; ++t) y = sigmoidf_(y);
    if (valid && l == 0) a.head_out[b] = y;
  }
}

// Sum / mean pooling, k % 4 == 0: NWP waves per workgroup split the fields
// (wave w takes fields w, w+NWP, ...: its ids first, then all its rows in
// flight), each lane keeps float4 partials of sum e and sum e^2 for its 4
// dims, and wave 0 adds the NWP partials in wave order (LDS) and finishes.
// 64/G samples per workgroup (16 at k = 16 -> 256 workgroups at B = 4096).
template <int G, int KIND, int NWP>
__global__ __launch_bounds__(NWP * 64) void pair_pool_ksplit(PoolArgs a) {
  typedef Ids<KIND> I;
  constexpr int CH = (32 + NWP - 1) / NWP;  // fields per wave (one pass up to 32 fields)
  __shared__ floatx4 sp[NWP][64], qp[NWP][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * (64 / G) + lane / G;
  const int l = lane & (G - 1);
  const bool valid = b < a.batch;
  const int64_t bb = valid ? b : a.batch - 1;
  const bool lane_ok = 4 * l < a.k;
  const int jj = lane_ok ? 4 * l : 0;
  floatx4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
  bool bad = false;
  for (int c0 = w; c0 < a.F; c0 += NWP * CH) {
    int64_t row[CH];
    bool okc[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int cu = c0 + NWP * u;
      const int c = cu < a.F ? cu : a.F - 1;
      int64_t id;
      okc[u] = I::decode(I::load(a.ids, bb * a.id_stride + c), a.vocab[c], id) && cu < a.F;
      bad |= cu < a.F && !okc[u];
      row[u] = a.offs[c] + id;
    }
    floatx4 v[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u)
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + row[u] * a.k + jj));
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const floatx4 x = okc[u] ? v[u] : floatx4{0.f, 0.f, 0.f, 0.f};
      s += x;
      q += x * x;
    }
  }
  if (bad && valid && lane_ok) flag_error(a.err);
  sp[w][lane] = s;
  qp[w][lane] = q;
  __syncthreads();
  if (w != 0) return;
  s = sp[0][lane];
  q = qp[0][lane];
#pragma unroll
  for (int ww = 1; ww < NWP; ++ww) {
    s += sp[ww][lane];
    q += qp[ww][lane];
  }
  floatx4 pooled = 0.5f * (s * s - q);
  if (a.mode == 1) pooled = a.F >= 2 ? pooled * (1.0f / (0.5f * (float)a.F * (float)(a.F - 1))) : floatx4{0.f, 0.f, 0.f, 0.f};
  if (valid && a.out) {
    float* o = a.out + b * a.out_stride;
    if (lane_ok) {
      if (((a.out_col | (int)a.out_stride) & 3) == 0) {
        *reinterpret_cast<floatx4*>(o + a.out_col + jj) = pooled;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) o[a.out_col + jj + t] = pooled[t];
      }
    }
    for (int d = l; d < a.nd; d += G) o[d] = a.dense[b * a.dense_stride + d];
  }
  if (a.head_w) {
    float y = 0.f;
    if (lane_ok) {
      const floatx4 hw = *reinterpret_cast<const floatx4*>(a.head_w + jj);
      const floatx4 p = pooled * hw;
      y = (p[0] + p[1]) + (p[2] + p[3]);
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) y += __shfl_xor(y, o, G);
    y += a.head_b ? a.head_b[0] : 0.f;
    for (int t = 0; t < a.n_sig; ++t) y = sigmoidf_(y);
    if (valid && l == 0) a.head_out[b] = y;
  }
}

// InteractionLayer: out[b, p, j] = e[b, i_p, j] * e[b, j_p, j], pairs row-major.
__global__ __launch_bounds__(256) void pair_products_kernel(const float* __restrict__ e, int64_t e_stride, int F,
                                                            int k, int64_t batch, float* __restrict__ out) {
  const int P = F * (F - 1) / 2;
  const int64_t total = batch * P * k;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t b = idx / ((int64_t)P * k);
    const int r = (int)(idx - b * P * k);
    const int p = r / k, j = r - p * k;
    // closed-form row-major pair index: first i with cum(i+1) > p
    int i = 0, base = 0;
    while (base + (F - 1 - i) <= p) {
      base += F - 1 - i;
      ++i;
    }
    const int jf = i + 1 + (p - base);
    const float* eb = e + b * e_stride;
    out[idx] = eb[i * k + j] * eb[jf * k + j];
  }
}

// ------------------------------------------------------------------ FFM
// One wave per sample.  Element e = f*k + d of the field matrix [NF, k]
// (NF = nd + F fields) lives on lane e % 64 (slot e / 64); k divides 64, so a
// lane's elements share one latent dim d = lane % k.
//   field_f = sum_dense x_i V[i] + sum_c V[nd + off_c + id_c]    (one-hot x)
//   inter   = 0.5 * (sum_d (sum_f F[f,d])^2 - sum_{f,d} F[f,d]^2)
//   logit   = w0 + sum_i x_i w[i] + sum_c w[nd + off_c + id_c] + inter
struct FfmArgs {
  const void* ids;
  int64_t id_stride;
  const float* dense;
  int64_t dense_stride;
  int nd;
  const float* v;  // [feature_num, NF * k]
  const float* w;  // [feature_num]
  const float* w0;
  const int64_t* offs;  // one-hot offsets of the sparse fields (without nd)
  const int64_t* vocab;
  int F, k;
  int n_sig;
  float* out;
  int64_t batch;
  int* err;
};

template <int KIND, int NS>
__global__ __launch_bounds__(256) void ffm_kernel(FfmArgs a) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.batch) return;  // wave-uniform
  const int NF = a.nd + a.F;
  const int E = NF * a.k;
  float acc[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) acc[t] = 0.f;
  // sparse rows first (the HBM gathers), then the dense rows (L2-resident)
  float lin = 0.f;
  // every field's id and table row up front (lane c = field c, F <= 64), as
  // in ffm4_kernel; then CH fields per step with CH * NS row loads in flight
  int64_t frow = 0;
  bool fok = false;
  if (lane < a.F) {
    int64_t id;
    fok = I::decode(I::load(a.ids, b * a.id_stride + lane), a.vocab[lane], id);
    frow = a.nd + a.offs[lane] + id;
  }
  const bool bad = lane < a.F && !fok;
  const uint64_t okm = __ballot(fok);
  const int frow_lo = (int)(uint32_t)frow, frow_hi = (int)(uint32_t)((uint64_t)frow >> 32);
  constexpr int CH = NS >= 8 ? 4 : 8;
  for (int c0 = 0; c0 < a.F; c0 += CH) {
    int64_t row[CH];
    bool okc[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int c = c0 + u < a.F ? c0 + u : a.F - 1;  // wave-uniform
      okc[u] = ((okm >> c) & 1) && c0 + u < a.F;
      row[u] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(frow_hi, c) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane(frow_lo, c));
    }
    float x[CH][NS];
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const int e = lane + 64 * t;
        x[u][t] = e < E ? a.v[row[u] * E + e] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
#pragma unroll
      for (int t = 0; t < NS; ++t) acc[t] += okc[u] ? x[u][t] : 0.f;
      if (lane == c0 + u && okc[u]) lin += a.w[row[u]];
    }
  }
  for (int i = 0; i < a.nd; ++i) {
    const float x = a.dense[b * a.dense_stride + i];
    const float* r = a.v + (int64_t)i * E;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int e = lane + 64 * t;
      if (e < E) acc[t] = fmaf(x, r[e], acc[t]);
    }
    if (lane == i) lin = fmaf(x, a.w[i], lin);  // lanes < nd; the sparse w's above use lanes < F
  }
  if (__any(bad) && lane == 0) flag_error(a.err);
  float tsum = 0.f, q = 0.f;
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    tsum += acc[t];
    q = fmaf(acc[t], acc[t], q);
  }
  // T_d: sum over lanes with the same d = lane % k
  for (int o = a.k; o < 64; o <<= 1) tsum += __shfl_xor(tsum, o);
  float t2 = lane < a.k ? tsum * tsum : 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    t2 += __shfl_xor(t2, o);
    q += __shfl_xor(q, o);
    lin += __shfl_xor(lin, o);
  }
  float y = (a.w0[0] + lin) + 0.5f * (t2 - q);
  for (int t = 0; t < a.n_sig; ++t) y = sigmoidf_(y);
  if (lane == 0) a.out[b] = y;
}

// float4 form (k % 4 == 0, k/4 | 64): lane l, slot t holds elements
// 4(l + 64t) .. +3 of the field matrix; their latent dims are
// 4(l mod k/4) .. +3 for every t, so T_d reduces over lanes l' = l mod k/4.
// A 1,248-B row (k = 8) is 2 wave-instructions of 16-B loads instead of 5 of 4 B.
template <int KIND, int NS>
__global__ __launch_bounds__(256) void ffm4_kernel(FfmArgs a) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.batch) return;  // wave-uniform
  const int NF = a.nd + a.F;
  const int E4 = NF * a.k / 4;  // float4 per row
  const floatx4* v4 = reinterpret_cast<const floatx4*>(a.v);
  floatx4 acc[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  float lin = 0.f;
  // every field's id, validity and table row up front, lane c = field c (F <=
  // 64): one id trip for the sample instead of one per chunk of fields (the
  // chunks' row loads then wait on nothing but their own trip)
  int64_t frow = 0;
  bool fok = false;
  if (lane < a.F) {
    int64_t id;
    fok = I::decode(I::load(a.ids, b * a.id_stride + lane), a.vocab[lane], id);
    frow = a.nd + a.offs[lane] + id;
  }
  const bool bad = lane < a.F && !fok;
  const uint64_t okm = __ballot(fok);
  const int frow_lo = (int)(uint32_t)frow, frow_hi = (int)(uint32_t)((uint64_t)frow >> 32);
  constexpr int CH = NS >= 4 ? 4 : 8;  // 13 at NS = 2 ran 37 % slower (occupancy), 4 the same as 8
  for (int c0 = 0; c0 < a.F; c0 += CH) {
    int64_t row[CH];
    bool okc[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int c = c0 + u < a.F ? c0 + u : a.F - 1;  // wave-uniform
      okc[u] = ((okm >> c) & 1) && c0 + u < a.F;
      row[u] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(frow_hi, c) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane(frow_lo, c));
    }
    floatx4 x[CH][NS];
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const int e = lane + 64 * t;
        x[u][t] = e < E4 ? __builtin_nontemporal_load(v4 + row[u] * E4 + e) : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
#pragma unroll
      for (int t = 0; t < NS; ++t)
        if (okc[u]) acc[t] += x[u][t];
      if (lane == c0 + u && okc[u]) lin += a.w[row[u]];
    }
  }
  for (int i = 0; i < a.nd; ++i) {
    const float xi = a.dense[b * a.dense_stride + i];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int e = lane + 64 * t;
      if (e < E4) acc[t] += xi * v4[(int64_t)i * E4 + e];
    }
    if (lane == i) lin = fmaf(xi, a.w[i], lin);
  }
  if (__any(bad) && lane == 0) flag_error(a.err);
  floatx4 ts = floatx4{0.f, 0.f, 0.f, 0.f};
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    ts += acc[t];
    q += acc[t][0] * acc[t][0] + acc[t][1] * acc[t][1] + acc[t][2] * acc[t][2] + acc[t][3] * acc[t][3];
  }
  const int KQ = a.k / 4;
  for (int o = KQ; o < 64; o <<= 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) ts[c] += __shfl_xor(ts[c], o);
  float t2 = lane < KQ ? ts[0] * ts[0] + ts[1] * ts[1] + ts[2] * ts[2] + ts[3] * ts[3] : 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    t2 += __shfl_xor(t2, o);
    q += __shfl_xor(q, o);
    lin += __shfl_xor(lin, o);
  }
  float y = (a.w0[0] + lin) + 0.5f * (t2 - q);
  for (int t = 0; t < a.n_sig; ++t) y = sigmoidf_(y);
  if (lane == 0) a.out[b] = y;
}

template <int KIND>
static void launch_ffm4(const FfmArgs& a, int ns, hipStream_t st) {
  const unsigned grid = (unsigned)((a.batch + 3) / 4);
  switch (ns) {
    case 1: ffm4_kernel<KIND, 1><<<grid, 256, 0, st>>>(a); break;
    case 2: ffm4_kernel<KIND, 2><<<grid, 256, 0, st>>>(a); break;
    default: ffm4_kernel<KIND, 4><<<grid, 256, 0, st>>>(a); break;
  }
}

template <int KIND>
static void launch_ffm(const FfmArgs& a, int ns, hipStream_t st) {
  const unsigned grid = (unsigned)((a.batch + 3) / 4);
  switch (ns) {
    case 1: ffm_kernel<KIND, 1><<<grid, 256, 0, st>>>(a); break;
    case 2: ffm_kernel<KIND, 2><<<grid, 256, 0, st>>>(a); break;
    case 4: ffm_kernel<KIND, 4><<<grid, 256, 0, st>>>(a); break;
    case 8: ffm_kernel<KIND, 8><<<grid, 256, 0, st>>>(a); break;
    default: ffm_kernel<KIND, 16><<<grid, 256, 0, st>>>(a); break;
  }
}

}  // namespace rs

using namespace rs;

extern "C" int rs_embed_pair_pool_fwd(const void* ids, int id_kind, int64_t id_stride, const float* table,
                                      const int64_t* field_offsets, const int64_t* field_vocab, int n_fields, int k,
                                      int mode, const float* dense, int64_t dense_stride, int nd, float* out,
                                      int64_t out_stride, int out_col, const float* head_w, const float* head_b,
                                      int n_sigmoid, float* head_out, int64_t batch, int* err_flag,
                                      rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch
  RS_REQUIRE(batch > 0 && n_fields >= 1 && k >= 1 && k <= 64 && mode >= 0 && mode <= 2 && nd >= 0 && n_sigmoid >= 0,
             "rs_embed_pair_pool_fwd: bad shape (1 <= k <= 64, mode 0..2)");
  RS_REQUIRE(mode != 2 || n_fields <= PMAXF, "rs_embed_pair_pool_fwd: 'max' pooling supports at most %d fields",
             PMAXF);
  RS_REQUIRE(ids && table && field_offsets && field_vocab, "rs_embed_pair_pool_fwd: null pointer");
  RS_REQUIRE(out || head_out, "rs_embed_pair_pool_fwd: no output requested");
  RS_REQUIRE(!out || (out_col >= 0 && out_col + k <= out_stride && nd <= out_stride && (nd == 0 || dense)),
             "rs_embed_pair_pool_fwd: bad output layout");
  RS_REQUIRE(!head_out || head_w, "rs_embed_pair_pool_fwd: head_out needs head_w");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_pair_pool_fwd: bad id_kind");
  PoolArgs a{ids, id_stride, table, field_offsets, field_vocab, n_fields, k, mode, dense, dense_stride,
             out ? nd : 0, out, out_stride, out_col, head_out ? head_w : nullptr, head_b, n_sigmoid, head_out,
             batch, err_flag};
  const bool v4 = k % 4 == 0 && (uintptr_t)table % 16 == 0 && (!head_w || (uintptr_t)head_w % 16 == 0);
  int G = 1;
  while (G * (v4 ? 4 : 1) < k) G <<= 1;
  // one wave per workgroup on the float4 path (16 samples per wave at k = 16):
  // B = 4096 spreads over 256 workgroups, every CU's rows in flight at once
  const int nth = v4 ? 64 : 256;
  const unsigned grid = (unsigned)((batch * G + nth - 1) / nth);
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KD = decltype(K)::value;
    auto go = [&](auto FMc) {
      constexpr int FM = decltype(FMc)::value;
      if (v4) {
        switch (G) {
          case 1: pair_pool_kernel<1, 4, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 2: pair_pool_kernel<2, 4, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 4: pair_pool_kernel<4, 4, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 8: pair_pool_kernel<8, 4, KD, FM><<<grid, nth, 0, st>>>(a); break;
          default: pair_pool_kernel<16, 4, KD, FM><<<grid, nth, 0, st>>>(a); break;
        }
      } else {
        switch (G) {
          case 1: pair_pool_kernel<1, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 2: pair_pool_kernel<2, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 4: pair_pool_kernel<4, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 8: pair_pool_kernel<8, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 16: pair_pool_kernel<16, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
          case 32: pair_pool_kernel<32, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
          default: pair_pool_kernel<64, 1, KD, FM><<<grid, nth, 0, st>>>(a); break;
        }
      }
    };
    if (mode != 2 && v4) {
      const unsigned g2 = (unsigned)((batch + 64 / G - 1) / (64 / G));
      // 8 waves per workgroup (<= 4 fields each at F = 26): 6.3-6.4 us at
      // B = 4096 against 6.7 with 4 waves and 6.6 with 16
      constexpr int NWP = 8;
      switch (G) {
        case 1: pair_pool_ksplit<1, KD, NWP><<<g2, NWP * 64, 0, st>>>(a); break;
        case 2: pair_pool_ksplit<2, KD, NWP><<<g2, NWP * 64, 0, st>>>(a); break;
        case 4: pair_pool_ksplit<4, KD, NWP><<<g2, NWP * 64, 0, st>>>(a); break;
        case 8: pair_pool_ksplit<8, KD, NWP><<<g2, NWP * 64, 0, st>>>(a); break;
        default: pair_pool_ksplit<16, KD, NWP><<<g2, NWP * 64, 0, st>>>(a); break;
      }
    } else if (mode != 2) {
      go(std::integral_constant<int, 0>());
    } else {
      go(std::integral_constant<int, PMAXF>());
    }
  });
  return launch_status("rs_embed_pair_pool_fwd");
}

extern "C" int rs_pair_products_fwd(const float* e, int64_t e_stride, int n_fields, int k, int64_t batch,
                                    float* out, rs_stream_t stream) {
  if (batch == 0 || n_fields < 2) return RS_OK;  // nothing to compute (P = 0)
  RS_REQUIRE(e && out && k >= 1 && batch > 0 && e_stride >= (int64_t)n_fields * k,
             "rs_pair_products_fwd: bad arguments");
  const int64_t total = batch * (int64_t)(n_fields * (n_fields - 1) / 2) * k;
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  pair_products_kernel<<<(unsigned)g, 256, 0, as_stream(stream)>>>(e, e_stride, n_fields, k, batch, out);
  return launch_status("rs_pair_products_fwd");
}

extern "C" int rs_ffm_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense, int64_t dense_stride,
                          int nd, const float* v, const float* w, const float* w0, const int64_t* field_offsets,
                          const int64_t* field_vocab, int n_fields, int k, int n_sigmoid, float* out, int64_t batch,
                          int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch
  RS_REQUIRE(batch > 0 && nd >= 0 && n_fields >= 0 && k >= 1 && 64 % k == 0 && n_sigmoid >= 0,
             "rs_ffm_fwd: bad shape (k must divide 64)");
  RS_REQUIRE(nd <= 64 && n_fields <= 64, "rs_ffm_fwd: at most 64 dense and 64 sparse fields");
  const int E = (nd + n_fields) * k;
  RS_REQUIRE(E >= 1 && E <= 16 * 64, "rs_ffm_fwd: field matrix (nd + n_fields) * k must be <= 1024");
  RS_REQUIRE(v && w && w0 && out && (nd == 0 || dense) && (n_fields == 0 || (ids && field_offsets && field_vocab)),
             "rs_ffm_fwd: null pointer");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_ffm_fwd: bad id_kind");
  FfmArgs a{ids, id_stride, dense, dense_stride, nd, v, w, w0, field_offsets, field_vocab, n_fields, k, n_sigmoid,
            out, batch, err_flag};
  hipStream_t st = as_stream(stream);
  if (k % 4 == 0 && (uintptr_t)v % 16 == 0) {  // (k | 64 already checked: k/4 | 64)
    const int s4 = (E / 4 + 63) / 64;          // <= 4
    const int ns = s4 <= 1 ? 1 : s4 <= 2 ? 2 : 4;
    with_id_kind(id_kind, [&](auto K) { launch_ffm4<decltype(K)::value>(a, ns, st); });
  } else {
    const int slots = (E + 63) / 64;
    const int ns = slots <= 1 ? 1 : slots <= 2 ? 2 : slots <= 4 ? 4 : slots <= 8 ? 8 : 16;
    with_id_kind(id_kind, [&](auto K) { launch_ffm<decltype(K)::value>(a, ns, st); });
  }
  return launch_status("rs_ffm_fwd");
}

// AttentionLayer on a [B, P, k] input (layer/interaction.py:310-319): the
// softmax runs over an axis of size 1, so every score is exactly 1 and the
// output is the plain sum over the P rows.  One thread per (b, j), rows
// summed in order.
namespace rs {
__global__ __launch_bounds__(256) void sum_rows_kernel(const float* __restrict__ x, int64_t x_stride, int P, int k,
                                                       int64_t batch, float* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= batch * k) return;
  const int64_t b = idx / k;
  const int j = (int)(idx - b * k);
  const float* xb = x + b * x_stride + j;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += xb[(int64_t)p * k];
  out[idx] = s;
}
}  // namespace rs

extern "C" int rs_attention_pool_fwd(const float* x, int64_t x_stride, int n_rows, int k, int64_t batch, float* out,
                                     rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(x && out && n_rows >= 0 && k >= 1 && batch > 0 && x_stride >= (int64_t)n_rows * k,
             "rs_attention_pool_fwd: bad arguments");
  sum_rows_kernel<<<(unsigned)((batch * k + 255) / 256), 256, 0, as_stream(stream)>>>(x, x_stride, n_rows, k, batch,
                                                                                       out);
  return launch_status("rs_attention_pool_fwd");
}
