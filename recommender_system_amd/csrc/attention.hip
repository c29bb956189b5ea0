// attention.hip — DIN attention unit (Attention, layer/interaction.py:355-406)
// and its Dice variant (Dice, layer/interaction.py:410-425).
//
// 'prelu' mode, per sample b and behaviour position t:
//   e_t = [q, key_t, q-key_t, q*key_t]                      (4k, :381-391)
//   h1  = PReLU_{alpha1[t]}(e_t W1 + b1)                     (:366,393-394)
//   h2  = PReLU_{alpha2[t]}(h1 W2 + b2)
//   s_t = h2 w3 + b3; s_t = -4294967296 where mask==0        (:396-401)
//   out = softmax_t(s) @ value                               (:403-405)
//
// MI355X mapping: one wave owns one sample; positions go 16 at a time through
// v_mfma_f32_16x16x4_f32 in the "swapped" orientation (C^T = W^T e^T), so the
// accumulator of layer 1 (lane = position t, registers = 4 hidden units) is
// directly the B operand of layer 2 with the k order permuted to match the
// registers (no LDS round trip between layers).  W1^T / W2^T live in LDS as
// per-lane operand images (one conflict-free ds_read_b32 per MFMA), staged
// once per workgroup; alpha1/alpha2 (shape [T,H], Keras PReLU on 3-D input)
// are read as float4 per lane from L2.  Scores for all T positions stay in
// LDS; the masked softmax and the weighted sum over value rows finish in the
// same wave.
#include "rs_common.hpp"

namespace rs {

constexpr int ATT_WAVES = 4;
constexpr int ATT_TMAX = 1024;

struct AttArgs {
  const float* q;
  const float* keys;
  const float* values;
  const float* mask;
  int T, k;
  const float* W1;
  const float* b1;
  const float* alpha1;
  int H1;
  const float* W2;
  const float* b2;
  const float* alpha2;
  int H2;
  const float* w3;
  const float* b3;
  float* out;
  int64_t batch;
  int HT1, HT2;
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// masked softmax over sc[0..T) and out[b] = sum_t a_t * value[b,t,:]
__device__ __forceinline__ void softmax_weighted_sum(float* sc, int T, int k, const float* values, int64_t b,
                                                     float* out, int lane) {
  wave_lds_sync();
  float mx = -INFINITY;
  for (int t = lane; t < T; t += 64) mx = fmaxf(mx, sc[t]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float sum = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float e = expf(sc[t] - mx);
    sc[t] = e;
    sum += e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  wave_lds_sync();
  // lanes = (tg, j): j = lane % k, tg = lane / k
  const int ntg = 64 / k;
  const int j = lane % k, tg = lane / k;
  float acc = 0.f;
  const float* vb = values + b * (int64_t)T * k;
  if (tg < ntg)
    for (int t = tg; t < T; t += ntg) acc = fmaf(sc[t] / sum, vb[(int64_t)t * k + j], acc);
  float tot = 0.f;
  for (int u = 0; u < ntg; ++u) tot += __shfl(acc, u * k + j);
  if (lane < k) out[b * k + lane] = tot;
  wave_lds_sync();
}

template <int KQ, int HT1M, int HT2M>
__global__ __launch_bounds__(ATT_WAVES * 64) void din_attention_mfma(AttArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int K = 4 * KQ;     // embedding dim
  constexpr int KS1 = 4 * KQ;   // layer-1 k-steps (4k / 4)
  const int HT1 = a.HT1, HT2 = a.HT2;
  float* w1img = smem;                                   // [HT1][KS1][64]
  float* w2img = w1img + HT1 * KS1 * 64;                 // [HT2][HT1][4][64]
  float* scores = w2img + HT2 * HT1 * 4 * 64;            // [ATT_WAVES][ATT_TMAX]

  // stage operand images (A operand: lane = (row i = l&15, k-slot kk = l>>4))
  for (int idx = threadIdx.x; idx < HT1 * KS1 * 64; idx += blockDim.x) {
    const int lane = idx & 63, st = idx >> 6;
    const int s = st % KS1, ht = st / KS1;
    const int h = 16 * ht + (lane & 15), kk = lane >> 4;
    const int sigma = s / KQ, m = s % KQ, j = kk * KQ + m;
    const int kin = sigma * K + j;
    w1img[idx] = h < a.H1 ? a.W1[(int64_t)kin * a.H1 + h] : 0.f;
  }
  for (int idx = threadIdx.x; idx < HT2 * HT1 * 4 * 64; idx += blockDim.x) {
    const int lane = idx & 63, st = idx >> 6;
    const int r = st & 3, ht = (st >> 2) % HT1, ht2 = (st >> 2) / HT1;
    const int h2 = 16 * ht2 + (lane & 15), h1 = 16 * ht + 4 * (lane >> 4) + r;
    w2img[idx] = (h2 < a.H2 && h1 < a.H1) ? a.W2[(int64_t)h1 * a.H2 + h2] : 0.f;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15;  // position within the 16-position tile
  const int g = lane >> 4;    // k-slot / accumulator row group
  float* sc = scores + w * ATT_TMAX;

  // per-lane constants: biases and w3 for the lane's accumulator rows
  float bias1[HT1M][4], bias2[HT2M][4], w3v[HT2M][4];
#pragma unroll
  for (int ht = 0; ht < HT1M; ++ht)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * ht + 4 * g + r;
      bias1[ht][r] = (ht < HT1 && h < a.H1) ? a.b1[h] : 0.f;
    }
#pragma unroll
  for (int ht = 0; ht < HT2M; ++ht)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * ht + 4 * g + r;
      const bool ok = ht < HT2 && h < a.H2;
      bias2[ht][r] = ok ? a.b2[h] : 0.f;
      w3v[ht][r] = ok ? a.w3[h] : 0.f;
    }
  const float b3 = a.b3[0];
  const bool a1vec = (a.H1 % 4) == 0, a2vec = (a.H2 % 4) == 0;

  for (int64_t b = (int64_t)blockIdx.x * ATT_WAVES + w; b < a.batch; b += (int64_t)gridDim.x * ATT_WAVES) {
    float qc[KQ];
#pragma unroll
    for (int m = 0; m < KQ; ++m) qc[m] = a.q[b * K + g * KQ + m];
    const float* kb = a.keys + b * (int64_t)a.T * K;
    for (int t0 = 0; t0 < a.T; t0 += 16) {
      const int t = t0 + col;
      const bool tv = t < a.T;
      float kc[KQ];
#pragma unroll
      for (int m = 0; m < KQ; ++m) kc[m] = tv ? kb[(int64_t)t * K + g * KQ + m] : 0.f;
      float bf[KS1];
#pragma unroll
      for (int s = 0; s < KS1; ++s) {
        const int sigma = s / KQ, m = s % KQ;
        bf[s] = sigma == 0 ? qc[m] : sigma == 1 ? kc[m] : sigma == 2 ? qc[m] - kc[m] : qc[m] * kc[m];
      }
      // layer 1: C1^T[h][t], lane holds h = 16ht + 4g + r
      float y1[HT1M][4];
#pragma unroll
      for (int ht = 0; ht < HT1M; ++ht) {
        if (ht < HT1) {
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
          const float* wi = w1img + ht * KS1 * 64 + lane;
#pragma unroll
          for (int s = 0; s < KS1; ++s) acc = mfma16x16x4(wi[s * 64], bf[s], acc);
          float al[4] = {0.f, 0.f, 0.f, 0.f};
          const int h0 = 16 * ht + 4 * g;
          if (tv) {
            const float* ap = a.alpha1 + (int64_t)t * a.H1 + h0;
            if (a1vec && h0 + 3 < a.H1) {
              const floatx4 v = *reinterpret_cast<const floatx4*>(ap);
              al[0] = v[0]; al[1] = v[1]; al[2] = v[2]; al[3] = v[3];
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) al[r] = (h0 + r < a.H1) ? ap[r] : 0.f;
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = acc[r] + bias1[ht][r];
            y1[ht][r] = fmaxf(x, 0.f) + al[r] * fminf(x, 0.f);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) y1[ht][r] = 0.f;
        }
      }
      // layer 2 (B operand = layer-1 accumulators, k index h1 = 16ht + 4kk + r)
      float part = 0.f;
#pragma unroll
      for (int ht2 = 0; ht2 < HT2M; ++ht2) {
        if (ht2 < HT2) {
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ht = 0; ht < HT1M; ++ht) {
            if (ht < HT1) {
              const float* wi = w2img + ((ht2 * HT1 + ht) * 4) * 64 + lane;
#pragma unroll
              for (int r = 0; r < 4; ++r) acc = mfma16x16x4(wi[r * 64], y1[ht][r], acc);
            }
          }
          float al[4] = {0.f, 0.f, 0.f, 0.f};
          const int h0 = 16 * ht2 + 4 * g;
          if (tv) {
            const float* ap = a.alpha2 + (int64_t)t * a.H2 + h0;
            if (a2vec && h0 + 3 < a.H2) {
              const floatx4 v = *reinterpret_cast<const floatx4*>(ap);
              al[0] = v[0]; al[1] = v[1]; al[2] = v[2]; al[3] = v[3];
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) al[r] = (h0 + r < a.H2) ? ap[r] : 0.f;
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = acc[r] + bias2[ht2][r];
            const float y = fmaxf(x, 0.f) + al[r] * fminf(x, 0.f);
            part = fmaf(y, w3v[ht2][r], part);
          }
        }
      }
      part += __shfl_xor(part, 16);
      part += __shfl_xor(part, 32);
      if (g == 0 && tv) {
        float s = part + b3;
        if (a.mask[b * a.T + t] == 0.f) s = -4294967296.0f;
        sc[t] = s;
      }
    }
    softmax_weighted_sum(sc, a.T, K, a.values, b, a.out, lane);
  }
}

// Dice mode: no Dense in the activation stack; every Dice is per-channel, so
// each lane walks its position's 4k channels through the n_dice Dice layers
// and accumulates the Dense(1) score directly.
struct DiceArgs {
  const float* q;
  const float* keys;
  const float* values;
  const float* mask;
  int T, k, n_dice;
  const float* alpha;
  const float* mean;
  const float* var;
  float eps;
  const float* w_out;
  const float* b_out;
  float* out;
  int64_t batch;
};

__global__ __launch_bounds__(ATT_WAVES * 64) void din_attention_dice(DiceArgs a) {
  __shared__ float scores[ATT_WAVES][ATT_TMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* sc = scores[w];
  const int K = a.k, C = 4 * a.k;
  for (int64_t b = (int64_t)blockIdx.x * ATT_WAVES + w; b < a.batch; b += (int64_t)gridDim.x * ATT_WAVES) {
    const float* qb = a.q + b * K;
    const float* kb = a.keys + b * (int64_t)a.T * K;
    for (int t = lane; t < a.T; t += 64) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) {
        const int sigma = c / K, j = c % K;
        const float qv = qb[j], kv = kb[(int64_t)t * K + j];
        float x = sigma == 0 ? qv : sigma == 1 ? kv : sigma == 2 ? qv - kv : qv * kv;
        for (int l = 0; l < a.n_dice; ++l) {
          const int o = l * C + c;
          const float xn = (x - a.mean[o]) / sqrtf(a.var[o] + a.eps);
          const float p = 1.0f / (1.0f + expf(-xn));
          x = a.alpha[o] * (1.0f - p) * x + p * x;
        }
        s = fmaf(x, a.w_out[c], s);
      }
      s += a.b_out[0];
      if (a.mask[b * a.T + t] == 0.f) s = -4294967296.0f;
      sc[t] = s;
    }
    softmax_weighted_sum(sc, a.T, K, a.values, b, a.out, lane);
  }
}

// Generic-depth 'prelu' path (any len(hidden_units), any H, k <= 64): the
// activation-unit input e = [q, key_t, q-key_t, q*key_t] is formed once per
// (b, t) row, every Dense(h, PReLU()) runs as an fp32 MFMA GEMM over the B*T
// rows (rs_dense_prelu_rows_fwd: alpha [T, h] indexed by row mod T), the
// Dense(1) score as the small-N GEMM, then the masked softmax + weighted sum.
__global__ void att_concat_kernel(const float* __restrict__ q, const float* __restrict__ keys, int T, int k,
                                  int64_t n, float* __restrict__ e) {
  // n = B*T*k elements (b, t, j)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bt = i / k;
    const int j = (int)(i - bt * k);
    const int64_t b = bt / T;
    const float qv = q[b * k + j], kv = keys[i];
    float* row = e + bt * 4 * k;
    row[j] = qv;
    row[k + j] = kv;
    row[2 * k + j] = qv - kv;
    row[3 * k + j] = qv * kv;
  }
}

__global__ __launch_bounds__(ATT_WAVES * 64) void att_masked_pool(const float* __restrict__ scores,
                                                                  const float* __restrict__ mask,
                                                                  const float* __restrict__ values, int T, int k,
                                                                  float* __restrict__ out, int64_t batch) {
  __shared__ float sbuf[ATT_WAVES][ATT_TMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* sc = sbuf[w];
  for (int64_t b = (int64_t)blockIdx.x * ATT_WAVES + w; b < batch; b += (int64_t)gridDim.x * ATT_WAVES) {
    for (int t = lane; t < T; t += 64) {
      const float sv = scores[b * T + t];
      sc[t] = mask[b * T + t] == 0.f ? -4294967296.0f : sv;
    }
    if (k <= 64) {
      softmax_weighted_sum(sc, T, k, values, b, out, lane);
      continue;
    }
    wave_lds_sync();
    float mx = -INFINITY;
    for (int t = lane; t < T; t += 64) mx = fmaxf(mx, sc[t]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float ev = expf(sc[t] - mx);
      sc[t] = ev;
      sum += ev;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    wave_lds_sync();
    const float* vb = values + b * (int64_t)T * k;
    for (int j = lane; j < k; j += 64) {
      float acc = 0.f;
      for (int t = 0; t < T; ++t) acc = fmaf(sc[t] / sum, vb[(int64_t)t * k + j], acc);
      out[b * k + j] = acc;
    }
    wave_lds_sync();
  }
}

static unsigned att_grid(int64_t batch) {
  int64_t g = (batch + ATT_WAVES - 1) / ATT_WAVES;
  if (g > 4096) g = 4096;
  return (unsigned)(g < 1 ? 1 : g);
}

template <int KQ, int HT1M, int HT2M>
static int launch_att(const AttArgs& a, hipStream_t st) {
  const size_t lds = (size_t)(a.HT1 * 4 * KQ * 64 + a.HT2 * a.HT1 * 4 * 64 + ATT_WAVES * ATT_TMAX) * sizeof(float);
  auto fn = din_attention_mfma<KQ, HT1M, HT2M>;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  fn<<<att_grid(a.batch), ATT_WAVES * 64, lds, st>>>(a);
  return launch_status("rs_din_attention_fwd");
}

template <int KQ>
static int launch_att_kq(const AttArgs& a, hipStream_t st) {
  if (a.HT1 <= 5 && a.HT2 <= 3) return launch_att<KQ, 5, 3>(a, st);
  return launch_att<KQ, 8, 8>(a, st);
}

}  // namespace rs

using namespace rs;

extern "C" int rs_din_attention_fwd(const float* query, const float* keys, const float* values, const float* mask,
                                    int T, int k, const float* W1, const float* b1, const float* alpha1, int H1,
                                    const float* W2, const float* b2, const float* alpha2, int H2, const float* w3,
                                    const float* b3, float* out, int64_t batch, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(query && keys && values && mask && W1 && b1 && alpha1 && W2 && b2 && alpha2 && w3 && b3 && out,
             "rs_din_attention_fwd: null pointer");
  RS_REQUIRE(T >= 1 && T <= ATT_TMAX && batch >= 0, "rs_din_attention_fwd: need 1 <= T <= %d", ATT_TMAX);
  RS_REQUIRE(k == 4 || k == 8 || k == 16 || k == 32, "rs_din_attention_fwd: k must be 4, 8, 16 or 32");
  RS_REQUIRE(H1 >= 1 && H1 <= 128 && H2 >= 1 && H2 <= 128, "rs_din_attention_fwd: hidden sizes must be <= 128");
  if (batch == 0) return RS_OK;
  AttArgs a{query, keys, values, mask, T, k, W1, b1, alpha1, H1, W2, b2, alpha2, H2, w3, b3, out, batch,
            (H1 + 15) / 16, (H2 + 15) / 16};
  hipStream_t st = as_stream(stream);
  switch (k) {
    case 4: return launch_att_kq<1>(a, st);
    case 8: return launch_att_kq<2>(a, st);
    case 16: return launch_att_kq<4>(a, st);
    default: return launch_att_kq<8>(a, st);
  }
}

extern "C" int rs_din_attention_dice_fwd(const float* query, const float* keys, const float* values,
                                         const float* mask, int T, int k, int n_dice, const float* dice_alpha,
                                         const float* dice_mean, const float* dice_var, float dice_eps,
                                         const float* w_out, const float* b_out, float* out, int64_t batch,
                                         rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(query && keys && values && mask && w_out && b_out && out, "rs_din_attention_dice_fwd: null pointer");
  RS_REQUIRE(n_dice == 0 || (dice_alpha && dice_mean && dice_var), "rs_din_attention_dice_fwd: null Dice params");
  RS_REQUIRE(T >= 1 && T <= ATT_TMAX && k >= 1 && k <= 64 && n_dice >= 0 && batch >= 0,
             "rs_din_attention_dice_fwd: bad shape");
  if (batch == 0) return RS_OK;
  DiceArgs a{query, keys, values, mask, T, k, n_dice, dice_alpha, dice_mean, dice_var, dice_eps, w_out, b_out, out,
             batch};
  din_attention_dice<<<att_grid(batch), ATT_WAVES * 64, 0, as_stream(stream)>>>(a);
  return launch_status("rs_din_attention_dice_fwd");
}

static int64_t att_gen_max_width(int k, int n_layers, const int* hidden) {
  int64_t mx = 1;
  for (int l = 0; l < n_layers; ++l) mx = hidden[l] > mx ? hidden[l] : mx;
  (void)k;
  return mx;
}

extern "C" int64_t rs_din_attention_gen_workspace_size(int64_t batch, int T, int k, int n_layers,
                                                       const int* hidden) {
  if (batch < 0 || T < 1 || k < 1 || n_layers < 0 || (n_layers > 0 && !hidden)) return -1;
  for (int l = 0; l < n_layers; ++l)
    if (hidden[l] < 1) return -1;
  const int64_t rows = batch * T;
  const int64_t h = att_gen_max_width(k, n_layers, hidden);
  // e [rows, 4k] | ping / pong [rows, h] | scores [rows], each 256-B aligned
  auto al = [](int64_t floats) { return (floats * 4 + 255) / 256 * 256; };
  return al(rows * 4 * k) + 2 * al(rows * h) + al(rows);
}

extern "C" int rs_din_attention_gen_fwd(const float* query, const float* keys, const float* values,
                                        const float* mask, int T, int k, int n_layers, const int* hidden,
                                        const float* const* W, const float* const* b, const float* const* alpha,
                                        const float* w_out, const float* b_out, float* out, int64_t batch,
                                        void* workspace, int64_t workspace_bytes, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(query && keys && values && mask && w_out && b_out && out && workspace,
             "rs_din_attention_gen_fwd: null pointer");
  RS_REQUIRE(T >= 1 && T <= ATT_TMAX && k >= 1 && n_layers >= 0 && batch > 0,
             "rs_din_attention_gen_fwd: bad shape (1 <= T <= %d)", ATT_TMAX);
  RS_REQUIRE(n_layers == 0 || (hidden && W && b && alpha), "rs_din_attention_gen_fwd: null layer arrays");
  for (int l = 0; l < n_layers; ++l)
    RS_REQUIRE(hidden[l] >= 1 && W[l] && b[l] && alpha[l], "rs_din_attention_gen_fwd: bad layer %d", l);
  const int64_t need = rs_din_attention_gen_workspace_size(batch, T, k, n_layers, hidden);
  RS_REQUIRE(workspace_bytes >= need, "rs_din_attention_gen_fwd: workspace needs %lld bytes", (long long)need);
  hipStream_t st = as_stream(stream);
  const int64_t rows = batch * T;
  const int64_t h = att_gen_max_width(k, n_layers, hidden);
  auto al = [](int64_t floats) { return (floats * 4 + 255) / 256 * 256; };
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  float* e = reinterpret_cast<float*>(ws);
  float* buf[2] = {reinterpret_cast<float*>(ws + al(rows * 4 * k)),
                   reinterpret_cast<float*>(ws + al(rows * 4 * k) + al(rows * h))};
  float* scores = reinterpret_cast<float*>(ws + al(rows * 4 * k) + 2 * al(rows * h));
  const int64_t n = rows * k;
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  att_concat_kernel<<<(unsigned)g, 256, 0, st>>>(query, keys, T, k, n, e);
  if (hipPeekAtLastError() != hipSuccess) return launch_status("rs_din_attention_gen_fwd");
  const float* in = e;
  int kin = 4 * k;
  for (int l = 0; l < n_layers; ++l) {
    const int rc = rs_dense_prelu_rows_fwd(in, kin, W[l], b[l], alpha[l], T, buf[l & 1], hidden[l], rows, kin,
                                           hidden[l], stream);
    if (rc != RS_OK) return rc;
    in = buf[l & 1];
    kin = hidden[l];
  }
  const int rc = rs_dense_fwd(in, kin, w_out, b_out, nullptr, RS_ACT_NONE, scores, 1, rows, kin, 1, stream);
  if (rc != RS_OK) return rc;
  att_masked_pool<<<att_grid(batch), ATT_WAVES * 64, 0, st>>>(scores, mask, values, T, k, out, batch);
  return launch_status("rs_din_attention_gen_fwd");
}
