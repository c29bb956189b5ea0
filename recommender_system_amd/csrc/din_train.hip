// din_train.hip — DIN training kernels (compile_fit on DIN: utils/compile_fit.py:9-15,
// model/din.py:56-95 with training=True).
//
// DIN.train_step composes these with rs_dense_fwd / rs_gemm / rs_col_sum /
// rs_sgd_update / rs_embedding_sgd:
//   rs_din_att_concat[_bwd]   the attention unit's input [q, k, q-k, q*k]
//                             (layer/interaction.py:381-391) and its backward
//   rs_prelu_rows_fwd / _bwd  Keras PReLU with alpha[(row mod period), col]
//                             (the attention's [T, h] alphas: period T; the
//                             DNN's [units]: period 1); dalpha by a fixed-
//                             order sum over the rows of each alpha
//   rs_masked_softmax_pool[_bwd]  score masking (-2^32+1 where the first
//                             behaviour id is 0), softmax over T, the weighted
//                             sum of the values (:396-404) and its backward
//   rs_bn_train_stats / _apply / _bwd  BatchNormalization in training mode
//                             (batch mean / biased variance, eps; moving
//                             averages with momentum) and its backward
// Every reduction runs in a fixed order: the step is bitwise reproducible.
#include "rs_common.hpp"

namespace rs {

__global__ __launch_bounds__(256) void din_concat_kernel(const float* __restrict__ item, const float* __restrict__ seq,
                                                         int64_t B, int T, int K, float* __restrict__ out) {
  const int64_t n = B * T * (int64_t)K;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / K;  // row b*T + t
    const int c = (int)(i - r * K);
    const float q = item[(r / T) * K + c], s = seq[i];
    float* o = out + r * 4 * K;
    o[c] = q;
    o[K + c] = s;
    o[2 * K + c] = q - s;
    o[3 * K + c] = q * s;
  }
}

// dq[b,c] (+)= sum_t (d0 + d2 + s d3); dseq[r,c] += d1 - d2 + q d3
__global__ __launch_bounds__(256) void din_concat_bwd_kernel(const float* __restrict__ d, const float* __restrict__ item,
                                                             const float* __restrict__ seq, int64_t B, int T, int K,
                                                             float* __restrict__ dq, int64_t lddq,
                                                             float* __restrict__ dseq) {
  const int64_t n = B * (int64_t)K;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / K;
    const int c = (int)(i - b * K);
    const float q = item[i];
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
      const int64_t r = b * T + t;
      const float* dr = d + r * 4 * K;
      const float s = seq[r * K + c];
      acc += dr[c] + dr[2 * K + c] + s * dr[3 * K + c];
      dseq[r * K + c] += dr[K + c] - dr[2 * K + c] + q * dr[3 * K + c];
    }
    dq[b * lddq + c] += acc;
  }
}

// The same with one block per sample when K divides 256: the B*T*K updates
// of dseq coalesced, dq[c] from the 256/K lanes of column c combined in lane
// order through LDS (T*K loads in flight per block instead of T per thread)
__global__ __launch_bounds__(256) void din_concat_bwd_block_kernel(const float* __restrict__ d,
                                                                   const float* __restrict__ item,
                                                                   const float* __restrict__ seq, int T, int K,
                                                                   float* __restrict__ dq, int64_t lddq,
                                                                   float* __restrict__ dseq) {
  __shared__ float red[256];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, c = tid % K, step = 256 / K;
  const float q = item[b * K + c];
  float acc = 0.f;
  for (int t = tid / K; t < T; t += step) {
    const int64_t r = b * T + t;
    const float* dr = d + r * 4 * K;
    const float d0 = dr[c], d1 = dr[K + c], d2 = dr[2 * K + c], d3 = dr[3 * K + c];
    const float sv = seq[r * K + c];
    acc += d0 + d2 + sv * d3;
    dseq[r * K + c] += d1 - d2 + q * d3;
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < K) {
    float v = 0.f;
    for (int j = tid; j < 256; j += K) v += red[j];
    dq[b * lddq + c] += v;
  }
}

__global__ __launch_bounds__(256) void prelu_rows_fwd_kernel(const float* __restrict__ z, int64_t M, int N,
                                                             const float* __restrict__ alpha, int period,
                                                             float* __restrict__ y) {
  const int64_t n = M * (int64_t)N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / N;
    const int c = (int)(i - r * N);
    const float v = z[i];
    y[i] = fmaxf(v, 0.f) + alpha[(r % period) * N + c] * fminf(v, 0.f);
  }
}

// PReLU backward elementwise part: dz = dy (z > 0 ? 1 : alpha[row mod period]),
// prod = dy min(z, 0) (dalpha = column sums of prod viewed as [M/period, period*N])
__global__ __launch_bounds__(256) void prelu_rows_bwd_kernel(const float* __restrict__ z, const float* __restrict__ dy,
                                                             int64_t M, int N, const float* __restrict__ alpha,
                                                             int period, float* __restrict__ dz,
                                                             float* __restrict__ prod) {
  const int64_t n = M * (int64_t)N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / N;
    const int c = (int)(i - r * N);
    const float v = z[i], g = dy[i];
    dz[i] = g * (v > 0.f ? 1.f : alpha[(r % period) * N + c]);
    prod[i] = g * fminf(v, 0.f);
  }
}

// one wave per sample: score masking, softmax over T (T <= 64 * 8), pool
constexpr int SP_MAXT = 512;
template <int KIND>
__global__ __launch_bounds__(256) void masked_softmax_pool_kernel(const float* __restrict__ score, const void* hist,
                                                                  int64_t hist_stride, const float* __restrict__ seq,
                                                                  int64_t B, int T, int K, float* __restrict__ a,
                                                                  float* __restrict__ out, int64_t ldo) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  constexpr int NT = SP_MAXT / 64;
  float s[NT];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int t = lane + 64 * j;
    s[j] = -INFINITY;
    if (t < T) {
      const bool live = I::load(hist, b * hist_stride + t) != (typename I::raw_t)0;
      s[j] = live ? score[b * T + t] : -4294967296.0f;  // -2**32+1 in fp32
      m = fmaxf(m, s[j]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    s[j] = (lane + 64 * j < T) ? expf(s[j] - m) : 0.f;
    sum += s[j];
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  const float inv = 1.f / sum;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int t = lane + 64 * j;
    if (t < T) a[b * T + t] = s[j] * inv;
  }
  if (K < 64 && 64 % K == 0) {
    // pool with G = 64/K row groups: lane (g, c) sums rows t = g (mod G) of
    // column c (a_t fetched from lane t % 64), then a butterfly over the
    // groups (fixed order): the wave reads 64 contiguous floats per step
    const int G = 64 / K, g = lane / K, c = lane - g * K;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if (64 * j >= T) break;
      const float w = s[j] * inv;
      for (int l0 = 0; l0 < 64 && 64 * j + l0 < T; l0 += G) {
        const int t = 64 * j + l0 + g;
        const float wl = __shfl(w, (l0 + g) & 63);
        if (t < T) acc += wl * seq[(b * T + t) * K + c];
      }
    }
    for (int o = K; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    if (g == 0) out[b * ldo + c] = acc;
    return;
  }
  // pool: lanes own columns; a_t is broadcast from lane t % 64 (t ascending)
  for (int c0 = 0; c0 < K; c0 += 64) {
    const int c = c0 + lane;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if (64 * j >= T) break;
      const float w = s[j] * inv;
      const int tn = min(64, T - 64 * j);
      for (int l = 0; l < tn; ++l) {
        const float wl = __shfl(w, l);
        if (c < K) acc += wl * seq[(b * T + 64 * j + l) * K + c];
      }
    }
    if (c < K) out[b * ldo + c] = acc;
  }
}

// backward: da_t = datt . seq_t; ds_t = live ? a_t (da_t - sum_s a_s da_s) : 0;
// dseq_t = a_t datt (stored, not accumulated)
template <int KIND>
__global__ __launch_bounds__(256) void masked_softmax_pool_bwd_kernel(const float* __restrict__ a, const void* hist,
                                                                      int64_t hist_stride,
                                                                      const float* __restrict__ seq,
                                                                      const float* __restrict__ datt, int64_t ldd,
                                                                      int64_t B, int T, int K,
                                                                      float* __restrict__ ds,
                                                                      float* __restrict__ dseq) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  constexpr int NT = SP_MAXT / 64;
  float da[NT];
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int t = lane + 64 * j;
    da[j] = 0.f;
    if (t < T) {
      float acc = 0.f;
      for (int c = 0; c < K; ++c) acc += datt[b * ldd + c] * seq[(b * T + t) * K + c];
      da[j] = acc;
      dot += a[b * T + t] * acc;
    }
  }
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int t = lane + 64 * j;
    if (t < T) {
      const bool live = I::load(hist, b * hist_stride + t) != (typename I::raw_t)0;
      const float at = a[b * T + t];
      ds[b * T + t] = live ? at * (da[j] - dot) : 0.f;
      for (int c = 0; c < K; ++c) dseq[(b * T + t) * K + c] = at * datt[b * ldd + c];
    }
  }
}

// BatchNormalization, training mode: one block per column
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ x, int64_t ldx, int64_t B,
                                                       float momentum, float* __restrict__ mean,
                                                       float* __restrict__ var, float* __restrict__ mov_mean,
                                                       float* __restrict__ mov_var) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 256) acc += x[b * ldx + c];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const float mu = red[0] / (float)B;
  __syncthreads();
  acc = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 256) {
    const float d = x[b * ldx + c] - mu;
    acc += d * d;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float v = red[0] / (float)B;  // biased (tf.nn.moments)
    mean[c] = mu;
    var[c] = v;
    if (mov_mean) mov_mean[c] = momentum * mov_mean[c] + (1.f - momentum) * mu;
    if (mov_var) mov_var[c] = momentum * mov_var[c] + (1.f - momentum) * v;
  }
}

__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, int64_t ldx, int64_t B, int D,
                                                       const float* __restrict__ mean, const float* __restrict__ var,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       float* __restrict__ y, int64_t ldy) {
  const int64_t n = B * (int64_t)D;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / D;
    const int c = (int)(i - b * D);
    y[b * ldy + c] = (x[b * ldx + c] - mean[c]) * rsqrtf(var[c] + eps) * gamma[c] + beta[c];
  }
}

// per column: dbeta = sum dy, dgamma = sum dy xhat; dx = gamma/sigma (dy -
// dbeta/B - xhat dgamma/B)
__global__ __launch_bounds__(256) void bn_bwd_kernel(const float* __restrict__ x, int64_t ldx, int64_t B,
                                                     const float* __restrict__ mean, const float* __restrict__ var,
                                                     const float* __restrict__ gamma, float eps,
                                                     const float* __restrict__ dy, int64_t ldy,
                                                     float* __restrict__ dx, int64_t lddx,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float r1[256], r2[256];
  const int c = blockIdx.x;
  const float mu = mean[c], is = rsqrtf(var[c] + eps);
  float s1 = 0.f, s2 = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 256) {
    const float g = dy[b * ldy + c];
    s1 += g;
    s2 += g * (x[b * ldx + c] - mu) * is;
  }
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      r1[threadIdx.x] += r1[threadIdx.x + s];
      r2[threadIdx.x] += r2[threadIdx.x + s];
    }
    __syncthreads();
  }
  const float db = r1[0], dg = r2[0];
  if (threadIdx.x == 0) {
    dgamma[c] = dg;
    dbeta[c] = db;
  }
  const float k = gamma[c] * is, inB = 1.f / (float)B;
  for (int64_t b = threadIdx.x; b < B; b += 256) {
    const float xh = (x[b * ldx + c] - mu) * is;
    dx[b * lddx + c] = k * (dy[b * ldy + c] - db * inB - xh * dg * inB);
  }
}

// ---- Dice in training (layer/interaction.py:416-425 under fit): its
// BatchNormalization(center=False, scale=False) uses the batch's mean and
// biased variance per column (every row of [M, N]); y = alpha (1-p) x + p x,
// p = sigmoid(xhat).  Column statistics through the split column sums
// (rs_col_sum_split: fixed slice order), the rest elementwise.
__global__ __launch_bounds__(256) void dice_sq_kernel(const float* __restrict__ x, int64_t M, int N,
                                                      const float* __restrict__ sum, float* __restrict__ sq) {
  const int64_t n = M * (int64_t)N;
  const float inv = 1.f / (float)M;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % N);
    const float d = x[i] - sum[c] * inv;
    sq[i] = d * d;
  }
}

// sums -> mean / var (biased); moving averages with momentum
__global__ __launch_bounds__(256) void dice_stats_kernel(int64_t M, int N, float momentum, float* __restrict__ mean,
                                                         float* __restrict__ var, float* __restrict__ mov_mean,
                                                         float* __restrict__ mov_var) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N) return;
  const float mu = mean[c] / (float)M, v = var[c] / (float)M;
  mean[c] = mu;
  var[c] = v;
  if (mov_mean) mov_mean[c] = momentum * mov_mean[c] + (1.f - momentum) * mu;
  if (mov_var) mov_var[c] = momentum * mov_var[c] + (1.f - momentum) * v;
}

__global__ __launch_bounds__(256) void dice_apply_kernel(const float* __restrict__ x, int64_t M, int N,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ var, float eps,
                                                         const float* __restrict__ alpha, float* __restrict__ y) {
  const int64_t n = M * (int64_t)N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % N);
    const float v = x[i];
    const float pz = 1.f / (1.f + expf(-(v - mean[c]) * rsqrtf(var[c] + eps)));
    y[i] = alpha[c] * (1.f - pz) * v + pz * v;
  }
}

// backward, elementwise part: dx = dy (alpha (1-p) + p); dxh = dy (1-alpha) x
// p (1-p) (dL/dxhat); dxh * xhat; prod = dy (1-p) x (dalpha = its column sums)
__global__ __launch_bounds__(256) void dice_bwd_elem_kernel(const float* __restrict__ x, int64_t M, int N,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ var, float eps,
                                                            const float* __restrict__ alpha,
                                                            const float* __restrict__ dy, float* __restrict__ dx,
                                                            float* __restrict__ dxh, float* __restrict__ dxhx,
                                                            float* __restrict__ prod) {
  const int64_t n = M * (int64_t)N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % N);
    const float v = x[i], g = dy[i], a = alpha[c];
    const float xh = (v - mean[c]) * rsqrtf(var[c] + eps);
    const float pz = 1.f / (1.f + expf(-xh));
    dx[i] = g * (a * (1.f - pz) + pz);
    const float d = g * (1.f - a) * v * pz * (1.f - pz);
    dxh[i] = d;
    dxhx[i] = d * xh;
    prod[i] = g * (1.f - pz) * v;
  }
}

// dx += (dxh - S1/M - xhat S2/M) rsqrt(var + eps)   (batch-norm backward, no gamma)
__global__ __launch_bounds__(256) void dice_bwd_fin_kernel(const float* __restrict__ x, int64_t M, int N,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ var, float eps,
                                                           const float* __restrict__ dxh,
                                                           const float* __restrict__ s1,
                                                           const float* __restrict__ s2, float* __restrict__ dx) {
  const int64_t n = M * (int64_t)N;
  const float inv = 1.f / (float)M;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % N);
    const float is = rsqrtf(var[c] + eps);
    const float xh = (x[i] - mean[c]) * is;
    dx[i] += (dxh[i] - s1[c] * inv - xh * s2[c] * inv) * is;
  }
}

static unsigned dt_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// ---------------------------------------------------------------------------
// Fused backward of the PReLU attention unit (layer/interaction.py:366-395 with
// two hidden Dense+PReLU layers, the reference default (80, 40)): from the
// saved h0 = [q, k, q-k, q*k] [B*T, K0], the pre-activations z1 [B*T, h1], z2
// [B*T, h2] and dL/dscore ds [B*T]:
//   dy2 = ds wo^T, dz2 = dy2 prelu'(z2), dy1 = dz2 W2^T, dz1 = dy1 prelu'(z1),
//   dh0 = dz1 W1^T, and the parameter gradients dW1 = h0^T dz1, dW2 =
//   y1^T dz2, dwo = y2^T ds, biases = column sums, dalpha[t] = sum over the
//   batch of dy min(z, 0).
// One workgroup (8 waves) per sample at a time: the sample's T rows (padded
// to Rp = 16 * ceil(T/16)) sit in LDS; the four products run on MFMA
// 16x16x4 f32 tiles; the weight gradients stay in MFMA accumulators across
// the workgroup's samples, the layer-2 elementwise sums in registers of the
// thread that owns each element, so every sum runs in a fixed order.  The
// next sample's h0 / z1 / z2 / ds are loaded into registers (float4, every
// load issued at once) while the current one runs its products.  The
// per-workgroup partials are then summed in workgroup order (fin kernel).
constexpr int AB_NW = 8;  // waves per workgroup
struct AttBwdArgs {
  const float *h0, *z1, *z2, *ds, *W1, *W2, *al1, *al2, *wo;
  int64_t B;
  int T, K0, h1, h2, Rp, K0p, h1p, h2p;
  int sW1, sW2, sH0, sY1, sZ2;                 // LDS row strides (odd; z1 / dz1 use sY1)
  int oW1, oW2, oH0, oY1, oZ1, oZ2, oDS, oWo;  // LDS offsets (floats)
  int lds_floats;
  int64_t P;                                   // partial floats per workgroup
  int64_t pW1, pW2, pA1, pA2, pB1, pB2, pWo, pBo;  // partial layout
  float* dh0;
  float* part;
};

__device__ __forceinline__ floatx4 ab_ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

// c += sum over k < n (n % 16 == 0) of the 16x16x4 MFMA steps whose operands
// are pa[k * sa] / pb[k * sb] (k = 0, 4, 8, ...): the next 4 steps' LDS reads
// are issued before the current 4 MFMAs (the last group re-reads in bounds)
__device__ __forceinline__ floatx4 ab_mfma_loop(const float* pa, int sa, const float* pb, int sb, int n, floatx4 c) {
  float a0[4], b0[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    a0[u] = pa[4 * u * sa];
    b0[u] = pb[4 * u * sb];
  }
  for (int k = 0; k < n; k += 16) {
    const int kn = min(k + 16, n - 16);
    float a1[4], b1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a1[u] = pa[(kn + 4 * u) * sa];
      b1[u] = pb[(kn + 4 * u) * sb];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) c = mfma16x16x4(a0[u], b0[u], c);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0[u] = a1[u];
      b0[u] = b1[u];
    }
  }
  return c;
}

// SA / SB / SC: tile slots per wave (ceil(tiles / AB_NW)) of the dy1, dW2
// and dW1 products; V0 / V1 / V2: float4 vectors per thread of a sample's
// h0 / z1 / z2 block
template <int SA, int SB, int SC, int V0, int V1, int V2>
__global__ __launch_bounds__(512) void din_att_bwd_kernel(const AttBwdArgs a) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lg = lane >> 4;
  const int T = a.T, K0 = a.K0, h1 = a.h1, h2 = a.h2;
  const int n0 = T * K0, n1 = T * h1, n2 = T * h2;
  float *sW1 = sm + a.oW1, *sW2 = sm + a.oW2, *sH0 = sm + a.oH0, *sY1 = sm + a.oY1, *sZ1 = sm + a.oZ1;
  float *sZ2 = sm + a.oZ2, *sWo = sm + a.oWo;
  // zero every region once (pads stay zero: nothing writes them except as 0)
  for (int e = tid; e < a.lds_floats; e += 512) sm[e] = 0.f;
  __syncthreads();
  for (int e = tid; e < K0 * h1; e += 512) {
    const int k = e / h1;
    sW1[k * a.sW1 + (e - k * h1)] = a.W1[e];
  }
  for (int e = tid; e < h1 * h2; e += 512) {
    const int i = e / h2;
    sW2[i * a.sW2 + (e - i * h2)] = a.W2[e];
  }
  for (int j = tid; j < h2; j += 512) sWo[j] = a.wo[j];
  const int RT = a.Rp >> 4, IT = a.h1p >> 4, JT = a.h2p >> 4, KT = a.K0p >> 4;
  const int Ta = RT * IT, Tb = IT * JT, Tc = KT * IT, Td = RT * KT;
  floatx4 accB[SB], accC[SC], accA[SA];
  float s1[SA];
#pragma unroll
  for (int s = 0; s < SB; ++s) accB[s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < SC; ++s) accC[s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < SA; ++s) {
    accA[s] = floatx4{0.f, 0.f, 0.f, 0.f};
    s1[s] = 0.f;
  }
  // the alphas of this lane's dy1 tile elements (the same for every sample)
  float al[SA][4];
#pragma unroll
  for (int s = 0; s < SA; ++s) {
    const int rt = (w + s * AB_NW) / IT, i = min((w + s * AB_NW - rt * IT) * 16 + l16, h1 - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) al[s][r] = a.al1[min(rt * 16 + 4 * lg + r, T - 1) * h1 + i];
  }
  // this thread's elements (4 consecutive floats of one row, fixed for every
  // sample): their alphas / score weights and the layer-2 sums
  floatx4 al1v[V1], al2v[V2], sA2[V2], sSW[V2], sS2[V2];
  const floatx4 zero4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < V1; ++i) {
    const int e = 4 * (tid + 512 * i);
    al1v[i] = e < n1 ? ab_ld4(a.al1 + e) : zero4;
  }
#pragma unroll
  for (int i = 0; i < V2; ++i) {
    const int e = 4 * (tid + 512 * i);
    al2v[i] = e < n2 ? ab_ld4(a.al2 + e) : zero4;
    sA2[i] = sSW[i] = sS2[i] = zero4;
  }
  float dbo = 0.f;  // sum of ds over the rows whose (t, 0) element this thread owns
  // every load above has landed before the loop: inside it only the
  // prefetches below are outstanding (vmcnt counts in order)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  // the next sample's inputs, every load unconditional at a clamped address
  floatx4 ph0[V0], pz1[V1], pz2[V2];
  float pds[V2];
  auto prefetch = [&](int64_t b) {
    const int64_t r0 = b * T;
#pragma unroll
    for (int i = 0; i < V0; ++i) ph0[i] = ab_ld4(a.h0 + r0 * K0 + min(4 * (tid + 512 * i), n0 - 4));
#pragma unroll
    for (int i = 0; i < V1; ++i) pz1[i] = ab_ld4(a.z1 + r0 * h1 + min(4 * (tid + 512 * i), n1 - 4));
#pragma unroll
    for (int i = 0; i < V2; ++i) {
      const int e = min(4 * (tid + 512 * i), n2 - 4);
      pz2[i] = ab_ld4(a.z2 + r0 * h2 + e);
      pds[i] = a.ds[r0 + e / h2];
    }
  };
  if ((int64_t)blockIdx.x < a.B) prefetch(blockIdx.x);

  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    __syncthreads();  // the previous sample's readers are done
    const int64_t r0 = b * T;
    // stage h0, z1, y1 = prelu(z1); layer 2 + the score Dense elementwise
#pragma unroll
    for (int i = 0; i < V0; ++i) {
      const int e = 4 * (tid + 512 * i);
      if (e < n0) {
        const int t = e / K0;
        float* d = sH0 + t * a.sH0 + (e - t * K0);
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = ph0[i][q];
      }
    }
#pragma unroll
    for (int i = 0; i < V1; ++i) {
      const int e = 4 * (tid + 512 * i);
      if (e < n1) {
        const int t = e / h1, o = t * a.sY1 + (e - t * h1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float z = pz1[i][q];
          sZ1[o + q] = z;
          sY1[o + q] = fmaxf(z, 0.f) + al1v[i][q] * fminf(z, 0.f);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < V2; ++i) {
      const int e = 4 * (tid + 512 * i);
      if (e < n2) {
        const int t = e / h2, o = t * a.sZ2 + (e - t * h2);
        const float dsv = pds[i];
        const floatx4 wv = ab_ld4(sWo + (e - t * h2));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float z = pz2[i][q], al = al2v[i][q];
          const float dy = dsv * wv[q], mn = fminf(z, 0.f);
          const float dz = z > 0.f ? dy : dy * al;
          sA2[i][q] += dy * mn;
          sSW[i][q] += (fmaxf(z, 0.f) + al * mn) * dsv;
          sS2[i][q] += dz;
          sZ2[o + q] = dz;
        }
        if (e - t * h2 == 0) dbo += dsv;
      }
    }
    // the next sample's loads fly during this sample's products
    if (b + gridDim.x < a.B) prefetch(b + gridDim.x);
    __syncthreads();
    // dW2 += y1^T dz2   (tile (it, jt); k runs over the sample's rows)
#pragma unroll
    for (int s = 0; s < SB; ++s) {
      const int q = w + s * AB_NW;
      if (q < Tb) {
        const int it = q / JT, jt = q - it * JT;
        const float* pa = sY1 + lg * a.sY1 + it * 16 + l16;
        const float* pb = sZ2 + lg * a.sZ2 + jt * 16 + l16;
        accB[s] = ab_mfma_loop(pa, a.sY1, pb, a.sZ2, a.Rp, accB[s]);
      }
    }
    // dy1 = dz2 W2^T -> dz1 (in z1's place: each element read and rewritten
    // by its own lane), dalpha1, db1
#pragma unroll
    for (int s = 0; s < SA; ++s) {
      const int q = w + s * AB_NW;
      if (q < Ta) {
        const int rt = q / IT, it = q - rt * IT;
        const float* pa = sZ2 + (rt * 16 + l16) * a.sZ2 + lg;
        const float* pb = sW2 + (it * 16 + l16) * a.sW2 + lg;
        const floatx4 c = ab_mfma_loop(pa, 1, pb, 1, a.h2p, floatx4{0.f, 0.f, 0.f, 0.f});
        const int i = it * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = rt * 16 + 4 * lg + r;
          float* zp = sZ1 + t * a.sY1 + i;
          float dz = 0.f;
          if (t < T && i < h1) {
            const float z = *zp, dy = c[r];
            dz = z > 0.f ? dy : dy * al[s][r];
            accA[s][r] += dy * fminf(z, 0.f);
            s1[s] += dz;
          }
          *zp = dz;
        }
      }
    }
    __syncthreads();
    // dW1 += h0^T dz1
#pragma unroll
    for (int s = 0; s < SC; ++s) {
      const int q = w + s * AB_NW;
      if (q < Tc) {
        const int kt = q / IT, it = q - kt * IT;
        const float* pa = sH0 + lg * a.sH0 + kt * 16 + l16;
        const float* pb = sZ1 + lg * a.sY1 + it * 16 + l16;
        accC[s] = ab_mfma_loop(pa, a.sH0, pb, a.sY1, a.Rp, accC[s]);
      }
    }
    // dh0 = dz1 W1^T
    for (int q = w; q < Td; q += AB_NW) {
      const int rt = q / KT, kt = q - rt * KT;
      const float* pa = sZ1 + (rt * 16 + l16) * a.sY1 + lg;
      const float* pb = sW1 + (kt * 16 + l16) * a.sW1 + lg;
      const floatx4 c = ab_mfma_loop(pa, 1, pb, 1, a.h1p, floatx4{0.f, 0.f, 0.f, 0.f});
      const int col = kt * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = rt * 16 + 4 * lg + r;
        if (t < T && col < K0) a.dh0[(r0 + t) * K0 + col] = c[r];
      }
    }
  }

  // this workgroup's partial sums
  __syncthreads();
  float* part = a.part + blockIdx.x * a.P;
  float* sS1 = sY1;  // [Ta][64] per-lane column sums of dz1
#pragma unroll
  for (int s = 0; s < SB; ++s) {
    const int q = w + s * AB_NW;
    if (q < Tb) {
      const int it = q / JT, jt = q - it * JT, j = jt * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = it * 16 + 4 * lg + r;
        if (i < h1 && j < h2) part[a.pW2 + i * h2 + j] = accB[s][r];
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SC; ++s) {
    const int q = w + s * AB_NW;
    if (q < Tc) {
      const int kt = q / IT, it = q - kt * IT, i = it * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = kt * 16 + 4 * lg + r;
        if (c < K0 && i < h1) part[a.pW1 + c * h1 + i] = accC[s][r];
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SA; ++s) {
    const int q = w + s * AB_NW;
    if (q < Ta) {
      const int rt = q / IT, it = q - rt * IT, i = it * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = rt * 16 + 4 * lg + r;
        if (t < T && i < h1) part[a.pA1 + t * h1 + i] = accA[s][r];
      }
      sS1[q * 64 + lane] = s1[s];
    }
  }
  float* sT = sZ2;  // [T][h2] staging of the per-element layer-2 sums
#pragma unroll
  for (int i = 0; i < V2; ++i) {
    const int e = 4 * (tid + 512 * i);
    if (e < n2)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        part[a.pA2 + e + q] = sA2[i][q];
        sT[e + q] = sSW[i][q];
      }
  }
  __syncthreads();
  for (int i = tid; i < h1; i += 512) {
    const int it = i >> 4;
    float v = 0.f;
    for (int rt = 0; rt < RT; ++rt)
      for (int g = 0; g < 4; ++g) v += sS1[(rt * IT + it) * 64 + g * 16 + (i & 15)];
    part[a.pB1 + i] = v;
  }
  for (int j = tid; j < h2; j += 512) {
    float v = 0.f;
    for (int t = 0; t < T; ++t) v += sT[t * h2 + j];
    part[a.pWo + j] = v;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < V2; ++i) {
    const int e = 4 * (tid + 512 * i);
    if (e < n2)
#pragma unroll
      for (int q = 0; q < 4; ++q) sT[e + q] = sS2[i][q];
  }
  __syncthreads();
  for (int j = tid; j < h2; j += 512) {
    float v = 0.f;
    for (int t = 0; t < T; ++t) v += sT[t * h2 + j];
    part[a.pB2 + j] = v;
  }
  __syncthreads();
  sm[tid] = dbo;  // (every region is free by now; LDS holds >= 512 floats)
  __syncthreads();
  if (tid == 0) {
    float v = 0.f;
    for (int t = 0; t < 512; ++t) v += sm[t];
    part[a.pBo] = v;
  }
}

// Forward of the same unit under fit: z1 = h0 W1 + b1, y1 = prelu(z1),
// z2 = y1 W2 + b2, y2 = prelu(z2), score = y2 wo + bo, keeping z1 / z2 for
// the backward.  Same layout as din_att_bwd_kernel: one sample's rows in LDS
// at a time, the next sample's h0 in registers, MFMA 16x16x4 f32 tiles.
struct AttFwdArgs {
  const float *h0, *W1, *b1, *al1, *W2, *b2, *al2, *wo, *bo;
  int64_t B;
  int T, K0, h1, h2, Rp, K0p, h1p, h2p;
  int sW1, sW2, sH0, sY1, sP;
  int oW1, oW2, oH0, oY1, oP;
  int lds_floats;
  float *z1, *z2, *score;
};

template <int SA, int SB, int V0>
__global__ __launch_bounds__(512) void din_att_fwd_kernel(const AttFwdArgs a) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lg = lane >> 4;
  const int T = a.T, K0 = a.K0, h1 = a.h1, h2 = a.h2, n0 = T * K0;
  float *sW1 = sm + a.oW1, *sW2 = sm + a.oW2, *sH0 = sm + a.oH0, *sY1 = sm + a.oY1, *sP = sm + a.oP;
  for (int e = tid; e < a.lds_floats; e += 512) sm[e] = 0.f;
  __syncthreads();
  for (int e = tid; e < K0 * h1; e += 512) {
    const int k = e / h1;
    sW1[k * a.sW1 + (e - k * h1)] = a.W1[e];
  }
  for (int e = tid; e < h1 * h2; e += 512) {
    const int i = e / h2;
    sW2[i * a.sW2 + (e - i * h2)] = a.W2[e];
  }
  const int RT = a.Rp >> 4, IT = a.h1p >> 4, JT = a.h2p >> 4;
  const int Ta = RT * IT, Tb = RT * JT;
  // per-lane constants of this wave's tiles (the same for every sample)
  float al1[SA][4], b1[SA], al2[SB][4], b2[SB], wo[SB];
#pragma unroll
  for (int s = 0; s < SA; ++s) {
    const int q = w + s * AB_NW, rt = q / IT, i = min((q - rt * IT) * 16 + l16, h1 - 1);
    b1[s] = a.b1[i];
#pragma unroll
    for (int r = 0; r < 4; ++r) al1[s][r] = a.al1[min(rt * 16 + 4 * lg + r, T - 1) * h1 + i];
  }
#pragma unroll
  for (int s = 0; s < SB; ++s) {
    const int q = w + s * AB_NW, rt = q / JT, j = min((q - rt * JT) * 16 + l16, h2 - 1);
    b2[s] = a.b2[j];
    wo[s] = a.wo[j];
#pragma unroll
    for (int r = 0; r < 4; ++r) al2[s][r] = a.al2[min(rt * 16 + 4 * lg + r, T - 1) * h2 + j];
  }
  const float bo = a.bo[0];
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): only the prefetches are outstanding in the loop

  floatx4 ph0[V0];
  auto prefetch = [&](int64_t b) {
#pragma unroll
    for (int i = 0; i < V0; ++i) ph0[i] = ab_ld4(a.h0 + b * n0 + min(4 * (tid + 512 * i), n0 - 4));
  };
  if ((int64_t)blockIdx.x < a.B) prefetch(blockIdx.x);
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    __syncthreads();
    const int64_t r0 = b * T;
#pragma unroll
    for (int i = 0; i < V0; ++i) {
      const int e = 4 * (tid + 512 * i);
      if (e < n0) {
        const int t = e / K0;
        float* d = sH0 + t * a.sH0 + (e - t * K0);
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = ph0[i][q];
      }
    }
    if (b + gridDim.x < a.B) prefetch(b + gridDim.x);
    __syncthreads();
    // z1 = h0 W1 + b1 -> HBM; y1 = prelu(z1) -> LDS
#pragma unroll
    for (int s = 0; s < SA; ++s) {
      const int q = w + s * AB_NW;
      if (q < Ta) {
        const int rt = q / IT, it = q - rt * IT;
        const floatx4 c = ab_mfma_loop(sH0 + (rt * 16 + l16) * a.sH0 + lg, 1, sW1 + lg * a.sW1 + it * 16 + l16, a.sW1,
                                       a.K0p, floatx4{0.f, 0.f, 0.f, 0.f});
        const int i = it * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = rt * 16 + 4 * lg + r;
          float y = 0.f;
          if (t < T && i < h1) {
            const float z = c[r] + b1[s];
            a.z1[(r0 + t) * h1 + i] = z;
            y = fmaxf(z, 0.f) + al1[s][r] * fminf(z, 0.f);
          }
          sY1[t * a.sY1 + i] = y;
        }
      }
    }
    __syncthreads();
    // z2 = y1 W2 + b2 -> HBM; y2 wo -> LDS (summed per row below)
#pragma unroll
    for (int s = 0; s < SB; ++s) {
      const int q = w + s * AB_NW;
      if (q < Tb) {
        const int rt = q / JT, jt = q - rt * JT;
        const floatx4 c = ab_mfma_loop(sY1 + (rt * 16 + l16) * a.sY1 + lg, 1, sW2 + lg * a.sW2 + jt * 16 + l16, a.sW2,
                                       a.h1p, floatx4{0.f, 0.f, 0.f, 0.f});
        const int j = jt * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = rt * 16 + 4 * lg + r;
          float v = 0.f;
          if (t < T && j < h2) {
            const float z = c[r] + b2[s];
            a.z2[(r0 + t) * h2 + j] = z;
            v = (fmaxf(z, 0.f) + al2[s][r] * fminf(z, 0.f)) * wo[s];
          }
          sP[t * a.sP + j] = v;
        }
      }
    }
    __syncthreads();
    if (tid < T) {
      float v = 0.f;
      for (int j = 0; j < h2; ++j) v += sP[tid * a.sP + j];
      a.score[r0 + tid] = v + bo;
    }
  }
}

struct AttBwdOut {
  float *dW1, *db1, *dal1, *dW2, *db2, *dal2, *dwo, *dbo;
};
// out[e] = the G partials in a fixed order: a block takes 64 consecutive
// elements (coalesced rows of the partials) x 4 lanes of workgroups (g = q
// mod 4, each in seg_sum8's tree), the 4 lane sums added in order
__global__ __launch_bounds__(256) void din_att_bwd_fin(const float* __restrict__ part, int G, const AttBwdArgs a,
                                                       const AttBwdOut o) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + c;
  const int ng = G > q ? (G - q + 3) / 4 : 0;
  red[q][c] = e < a.P ? seg_sum8(0, ng, [&](int64_t i) { return part[(q + 4 * i) * a.P + e]; }) : 0.f;
  __syncthreads();
  if (q != 0 || e >= a.P) return;
  const float v = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  if (e < a.pW2) o.dW1[e - a.pW1] = v;
  else if (e < a.pA1) o.dW2[e - a.pW2] = v;
  else if (e < a.pA2) o.dal1[e - a.pA1] = v;
  else if (e < a.pB1) o.dal2[e - a.pA2] = v;
  else if (e < a.pB2) o.db1[e - a.pB1] = v;
  else if (e < a.pWo) o.db2[e - a.pB2] = v;
  else if (e < a.pBo) o.dwo[e - a.pWo] = v;
  else o.dbo[0] = v;
}

// geometry; false when the dims do not fit (T, K0, h1, h2 <= 128 and the LDS)
// LDS row strides for the two MFMA operand patterns of ds_read_b32 (32 banks
// per 32-lane group): "rows": 16 rows x 2 consecutive columns per group
// (operand[(16t + l16) * S + k + lg]) is conflict-free for S = 2 * odd;
// "cols": 2 rows x 16 columns (operand[(k + lg) * S + 16t + l16]) for
// S = 16 (mod 32).  Arrays read both ways take the "rows" stride.
static int lds_stride_rows(int n) { return (n + 3) / 4 * 4 + 2; }
static int lds_stride_cols(int n) {
  const int v = (n + 15) / 32 * 32 + 16;
  return v >= n ? v : v + 32;
}
// vectors per thread of a [T, X] block (X % 4 == 0) read as float4 by 512 threads
static int att_bwd_nv(int T, int X) { return (T * X / 4 + 511) / 512; }
static bool att_bwd_geom(int64_t B, int T, int K0, int h1, int h2, AttBwdArgs& a, int& G) {
  if (B < 0 || T < 1 || T > 128 || K0 < 4 || K0 > 128 || h1 < 4 || h1 > 128 || h2 < 4 || h2 > 128) return false;
  if (K0 % 4 || h1 % 4 || h2 % 4) return false;  // float4 rows
  if (att_bwd_nv(T, K0) > 4 || att_bwd_nv(T, h1) > 4 || att_bwd_nv(T, h2) > 4) return false;
  auto r16 = [](int v) { return (v + 15) / 16 * 16; };
  a.B = B;
  a.T = T;
  a.K0 = K0;
  a.h1 = h1;
  a.h2 = h2;
  a.Rp = r16(T);
  a.K0p = r16(K0);
  a.h1p = r16(h1);
  a.h2p = r16(h2);
  a.sW1 = lds_stride_rows(a.h1p);  // (dh0: rows)
  a.sW2 = lds_stride_rows(a.h2p);  // (dy1: rows)
  a.sH0 = lds_stride_cols(a.K0p);  // (dW1: cols)
  a.sY1 = lds_stride_rows(a.h1p);  // y1 (dW2: cols) and z1 / dz1 (rows and cols) share it
  a.sZ2 = lds_stride_rows(a.h2p);  // dz2: rows and cols
  int o = 0;
  a.oW1 = o;
  o += a.K0p * a.sW1;
  a.oW2 = o;
  o += a.h1p * a.sW2;
  a.oH0 = o;
  o += a.Rp * a.sH0;
  a.oY1 = o;
  o += a.Rp * a.sY1;
  a.oZ1 = o;
  o += a.Rp * a.sY1;
  a.oZ2 = o;
  o += a.Rp * a.sZ2;
  a.oDS = o;
  o += a.Rp;
  a.oWo = o;
  o += a.h2p;
  a.lds_floats = o;
  if ((size_t)o * sizeof(float) > 160 * 1024) return false;
  int64_t p = 0;
  a.pW1 = p;
  p += (int64_t)K0 * h1;
  a.pW2 = p;
  p += (int64_t)h1 * h2;
  a.pA1 = p;
  p += (int64_t)T * h1;
  a.pA2 = p;
  p += (int64_t)T * h2;
  a.pB1 = p;
  p += h1;
  a.pB2 = p;
  p += h2;
  a.pWo = p;
  p += h2;
  a.pBo = p;
  p += 1;
  a.P = p;
  G = (int)std::max<int64_t>(1, std::min<int64_t>(B, 256));
  return true;
}

}  // namespace rs

using namespace rs;

extern "C" int rs_din_att_concat(const float* item, const float* seq, int64_t batch, int T, int K, float* out,
                                 rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(item && seq && out && batch > 0 && T >= 1 && K >= 1, "rs_din_att_concat: bad arguments");
  din_concat_kernel<<<dt_grid(batch * T * (int64_t)K), 256, 0, as_stream(stream)>>>(item, seq, batch, T, K, out);
  return launch_status("rs_din_att_concat");
}

extern "C" int rs_din_att_concat_bwd(const float* d, const float* item, const float* seq, int64_t batch, int T, int K,
                                     float* dq, int64_t dq_stride, float* dseq, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(d && item && seq && dq && dseq && batch > 0 && T >= 1 && K >= 1 && dq_stride >= K,
             "rs_din_att_concat_bwd: bad arguments");
  if (K <= 256 && 256 % K == 0)
    din_concat_bwd_block_kernel<<<(unsigned)batch, 256, 0, as_stream(stream)>>>(d, item, seq, T, K, dq, dq_stride,
                                                                                 dseq);
  else
    din_concat_bwd_kernel<<<dt_grid(batch * (int64_t)K), 256, 0, as_stream(stream)>>>(d, item, seq, batch, T, K, dq,
                                                                                     dq_stride, dseq);
  return launch_status("rs_din_att_concat_bwd");
}

extern "C" int rs_prelu_rows_fwd(const float* z, int64_t M, int N, const float* alpha, int period, float* y,
                                 rs_stream_t stream) {
  if (M == 0) return RS_OK;
  RS_REQUIRE(z && alpha && y && M > 0 && N >= 1 && period >= 1, "rs_prelu_rows_fwd: bad arguments");
  prelu_rows_fwd_kernel<<<dt_grid(M * (int64_t)N), 256, 0, as_stream(stream)>>>(z, M, N, alpha, period, y);
  return launch_status("rs_prelu_rows_fwd");
}

extern "C" int64_t rs_prelu_rows_bwd_workspace_size(int64_t M, int N, int period) {
  if (M < 0 || N < 1 || period < 1) return -1;
  return (M * N * 4 + 255) / 256 * 256 + rs_col_sum_workspace_size(M / period, (int64_t)period * N);
}

extern "C" int rs_prelu_rows_bwd(const float* z, const float* dy, int64_t M, int N, const float* alpha, int period,
                                 float* dz, float* dalpha, void* workspace, int64_t workspace_bytes,
                                 rs_stream_t stream) {
  if (M == 0) return RS_OK;
  RS_REQUIRE(z && dy && alpha && dz && dalpha && workspace && M > 0 && N >= 1 && period >= 1 && M % period == 0 &&
                 dz != dy,
             "rs_prelu_rows_bwd: bad arguments (rows a multiple of period)");
  RS_REQUIRE(workspace_bytes >= rs_prelu_rows_bwd_workspace_size(M, N, period),
             "rs_prelu_rows_bwd: workspace too small");
  hipStream_t st = as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  float* prod = reinterpret_cast<float*>(ws);
  const int64_t pb = (M * N * 4 + 255) / 256 * 256;
  prelu_rows_bwd_kernel<<<dt_grid(M * (int64_t)N), 256, 0, st>>>(z, dy, M, N, alpha, period, dz, prod);
  // dalpha[p, c] = column (p*N + c) sum of prod viewed as [M/period, period*N]
  const int64_t W = (int64_t)period * N;
  return rs_col_sum_split(prod, W, M / period, W, dalpha, ws + pb, workspace_bytes - pb, stream);
}

extern "C" int rs_din_att_prelu_fwd(const float* h0, const float* W1, const float* b1, const float* alpha1,
                                    const float* W2, const float* b2, const float* alpha2, const float* wo,
                                    const float* bo, int64_t batch, int T, int K0, int h1, int h2, float* z1, float* z2,
                                    float* score, rs_stream_t stream) {
  AttBwdArgs g{};
  int G = 0;
  RS_REQUIRE(att_bwd_geom(batch, T, K0, h1, h2, g, G),
             "rs_din_att_prelu_fwd: unsupported shape (T, K0, h1, h2 <= 128, multiples of 4, the rows in LDS)");
  RS_REQUIRE(h0 && W1 && b1 && alpha1 && W2 && b2 && alpha2 && wo && bo && z1 && z2 && score,
             "rs_din_att_prelu_fwd: null pointer");
  RS_REQUIRE(reinterpret_cast<uintptr_t>(h0) % 16 == 0, "rs_din_att_prelu_fwd: h0 16-B aligned");
  if (batch == 0) return RS_OK;
  AttFwdArgs a{};
  a.h0 = h0;
  a.W1 = W1;
  a.b1 = b1;
  a.al1 = alpha1;
  a.W2 = W2;
  a.b2 = b2;
  a.al2 = alpha2;
  a.wo = wo;
  a.bo = bo;
  a.B = batch;
  a.T = T;
  a.K0 = K0;
  a.h1 = h1;
  a.h2 = h2;
  a.Rp = g.Rp;
  a.K0p = g.K0p;
  a.h1p = g.h1p;
  a.h2p = g.h2p;
  a.sW1 = lds_stride_cols(g.h1p);  // z1 product B: cols
  a.sW2 = lds_stride_cols(g.h2p);  // z2 product B: cols
  a.sH0 = lds_stride_rows(g.K0p);  // z1 product A: rows
  a.sY1 = lds_stride_rows(g.h1p);  // z2 product A: rows
  a.sP = g.h2p + 1;
  int o = 0;
  a.oW1 = o;
  o += a.K0p * a.sW1;
  a.oW2 = o;
  o += a.h1p * a.sW2;
  a.oH0 = o;
  o += a.Rp * a.sH0;
  a.oY1 = o;
  o += a.Rp * a.sY1;
  a.oP = o;
  o += a.Rp * a.sP;
  a.lds_floats = o;
  a.z1 = z1;
  a.z2 = z2;
  a.score = score;
  auto slots = [](int tiles) { return (tiles + AB_NW - 1) / AB_NW; };
  const int SA = slots((a.Rp >> 4) * (a.h1p >> 4)), SB = slots((a.Rp >> 4) * (a.h2p >> 4));
  const size_t lds = (size_t)o * sizeof(float);
  hipStream_t st = as_stream(stream);
  auto go = [&](auto fn) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<(unsigned)G, 512, lds, st>>>(a);
  };
  if (SA <= 5 && SB <= 3 && att_bwd_nv(T, K0) <= 2)
    go(din_att_fwd_kernel<5, 3, 2>);
  else
    go(din_att_fwd_kernel<8, 8, 4>);
  return launch_status("rs_din_att_prelu_fwd");
}

extern "C" int64_t rs_din_att_prelu_bwd_workspace_size(int64_t batch, int T, int K0, int h1, int h2) {
  AttBwdArgs a{};
  int G = 0;
  if (!att_bwd_geom(batch, T, K0, h1, h2, a, G)) return -1;
  return (int64_t)G * a.P * (int64_t)sizeof(float);
}

extern "C" int rs_din_att_prelu_bwd(const float* h0, const float* z1, const float* z2, const float* ds, const float* W1,
                                    const float* W2, const float* alpha1, const float* alpha2, const float* wo,
                                    int64_t batch, int T, int K0, int h1, int h2, float* dh0, float* dW1, float* db1,
                                    float* dalpha1, float* dW2, float* db2, float* dalpha2, float* dwo, float* dbo,
                                    void* workspace, int64_t workspace_bytes, rs_stream_t stream) {
  AttBwdArgs a{};
  int G = 0;
  RS_REQUIRE(att_bwd_geom(batch, T, K0, h1, h2, a, G),
             "rs_din_att_prelu_bwd: unsupported shape (T, K0, h1, h2 <= 128 and the sample's rows in LDS)");
  RS_REQUIRE(h0 && z1 && z2 && ds && W1 && W2 && alpha1 && alpha2 && wo && dh0 && dW1 && db1 && dalpha1 && dW2 &&
                 db2 && dalpha2 && dwo && dbo && workspace,
             "rs_din_att_prelu_bwd: null pointer");
  RS_REQUIRE(workspace_bytes >= (int64_t)G * a.P * (int64_t)sizeof(float), "rs_din_att_prelu_bwd: workspace too small");
  for (const void* p : {(const void*)h0, (const void*)z1, (const void*)z2, (const void*)alpha1, (const void*)alpha2,
                        (const void*)wo})
    RS_REQUIRE(reinterpret_cast<uintptr_t>(p) % 16 == 0, "rs_din_att_prelu_bwd: h0, z1, z2, alphas, wo 16-B aligned");
  hipStream_t st = as_stream(stream);
  a.h0 = h0;
  a.z1 = z1;
  a.z2 = z2;
  a.ds = ds;
  a.W1 = W1;
  a.W2 = W2;
  a.al1 = alpha1;
  a.al2 = alpha2;
  a.wo = wo;
  a.dh0 = dh0;
  a.part = static_cast<float*>(workspace);
  const size_t lds = (size_t)a.lds_floats * sizeof(float);
  auto slots = [](int tiles) { return (tiles + AB_NW - 1) / AB_NW; };
  const int SA = slots((a.Rp >> 4) * (a.h1p >> 4)), SB = slots((a.h1p >> 4) * (a.h2p >> 4)),
            SC = slots((a.K0p >> 4) * (a.h1p >> 4));
  auto go = [&](auto fn) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<(unsigned)G, 512, lds, st>>>(a);
  };
  // fewer slots / vectors = fewer live registers: the (80, 40) default at
  // T <= 112 (K0 = 32) takes the small instance; the general one spills
  if (SA <= 5 && SB <= 2 && SC <= 2 && att_bwd_nv(T, K0) <= 2 && att_bwd_nv(T, h1) <= 4 && att_bwd_nv(T, h2) <= 2)
    go(din_att_bwd_kernel<5, 2, 2, 2, 4, 2>);
  else
    go(din_att_bwd_kernel<8, 8, 8, 4, 4, 4>);
  const AttBwdOut o{dW1, db1, dalpha1, dW2, db2, dalpha2, dwo, dbo};
  din_att_bwd_fin<<<(unsigned)((a.P + 63) / 64), 256, 0, st>>>(a.part, G, a, o);
  return launch_status("rs_din_att_prelu_bwd");
}

extern "C" int rs_masked_softmax_pool(const float* score, const void* hist, int hist_kind, int64_t hist_stride,
                                      const float* seq, int64_t batch, int T, int K, float* a, float* out,
                                      int64_t out_stride, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(score && hist && seq && a && out && batch > 0 && T >= 1 && T <= SP_MAXT && K >= 1 && out_stride >= K &&
                 hist_kind >= RS_ID_I32 && hist_kind <= RS_ID_F32,
             "rs_masked_softmax_pool: bad arguments (T <= %d)", SP_MAXT);
  const unsigned g = (unsigned)((batch + 3) / 4);
  hipStream_t st = as_stream(stream);
  with_id_kind(hist_kind, [&](auto kc) {
    masked_softmax_pool_kernel<decltype(kc)::value>
        <<<g, 256, 0, st>>>(score, hist, hist_stride, seq, batch, T, K, a, out, out_stride);
  });
  return launch_status("rs_masked_softmax_pool");
}

extern "C" int rs_masked_softmax_pool_bwd(const float* a, const void* hist, int hist_kind, int64_t hist_stride,
                                          const float* seq, const float* datt, int64_t datt_stride, int64_t batch,
                                          int T, int K, float* ds, float* dseq, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(a && hist && seq && datt && ds && dseq && batch > 0 && T >= 1 && T <= SP_MAXT && K >= 1 &&
                 datt_stride >= K && hist_kind >= RS_ID_I32 && hist_kind <= RS_ID_F32,
             "rs_masked_softmax_pool_bwd: bad arguments (T <= %d)", SP_MAXT);
  const unsigned g = (unsigned)((batch + 3) / 4);
  hipStream_t st = as_stream(stream);
  with_id_kind(hist_kind, [&](auto kc) {
    masked_softmax_pool_bwd_kernel<decltype(kc)::value>
        <<<g, 256, 0, st>>>(a, hist, hist_stride, seq, datt, datt_stride, batch, T, K, ds, dseq);
  });
  return launch_status("rs_masked_softmax_pool_bwd");
}

extern "C" int rs_bn_train_fwd(const float* x, int64_t x_stride, int64_t batch, int D, const float* gamma,
                               const float* beta, float eps, float momentum, float* moving_mean,
                               float* moving_var, float* mean, float* var, float* y, int64_t y_stride,
                               rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(x && gamma && beta && mean && var && y && batch > 0 && D >= 1 && x_stride >= D && y_stride >= D,
             "rs_bn_train_fwd: bad arguments");
  hipStream_t st = as_stream(stream);
  bn_stats_kernel<<<(unsigned)D, 256, 0, st>>>(x, x_stride, batch, momentum, mean, var, moving_mean, moving_var);
  bn_apply_kernel<<<dt_grid(batch * (int64_t)D), 256, 0, st>>>(x, x_stride, batch, D, mean, var, gamma, beta, eps, y,
                                                               y_stride);
  return launch_status("rs_bn_train_fwd");
}

extern "C" int rs_bn_train_bwd(const float* x, int64_t x_stride, int64_t batch, int D, const float* mean,
                               const float* var, const float* gamma, float eps, const float* dy, int64_t dy_stride,
                               float* dx, int64_t dx_stride, float* dgamma, float* dbeta, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(x && mean && var && gamma && dy && dx && dgamma && dbeta && batch > 0 && D >= 1 && x_stride >= D &&
                 dy_stride >= D && dx_stride >= D && dx != dy,
             "rs_bn_train_bwd: bad arguments");
  bn_bwd_kernel<<<(unsigned)D, 256, 0, as_stream(stream)>>>(x, x_stride, batch, mean, var, gamma, eps, dy, dy_stride,
                                                            dx, dx_stride, dgamma, dbeta);
  return launch_status("rs_bn_train_bwd");
}

static int64_t dt_al(int64_t b) { return (b + 255) / 256 * 256; }

extern "C" int64_t rs_dice_train_workspace_size(int64_t M, int N) {
  if (M < 0 || N < 1) return -1;
  return 3 * dt_al(M * N * 4) + 2 * dt_al((int64_t)N * 4) + dt_al(rs_col_sum_workspace_size(M, N));
}

extern "C" int rs_dice_train_fwd(const float* x, int64_t M, int N, const float* alpha, float eps, float momentum,
                                 float* moving_mean, float* moving_var, float* mean, float* var, float* y,
                                 void* workspace, int64_t workspace_bytes, rs_stream_t stream) {
  if (M == 0) return RS_OK;
  RS_REQUIRE(x && alpha && mean && var && y && workspace && M > 0 && N >= 1 && mean != var,
             "rs_dice_train_fwd: bad arguments");
  RS_REQUIRE(workspace_bytes >= rs_dice_train_workspace_size(M, N), "rs_dice_train_fwd: workspace too small");
  hipStream_t st = as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  float* sq = reinterpret_cast<float*>(ws);
  uint8_t* cws = ws + 3 * dt_al(M * N * 4) + 2 * dt_al((int64_t)N * 4);
  const int64_t cb = rs_col_sum_workspace_size(M, N);
  int rc = rs_col_sum_split(x, N, M, N, mean, cws, cb, stream);  // column sums
  if (rc != RS_OK) return rc;
  dice_sq_kernel<<<dt_grid(M * (int64_t)N), 256, 0, st>>>(x, M, N, mean, sq);
  rc = rs_col_sum_split(sq, N, M, N, var, cws, cb, stream);
  if (rc != RS_OK) return rc;
  dice_stats_kernel<<<(unsigned)((N + 255) / 256), 256, 0, st>>>(M, N, momentum, mean, var, moving_mean, moving_var);
  dice_apply_kernel<<<dt_grid(M * (int64_t)N), 256, 0, st>>>(x, M, N, mean, var, eps, alpha, y);
  return launch_status("rs_dice_train_fwd");
}

extern "C" int rs_dice_train_bwd(const float* x, int64_t M, int N, const float* alpha, const float* mean,
                                 const float* var, float eps, const float* dy, float* dx, float* dalpha,
                                 void* workspace, int64_t workspace_bytes, rs_stream_t stream) {
  if (M == 0) return RS_OK;
  RS_REQUIRE(x && alpha && mean && var && dy && dx && dalpha && workspace && M > 0 && N >= 1 && dx != dy,
             "rs_dice_train_bwd: bad arguments");
  RS_REQUIRE(workspace_bytes >= rs_dice_train_workspace_size(M, N), "rs_dice_train_bwd: workspace too small");
  hipStream_t st = as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  const int64_t slab = dt_al(M * N * 4);
  float* dxh = reinterpret_cast<float*>(ws);
  float* dxhx = reinterpret_cast<float*>(ws + slab);
  float* prod = reinterpret_cast<float*>(ws + 2 * slab);
  float* s1 = reinterpret_cast<float*>(ws + 3 * slab);
  float* s2 = reinterpret_cast<float*>(ws + 3 * slab + dt_al((int64_t)N * 4));
  uint8_t* cws = ws + 3 * slab + 2 * dt_al((int64_t)N * 4);
  const int64_t cb = rs_col_sum_workspace_size(M, N);
  dice_bwd_elem_kernel<<<dt_grid(M * (int64_t)N), 256, 0, st>>>(x, M, N, mean, var, eps, alpha, dy, dx, dxh, dxhx,
                                                                prod);
  int rc = rs_col_sum_split(dxh, N, M, N, s1, cws, cb, stream);
  if (rc == RS_OK) rc = rs_col_sum_split(dxhx, N, M, N, s2, cws, cb, stream);
  if (rc == RS_OK) rc = rs_col_sum_split(prod, N, M, N, dalpha, cws, cb, stream);
  if (rc != RS_OK) return rc;
  dice_bwd_fin_kernel<<<dt_grid(M * (int64_t)N), 256, 0, st>>>(x, M, N, mean, var, eps, dxh, s1, s2, dx);
  return launch_status("rs_dice_train_bwd");
}
