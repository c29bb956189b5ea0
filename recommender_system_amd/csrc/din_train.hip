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
