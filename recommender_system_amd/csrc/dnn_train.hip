// dnn_train.hip — building blocks of the DeepFM training step (SURVEY §8(f)
// rank 4: compile_fit on model/deepFM.py): a deterministic fp32 GEMM for the
// DNN backward, column sums, SGD updates, the DeepFM head gradient, the FM
// gradients w.r.t. x and (w0, w1, v), and the row-sparse SGD of the
// embedding tables (EmbedLayer's Embedding, layer/core.py:271 — Keras applies
// its IndexedSlices gradient with a scatter-add; here a stable sort by row
// plus an in-order segmented sum, bitwise reproducible).
//
// Reference semantics (utils/compile_fit.py:9-15, model/deepFM.py:23-31):
//   z = 0.5 (FM(x) + DNN(x)),  p = sigmoid(z),  L = mean_b BCE(t_b, p_b)
//   + l2(reg_w) |w1|^2 + l2(reg_b) |v|^2 (FMLayer.build); Dense layers and
//   embeddings carry no regulariser; SGD(lr): w -= lr dL/dw.
#include "radix_sort.hpp"

#include "rs_common.hpp"

namespace rs {

// ------------------------------------------------------------------ GEMM
// C[M,N] = alpha * op(A)[M,K] op(B)[K,N] + beta * C, row-major, optionally
// masked: C[m,n] *= (mask[m,n] > 0) (ReLU backward: a = relu(z) > 0 <=> z > 0).
// 64x64 tiles, 256 threads = four waves in 2x2, each a 32x32 tile of
// v_mfma_f32_32x32x2_f32 (lane l: A row / B column l&31, k-slot l>>5; C:
// column l&31, rows (r&3) + 8(r>>2) + 4(l>>5)); K in steps of 16 through LDS.
// The f32 MFMA is a k-ordered fmaf chain, so each output's K sum runs in one
// fixed order (deterministic, the same order as a scalar k loop).
constexpr int GT = 64, GK = 16;
// Split-K launches (the weight gradients: a tall K = batch or batch*T, few
// output tiles) stage 64 k-rows per round trip instead of 16: each slice is a
// chain of dependent load -> MFMA steps, so 4x the bytes per step is 4x fewer
// steps.
constexpr int GK_SPLIT = 64;
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Split-K (part != nullptr): block z of gridDim.z covers K range
// [z*kslice, (z+1)*kslice) and stores its raw partial tile to part[z][M][N];
// gemm_reduce sums the slices in z order (deterministic).
template <int GK>
__global__ __launch_bounds__(256) void gemm_kernel(int ta, int tb, int M, int N, int K, float alpha,
                                                   const float* __restrict__ A, int64_t lda,
                                                   const float* __restrict__ B, int64_t ldb, float beta,
                                                   float* __restrict__ C, int64_t ldc,
                                                   const float* __restrict__ mask, int64_t ldm, int kslice,
                                                   float* __restrict__ part) {
  __shared__ float As[GK][GT + 4];
  __shared__ float Bs[GK][GT + 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1, li = lane & 31, lk = lane >> 5;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int kb = part ? blockIdx.z * kslice : 0;
  const int ke = part ? min(K, kb + kslice) : K;
  // stage op(A)[m0:m0+64, k0:k0+GK] as As[k][m] and op(B)[k0:k0+GK, n0:n0+64]
  // as Bs[k][n]; consecutive threads walk each operand's contiguous memory
  // dimension (k for a row-major A / transposed B, m or n otherwise).  Every
  // load is unconditional (an out-of-range element reads a clamped address in
  // the tile's own lines and is zeroed by a select: a load under a branch
  // merged with a default makes the compiler wait for it before the next one,
  // and a common dummy address would be a chip-wide L2 hot spot), and the next
  // stage's loads are in flight while this stage's MFMAs run.
  constexpr int NE = GK * GT / 256;
  float av[NE], bv[NE];
  auto load_stage = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int ka = ta ? e / GT : e % GK, ma = ta ? e % GT : e / GK;
      const int m = m0 + ma, k = k0 + ka;
      const bool oka = m < M && k < ke;
      const int mc = min(m, M - 1), kc = min(k, ke - 1);  // clamped into the tile's own lines
      const float x = A[ta ? (int64_t)kc * lda + mc : (int64_t)mc * lda + kc];
      av[i] = oka ? x : 0.f;
      const int kb2 = tb ? e % GK : e / GT, nb = tb ? e / GK : e % GT;
      const int n = n0 + nb, k2 = k0 + kb2;
      const bool okb = n < N && k2 < ke;
      const int nc = min(n, N - 1), kc2 = min(k2, ke - 1);
      const float y = B[tb ? (int64_t)nc * ldb + kc2 : (int64_t)kc2 * ldb + nc];
      bv[i] = okb ? y : 0.f;
    }
  };
  if (kb < ke) load_stage(kb);
  for (int k0 = kb; k0 < ke; k0 += GK) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = threadIdx.x + 256 * i;
      As[ta ? e / GT : e % GK][ta ? e % GT : e / GK] = av[i];
      Bs[tb ? e % GK : e / GT][tb ? e / GK : e % GT] = bv[i];
    }
    __syncthreads();
    if (k0 + GK < ke) load_stage(k0 + GK);
#pragma unroll
    for (int ks = 0; ks < GK / 2; ++ks)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[2 * ks + lk][wm * 32 + li], Bs[2 * ks + lk][wn * 32 + li], acc,
                                                 0, 0, 0);
    __syncthreads();
  }
  const int n = n0 + wn * 32 + li;
  if (n >= N) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
    if (m >= M) continue;
    if (part) {
      part[((int64_t)blockIdx.z * M + m) * N + n] = acc[r];
      continue;
    }
    float v = alpha * acc[r];
    if (beta != 0.f) v += beta * C[(int64_t)m * ldc + n];
    if (mask && !(mask[(int64_t)m * ldm + n] > 0.f)) v = 0.f;
    C[(int64_t)m * ldc + n] = v;
  }
}

__global__ __launch_bounds__(256) void gemm_reduce(int M, int N, int S, float alpha, const float* __restrict__ part,
                                                   float beta, float* __restrict__ C, int64_t ldc,
                                                   const float* __restrict__ mask, int64_t ldm) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)M * N) return;
  const int m = (int)(idx / N), n = (int)(idx - (int64_t)m * N);
  const int64_t MN = (int64_t)M * N;
  const float acc = seg_sum8(0, S, [&](int64_t z) { return part[z * MN + idx]; });
  float v = alpha * acc;
  if (beta != 0.f) v += beta * C[(int64_t)m * ldc + n];
  if (mask && !(mask[(int64_t)m * ldm + n] > 0.f)) v = 0.f;
  C[(int64_t)m * ldc + n] = v;
}

// The same reduction with one wave per output when the slices are many
// (S >= 64): lane l sums slices l, l+64, ... (8 partial sums), then a fixed
// butterfly over the lanes; the epilogue as gemm_reduce
__device__ __forceinline__ float wave_sum_fixed(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void gemm_reduce_wave(int M, int N, int S, float alpha,
                                                        const float* __restrict__ part, float beta,
                                                        float* __restrict__ C, int64_t ldc,
                                                        const float* __restrict__ mask, int64_t ldm) {
  const int64_t idx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (idx >= (int64_t)M * N) return;
  const int64_t MN = (int64_t)M * N;
  const int ns = S > lane ? (S - lane + 63) / 64 : 0;  // slices lane, lane+64, ...
  const float acc = wave_sum_fixed(seg_sum8(0, ns, [&](int64_t i) { return part[(lane + 64 * i) * MN + idx]; }));
  if (lane) return;
  const int m = (int)(idx / N), n = (int)(idx - (int64_t)m * N);
  float v = alpha * acc;
  if (beta != 0.f) v += beta * C[(int64_t)m * ldc + n];
  if (mask && !(mask[(int64_t)m * ldm + n] > 0.f)) v = 0.f;
  C[(int64_t)m * ldc + n] = v;
}

// out[n] = sum_m A[m, n] (fixed-shape tree per column; one block per column)
__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ A, int64_t lda, int M, int N,
                                                      float* __restrict__ out) {
  __shared__ float red[256];
  const int n = blockIdx.x;
  float acc = 0.f;
  for (int m = threadIdx.x; m < M; m += 256) acc += A[(int64_t)m * lda + n];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[n] = red[0];
}

// Split column sums (rs_col_sum_split): slice s of R rows -> part[s][n]
// (64 columns x 4 row lanes per block, the lanes combined in order), then
// out[n] = the slices in order (seg_sum8).  R = 256 rows, halved (down to 16)
// while there would be fewer than 64 slices, so a short matrix still spreads
// over the chip.  Deterministic for a given shape.
constexpr int CS_R = 256;
__global__ __launch_bounds__(256) void col_sum_part_kernel(const float* __restrict__ A, int64_t lda, int64_t M, int N,
                                                           int R, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int64_t m0 = (int64_t)blockIdx.y * R;
  const int64_t m1 = m0 + R < M ? m0 + R : M;
  float acc = 0.f;
  if (n < N)
    for (int64_t m = m0 + rl; m < m1; m += 4) acc += A[m * lda + n];
  red[rl][c] = acc;
  __syncthreads();
  if (rl == 0 && n < N) part[(int64_t)blockIdx.y * N + n] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

__global__ __launch_bounds__(256) void col_sum_fin_kernel(const float* __restrict__ part, int S, int N,
                                                          float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  out[n] = seg_sum8(0, S, [&](int64_t s) { return part[s * N + n]; });
}

// one wave per column when the slices are many (S >= 64; as gemm_reduce_wave)
__global__ __launch_bounds__(256) void col_sum_fin_wave(const float* __restrict__ part, int S, int N,
                                                        float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (n >= N) return;
  const int ns = S > lane ? (S - lane + 63) / 64 : 0;
  const float v = wave_sum_fixed(seg_sum8(0, ns, [&](int64_t i) { return part[(lane + 64 * i) * (int64_t)N + n]; }));
  if (lane == 0) out[n] = v;
}

// w -= lr * (g + 2 l2 w)
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ w, const float* __restrict__ g, int64_t n,
                                                  float lr, float l2) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    w[i] -= lr * (g[i] + 2.f * l2 * w[i]);
}

// The same update over up to SGD_MT tensors in one launch: tensor j owns
// blocks [first[j], first[j+1]) of 1024 elements (4 per thread).
constexpr int SGD_MT = 32;
struct SgdMulti {
  float* w[SGD_MT];
  const float* g[SGD_MT];
  int64_t n[SGD_MT];
  float l2[SGD_MT];
  int first[SGD_MT + 1];
  int count;
  float lr;
};
__global__ __launch_bounds__(256) void sgd_multi_kernel(const SgdMulti a) {
  const int blk = blockIdx.x;
  int j = 0;
  while (j + 1 < a.count && blk >= a.first[j + 1]) ++j;  // uniform, <= 32 steps
  float* __restrict__ w = a.w[j];
  const float* __restrict__ g = a.g[j];
  const int64_t base = (int64_t)(blk - a.first[j]) * 1024 + threadIdx.x;
  const float lr = a.lr, l2 = a.l2[j];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = base + 256 * u;
    if (i < a.n[j]) w[i] -= lr * (g[i] + 2.f * l2 * w[i]);
  }
}

// DeepFM head: z = c_fm*fm + c_dnn*dnn, g = (sigmoid(z) - t)/B, outputs
// g_fm = c_fm*g, g_dnn = c_dnn*g (dL/dfm, dL/ddnn) and the BCE loss.
__global__ __launch_bounds__(256) void head_grad_kernel(const float* __restrict__ fm, const float* __restrict__ dnn,
                                                        const float* __restrict__ t, int64_t B, float c_fm,
                                                        float c_dnn, float scale, float* __restrict__ g_fm,
                                                        float* __restrict__ g_dnn, float* __restrict__ loss) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float z = c_fm * fm[b] + c_dnn * dnn[b];
  // scale = 0: the batch mean 1/B (rs_head_grad)
  const float g = scale == 0.f ? (sigmoidf_(z) - t[b]) / (float)B : scale * (sigmoidf_(z) - t[b]);
  g_fm[b] = c_fm * g;
  g_dnn[b] = c_dnn * g;
  if (loss) loss[b] = fmaxf(z, 0.f) - z * t[b] + log1pf(expf(-fabsf(z)));
}

// PNN's training loss (model/pnn.py:79): tf.reduce_mean(
// losses.binary_crossentropy(y[B], pre[B,1])) on the DNN's LOGIT (no
// sigmoid), i.e. Keras' probability form: pre clipped to [eps, 1-eps], eps =
// 1e-7, and the label vector broadcast against the [B,1] output, so per
// sample i the loss is the mean over j of BCE(y_j, pre_i):
//   loss_i = -(ybar log(q_i + eps) + (1 - ybar) log(1 - q_i + eps)),
//   q_i = clip(pre_i), ybar = mean_j y_j,
//   dL/dpre_i = (-ybar/(q_i + eps) + (1 - ybar)/(1 - q_i + eps)) / B inside
//   the clip range, 0 outside (tf.clip_by_value's gradient).
// One workgroup: ybar by a fixed-order tree, then every sample.
__global__ __launch_bounds__(1024) void bce_prob_grad_kernel(const float* __restrict__ pre, int64_t ldp,
                                                             const float* __restrict__ t, int64_t B,
                                                             float* __restrict__ g, float* __restrict__ loss) {
  __shared__ float red[1024];
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 1024) acc += t[b];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const float ybar = red[0] / (float)B;
  const float eps = 1e-7f;
  for (int64_t b = threadIdx.x; b < B; b += 1024) {
    const float p = pre[b * ldp];
    const float q = fminf(fmaxf(p, eps), 1.f - eps);
    const bool inside = p >= eps && p <= 1.f - eps;
    g[b] = inside ? (-ybar / (q + eps) + (1.f - ybar) / (1.f - q + eps)) / (float)B : 0.f;
    if (loss) loss[b] = -(ybar * logf(q + eps) + (1.f - ybar) * logf(1.f - q + eps));
  }
}

// InnerProductLayer backward (layer/interaction.py:170-183, pairs i < j in
// row-major order p(i,j) = i(2F-i-1)/2 + j-i-1): with the DNN's gradient
// w.r.t. its input [flat | inner], de[b,i,:] = dflat[b,i,:] + sum_{j != i}
// dinner[b, p(i,j)] e[b,j,:].  One wave per sample; the sample's rows and
// pair gradients staged in LDS; the j sum in fixed order.
constexpr int IPB_MAXF = 64, IPB_MAXK = 64;
__global__ __launch_bounds__(256) void inner_product_bwd_kernel(const float* __restrict__ e, int64_t lde,
                                                                const float* __restrict__ dinner, int64_t ldi,
                                                                const float* __restrict__ dflat, int64_t ldf, int F,
                                                                int k, int64_t B, float* __restrict__ de,
                                                                int64_t ldo) {
  __shared__ float se[4][IPB_MAXF * IPB_MAXK];
  __shared__ float sp[4][IPB_MAXF * (IPB_MAXF - 1) / 2];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + w;
  if (b >= B) return;  // wave-uniform; no block barrier below
  const int n = F * k, P = F * (F - 1) / 2;
  for (int t = lane; t < n; t += 64) se[w][t] = e[b * lde + t];
  for (int t = lane; t < P; t += 64) sp[w][t] = dinner[b * ldi + t];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  for (int t = lane; t < n; t += 64) {
    const int i = t / k, f = t - i * k;
    float acc = dflat[b * ldf + t];
    for (int j = 0; j < F; ++j) {
      if (j == i) continue;
      const int lo = i < j ? i : j, hi = i < j ? j : i;
      acc = fmaf(sp[w][lo * (2 * F - lo - 1) / 2 + hi - lo - 1], se[w][j * k + f], acc);
    }
    de[b * ldo + t] = acc;
  }
}

// FM gradient w.r.t. x: dx[b,i] (+)= g_b (w1_i + sum_f v_if s_bf - x_bi
// sum_f v_if^2); one thread per (b, i).  s rows lds apart, g ldg apart
// (the sharded backward reads both out of interleaved [s | g] records);
// ACC: accumulate into dx, else store.
template <bool ACC>
__global__ __launch_bounds__(256) void fm_x_grad_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ s, int64_t lds,
                                                        const float* __restrict__ w1, const float* __restrict__ v,
                                                        int64_t B, int d, int kfm, const float* __restrict__ g,
                                                        int64_t ldg, float* __restrict__ dx, int64_t lddx) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * d) return;
  const int64_t b = idx / d;
  const int i = (int)(idx - b * d);
  float vs = 0.f, vv = 0.f;
  for (int f = 0; f < kfm; ++f) {
    const float vf = v[(int64_t)i * kfm + f];
    vs = fmaf(vf, s[b * lds + f], vs);
    vv = fmaf(vf, vf, vv);
  }
  const float r = g[b * ldg] * ((w1[i] + vs) - x[b * ldx + i] * vv);
  if (ACC) dx[b * lddx + i] += r;
  else dx[b * lddx + i] = r;
}

// FM parameter gradients (without the l2 terms), kfm <= KF: one block per
// feature i (block d: dw0 = sum_b g_b), fixed-shape trees over the batch,
//   dw1_i = sum_b g_b x_bi,  dv_if = sum_b g_b x_bi s_bf - (sum_b g_b x_bi^2) v_if;
// KF is a compile-time bound so the KF + 2 partial sums stay in registers
template <int KF>
__global__ __launch_bounds__(256) void fm_param_grad_col(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ s, int64_t lds,
                                                         const float* __restrict__ v, int64_t B, int d, int kfm,
                                                         const float* __restrict__ g, int64_t ldg,
                                                         float* __restrict__ dw1, float* __restrict__ dv,
                                                         float* __restrict__ dw0) {
  __shared__ float red[KF + 2][256];
  const int i = blockIdx.x;
  float acc[KF + 2];
#pragma unroll
  for (int q = 0; q < KF + 2; ++q) acc[q] = 0.f;
  if (i == d) {
    for (int64_t b = threadIdx.x; b < B; b += 256) acc[0] += g[b * ldg];
  } else {
    for (int64_t b = threadIdx.x; b < B; b += 256) {
      const float xv = x[b * ldx + i];
      const float xg = g[b * ldg] * xv;
#pragma unroll
      for (int f = 0; f < KF; ++f) {
        const float sv = s[b * lds + (f < kfm ? f : 0)];
        acc[f] = fmaf(xg, f < kfm ? sv : 0.f, acc[f]);
      }
      acc[KF] += xg;
      acc[KF + 1] = fmaf(xg, xv, acc[KF + 1]);
    }
  }
#pragma unroll
  for (int q = 0; q < KF + 2; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
#pragma unroll
      for (int q = 0; q < KF + 2; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (i == d) {
    if (threadIdx.x == 0) dw0[0] = red[0][0];
    return;
  }
  if ((int)threadIdx.x < kfm) {
    const int f = threadIdx.x;
    dv[(int64_t)i * kfm + f] = red[f][0] - red[KF + 1][0] * v[(int64_t)i * kfm + f];
  }
  if (threadIdx.x == 0) dw1[i] = red[KF][0];
}

static void launch_fm_param_grads(const float* x, int64_t ldx, const float* s, int64_t lds, const float* v,
                                  int64_t B, int d, int kfm, const float* g, int64_t ldg, float* dw1, float* dv,
                                  float* dw0, hipStream_t st) {
  const unsigned grid = (unsigned)(d + (dw0 ? 1 : 0));
  if (grid == 0) return;
  if (kfm <= 16)
    fm_param_grad_col<16><<<grid, 256, 0, st>>>(x, ldx, s, lds, v, B, d, kfm, g, ldg, dw1, dv, dw0);
  else
    fm_param_grad_col<32><<<grid, 256, 0, st>>>(x, ldx, s, lds, v, B, d, kfm, g, ldg, dw1, dv, dw0);
}


// Sharded FM backward, owner side: x rows of the owned slots of every
// (requester, sample) record, [n_pairs][n_owned * k] (absent slot -> 0).
__global__ __launch_bounds__(256) void owner_rows_kernel(const int32_t* __restrict__ recv, int64_t rec, int n_owned,
                                                         const float* __restrict__ shard, int64_t shard_rows, int k,
                                                         int64_t n_pairs, float* __restrict__ xo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t w = (int64_t)n_owned * k;
  if (idx >= n_pairs * w) return;
  const int64_t p = idx / w;
  const int e = (int)(idx - p * w);
  const int u = e / k;
  const int64_t r = recv[p * rec + u];
  xo[idx] = (r >= 0 && r < shard_rows) ? shard[r * k + (e - u * k)] : 0.f;
}

// ------------------------------------------ OuterProductLayer backward
// layer/interaction.py:200-215: o_p = e_j^T W_p e_i with W_p[a][c] = W[a,p,c]
// (W [k, P, k]), i = row(p) < j = col(p).  With g = dL/do:
//   de_f += sum_{j>f} g_p (e_j W_p) + sum_{i<f} g_p (e_i W_p^T)    (outer_bwd)
//   dW[a,p,c] = sum_b g_bp e_j[b,a] e_i[b,c]                       (outer_w_grad)
// Both on v_mfma_f32_16x16x4f32 (k <= 16 padded to 16 columns): the scaling by
// g rides in the A fragment, so every field's contributions accumulate in one
// MFMA chain in pair order (deterministic).
__device__ __forceinline__ int pair_of(int i, int j, int F) { return i * (2 * F - i - 1) / 2 + j - i - 1; }

// one workgroup per 16-sample tile: the tile's [16][F*k] embeddings in LDS;
// wave w owns fields f = w, w + NW, ... and adds its MFMA tile into demb
__global__ __launch_bounds__(1024) void outer_bwd_kernel(const float* __restrict__ emb, int64_t lde,
                                                         const float* __restrict__ dout, int64_t ldd,
                                                         const float* __restrict__ W, int F, int k, int64_t B,
                                                         float* __restrict__ demb, int64_t lddm) {
  extern __shared__ float se[];
  const int Fk = F * k, LS = Fk + 1, P = F * (F - 1) / 2;
  const int64_t b0 = (int64_t)blockIdx.x * 16;
  for (int e = threadIdx.x; e < 16 * Fk; e += 1024) {
    const int r = e / Fk, c = e - r * Fk;
    const int64_t b = b0 + r < B ? b0 + r : B - 1;
    se[r * LS + c] = emb[b * lde + c];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s = lane & 15, kk = lane >> 4;
  const int64_t bs = b0 + s < B ? b0 + s : B - 1;
  const bool vs = b0 + s < B;
  for (int f = w; f < F; f += 16) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int o = 0; o < F; ++o) {
      if (o == f) continue;
      const int p = o > f ? pair_of(f, o, F) : pair_of(o, f, F);
      const float gx = dout[bs * ldd + p];
      const float g = vs ? gx : 0.f;
      const float* eo = se + s * LS + o * k;
      for (int k0 = 0; k0 < k; k0 += 4) {
        const int kr = k0 + kk;
        const float av = kr < k ? g * eo[kr] : 0.f;
        // B[kr][col]: W[kr, p, col] (e_o W_p, o = j > f) or W[col, p, kr] (e_o W_p^T, o = i < f)
        const int ac = s < k ? s : 0, ak = kr < k ? kr : 0;
        const float wx = o > f ? W[((int64_t)ak * P + p) * k + ac] : W[((int64_t)ac * P + p) * k + ak];
        const float bv = (s < k && kr < k) ? wx : 0.f;
        acc = mfma16x16x4(av, bv, acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t b = b0 + 4 * kk + r;
      if (b < B && s < k) demb[b * lddm + (int64_t)f * k + s] += acc[r];
    }
  }
}

// one workgroup per pair: 4 waves stride the batch 4 samples per MFMA, the
// 4 partial tiles added in wave order
__global__ __launch_bounds__(256) void outer_w_grad_kernel(const float* __restrict__ emb, int64_t lde,
                                                           const float* __restrict__ dout, int64_t ldd, int F, int k,
                                                           int64_t B, float* __restrict__ dW) {
  __shared__ floatx4 red[4][64];
  const int p = blockIdx.x, P = F * (F - 1) / 2;
  int i = 0, rem = p;
  while (rem >= F - 1 - i) {
    rem -= F - 1 - i;
    ++i;
  }
  const int j = i + 1 + rem;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s = lane & 15, kk = lane >> 4;
  const int sc = s < k ? s : 0;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t bb = 4 * w; bb < B; bb += 16) {
    const int64_t b = bb + kk;
    const int64_t bc = b < B ? b : B - 1;  // clamped: the loads stay unconditional
    const float g = dout[bc * ldd + p];
    const float ej = emb[bc * lde + (int64_t)j * k + sc];
    const float ei = emb[bc * lde + (int64_t)i * k + sc];
    const bool ok = b < B && s < k;
    // A[row a = s][kdim = kk] = g_b e_j[b][a];  B[kdim = kk][col c = s] = e_i[b][c]
    acc = mfma16x16x4(ok ? g * ej : 0.f, ok ? ei : 0.f, acc);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0) {
    floatx4 t = red[0][lane];
#pragma unroll
    for (int u = 1; u < 4; ++u) t += red[u][lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 4 * kk + r;
      if (a < k && s < k) dW[((int64_t)a * P + p) * k + s] = t[r];
    }
  }
}

// ------------------------------------------- NFM Bi-Interaction backward
// model/nfm.py:28 on [B, F, k]: bi_c = 0.5((sum_f e_fc)^2 - sum_f e_fc^2) ->
// de_fc = dbi_c (S_c - e_fc), S_c = sum_f e_fc (fields summed in order).
// One thread per (sample, column).
__global__ __launch_bounds__(256) void bi_interaction_bwd_kernel(const float* __restrict__ emb, int64_t lde,
                                                                 const float* __restrict__ dbi, int64_t ldd, int F,
                                                                 int k, int64_t B, float* __restrict__ demb,
                                                                 int64_t lddm) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= B * k) return;
  const int64_t b = t / k;
  const int c = (int)(t - b * k);
  const float* e = emb + b * lde + c;
  float S = 0.f;
  for (int f = 0; f < F; ++f) S += e[(int64_t)f * k];
  const float g = dbi[b * ldd + c];
  for (int f = 0; f < F; ++f) demb[b * lddm + (int64_t)f * k + c] = g * (S - e[(int64_t)f * k]);
}

// ------------------------------------------- row-sparse SGD of the tables
template <int KIND>
__global__ __launch_bounds__(256) void emb_keys_kernel(const void* ids, int64_t id_stride,
                                                       const int64_t* __restrict__ offs,
                                                       const int64_t* __restrict__ vocab, int F, int64_t B,
                                                       uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                                                       int* err) {
  typedef Ids<KIND> I;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= B * F) return;
  const int64_t b = j / F;
  const int c = (int)(j - b * F);
  int64_t id;
  const bool ok = I::decode(I::load(ids, b * id_stride + c), vocab[c], id);
  if (!ok) flag_error(err);
  key[j] = ok ? (uint32_t)(offs[c] + id) : 0xffffffffu;  // bad ids sort last and are skipped
  val[j] = (uint32_t)j;
}

// Sorted lookups -> table[r] -= lr * (sum of the segment's gradient rows);
// grad row of lookup j = b*F + c at grad[b*ldg + c*k].  One thread per
// (position, column): the k columns of a segment are summed by k adjacent
// lanes, in chunk pieces (seg_piece / seg_cross, rs_common.hpp), so a hot row
// (the DIN padding id: 10^5 lookups per batch) stays parallel and the result
// bitwise reproducible.
// (grad row of lookup (b, c) at grad[b*ldg + c*gfs]: gfs = k for one row per
// lookup, 0 for one row per sample shared by its fields — FFM)
__global__ __launch_bounds__(256) void emb_piece_kernel(const uint32_t* __restrict__ key,
                                                        const uint32_t* __restrict__ val, int64_t n, int F, int k,
                                                        const float* __restrict__ grad, int64_t ldg, int64_t gfs,
                                                        float lr, int64_t C, float* __restrict__ part_first,
                                                        float* __restrict__ part_last, float* __restrict__ table) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t p = t / k;
  const int f = (int)(t - p * k);
  if (p >= n) return;
  uint32_t r;
  float s;
  // 32 gathers in flight per round: a hot row's chunk-long piece (the padding
  // id of a DIN history) is 8 dependent rounds, not 32 (positions < 2^31)
  if (seg_piece<32>(key, n, C, p, k, f, [&](int64_t q) {
        const uint32_t j = val[q];
        const uint32_t b = j / (uint32_t)F;
        const int cc = (int)(j - b * (uint32_t)F);
        return grad[(int64_t)b * ldg + (int64_t)cc * gfs + f];
      }, part_first, part_last, r, s))
    table[(int64_t)r * k + f] -= lr * s;
}

__global__ __launch_bounds__(256) void emb_cross_kernel(const uint32_t* __restrict__ key, int64_t n, int k,
                                                        float lr, int64_t C, const float* __restrict__ part_first,
                                                        const float* __restrict__ part_last,
                                                        float* __restrict__ table) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t p = t / k;
  const int f = (int)(t - p * k);
  if (p >= n) return;
  uint32_t r;
  float s;
  if (seg_cross(key, n, C, p, k, f, part_first, part_last, r, s)) table[(int64_t)r * k + f] -= lr * s;
}

// ------------------------------------------------------ CrossNet training
// layer/interaction.py:75-83: x_{l+1} = x0 (x_l . w_l) + b_l + x_l.
// Forward, one wave per sample: every x_l (l = 1..L; x_0 = x0 itself) and
// g_l = x_l . w_l are kept for the backward; x_L also goes to xl_out (the
// output Dense's input, row stride ldo).
constexpr int CR_MAXE = 32;  // d <= 64 * CR_MAXE

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void cross_train_fwd(const float* __restrict__ x0, int64_t ldx, int d, int L,
                                                       const float* __restrict__ W, const float* __restrict__ Bv,
                                                       int64_t B, float* __restrict__ xs, float* __restrict__ gl,
                                                       float* __restrict__ xl_out, int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // wave-uniform
  const int ne = (d + 63) / 64;
  float x0r[CR_MAXE], xr[CR_MAXE];
#pragma unroll
  for (int t = 0; t < CR_MAXE; ++t) {
    const int e = lane + 64 * t;
    x0r[t] = (t < ne && e < d) ? x0[b * ldx + e] : 0.f;
    xr[t] = x0r[t];
  }
  for (int l = 0; l < L; ++l) {
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < CR_MAXE; ++t) {
      const int e = lane + 64 * t;
      if (t < ne && e < d) dot = fmaf(xr[t], W[(int64_t)l * d + e], dot);
    }
    const float g = wave_sum(dot);
    if (lane == 0) gl[(int64_t)l * B + b] = g;
    float* xo = xs + ((int64_t)l * B + b) * d;  // x_{l+1}
#pragma unroll
    for (int t = 0; t < CR_MAXE; ++t) {
      const int e = lane + 64 * t;
      if (t < ne && e < d) {
        xr[t] = fmaf(x0r[t], g, Bv[(int64_t)l * d + e]) + xr[t];
        xo[e] = xr[t];
      }
    }
  }
  if (xl_out) {
#pragma unroll
    for (int t = 0; t < CR_MAXE; ++t) {
      const int e = lane + 64 * t;
      if (t < ne && e < d) xl_out[b * ldo + e] = xr[t];
    }
  }
}

// Backward, one wave per sample, from delta_L = dL/dx_L (row stride ldd):
// for l = L-1 .. 0:  keep delta_{l+1} (db_l = sum_b delta_{l+1}) and
// s_l = x0 . delta_{l+1} (dw_l = sum_b s_l x_l); dL/dx0 += g_l delta_{l+1};
// delta_l = delta_{l+1} + s_l w_l.  Finally dx (row stride lddx) += delta_0
// + sum_l g_l delta_{l+1}.
__global__ __launch_bounds__(256) void cross_train_bwd(const float* __restrict__ x0, int64_t ldx, int d, int L,
                                                       const float* __restrict__ W, int64_t B,
                                                       const float* __restrict__ gl, const float* __restrict__ dL,
                                                       int64_t ldd, float* __restrict__ deltas,
                                                       float* __restrict__ sl, float* __restrict__ dx,
                                                       int64_t lddx) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int ne = (d + 63) / 64;
  float x0r[CR_MAXE], dr[CR_MAXE], acc[CR_MAXE];
#pragma unroll
  for (int t = 0; t < CR_MAXE; ++t) {
    const int e = lane + 64 * t;
    const bool in = t < ne && e < d;
    x0r[t] = in ? x0[b * ldx + e] : 0.f;
    dr[t] = in ? dL[b * ldd + e] : 0.f;
    acc[t] = 0.f;
  }
  for (int l = L - 1; l >= 0; --l) {
    float* dout = deltas + ((int64_t)l * B + b) * d;  // delta_{l+1}
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < CR_MAXE; ++t) {
      const int e = lane + 64 * t;
      if (t < ne && e < d) {
        dout[e] = dr[t];
        dot = fmaf(x0r[t], dr[t], dot);
      }
    }
    const float s = wave_sum(dot);
    const float g = gl[(int64_t)l * B + b];
    if (lane == 0) sl[(int64_t)l * B + b] = s;
#pragma unroll
    for (int t = 0; t < CR_MAXE; ++t) {
      const int e = lane + 64 * t;
      if (t < ne && e < d) {
        acc[t] = fmaf(g, dr[t], acc[t]);
        dr[t] = fmaf(s, W[(int64_t)l * d + e], dr[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < CR_MAXE; ++t) {
    const int e = lane + 64 * t;
    if (t < ne && e < d) dx[b * lddx + e] += dr[t] + acc[t];
  }
}

}  // namespace rs

using namespace rs;

// K slices for a launch of few output tiles (the weight gradients x^T delta:
// M x N small, K = batch): aim for ~1024 workgroups (4 per CU: each slice is
// a latency-bound chain of stages), slices of >= 64.
static int gemm_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + GT - 1) / GT) * ((N + GT - 1) / GT);
  int64_t s = 1024 / (tiles > 0 ? tiles : 1);
  s = std::min<int64_t>(s, K / 64);
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 1024));
}

extern "C" int64_t rs_gemm_workspace_size(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return -1;
  const int s = gemm_splits(M, N, K);
  return s > 1 ? (int64_t)s * M * N * 4 : 0;
}

extern "C" int rs_gemm(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                       int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                       const float* mask, int64_t ldm, void* workspace, int64_t workspace_bytes,
                       rs_stream_t stream) {
  if (M == 0 || N == 0) return RS_OK;
  RS_REQUIRE(M > 0 && N > 0 && K >= 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "rs_gemm: bad shape");
  RS_REQUIRE(C && (K == 0 || (A && B)), "rs_gemm: null pointer");
  RS_REQUIRE(lda >= (trans_a ? M : K) && ldb >= (trans_b ? K : N) && ldc >= N && (!mask || ldm >= N),
             "rs_gemm: leading dimension too small");
  hipStream_t st = as_stream(stream);
  int S = gemm_splits(M, N, K);
  if (S > 1 && (!workspace || workspace_bytes < (int64_t)S * M * N * 4)) S = 1;  // no room: one pass over K
  dim3 grid((unsigned)((N + GT - 1) / GT), (unsigned)((M + GT - 1) / GT), (unsigned)S);
  const int gk = S > 1 ? GK_SPLIT : GK;
  const int kslice = (int)((K + S - 1) / S + gk - 1) / gk * gk;
  float* part = S > 1 ? static_cast<float*>(workspace) : nullptr;
  if (part)
    gemm_kernel<GK_SPLIT><<<grid, 256, 0, st>>>(trans_a, trans_b, (int)M, (int)N, (int)K, alpha, A, lda, B, ldb, beta,
                                                C, ldc, mask, ldm, kslice, part);
  else
    gemm_kernel<GK><<<grid, 256, 0, st>>>(trans_a, trans_b, (int)M, (int)N, (int)K, alpha, A, lda, B, ldb, beta, C,
                                          ldc, mask, ldm, kslice, part);
  if (part && S >= 64 && M * N <= (1 << 20))
    gemm_reduce_wave<<<(unsigned)((M * N + 3) / 4), 256, 0, st>>>((int)M, (int)N, S, alpha, part, beta, C, ldc, mask,
                                                                 ldm);
  else if (part)
    gemm_reduce<<<(unsigned)((M * N + 255) / 256), 256, 0, st>>>((int)M, (int)N, S, alpha, part, beta, C, ldc, mask,
                                                                 ldm);
  return launch_status("rs_gemm");
}

extern "C" int rs_col_sum(const float* A, int64_t lda, int64_t M, int64_t N, float* out, rs_stream_t stream) {
  if (N == 0) return RS_OK;
  RS_REQUIRE(A && out && M >= 0 && N > 0 && M < (1ll << 31) && lda >= N, "rs_col_sum: bad arguments");
  col_sum_kernel<<<(unsigned)N, 256, 0, as_stream(stream)>>>(A, lda, (int)M, (int)N, out);
  return launch_status("rs_col_sum");
}

static int col_sum_rows(int64_t M) {
  int R = CS_R;
  while (R > 16 && (M + R - 1) / R < 64) R >>= 1;
  return R;
}
static int64_t col_sum_slices(int64_t M) { return (M + col_sum_rows(M) - 1) / col_sum_rows(M); }

extern "C" int64_t rs_col_sum_workspace_size(int64_t M, int64_t N) {
  if (M < 0 || N < 0) return -1;
  const int64_t S = col_sum_slices(M);
  return S > 1 ? S * N * 4 : 0;
}

static void col_sum_launch(const float* A, int64_t lda, int64_t M, int64_t N, float* out, void* ws, int64_t ws_bytes,
                           hipStream_t st) {
  const int64_t S = col_sum_slices(M);
  if (S <= 1 || !ws || ws_bytes < S * N * 4 || S > (1 << 20)) {
    col_sum_kernel<<<(unsigned)N, 256, 0, st>>>(A, lda, (int)M, (int)N, out);
    return;
  }
  float* part = static_cast<float*>(ws);
  col_sum_part_kernel<<<dim3((unsigned)((N + 63) / 64), (unsigned)S), 256, 0, st>>>(A, lda, M, (int)N,
                                                                                   col_sum_rows(M), part);
  if (S >= 64 && N <= (1 << 20))
    col_sum_fin_wave<<<(unsigned)((N + 3) / 4), 256, 0, st>>>(part, (int)S, (int)N, out);
  else
    col_sum_fin_kernel<<<(unsigned)((N + 255) / 256), 256, 0, st>>>(part, (int)S, (int)N, out);
}

extern "C" int rs_col_sum_split(const float* A, int64_t lda, int64_t M, int64_t N, float* out, void* workspace,
                                int64_t workspace_bytes, rs_stream_t stream) {
  if (N == 0) return RS_OK;
  RS_REQUIRE(A && out && M >= 0 && N > 0 && M < (1ll << 31) && N < (1ll << 30) && lda >= N,
             "rs_col_sum_split: bad arguments");
  col_sum_launch(A, lda, M, N, out, workspace, workspace_bytes, as_stream(stream));
  return launch_status("rs_col_sum_split");
}

extern "C" int rs_sgd_update(float* w, const float* grad, int64_t n, float lr, float l2, rs_stream_t stream) {
  if (n == 0) return RS_OK;
  RS_REQUIRE(w && grad && n > 0, "rs_sgd_update: bad arguments");
  sgd_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 8192), 256, 0, as_stream(stream)>>>(w, grad, n, lr, l2);
  return launch_status("rs_sgd_update");
}

extern "C" int rs_sgd_update_multi(int count, float* const* w, const float* const* grad, const int64_t* n,
                                   const float* l2, float lr, rs_stream_t stream) {
  if (count == 0) return RS_OK;
  RS_REQUIRE(count > 0 && w && grad && n && l2, "rs_sgd_update_multi: bad arguments");
  for (int j = 0; j < count; ++j)
    RS_REQUIRE(w[j] && grad[j] && n[j] >= 0 && n[j] < (1ll << 40), "rs_sgd_update_multi: bad tensor %d", j);
  hipStream_t st = as_stream(stream);
  for (int j0 = 0; j0 < count;) {
    SgdMulti a{};
    a.lr = lr;
    int blocks = 0;
    // pack tensors while the grid stays below 2^30 blocks; one huge tensor
    // goes alone through sgd_kernel's grid-stride loop
    while (j0 < count && a.count < SGD_MT) {
      const int64_t nb = (n[j0] + 1023) / 1024;
      if (nb > (1 << 20)) {
        if (a.count == 0) {
          sgd_kernel<<<8192, 256, 0, st>>>(w[j0], grad[j0], n[j0], lr, l2[j0]);
          ++j0;
          continue;
        }
        break;
      }
      if (nb > 0) {
        a.w[a.count] = w[j0];
        a.g[a.count] = grad[j0];
        a.n[a.count] = n[j0];
        a.l2[a.count] = l2[j0];
        a.first[a.count] = blocks;
        blocks += (int)nb;
        ++a.count;
      }
      ++j0;
    }
    if (a.count == 0) continue;
    a.first[a.count] = blocks;
    sgd_multi_kernel<<<(unsigned)blocks, 256, 0, st>>>(a);
  }
  return launch_status("rs_sgd_update_multi");
}

extern "C" int rs_bce_prob_grad(const float* pred, int64_t pred_stride, const float* labels, int64_t batch, float* g,
                                float* loss, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(pred && labels && g && batch > 0 && pred_stride >= 1, "rs_bce_prob_grad: bad arguments");
  bce_prob_grad_kernel<<<1, 1024, 0, as_stream(stream)>>>(pred, pred_stride, labels, batch, g, loss);
  return launch_status("rs_bce_prob_grad");
}

extern "C" int rs_outer_product_bwd(const float* emb, int64_t emb_stride, const float* dout, int64_t dout_stride,
                                    const float* W, int n_fields, int k, int64_t batch, float* demb,
                                    int64_t demb_stride, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(emb && dout && W && demb && batch > 0 && n_fields >= 2 && n_fields <= 64 && k >= 1 && k <= 16 &&
                 emb_stride >= n_fields * k && demb_stride >= n_fields * k &&
                 dout_stride >= n_fields * (n_fields - 1) / 2,
             "rs_outer_product_bwd: bad arguments (2 <= n_fields <= 64, 1 <= k <= 16)");
  const size_t lds = (size_t)16 * (n_fields * k + 1) * sizeof(float);
  outer_bwd_kernel<<<(unsigned)((batch + 15) / 16), 1024, lds, as_stream(stream)>>>(
      emb, emb_stride, dout, dout_stride, W, n_fields, k, batch, demb, demb_stride);
  return launch_status("rs_outer_product_bwd");
}

extern "C" int rs_outer_product_w_grad(const float* emb, int64_t emb_stride, const float* dout, int64_t dout_stride,
                                       int n_fields, int k, int64_t batch, float* dW, rs_stream_t stream) {
  RS_REQUIRE(emb && dout && dW && batch >= 0 && n_fields >= 2 && n_fields <= 64 && k >= 1 && k <= 16 &&
                 emb_stride >= n_fields * k && dout_stride >= n_fields * (n_fields - 1) / 2,
             "rs_outer_product_w_grad: bad arguments (2 <= n_fields <= 64, 1 <= k <= 16)");
  if (batch == 0) return RS_OK;  // (dW untouched: callers size the step on a non-empty batch)
  outer_w_grad_kernel<<<(unsigned)(n_fields * (n_fields - 1) / 2), 256, 0, as_stream(stream)>>>(
      emb, emb_stride, dout, dout_stride, n_fields, k, batch, dW);
  return launch_status("rs_outer_product_w_grad");
}

extern "C" int rs_bi_interaction_bwd(const float* emb, int64_t emb_stride, const float* dbi, int64_t dbi_stride,
                                     int n_fields, int k, int64_t batch, float* demb, int64_t demb_stride,
                                     rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(emb && dbi && demb && batch > 0 && n_fields >= 1 && k >= 1 && emb_stride >= (int64_t)n_fields * k &&
                 dbi_stride >= k && demb_stride >= (int64_t)n_fields * k,
             "rs_bi_interaction_bwd: bad arguments");
  bi_interaction_bwd_kernel<<<(unsigned)((batch * k + 255) / 256), 256, 0, as_stream(stream)>>>(
      emb, emb_stride, dbi, dbi_stride, n_fields, k, batch, demb, demb_stride);
  return launch_status("rs_bi_interaction_bwd");
}

extern "C" int rs_inner_product_bwd(const float* emb, int64_t emb_stride, const float* dinner, int64_t dinner_stride,
                                    const float* dflat, int64_t dflat_stride, int n_fields, int k, int64_t batch,
                                    float* demb, int64_t demb_stride, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(emb && dinner && dflat && demb && batch > 0 && n_fields >= 2 && n_fields <= IPB_MAXF && k >= 1 &&
                 k <= IPB_MAXK && n_fields * k <= 4096 && emb_stride >= n_fields * k &&
                 dflat_stride >= n_fields * k && demb_stride >= n_fields * k &&
                 dinner_stride >= n_fields * (n_fields - 1) / 2,
             "rs_inner_product_bwd: bad arguments (2 <= n_fields <= %d, k <= %d, n_fields*k <= 4096)", IPB_MAXF,
             IPB_MAXK);
  inner_product_bwd_kernel<<<(unsigned)((batch + 3) / 4), 256, 0, as_stream(stream)>>>(
      emb, emb_stride, dinner, dinner_stride, dflat, dflat_stride, n_fields, k, batch, demb, demb_stride);
  return launch_status("rs_inner_product_bwd");
}

extern "C" int rs_head_grad(const float* fm, const float* dnn, const float* labels, int64_t batch, float c_fm,
                            float c_dnn, float* g_fm, float* g_dnn, float* loss, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(fm && dnn && labels && g_fm && g_dnn && batch > 0, "rs_head_grad: bad arguments");
  head_grad_kernel<<<(unsigned)((batch + 255) / 256), 256, 0, as_stream(stream)>>>(fm, dnn, labels, batch, c_fm,
                                                                                   c_dnn, 0.f, g_fm, g_dnn, loss);
  return launch_status("rs_head_grad");
}

extern "C" int rs_head_grad_scaled(const float* fm, const float* dnn, const float* labels, int64_t batch, float c_fm,
                                   float c_dnn, float scale, float* g_fm, float* g_dnn, float* loss,
                                   rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(fm && dnn && labels && g_fm && g_dnn && batch > 0 && scale > 0.f, "rs_head_grad_scaled: bad arguments");
  head_grad_kernel<<<(unsigned)((batch + 255) / 256), 256, 0, as_stream(stream)>>>(fm, dnn, labels, batch, c_fm,
                                                                                   c_dnn, scale, g_fm, g_dnn, loss);
  return launch_status("rs_head_grad_scaled");
}

extern "C" int rs_fm_x_grad(const float* x, int64_t ldx, const float* s, const float* w1, const float* v,
                            int64_t batch, int d, int kfm, const float* g, float* dx, int64_t lddx,
                            rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(x && s && w1 && v && g && dx && batch > 0 && d > 0 && kfm >= 1 && ldx >= d && lddx >= d,
             "rs_fm_x_grad: bad arguments");
  fm_x_grad_kernel<true><<<(unsigned)((batch * d + 255) / 256), 256, 0, as_stream(stream)>>>(
      x, ldx, s, kfm, w1, v, batch, d, kfm, g, 1, dx, lddx);
  return launch_status("rs_fm_x_grad");
}

extern "C" int rs_fm_param_grads(const float* x, int64_t ldx, const float* s, const float* v, int64_t batch, int d,
                                 int kfm, const float* g, float* dw1, float* dv, float* dw0, rs_stream_t stream) {
  RS_REQUIRE(x && s && v && g && dw1 && dv && dw0 && batch >= 0 && d > 0 && kfm >= 1 && kfm <= 32 && ldx >= d,
             "rs_fm_param_grads: bad arguments (kfm <= 32)");
  launch_fm_param_grads(x, ldx, s, kfm, v, batch, d, kfm, g, 1, dw1, dv, dw0, as_stream(stream));
  return launch_status("rs_fm_param_grads");
}

extern "C" int rs_fm_param_grads_strided(const float* x, int64_t ldx, const float* s, int64_t lds, const float* g,
                                         int64_t ldg, const float* v, int64_t batch, int d, int kfm, float* dw1,
                                         float* dv, float* dw0, rs_stream_t stream) {
  if (d == 0 && !dw0) return RS_OK;
  RS_REQUIRE((x || d == 0) && s && v && g && dw1 && dv && batch >= 0 && d >= 0 && kfm >= 1 && kfm <= 32 &&
                 ldx >= d && lds >= kfm && ldg >= 1,
             "rs_fm_param_grads_strided: bad arguments (kfm <= 32)");
  launch_fm_param_grads(x, ldx, s, lds, v, batch, d, kfm, g, ldg, dw1, dv, dw0, as_stream(stream));
  return launch_status("rs_fm_param_grads_strided");
}

extern "C" int rs_shard_owner_fm_grad(const int32_t* recv, int64_t rec_stride, int field_lo, int n_owned,
                                      const float* shard, int64_t shard_rows, int nd, int k, const float* w1,
                                      const float* v, int kfm, const float* gs, int64_t gs_stride, int64_t n_pairs,
                                      float* rows_ws, float* drows, float* dw1, float* dv, rs_stream_t stream) {
  if (n_pairs == 0 || n_owned == 0) return RS_OK;
  RS_REQUIRE(recv && shard && w1 && v && gs && rows_ws && drows && dw1 && dv, "rs_shard_owner_fm_grad: null pointer");
  RS_REQUIRE(n_pairs > 0 && n_owned > 0 && rec_stride >= n_owned && field_lo >= 0 && nd >= 0 && k >= 1 &&
                 kfm >= 1 && kfm <= 32 && gs_stride >= kfm + 1 && shard_rows >= 0,
             "rs_shard_owner_fm_grad: bad shape (kfm <= 32)");
  hipStream_t st = as_stream(stream);
  const int w = n_owned * k;
  const int64_t col = nd + (int64_t)field_lo * k;  // first FM feature of the owned fields
  owner_rows_kernel<<<(unsigned)((n_pairs * w + 255) / 256), 256, 0, st>>>(recv, rec_stride, n_owned, shard,
                                                                             shard_rows, k, n_pairs, rows_ws);
  fm_x_grad_kernel<false><<<(unsigned)((n_pairs * w + 255) / 256), 256, 0, st>>>(
      rows_ws, w, gs, gs_stride, w1 + col, v + col * kfm, n_pairs, w, kfm, gs + kfm, gs_stride, drows, w);
  launch_fm_param_grads(rows_ws, w, gs, gs_stride, v + col * kfm, n_pairs, w, kfm, gs + kfm, gs_stride, dw1, dv,
                        nullptr, st);
  return launch_status("rs_shard_owner_fm_grad");
}

static int64_t emb_sort_bytes(int64_t n) { return sort_pairs_ws_bytes(n); }

extern "C" int64_t rs_embedding_sgd_workspace_size(int64_t n_lookups) {
  if (n_lookups < 0) return -1;
  return 5 * ((n_lookups * 4 + 255) / 256 * 256) + (emb_sort_bytes(n_lookups) + 255) / 256 * 256;
}

extern "C" int rs_embedding_sgd_strided(float* table, int64_t n_rows, int k, const void* ids, int id_kind,
                                        int64_t id_stride, const int64_t* field_offsets, const int64_t* field_vocab,
                                        int n_fields, int64_t batch, const float* grad, int64_t grad_stride,
                                        int64_t grad_field_stride, float lr, void* workspace, int* err_flag,
                                        rs_stream_t stream) {
  const int64_t n = batch * n_fields;
  if (n == 0) return RS_OK;
  RS_REQUIRE(table && ids && field_offsets && field_vocab && grad && workspace && k >= 1 && batch > 0 &&
                 grad_field_stride >= 0 && grad_stride >= (int64_t)(n_fields - 1) * grad_field_stride + k,
             "rs_embedding_sgd: bad arguments");
  RS_REQUIRE(n_rows < 0xffffffffll && n < (1ll << 31), "rs_embedding_sgd: rows must fit uint32, lookups int32");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embedding_sgd: bad id_kind");
  const int64_t slab = (n * 4 + 255) / 256 * 256;
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  uint32_t* key_in = reinterpret_cast<uint32_t*>(ws);
  uint32_t* key_out = reinterpret_cast<uint32_t*>(ws + slab);
  uint32_t* val_in = reinterpret_cast<uint32_t*>(ws + 2 * slab);
  uint32_t* val_out = reinterpret_cast<uint32_t*>(ws + 3 * slab);
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    emb_keys_kernel<decltype(K)::value><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
        ids, id_stride, field_offsets, field_vocab, n_fields, batch, key_in, val_in, err_flag);
  });
  // 2^bits > n_rows: a bad id's key 0xffffffff keeps its low bits all set,
  // so it still sorts after every valid row
  int bits = 1;
  while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)n_rows) ++bits;
  const hipError_t e = sort_pairs_u32(key_in, val_in, key_out, val_out, n, bits, ws + 5 * slab, st);
  if (e != hipSuccess) {
    set_error("rs_embedding_sgd: radix sort failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  const int64_t C = seg_chunk(k);
  const int64_t nchunk = (n + C - 1) / C;
  float* part_first = reinterpret_cast<float*>(ws + 4 * slab);
  float* part_last = part_first + nchunk * k;
  const unsigned g = (unsigned)((n * k + 255) / 256);
  emb_piece_kernel<<<g, 256, 0, st>>>(key_out, val_out, n, n_fields, k, grad, grad_stride, grad_field_stride, lr, C,
                                      part_first, part_last, table);
  if (nchunk > 1) emb_cross_kernel<<<g, 256, 0, st>>>(key_out, n, k, lr, C, part_first, part_last, table);
  return launch_status("rs_embedding_sgd");
}

extern "C" int rs_embedding_sgd(float* table, int64_t n_rows, int k, const void* ids, int id_kind, int64_t id_stride,
                                const int64_t* field_offsets, const int64_t* field_vocab, int n_fields,
                                int64_t batch, const float* grad, int64_t grad_stride, float lr, void* workspace,
                                int* err_flag, rs_stream_t stream) {
  if (batch * n_fields == 0) return RS_OK;
  RS_REQUIRE(grad_stride >= (int64_t)n_fields * k, "rs_embedding_sgd: bad arguments");
  return rs_embedding_sgd_strided(table, n_rows, k, ids, id_kind, id_stride, field_offsets, field_vocab, n_fields,
                                  batch, grad, grad_stride, k, lr, workspace, err_flag, stream);
}

extern "C" int rs_cross_train_fwd(const float* x0, int64_t ldx, int d, int n_layers, const float* W, const float* b,
                                  int64_t batch, float* xs, float* g, float* xl_out, int64_t ldo,
                                  rs_stream_t stream) {
  if (batch == 0 || n_layers == 0) return RS_OK;
  RS_REQUIRE(x0 && W && b && xs && g && batch > 0 && d >= 1 && d <= 64 * CR_MAXE && n_layers > 0 && ldx >= d &&
                 (!xl_out || ldo >= d),
             "rs_cross_train_fwd: bad arguments (d <= %d)", 64 * CR_MAXE);
  cross_train_fwd<<<(unsigned)((batch + 3) / 4), 256, 0, as_stream(stream)>>>(x0, ldx, d, n_layers, W, b, batch, xs,
                                                                              g, xl_out, ldo);
  return launch_status("rs_cross_train_fwd");
}

extern "C" int rs_cross_train_bwd(const float* x0, int64_t ldx, int d, int n_layers, const float* W, int64_t batch,
                                  const float* g, const float* dxl, int64_t lddxl, float* deltas, float* s,
                                  float* dx, int64_t lddx, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(x0 && dxl && dx && batch > 0 && d >= 1 && d <= 64 * CR_MAXE && n_layers >= 0 && ldx >= d &&
                 lddxl >= d && lddx >= d && (n_layers == 0 || (W && g && deltas && s)),
             "rs_cross_train_bwd: bad arguments (d <= %d)", 64 * CR_MAXE);
  cross_train_bwd<<<(unsigned)((batch + 3) / 4), 256, 0, as_stream(stream)>>>(x0, ldx, d, n_layers, W, batch, g, dxl,
                                                                              lddxl, deltas, s, dx, lddx);
  return launch_status("rs_cross_train_bwd");
}

// ------------------------------------------------------------------ dropout
// Inverted dropout of DNNLayer (layer/interaction.py:35,44: Dropout(0.2)
// after every hidden layer, active under compile_fit's model.fit,
// utils/compile_fit.py:14): x <- x * keep / (1 - rate), keep = (u >= rate)
// as tf.nn.dropout.  TF's own random draws cannot be reproduced, so the mask
// comes from a counter-based generator: Philox4x32-10 (Salmon et al., SC'11)
// with key = seed and counter = (offset + e) / 4 for element e = row * cols +
// col of the call; word (offset + e) % 4 of the block gives
// u = (word >> 8) * 2^-24.  The same (seed, offset) regenerates the mask, so
// the backward multiplies dL/dx by the same keep / (1 - rate) without storing
// it; oracle.dropout_multiplier restates it bit for bit.
namespace rs {
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
    c[0] = n0;
    c[1] = n1;
    c[2] = n2;
    c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// one thread per 4-element counter block of the call's [rows, cols] range;
// base (rs_dropout_at): the offset is *base + offset, read on the device
__global__ __launch_bounds__(256) void dropout_kernel(float* __restrict__ x, int64_t ld, int64_t rows, int64_t cols,
                                                      float rate, float scale, uint32_t k0, uint32_t k1,
                                                      uint64_t offset, const uint64_t* __restrict__ base) {
  if (base) offset += *base;
  const int64_t n = rows * cols, nblk = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nblk; q += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t ctr = (offset >> 2) + (uint64_t)q;
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    philox4x32_10(c, k0, k1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = 4 * q + j;
      if (e < n) {
        const float u = (float)(c[j] >> 8) * (1.0f / 16777216.0f);
        const int64_t r = e / cols, col = e - r * cols;
        float* p = x + r * ld + col;
        *p = u >= rate ? *p * scale : 0.f;
      }
    }
  }
}
}  // namespace rs

extern "C" int rs_dropout(float* x, int64_t ld, int64_t rows, int64_t cols, float rate, uint64_t seed,
                          uint64_t offset, rs_stream_t stream) {
  if (rows == 0 || cols == 0) return RS_OK;
  RS_REQUIRE(x && rows > 0 && cols > 0 && ld >= cols, "rs_dropout: bad arguments");
  RS_REQUIRE(rate >= 0.f && rate < 1.f, "rs_dropout: rate must be in [0, 1)");
  RS_REQUIRE(offset % 4 == 0, "rs_dropout: offset must be a multiple of 4");
  const int64_t nblk = (rows * cols + 3) / 4;
  const int grid = (int)std::min<int64_t>((nblk + 255) / 256, 8192);
  dropout_kernel<<<grid, 256, 0, as_stream(stream)>>>(x, ld, rows, cols, rate, 1.0f / (1.0f - rate), (uint32_t)seed,
                                                      (uint32_t)(seed >> 32), offset, nullptr);
  return launch_status("rs_dropout");
}

namespace rs {
__global__ void dropout_advance_kernel(uint64_t* base, uint64_t inc) {
  if (threadIdx.x == 0) base[0] += inc;
}
}  // namespace rs

extern "C" int rs_dropout_at(float* x, int64_t ld, int64_t rows, int64_t cols, float rate, uint64_t seed,
                             const uint64_t* base, uint64_t offset, rs_stream_t stream) {
  if (rows == 0 || cols == 0) return RS_OK;
  RS_REQUIRE(x && base && rows > 0 && cols > 0 && ld >= cols, "rs_dropout_at: bad arguments");
  RS_REQUIRE(rate >= 0.f && rate < 1.f, "rs_dropout_at: rate must be in [0, 1)");
  RS_REQUIRE(offset % 4 == 0, "rs_dropout_at: offset must be a multiple of 4");
  const int64_t nblk = (rows * cols + 3) / 4;
  const int grid = (int)std::min<int64_t>((nblk + 255) / 256, 8192);
  dropout_kernel<<<grid, 256, 0, as_stream(stream)>>>(x, ld, rows, cols, rate, 1.0f / (1.0f - rate), (uint32_t)seed,
                                                      (uint32_t)(seed >> 32), offset, base);
  return launch_status("rs_dropout_at");
}

extern "C" int rs_dropout_advance(uint64_t* base, uint64_t inc, rs_stream_t stream) {
  RS_REQUIRE(base && inc % 4 == 0, "rs_dropout_advance: bad arguments");
  if (inc == 0) return RS_OK;
  dropout_advance_kernel<<<1, 64, 0, as_stream(stream)>>>(base, inc);
  return launch_status("rs_dropout_advance");
}
