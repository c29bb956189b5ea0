// dense.hip — Keras Dense (+activation) for the DNN towers (DNNLayer,
// layer/interaction.py:30-46; DIN MLP, model/din.py:51-54,89-95), per-column
// affine (BatchNormalization at inference, model/din.py:89) and the sigmoid
// model heads (model/deepFM.py:30, model/dcn.py:33, model/fm.py:22).
//
// GEMM: y[M,N] = act(x[M,K] @ W[K,N] + bias) in fp32 on
// v_mfma_f32_32x32x2_f32 (exact f32 FMA chain).  Workgroup tile 64x64, four
// waves in 2x2, each a 32x32 accumulator (16 AGPR/VGPR per lane); K staged
// through LDS 16 deep, double-buffered through registers (the next tile's
// global loads are issued before the current tile's MFMAs).  LDS images are
// k-major so both operand reads are contiguous 128-B rows (conflict-free
// ds_read_b32).  Bias + ReLU/PReLU/sigmoid are fused into the epilogue.
#include "rs_common.hpp"

namespace rs {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 64, GBN = 64, GBK = 16;

struct DenseArgs {
  const float* x;
  int64_t xs;
  const float* W;
  const float* bias;
  const float* alpha;
  int act;
  float* y;
  int64_t ys;
  int64_t M;
  int K, N;
  int arows;  // PReLU alpha rows: 1 = alpha[n]; > 1 = alpha[(m % arows) * N + n]
};

// PReLU slope of output (m, n): per column, or per (row mod arows, column) —
// Keras PReLU() on a 3-D input [B, T, N] flattened to [B*T, N] has alpha [T, N]
__device__ __forceinline__ float prelu_alpha(const DenseArgs& a, int64_t m, int n, float col_alpha) {
  return a.arows > 1 ? a.alpha[(m % a.arows) * a.N + n] : col_alpha;
}

__device__ __forceinline__ float apply_act(float v, int act, float alpha) {
  switch (act) {
    case RS_ACT_RELU: return fmaxf(v, 0.f);
    case RS_ACT_PRELU: return fmaxf(v, 0.f) + alpha * fminf(v, 0.f);
    case RS_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}

__global__ __launch_bounds__(256) void dense_mfma(DenseArgs a) {
  __shared__ float As[2][GBK][GBM + 4];
  __shared__ float Bs[2][GBK][GBN + 4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.y * GBM;
  const int n0 = blockIdx.x * GBN;
  // global->register staging: A: 64 rows x 16 k (4 per thread), B: 16 k x 64 cols (4 per thread)
  const int ar = tid >> 2, ak = (tid & 3) * 4;
  const int bk = tid >> 4, bn = (tid & 15) * 4;
  float ra[4], rb[4];
  auto load_tiles = [&](int k0) {
    const int64_t m = m0 + ar;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kq = k0 + ak + q;
      ra[q] = (m < a.M && kq < a.K) ? a.x[m * a.xs + kq] : 0.f;
    }
    const int kb = k0 + bk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nq = n0 + bn + q;
      rb[q] = (kb < a.K && nq < a.N) ? a.W[(int64_t)kb * a.N + nq] : 0.f;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) As[buf][ak + q][ar] = ra[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) Bs[buf][bk][bn + q] = rb[q];
  };

  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int nk = (a.K + GBK - 1) / GBK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles((kt + 1) * GBK);
#pragma unroll
    for (int ks = 0; ks < GBK / 2; ++ks) {
      const float av = As[cur][2 * ks + lk][wm * 32 + li];
      const float bv = Bs[cur][2 * ks + lk][wn * 32 + li];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }
  // epilogue: lane holds col = lane&31, rows (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int n = n0 + wn * 32 + li;
  if (n < a.N) {
    const float bz = a.bias ? a.bias[n] : 0.f;
    const bool pre = a.act == RS_ACT_PRELU && a.alpha;
    const float al = (pre && a.arows <= 1) ? a.alpha[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
      if (m < a.M) a.y[m * a.ys + n] = apply_act(acc[r] + bz, a.act, pre ? prelu_alpha(a, m, n, al) : 0.f);
    }
  }
}

// Small-N path (N <= 4, e.g. the 64->1 output layer): one wave per row chunk,
// lanes split K, shuffle reduction.
__global__ __launch_bounds__(256) void dense_small_n(DenseArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t m = wave; m < a.M; m += nwaves) {
    for (int n = 0; n < a.N; ++n) {
      float p = 0.f;
      for (int k = lane; k < a.K; k += 64) p = fmaf(a.x[m * a.xs + k], a.W[(int64_t)k * a.N + n], p);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
      if (lane == 0) {
        const float bz = a.bias ? a.bias[n] : 0.f;
        const float al = (a.act == RS_ACT_PRELU && a.alpha) ? prelu_alpha(a, m, n, a.alpha[n]) : 0.f;
        a.y[m * a.ys + n] = apply_act(p + bz, a.act, al);
      }
    }
  }
}

__global__ void affine_act_kernel(const float* __restrict__ x, int64_t xs, const float* scale, const float* shift,
                                  const float* alpha, int act, float* y, int64_t ys, int64_t M, int N) {
  const int64_t total = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N;
    const int n = (int)(i - m * N);
    float v = x[m * xs + n];
    if (scale) v = v * scale[n];
    if (shift) v = v + shift[n];
    y[m * ys + n] = apply_act(v, act, (act == RS_ACT_PRELU && alpha) ? alpha[n] : 0.f);
  }
}

__global__ void sigmoid_combine_kernel(const float* a, const float* b, float c0, float c1, float* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float z = c0 * a[i];
    if (b) z = z + c1 * b[i];
    out[i] = 1.0f / (1.0f + expf(-z));
  }
}

static unsigned ew_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace rs

using namespace rs;

static int dense_launch(const DenseArgs& a, hipStream_t st, const char* what) {
  if (a.N <= 4) {
    int64_t g = (a.M * 64 + 255) / 256;
    if (g > 4096) g = 4096;
    dense_small_n<<<(unsigned)g, 256, 0, st>>>(a);
  } else {
    dim3 grid((a.N + GBN - 1) / GBN, (unsigned)((a.M + GBM - 1) / GBM));
    dense_mfma<<<grid, 256, 0, st>>>(a);
  }
  return launch_status(what);
}

extern "C" int rs_dense_fwd(const float* x, int64_t x_stride, const float* W, const float* bias, const float* alpha,
                            int act, float* y, int64_t y_stride, int64_t M, int K, int N, rs_stream_t stream) {
  if (M == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(x && W && y, "rs_dense_fwd: null pointer");
  RS_REQUIRE(M >= 0 && K >= 1 && N >= 1 && x_stride >= K && y_stride >= N, "rs_dense_fwd: bad shape");
  RS_REQUIRE(act >= RS_ACT_NONE && act <= RS_ACT_SIGMOID, "rs_dense_fwd: bad activation");
  RS_REQUIRE(act != RS_ACT_PRELU || alpha, "rs_dense_fwd: PReLU needs alpha");
  RS_REQUIRE((M + GBM - 1) / GBM < 65536, "rs_dense_fwd: M too large for one launch");
  DenseArgs a{x, x_stride, W, bias, alpha, act, y, y_stride, M, K, N, 1};
  return dense_launch(a, as_stream(stream), "rs_dense_fwd");
}

extern "C" int rs_dense_prelu_rows_fwd(const float* x, int64_t x_stride, const float* W, const float* bias,
                                       const float* alpha, int alpha_rows, float* y, int64_t y_stride, int64_t M,
                                       int K, int N, rs_stream_t stream) {
  if (M == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(x && W && y && alpha, "rs_dense_prelu_rows_fwd: null pointer");
  RS_REQUIRE(M >= 0 && K >= 1 && N >= 1 && x_stride >= K && y_stride >= N && alpha_rows >= 1,
             "rs_dense_prelu_rows_fwd: bad shape");
  RS_REQUIRE((M + GBM - 1) / GBM < 65536, "rs_dense_prelu_rows_fwd: M too large for one launch");
  DenseArgs a{x, x_stride, W, bias, alpha, RS_ACT_PRELU, y, y_stride, M, K, N, alpha_rows};
  return dense_launch(a, as_stream(stream), "rs_dense_prelu_rows_fwd");
}

extern "C" int rs_affine_act(const float* x, int64_t x_stride, const float* scale, const float* shift,
                             const float* alpha, int act, float* y, int64_t y_stride, int64_t M, int N,
                             rs_stream_t stream) {
  if (M == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(x && y && M >= 0 && N >= 1 && x_stride >= N && y_stride >= N, "rs_affine_act: bad arguments");
  RS_REQUIRE(act >= RS_ACT_NONE && act <= RS_ACT_SIGMOID && (act != RS_ACT_PRELU || alpha),
             "rs_affine_act: bad activation");
  if (M == 0) return RS_OK;
  affine_act_kernel<<<ew_grid(M * N), 256, 0, as_stream(stream)>>>(x, x_stride, scale, shift, alpha, act, y,
                                                                   y_stride, M, N);
  return launch_status("rs_affine_act");
}

extern "C" int rs_sigmoid_combine(const float* a, const float* b, float c0, float c1, float* out, int64_t n,
                                  rs_stream_t stream) {
  if (n == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(a && out && n >= 0, "rs_sigmoid_combine: bad arguments");
  if (n == 0) return RS_OK;
  sigmoid_combine_kernel<<<ew_grid(n), 256, 0, as_stream(stream)>>>(a, b, c0, c1, out, n);
  return launch_status("rs_sigmoid_combine");
}

namespace rs {
__global__ void dice_kernel(const float* __restrict__ x, int64_t xs, const float* mean, const float* var, float eps,
                            const float* alpha, float* y, int64_t ys, int64_t M, int N) {
  const int64_t total = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N;
    const int n = (int)(i - m * N);
    const float v = x[m * xs + n];
    const float xn = (v - mean[n]) / sqrtf(var[n] + eps);
    const float p = 1.0f / (1.0f + expf(-xn));
    y[m * ys + n] = alpha[n] * (1.0f - p) * v + p * v;
  }
}
}  // namespace rs

extern "C" int rs_dice_fwd(const float* x, int64_t x_stride, const float* mean, const float* var, float eps,
                           const float* alpha, float* y, int64_t y_stride, int64_t M, int N, rs_stream_t stream) {
  if (M == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(x && mean && var && alpha && y && M >= 0 && N >= 1 && x_stride >= N && y_stride >= N,
             "rs_dice_fwd: bad arguments");
  if (M == 0) return RS_OK;
  dice_kernel<<<ew_grid(M * N), 256, 0, as_stream(stream)>>>(x, x_stride, mean, var, eps, alpha, y, y_stride, M, N);
  return launch_status("rs_dice_fwd");
}
