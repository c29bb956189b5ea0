// inner.hip — PNN inner product (InnerProductLayer, layer/interaction.py:166-183)
// and the fused gather + flatten + inner product that builds PNN's DNN input
// (model/pnn.py:32-41, with 3-D embeddings).
//
// Per sample the F x k embedding tile is staged in LDS once (coalesced, one
// HBM read); each thread owns a balanced pair of Gram rows (i and F-2-i, so
// every thread computes ~F dot products), keeps e_i in registers and streams
// e_j from LDS.  Output column p enumerates pairs (i<j) in the reference's
// row-major order: p(i,j) = i*(2F-i-1)/2 + (j-i-1).
#include "rs_common.hpp"

namespace rs {

struct InnerArgs {
  const float* emb;  // [B, F, k] (when ids == nullptr)
  const void* ids;
  int id_kind;
  int64_t id_stride;
  const float* table;
  const int64_t* offs;
  const int64_t* vocab;
  int F, k, S, NG;
  float* out;
  int64_t out_stride;
  int inner_off;   // column of the first pair in out
  int write_flat;  // also write the flattened embeddings to out[:, 0:F*k]
  int64_t batch;
  int* err;
};

__device__ __forceinline__ bool inner_decode(const void* ids, int kind, int64_t off, int64_t vocab, int64_t& id) {
  if (kind == RS_ID_F32) {
    const float f = static_cast<const float*>(ids)[off];
    if (!(f > -1.0f && static_cast<double>(f) < static_cast<double>(vocab))) return false;
    id = static_cast<int64_t>(f);
    return true;
  }
  id = (kind == RS_ID_I64) ? static_cast<const int64_t*>(ids)[off] : static_cast<const int32_t*>(ids)[off];
  return id >= 0 && id < vocab;
}

template <int KMAX>
__global__ __launch_bounds__(256) void inner_kernel(InnerArgs a) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [S][F][KP]
  const int KP = a.k;  // row stride in LDS
  const int64_t b0 = (int64_t)blockIdx.x * a.S;
  const int vec = (a.k % 4 == 0);
  const int KQ = vec ? a.k / 4 : a.k;
  const int per_s = a.F * KQ;
  const int tot = a.S * per_s;
  for (int i = threadIdx.x; i < tot; i += blockDim.x) {
    const int s = i / per_s, r = i - s * per_s;
    const int c = r / KQ, q = r - c * KQ;
    const int64_t b = b0 + s;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (b < a.batch) {
      const float* src = nullptr;
      if (a.ids) {
        int64_t id;
        if (inner_decode(a.ids, a.id_kind, b * a.id_stride + c, a.vocab[c], id))
          src = a.table + (a.offs[c] + id) * a.k;
        else
          flag_error(a.err);
      } else {
        src = a.emb + (b * a.F + c) * a.k;
      }
      if (src) {
        if (vec) {
          const floatx4 t = *reinterpret_cast<const floatx4*>(src + 4 * q);
          v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
        } else {
          v[0] = src[q];
        }
      }
      if (a.write_flat) {
        float* dst = a.out + b * a.out_stride + c * a.k + (vec ? 4 * q : q);
        const int nv = vec ? 4 : 1;
        for (int t = 0; t < nv; ++t) dst[t] = v[t];
      }
    }
    float* d = tile + ((int64_t)s * a.F + c) * KP + (vec ? 4 * q : q);
    if (vec) {
      *reinterpret_cast<floatx4*>(d) = floatx4{v[0], v[1], v[2], v[3]};
    } else {
      d[0] = v[0];
    }
  }
  __syncthreads();

  const int s = threadIdx.x / a.NG, g = threadIdx.x - s * a.NG;
  if (s >= a.S) return;
  const int64_t b = b0 + s;
  if (b >= a.batch) return;
  const float* es = tile + (int64_t)s * a.F * KP;
  float* o = a.out + b * a.out_stride + a.inner_off;
  for (int pass = 0; pass < 2; ++pass) {
    const int i = pass == 0 ? g : a.F - 2 - g;
    if (pass == 1 && i <= g) break;
    if (i > a.F - 2) continue;
    float ei[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) ei[q] = q < a.k ? es[i * KP + q] : 0.f;
    const int p0 = i * (2 * a.F - i - 1) / 2;
    for (int j = i + 1; j < a.F; ++j) {
      const float* ej = es + j * KP;
      float dot = 0.f;
#pragma unroll
      for (int q = 0; q < KMAX; ++q)
        if (q < a.k) dot = fmaf(ei[q], ej[q], dot);
      o[p0 + j - i - 1] = dot;
    }
  }
}

// ---------------------------------------------------------------- fast path
// k in {4,8,16,32,64}, F <= 64.  Up to 16 samples per 256-thread workgroup:
//  1. the workgroup's S x F ids and the F (offset, vocab) pairs -> LDS
//     (coalesced, once), barrier;
//  2. every row chunk (float4) of the S x F x k tile is requested up front
//     (8 in flight per thread, non-temporal), then stored to LDS, barrier;
//  3. Gram rows: thread (s, g) owns rows g and F-2-g (balanced, ~F dot
//     products) with e_i in registers, e_j as float4 LDS reads; results to an
//     LDS output tile, barrier;
//  4. the S output rows [flat | inner] (or [inner]) leave as one coalesced
//     block of dword stores.
constexpr int IP_SMAX = 16;
constexpr int IP_FMAX = 64;

template <int K, int KIND>
__global__ __launch_bounds__(256) void inner_fast(InnerArgs a) {
  constexpr int KQ = K / 4;
  typedef Ids<KIND == 3 ? 0 : KIND> I;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ typename I::raw_t lid[IP_SMAX][IP_FMAX];
  __shared__ int64_t lmeta[2][IP_FMAX];
  const int F = a.F, P = F * (F - 1) / 2, S = a.S;
  float* tile = smem;                          // [S][F][K]
  float* gram = smem + S * F * K;              // [S][P]
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * S;
  const int nvalid = (int)(a.batch - b0 < S ? a.batch - b0 : S);

  if constexpr (KIND != 3) {
    for (int t = tid; t < S * F; t += 256) {
      const int s = t / F, c = t - s * F;
      const int64_t bb = b0 + (s < nvalid ? s : nvalid - 1);
      lid[s][c] = I::load(a.ids, bb * a.id_stride + c);
    }
    for (int t = tid; t < 2 * F; t += 256) {
      const int c = t < F ? t : t - F;
      lmeta[t < F ? 0 : 1][c] = t < F ? a.offs[c] : a.vocab[c];
    }
    __syncthreads();
  }

  bool bad = false;
  const float* src = KIND == 3 ? a.emb : a.table;  // embeddings given vs gathered
  const int total = S * F * KQ;
  for (int base = 0; base < total; base += 256 * 8) {
    floatx4 v[8];
    int dsti[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * 256 + tid;
      dsti[u] = -1;
      v[u] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (idx < total) {
        const int s = idx / (F * KQ), r = idx - s * (F * KQ);
        const int c = r / KQ, q = r - c * KQ;
        const int64_t bb = b0 + (s < nvalid ? s : nvalid - 1);
        int64_t row;
        bool ok = true;
        if constexpr (KIND == 3) {
          row = bb * F + c;
        } else {
          int64_t id;
          ok = I::decode(lid[s][c], lmeta[1][c], id);
          row = lmeta[0][c] + id;
          bad |= !ok && s < nvalid;
        }
        const floatx4 t = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(src + row * K + 4 * q));
        v[u] = ok ? t : floatx4{0.f, 0.f, 0.f, 0.f};
        dsti[u] = (s * F + c) * K + 4 * q;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (dsti[u] >= 0) *reinterpret_cast<floatx4*>(tile + dsti[u]) = v[u];
  }
  if (bad) flag_error(a.err);
  __syncthreads();

  const int NG = F / 2 > 0 ? F / 2 : 1;  // balanced row pairs (g, F-2-g)
  for (int t = tid; t < S * NG; t += 256) {
    const int s = t / NG, g = t - s * NG;
    const float* es = tile + s * F * K;
    float* gs = gram + s * P;
    for (int pass = 0; pass < 2; ++pass) {
      const int i = pass == 0 ? g : F - 2 - g;
      if (pass == 1 && i <= g) break;
      if (i > F - 2) continue;
      float ei[K];
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const floatx4 x = *reinterpret_cast<const floatx4*>(es + i * K + 4 * q);
        ei[4 * q] = x[0]; ei[4 * q + 1] = x[1]; ei[4 * q + 2] = x[2]; ei[4 * q + 3] = x[3];
      }
      const int p0 = i * (2 * F - i - 1) / 2 - i - 1;
      for (int j = i + 1; j < F; ++j) {
        float dot = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
          const floatx4 y = *reinterpret_cast<const floatx4*>(es + j * K + 4 * q);
          dot = fmaf(ei[4 * q], y[0], dot);
          dot = fmaf(ei[4 * q + 1], y[1], dot);
          dot = fmaf(ei[4 * q + 2], y[2], dot);
          dot = fmaf(ei[4 * q + 3], y[3], dot);
        }
        gs[p0 + j] = dot;
      }
    }
  }
  __syncthreads();

  const int FK = a.write_flat ? F * K : 0;
  const int W = FK + P;
  for (int e = tid; e < nvalid * W; e += 256) {
    const int s = e / W, col = e - s * W;
    const float val = col < FK ? tile[s * F * K + col] : gram[s * P + (col - FK)];
    const int oc = col < FK ? col : a.inner_off + (col - FK);
    a.out[(b0 + s) * a.out_stride + oc] = val;
  }
}

template <int KIND>
static void launch_inner_fast_k(const InnerArgs& a, size_t lds, unsigned grid, hipStream_t st) {
  switch (a.k) {
    case 4: inner_fast<4, KIND><<<grid, 256, lds, st>>>(a); break;
    case 8: inner_fast<8, KIND><<<grid, 256, lds, st>>>(a); break;
    case 16: inner_fast<16, KIND><<<grid, 256, lds, st>>>(a); break;
    case 32: inner_fast<32, KIND><<<grid, 256, lds, st>>>(a); break;
    default: inner_fast<64, KIND><<<grid, 256, lds, st>>>(a); break;
  }
}

static int launch_inner(InnerArgs a, hipStream_t st, const char* what) {
  if (a.batch == 0) return RS_OK;
  const bool fast_k = a.k == 4 || a.k == 8 || a.k == 16 || a.k == 32 || a.k == 64;
  if (fast_k && a.F >= 2 && a.F <= IP_FMAX) {
    const int P = a.F * (a.F - 1) / 2;
    const int64_t per = ((int64_t)a.F * a.k + P) * sizeof(float);
    int S = IP_SMAX;
    while (S > 1 && S * per > 96 * 1024) --S;
    a.S = S;
    const size_t lds = (size_t)S * per;
    const unsigned grid = (unsigned)((a.batch + S - 1) / S);
    if (a.ids == nullptr) {
      launch_inner_fast_k<3>(a, lds, grid, st);
    } else {
      with_id_kind(a.id_kind, [&](auto K) { launch_inner_fast_k<decltype(K)::value>(a, lds, grid, st); });
    }
    return launch_status(what);
  }
  a.NG = a.F / 2 > 0 ? a.F / 2 : 1;
  int S = 256 / a.NG;
  const int64_t per = (int64_t)a.F * a.k * sizeof(float);
  while (S > 1 && S * per > 48 * 1024) --S;
  RS_REQUIRE(S * per <= 150 * 1024, "%s: F*k too large for one LDS tile", what);
  a.S = S;
  const size_t lds = (size_t)S * per;
  const unsigned grid = (unsigned)((a.batch + S - 1) / S);
  if (a.k <= 8) inner_kernel<8><<<grid, 256, lds, st>>>(a);
  else if (a.k <= 16) inner_kernel<16><<<grid, 256, lds, st>>>(a);
  else if (a.k <= 32) inner_kernel<32><<<grid, 256, lds, st>>>(a);
  else inner_kernel<64><<<grid, 256, lds, st>>>(a);
  return launch_status(what);
}

}  // namespace rs

using namespace rs;

extern "C" int rs_inner_product_fwd(const float* emb, int n_fields, int k, float* out, int64_t out_stride,
                                    int64_t batch, rs_stream_t stream) {
  RS_REQUIRE(emb && out, "rs_inner_product_fwd: null pointer");
  RS_REQUIRE(n_fields >= 1 && k >= 1 && k <= 64 && batch >= 0, "rs_inner_product_fwd: bad shape (k<=64)");
  RS_REQUIRE(out_stride >= (int64_t)n_fields * (n_fields - 1) / 2, "rs_inner_product_fwd: out_stride too small");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)emb % 16 == 0, "rs_inner_product_fwd: emb must be 16-B aligned");
  InnerArgs a{};
  a.emb = emb;
  a.F = n_fields;
  a.k = k;
  a.out = out;
  a.out_stride = out_stride;
  a.inner_off = 0;
  a.write_flat = 0;
  a.batch = batch;
  return launch_inner(a, as_stream(stream), "rs_inner_product_fwd");
}

extern "C" int rs_embed_inner_fwd(const void* ids, int id_kind, int64_t id_stride, const float* table,
                                  const int64_t* field_offsets, const int64_t* field_vocab, int n_fields, int k,
                                  float* out, int64_t out_stride, int64_t batch, int* err_flag,
                                  rs_stream_t stream) {
  RS_REQUIRE(ids && table && field_offsets && field_vocab && out, "rs_embed_inner_fwd: null pointer");
  RS_REQUIRE(n_fields >= 1 && k >= 1 && k <= 64 && batch >= 0, "rs_embed_inner_fwd: bad shape (k<=64)");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_inner_fwd: bad id_kind");
  RS_REQUIRE(out_stride >= (int64_t)n_fields * k + (int64_t)n_fields * (n_fields - 1) / 2,
             "rs_embed_inner_fwd: out_stride too small");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)table % 16 == 0, "rs_embed_inner_fwd: table must be 16-B aligned");
  InnerArgs a{};
  a.ids = ids;
  a.id_kind = id_kind;
  a.id_stride = id_stride;
  a.table = table;
  a.offs = field_offsets;
  a.vocab = field_vocab;
  a.F = n_fields;
  a.k = k;
  a.out = out;
  a.out_stride = out_stride;
  a.inner_off = n_fields * k;
  a.write_flat = 1;
  a.batch = batch;
  a.err = err_flag;
  return launch_inner(a, as_stream(stream), "rs_embed_inner_fwd");
}
