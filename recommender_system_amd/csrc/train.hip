// train.hip — the FM model's training step: forward,
// binary cross-entropy gradient, L2 regularisers and SGD, with the sparse
// rows updated by a deterministic scatter-add (row-sparse SGD).
//
// Reference semantics:
//   FM.call / FMLayer.call   model/fm.py:19-23, layer/interaction.py:106-114
//     y = w0 + x@w1 + 0.5 * sum_f [(x@v)_f^2 - (x^2 @ v^2)_f],  p = sigmoid(y)
//   FMLayer.build            layer/interaction.py:94-104: w1 ~ l2(reg_w),
//                            v ~ l2(reg_b) (Keras l2: loss += l * sum(w^2))
//   compile_fit              utils/compile_fit.py:9-15: SGD(lr), loss
//                            'binary_crossentropy' on a sigmoid output —
//                            Keras takes the sigmoid's logits, so
//                            dL/dy_b = (sigmoid(y_b) - t_b) / B (batch mean)
// with x = [dense | one-hot] (utils/dataset.py:47-48): the one-hot block of
// sample b has a single 1 at column nd + offset_c + id(b,c) per field.
//
// Gradients (x one-hot, so x = x^2 = 1 on the sparse rows):
//   dy/dw0 = 1,  dy/dw1_i = x_i,  dy/dv_if = x_i s_f - x_i^2 v_if,
//   s_f = (x@v)_f.
// Update (one step, lr, l2 weights lw / lv; all from the OLD weights):
//   w0  -= lr * sum_b g_b
//   w1  -= lr * (G1 + 2 lw w1),   v -= lr * (Gv + 2 lv v)       (every row)
// The decay touches every row (as Keras' dense regulariser gradient does);
// G is non-zero only on the nd dense rows and the rows the batch looked up.
// Sparse rows: per-lookup contributions are sorted by row (the hand-written
// stable radix sort, radix_sort.hip) and each row's contributions are summed in lookup order, in chunk
// pieces added in chunk order, so the result is bitwise reproducible.
#include "radix_sort.hpp"
#include "rs_common.hpp"

namespace rs {

struct FmTrainArgs {
  const void* ids;
  int64_t id_stride;
  const float* dense;
  int64_t dense_stride;
  int nd;
  const int64_t* offs;  // one-hot field offsets (without nd)
  const int64_t* vocab;
  int F, k;
  float* w0;
  float* w1;  // [n_rows]
  float* v;   // [n_rows, k]
  int64_t n_rows;
  const float* labels;
  int64_t batch;
  float lr, l2_w, l2_v;
  // workspace
  float* g;        // [B]
  float* s;        // [B, k]
  float* contrib;  // [B*F, k+1]
  uint32_t* key_in;
  uint32_t* key_out;
  uint32_t* val_in;
  uint32_t* val_out;
  float* gdense;  // [nd, k+1] + 1 (w0)
  float* part;    // chunk-piece partials of crossing row segments (2 * nchunk * (k+1))
  int64_t chunk;
  float* loss;    // [B] (optional)
  int* err;
};

// One wave per sample, lane f < k: s_f and the (x^2 @ v^2)_f term; lane 0
// also the linear part.  Rows in the reference's column order (dense, then
// field by field).
template <int KIND>
__global__ __launch_bounds__(256) void fm_train_fwd(FmTrainArgs a) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.batch) return;  // wave-uniform
  const bool fl = lane < a.k;
  const int f = fl ? lane : 0;
  float s = 0.f, q = 0.f, lin = 0.f;
  for (int i = 0; i < a.nd; ++i) {
    const float x = a.dense[b * a.dense_stride + i];
    const float vv = a.v[(int64_t)i * a.k + f];
    s = fmaf(x, vv, s);
    q = fmaf(x * x, vv * vv, q);
    lin = fmaf(x, a.w1[i], lin);
  }
  bool bad = false;
  for (int c = 0; c < a.F; ++c) {
    int64_t id;
    const bool ok = I::decode(I::load(a.ids, b * a.id_stride + c), a.vocab[c], id);
    bad |= !ok;
    const int64_t row = a.nd + a.offs[c] + id;
    const float vv = ok ? a.v[row * a.k + f] : 0.f;
    s += vv;
    q = fmaf(vv, vv, q);
    lin += ok ? a.w1[row] : 0.f;
  }
  if (bad && lane == 0) flag_error(a.err);
  float t = fl ? s * s - q : 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
  const float y = (lin + a.w0[0]) + 0.5f * t;
  const float p = sigmoidf_(y);
  const float tb = a.labels[b];
  const float g = (p - tb) / (float)a.batch;
  if (fl) a.s[b * a.k + f] = s;
  if (lane == 0) {
    a.g[b] = g;
    if (a.loss) a.loss[b] = fmaxf(y, 0.f) - y * tb + log1pf(expf(-fabsf(y)));
  }
}

// Per lookup j = b*F + c: key = one-hot row, contribution
// [g_b (s_bf - v_rf) for f < k | g_b]   (x = 1 on the sparse rows).
template <int KIND>
__global__ __launch_bounds__(256) void fm_train_lookup_grads(FmTrainArgs a) {
  typedef Ids<KIND> I;
  const int K1 = a.k + 1;
  const int64_t total = a.batch * a.F * K1;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t j = idx / K1;
    const int f = (int)(idx - j * K1);
    const int64_t b = j / a.F;
    const int c = (int)(j - b * a.F);
    int64_t id;
    const bool ok = I::decode(I::load(a.ids, b * a.id_stride + c), a.vocab[c], id);
    const int64_t row = a.nd + a.offs[c] + id;
    const float g = ok ? a.g[b] : 0.f;  // a bad id contributes nothing (its row is a valid one)
    a.contrib[idx] = f < a.k ? g * (a.s[b * a.k + f] - a.v[row * a.k + f]) : g;
    if (f == 0) {
      a.key_in[j] = (uint32_t)row;
      a.val_in[j] = (uint32_t)j;
    }
  }
}

// Dense rows i < nd: G[i][f] = sum_b g_b (x_bi s_bf - x_bi^2 v_if),
// G[i][k] = sum_b g_b x_bi; G[nd*(k+1)] = sum_b g_b (w0).  One 256-thread
// block per output: strided partial sums, then a fixed-shape tree in LDS —
// the same order every run.
__global__ __launch_bounds__(256) void fm_train_dense_grads(FmTrainArgs a) {
  __shared__ float red[256];
  const int K1 = a.k + 1;
  const int idx = blockIdx.x;
  const bool is_w0 = idx == a.nd * K1;
  const int i = is_w0 ? 0 : idx / K1, f = is_w0 ? 0 : idx - i * K1;
  const float vi = (!is_w0 && f < a.k) ? a.v[(int64_t)i * a.k + f] : 0.f;
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < a.batch; b += 256) {
    const float g = a.g[b];
    if (is_w0) {
      acc += g;
    } else {
      const float x = a.dense[b * a.dense_stride + i];
      acc += f < a.k ? g * (x * a.s[b * a.k + f] - x * x * vi) : g * x;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
#pragma unroll
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.gdense[idx] = red[0];
}

// w[0, n4) (float4s) -= f * w, streamed with DECAY_U independent 16-B loads
// in flight per thread before their stores (one at a time left ~8 MB in
// flight chip-wide: ~54 % of HBM); grid-stride over the whole range.
constexpr int DECAY_U = 4;
__device__ __forceinline__ void decay_stream(floatx4* __restrict__ w4, int64_t n4, float f) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; q + (DECAY_U - 1) * stride < n4; q += DECAY_U * stride) {
    floatx4 x[DECAY_U];
#pragma unroll
    for (int u = 0; u < DECAY_U; ++u) x[u] = __builtin_nontemporal_load(w4 + q + u * stride);
#pragma unroll
    for (int u = 0; u < DECAY_U; ++u) {
      x[u] -= f * x[u];
      __builtin_nontemporal_store(x[u], w4 + q + u * stride);
    }
  }
  for (; q < n4; q += stride) {
    floatx4 x = __builtin_nontemporal_load(w4 + q);
    x -= f * x;
    __builtin_nontemporal_store(x, w4 + q);
  }
}

// L2 decay of every row: w -= lr * 2 l w  (the regulariser's gradient);
// float4 over v when it is 16-B aligned (k % 4 == 0), then w1.
__global__ __launch_bounds__(256) void fm_train_decay(FmTrainArgs a) {
  const int64_t nv = a.n_rows * a.k;
  const float cv = a.lr * 2.f * a.l2_v, cw = a.lr * 2.f * a.l2_w;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t done = 0;
  if ((nv & 3) == 0 && ((uintptr_t)a.v & 15) == 0) {
    decay_stream(reinterpret_cast<floatx4*>(a.v), nv / 4, cv);
    done = nv;
  }
  for (int64_t idx = done + t0; idx < nv + a.n_rows; idx += stride) {
    if (idx < nv) a.v[idx] -= cv * a.v[idx];
    else a.w1[idx - nv] -= cw * a.w1[idx - nv];
  }
}

// Sorted lookups: each row's contributions summed in lookup order in chunk
// pieces (seg_piece / seg_cross, rs_common.hpp: one lane per (position,
// column), a hot row's k+1 columns by adjacent lanes, pieces added in chunk
// order — bitwise reproducible, and a Zipf-hot row no longer serialises);
// then the dense rows and w0.
__device__ __forceinline__ void fm_apply_row(const FmTrainArgs& a, uint32_t r, int f, float acc) {
  if (f < a.k) a.v[(int64_t)r * a.k + f] -= a.lr * acc;
  else a.w1[r] -= a.lr * acc;
}

__global__ __launch_bounds__(256) void fm_train_apply(FmTrainArgs a) {
  const int64_t n = a.batch * a.F;
  const int K1 = a.k + 1;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n * K1) {
    const int64_t p = t / K1;
    const int f = (int)(t - p * K1);
    const int64_t nch = (n + a.chunk - 1) / a.chunk;
    uint32_t r;
    float acc;
    if (seg_piece(a.key_out, n, a.chunk, p, K1, f,
                  [&](int64_t q) { return a.contrib[(int64_t)a.val_out[q] * K1 + f]; }, a.part,
                  a.part + nch * K1, r, acc))
      fm_apply_row(a, r, f, acc);
  } else if (t < n * K1 + a.nd * K1 + 1) {
    const int idx = (int)(t - n * K1);
    const float gsum = a.gdense[idx];
    if (idx == a.nd * K1) {
      a.w0[0] -= a.lr * gsum;
    } else {
      const int i = idx / K1, f = idx - i * K1;
      if (f < a.k) a.v[(int64_t)i * a.k + f] -= a.lr * gsum;
      else a.w1[i] -= a.lr * gsum;
    }
  }
}

__global__ __launch_bounds__(256) void fm_train_apply_cross(FmTrainArgs a) {
  const int64_t n = a.batch * a.F;
  const int K1 = a.k + 1;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * K1) return;
  const int64_t p = t / K1;
  const int f = (int)(t - p * K1);
  const int64_t nch = (n + a.chunk - 1) / a.chunk;
  uint32_t r;
  float acc;
  if (seg_cross(a.key_out, n, a.chunk, p, K1, f, a.part, a.part + nch * K1, r, acc)) fm_apply_row(a, r, f, acc);
}

// ---- FFM training (compile_fit on FFM, model/ffm.py:20-22 over FFMLayer,
// layer/interaction.py:134-163).  One wave per sample: Fm[f, c] = sum_i x_i
// v[i, f, c] over the nd dense rows and the F looked-up rows (an out-of-range
// id is tf.one_hot's zero row), T_c = sum_f Fm[f, c], z = w0 + x.w +
// 0.5 (sum_c T_c^2 - sum Fm^2); g = (sigmoid(z) - t)/B and the per-sample
// gradient row G[f, c] = g (T_c - Fm[f, c]) (shared by the sample's looked-up
// rows: dv[row] += G; dense rows: dv[i] += x_i G).  Fixed orders throughout.
constexpr int FFMT_MAXE = 4096;  // NF * k
template <int KIND>
__global__ __launch_bounds__(256) void ffm_train_fwd_kernel(const void* ids, int64_t id_stride,
                                                            const float* __restrict__ dense, int64_t ds, int nd,
                                                            const float* __restrict__ v, const float* __restrict__ w,
                                                            const float* __restrict__ w0,
                                                            const int64_t* __restrict__ offs,
                                                            const int64_t* __restrict__ vocab, int F, int k,
                                                            const float* __restrict__ labels, int64_t B,
                                                            float* __restrict__ G, float* __restrict__ g,
                                                            float* __restrict__ loss) {
  typedef Ids<KIND> I;
  __shared__ float sfm[4][FFMT_MAXE];
  __shared__ float st[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * 4 + wv;
  if (b >= B) return;  // wave-uniform
  const int NF = nd + F, E = NF * k;
  float* fm = sfm[wv];
  float q = 0.f;  // sum Fm^2 (this lane's elements)
  for (int e = lane; e < E; e += 64) {
    float a = 0.f;
    for (int i = 0; i < nd; ++i) a = fmaf(dense[b * ds + i], v[(int64_t)i * E + e], a);
    for (int c = 0; c < F; ++c) {
      int64_t id;
      const bool ok = I::decode(I::load(ids, b * id_stride + c), vocab[c], id);
      const int64_t row = nd + offs[c] + (ok ? id : 0);
      const float x = v[row * E + e];
      a += ok ? x : 0.f;
    }
    fm[e] = a;
    q = fmaf(a, a, q);
  }
  // linear part: lanes over the dense features and the fields
  float lin = 0.f;
  for (int i = lane; i < nd + F; i += 64) {
    if (i < nd) {
      lin = fmaf(dense[b * ds + i], w[i], lin);
    } else {
      const int c = i - nd;
      int64_t id;
      const bool ok = I::decode(I::load(ids, b * id_stride + c), vocab[c], id);
      const float x = w[nd + offs[c] + (ok ? id : 0)];
      lin += ok ? x : 0.f;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  float tt = 0.f;  // T_c^2 for c = lane
  if (lane < k) {
    float T = 0.f;
    for (int f = 0; f < NF; ++f) T += fm[f * k + lane];
    st[wv][lane] = T;
    tt = T * T;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    q += __shfl_xor(q, o);
    lin += __shfl_xor(lin, o);
    tt += __shfl_xor(tt, o);
  }
  const float z = (w0[0] + lin) + 0.5f * (tt - q);
  const float t = labels[b];
  const float gb = (1.f / (1.f + expf(-z)) - t) / (float)B;
  if (lane == 0) {
    g[b] = gb;
    if (loss) loss[b] = fmaxf(z, 0.f) - z * t + log1pf(expf(-fabsf(z)));
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  for (int e = lane; e < E; e += 64) G[b * E + e] = gb * (st[wv][e % k] - fm[e]);
}

// Keras l2(l) regulariser's gradient on every row: w -= lr * 2 l w
__global__ __launch_bounds__(256) void l2_decay_kernel(float* __restrict__ w, int64_t n, float f) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t done = 0;
  if ((n & 3) == 0 && ((uintptr_t)w & 15) == 0) {
    decay_stream(reinterpret_cast<floatx4*>(w), n / 4, f);
    done = n;
  }
  for (int64_t i = done + t0; i < n; i += stride) w[i] -= f * w[i];
}

// workspace layout (all 256-B aligned)
struct TrainWs {
  int64_t g, s, contrib, key_in, key_out, val_in, val_out, gdense, part, sort, total;
  size_t sort_bytes;
};

static int64_t al256(int64_t x) { return (x + 255) / 256 * 256; }

static TrainWs train_ws(int64_t batch, int n_fields, int k, int nd) {
  TrainWs w{};
  const int64_t n = batch * n_fields;
  const int64_t sb = sort_pairs_ws_bytes(n);
  w.sort_bytes = (size_t)sb;
  int64_t o = 0;
  w.g = o; o = al256(o + batch * 4);
  w.s = o; o = al256(o + batch * k * 4);
  w.contrib = o; o = al256(o + n * (k + 1) * 4);
  w.key_in = o; o = al256(o + n * 4);
  w.key_out = o; o = al256(o + n * 4);
  w.val_in = o; o = al256(o + n * 4);
  w.val_out = o; o = al256(o + n * 4);
  w.gdense = o; o = al256(o + ((int64_t)nd * (k + 1) + 1) * 4);
  w.part = o; o = al256(o + n * 4);  // <= n floats (seg_chunk(k + 1))
  w.sort = o; o = al256(o + (int64_t)sb);
  w.total = o;
  return w;
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_fm_train_workspace_size(int64_t batch, int n_fields, int k, int nd) {
  if (batch < 0 || n_fields < 0 || k < 1 || nd < 0) return -1;
  return train_ws(batch, n_fields, k, nd).total;
}

extern "C" int rs_fm_train_step(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                int64_t dense_stride, int nd, const int64_t* field_offsets,
                                const int64_t* field_vocab, int n_fields, int k, float* w0, float* w1, float* v,
                                int64_t n_rows, const float* labels, int64_t batch, float lr, float l2_w, float l2_v,
                                void* workspace, float* loss, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: no step (Keras runs no step either)
  RS_REQUIRE(batch > 0 && nd >= 0 && n_fields >= 0 && k >= 1 && k <= 64 && n_rows >= nd,
             "rs_fm_train_step: bad shape (1 <= k <= 64)");
  RS_REQUIRE(n_rows < ((int64_t)1 << 32) && batch * n_fields < ((int64_t)1 << 31),
             "rs_fm_train_step: rows must fit uint32, lookups int32");
  RS_REQUIRE(w0 && w1 && v && labels && workspace && (nd == 0 || dense) &&
                 (n_fields == 0 || (ids && field_offsets && field_vocab)),
             "rs_fm_train_step: null pointer");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_fm_train_step: bad id_kind");
  const TrainWs w = train_ws(batch, n_fields, k, nd);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  FmTrainArgs a{ids, id_stride, dense, dense_stride, nd, field_offsets, field_vocab, n_fields, k, w0, w1, v, n_rows,
                labels, batch, lr, l2_w, l2_v,
                reinterpret_cast<float*>(ws + w.g), reinterpret_cast<float*>(ws + w.s),
                reinterpret_cast<float*>(ws + w.contrib), reinterpret_cast<uint32_t*>(ws + w.key_in),
                reinterpret_cast<uint32_t*>(ws + w.key_out), reinterpret_cast<uint32_t*>(ws + w.val_in),
                reinterpret_cast<uint32_t*>(ws + w.val_out), reinterpret_cast<float*>(ws + w.gdense),
                reinterpret_cast<float*>(ws + w.part), seg_chunk(k + 1), loss, err_flag};
  hipStream_t st = as_stream(stream);
  const int64_t n = batch * n_fields;
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KD = decltype(K)::value;
    fm_train_fwd<KD><<<(unsigned)((batch + 3) / 4), 256, 0, st>>>(a);
    if (n > 0) {
      const int64_t tot = n * (k + 1);
      fm_train_lookup_grads<KD><<<(unsigned)std::min<int64_t>((tot + 255) / 256, 8192), 256, 0, st>>>(a);
    }
  });
  fm_train_dense_grads<<<(unsigned)(nd * (k + 1) + 1), 256, 0, st>>>(a);
  if (n > 0) {
    int bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < (uint64_t)n_rows) ++bits;
    const hipError_t e = sort_pairs_u32(a.key_in, a.val_in, a.key_out, a.val_out, n, bits, ws + w.sort, st);
    if (e != hipSuccess) {
      set_error("rs_fm_train_step: radix sort failed: %s", hipGetErrorString(e));
      return RS_ERR_HIP;
    }
  }
  const int64_t dn = n_rows * (int64_t)(k + 1);
  fm_train_decay<<<(unsigned)std::min<int64_t>((dn / 4 + 255) / 256 + 1, 8192), 256, 0, st>>>(a);
  const int64_t ap = (n + nd) * (k + 1) + 1;
  fm_train_apply<<<(unsigned)((ap + 255) / 256), 256, 0, st>>>(a);
  if (n > a.chunk) fm_train_apply_cross<<<(unsigned)((n * (k + 1) + 255) / 256), 256, 0, st>>>(a);
  return launch_status("rs_fm_train_step");
}

extern "C" int rs_ffm_train_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                int64_t dense_stride, int nd, const float* v, const float* w, const float* w0,
                                const int64_t* field_offsets, const int64_t* field_vocab, int n_fields, int k,
                                const float* labels, int64_t batch, float* G, float* g, float* loss,
                                rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(v && w && w0 && labels && G && g && batch > 0 && nd >= 0 && n_fields >= 1 && k >= 1 && k <= 64 &&
                 (int64_t)(nd + n_fields) * k <= FFMT_MAXE && (nd == 0 || dense) && ids && field_offsets &&
                 field_vocab && id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32,
             "rs_ffm_train_fwd: bad arguments (k <= 64, (nd + n_fields) * k <= %d)", FFMT_MAXE);
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    ffm_train_fwd_kernel<decltype(K)::value><<<(unsigned)((batch + 3) / 4), 256, 0, st>>>(
        ids, id_stride, dense, dense_stride, nd, v, w, w0, field_offsets, field_vocab, n_fields, k, labels, batch, G,
        g, loss);
  });
  return launch_status("rs_ffm_train_fwd");
}

extern "C" int rs_l2_decay(float* w, int64_t n, float lr, float l2, rs_stream_t stream) {
  if (n == 0 || l2 == 0.f) return RS_OK;
  RS_REQUIRE(w && n > 0, "rs_l2_decay: bad arguments");
  l2_decay_kernel<<<(unsigned)std::min<int64_t>((n / 4 + 255) / 256 + 1, 8192), 256, 0, as_stream(stream)>>>(
      w, n, lr * 2.f * l2);
  return launch_status("rs_l2_decay");
}
