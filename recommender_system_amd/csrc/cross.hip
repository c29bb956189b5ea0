// cross.hip — DCN CrossNet forward (CrossLayer, layer/interaction.py:49-83).
//
// Reference: x_{l+1} = x0 * (x_l^T w_l) + b_l + x_l for l < L, out = x_L.
// Every x_l is affine in x0 per sample: x_l = alpha_l * x0 + beta_l with
//   beta_l  = sum_{j<l} b_j               (sample-independent vector)
//   alpha_0 = 1, alpha_{l+1} = alpha_l * (1 + g_l) + h_l,
//   g_l = x0^T w_l (per sample),  h_l = beta_l^T w_l (sample-independent).
// So the whole stack is one contraction G = X0 @ [w_0 .. w_{L-1}] — the
// x0 x_l^T w contraction of the north star — done on v_mfma_f32_16x16x4_f32
// with all L weight vectors as B columns, a 16-sample scalar recurrence, and
// one fused-multiply-add pass out = alpha_L * x0 + beta_L.  x0 is read from
// HBM once (staged in LDS), out is written once: the kernel is HBM-bound at
// 2*d*4 bytes per sample; MFMA utilisation is at most L/16 by construction.
#include "mlp_tower.hpp"
#include "rs_common.hpp"
#include "tile_gather.hpp"

namespace rs {

struct CrossGeom {
  int d, L, NT, DB;
  int64_t b_img, h_off, beta_off, size;
};

static inline CrossGeom cross_geom(int d, int L) {
  CrossGeom g{};
  g.d = d;
  g.L = L;
  g.NT = (L + 15) / 16;
  g.DB = (d + 3) / 4;
  g.b_img = (int64_t)g.DB * g.NT * 64;
  g.h_off = g.b_img;
  g.beta_off = g.h_off + ((L + 3) / 4) * 4;
  g.size = g.beta_off + ((d + 3) / 4) * 4;
  return g;
}

// B image: rec[t][nt][lane] = w[col][4t + kk] (col = nt*16 + (lane&15), kk = lane>>4)
__global__ void cross_prepare_img(const float* __restrict__ w, int d, int L, int NT, int64_t n,
                                  float* __restrict__ out) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(idx / (NT * 64));
    const int r = (int)(idx % (NT * 64));
    const int nt = r / 64, lane = r % 64;
    const int e = 4 * t + (lane >> 4), col = nt * 16 + (lane & 15);
    out[idx] = (e < d && col < L) ? w[(int64_t)col * d + e] : 0.f;
  }
}

// h_l = beta_l . w_l and beta_L = sum_l b_l (one workgroup, sequential over l).
__global__ void cross_prepare_bias(const float* __restrict__ w, const float* __restrict__ b, int d, int L,
                                   float* __restrict__ h, float* __restrict__ beta) {
  __shared__ float red[16];
  for (int j = threadIdx.x; j < d; j += blockDim.x) beta[j] = 0.f;
  __syncthreads();
  for (int l = 0; l < L; ++l) {
    float p = 0.f;
    for (int j = threadIdx.x; j < d; j += blockDim.x) p = fmaf(beta[j], w[(int64_t)l * d + j], p);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = p;
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
      h[l] = s;
    }
    for (int j = threadIdx.x; j < d; j += blockDim.x) beta[j] += b[(int64_t)l * d + j];
    __syncthreads();
  }
}

struct CrossArgs {
  const float* x0;
  int64_t x_stride;
  int d, L, DB;
  const float* img;
  const float* h;
  const float* beta;
  float* out;
  int64_t out_stride;
  int64_t batch;
  unsigned long long* dbg;  // diagnostics only: per-wave phase stamps (rs_diag_cross_set_dbg)
};
static unsigned long long* g_cross_dbg = nullptr;  // rs_diag_cross_set_dbg
// Phase stamps only in the diagnostic build (scripts/build_diag.sh), like
// MLP_STAMP / DIN_STAMP / IP_STAMP: no runtime check of a.dbg in the product.
#ifdef RS_DIAG_STAMPS
#define CR_STAMP(i)                                                                                   \
  do {                                                                                                \
    if (a.dbg && (threadIdx.x & 63) == 0)                                                             \
      a.dbg[((int64_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define CR_STAMP(i) \
  do {              \
  } while (0)
#endif

// The B fragments of 8 of a wave's k-steps (t0, t0 + NW, ..): L2-resident
// launch constants, so the fused kernels request the first 8 before their
// gather (they arrive inside the id / row trips).
template <int NT, int NW>
struct CrossB {
  float v[8][NT];
  __device__ __forceinline__ void load(const CrossArgs& a, int t0) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = min(t0 + u * NW, a.DB - 1);
      const float* rec = a.img + (int64_t)t * NT * 64;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) v[u][nt] = rec[nt * 64 + lane];
    }
  }
};

// G = X0 @ W on MFMA, K split across the NW waves: the wave's k-steps are
// t = w + NW*i, 8 at a time (B fragments requested before any MFMA waits on
// them; the first 8 from `pre` when the caller prefetched them).  tile rows
// are `ld` floats apart, columns >= a.d read as 0.
template <int NT, int NW>
__device__ __forceinline__ void cross_contract(const CrossArgs& a, const float* tile, int ld,
                                               const CrossB<NT, NW>* pre, floatx4 (&acc)[NT]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  // four accumulation chains: k-step u into chain u & 3 (compile-time, no
  // per-MFMA branch on a runtime flag)
  floatx4 ac[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int c = 0; c < 4; ++c) ac[nt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](int t0, const CrossB<NT, NW>& B) {
    float xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = 4 * (t0 + u * NW) + kk;
      xv[u] = (t0 + u * NW < a.DB && e < a.d) ? tile[s * ld + e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        ac[nt][u & 3] = mfma16x16x4(xv[u], B.v[u][nt], ac[nt][u & 3]);
      }
  };
  if (w < a.DB) {
    if (pre) {
      step(w, *pre);
    } else {
      CrossB<NT, NW> B;
      B.load(a, w);
      step(w, B);
    }
  }
  for (int t0 = w + 8 * NW; t0 < a.DB; t0 += 8 * NW) {
    CrossB<NT, NW> B;
    B.load(a, t0);
    step(t0, B);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[nt][i] = (ac[nt][0][i] + ac[nt][1][i]) + (ac[nt][2][i] + ac[nt][3][i]);
}

// Phases (2)-(4) on a staged 16 x d tile of x0 (rows >= `rows` zero).
// beta: beta_L (a.beta, or its LDS copy when the caller staged one).
template <int NT, int NW>
__device__ __forceinline__ void cross_finish(const CrossArgs& a, float* tile, float* cs, float* alpha, int64_t b0,
                                             int rows, const floatx4 (&acc)[NT], const float* beta);

template <int NT, int NW>
__device__ __forceinline__ void cross_tile(const CrossArgs& a, float* tile, float* cs, float* alpha, int64_t b0,
                                           int rows, const CrossB<NT, NW>* pre = nullptr,
                                           const float* beta = nullptr) {
  // (2) G = X0 @ W on MFMA
  floatx4 acc[NT];
  cross_contract<NT, NW>(a, tile, a.d, pre, acc);
  cross_finish<NT, NW>(a, tile, cs, alpha, b0, rows, acc, beta);
}

// Phases (3)-(4) from each wave's partial G tile `acc` (its share of the
// contraction): partials to LDS, the recurrence, the output pass.  The tile
// must be complete in LDS by the barrier below.
template <int NT, int NW>
__device__ __forceinline__ void cross_finish(const CrossArgs& a, float* tile, float* cs, float* alpha, int64_t b0,
                                             int rows, const floatx4 (&acc)[NT], const float* beta) {
  if (!beta) beta = a.beta;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  const int n = rows * a.d;
  constexpr int CW = NT * 16 + 1;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[(w * 16 + kk * 4 + r) * CW + nt * 16 + s] = acc[nt][r];
  CR_STAMP(3);
  __syncthreads();
  CR_STAMP(4);

  // (3) per-sample recurrence alpha_{l+1} = alpha_l (1 + g_l) + h_l
  if (threadIdx.x < 16) {
    float al = 1.f;
    for (int l = 0; l < a.L; ++l) {
      float g = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) g += cs[(ww * 16 + threadIdx.x) * CW + l];
      al = fmaf(al, 1.f + g, a.h[l]);
    }
    alpha[threadIdx.x] = al;
  }
  __syncthreads();
  CR_STAMP(5);

  // (4) out = alpha * x0 + beta_L.  The workgroup's rows are one contiguous
  // block when out_stride == d (16-B aligned: b0 is a multiple of 16): float4
  // stores over it, a chunk's four elements may straddle two rows (row /
  // column tracked incrementally, no per-element division); scalar stores
  // are issue-bound (~4 B/clk/CU), so they only take the strided case.
  if (a.out_stride == a.d && ((uintptr_t)(a.out + b0 * a.d) % 16 == 0)) {
    floatx4* dst = reinterpret_cast<floatx4*>(a.out + b0 * a.d);
    const int n4 = n / 4;
    const int step = 4 * NW * 64, dq = step / a.d, dr = step - dq * a.d;
    int i = threadIdx.x, r = (4 * i) / a.d, j = 4 * i - r * a.d;
    for (; i < n4; i += NW * 64) {
      const floatx4 x = reinterpret_cast<const floatx4*>(tile)[i];  // tile rows are d apart too
      floatx4 v;
      int rr = r, jj = j;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = fmaf(alpha[rr], x[q], beta[jj]);
        if (++jj == a.d) { jj = 0; ++rr; }
      }
      __builtin_nontemporal_store(v, dst + i);  // streamed: 8.6 -> 7.7 us (profiles/r6_ab_cross_nt_out.jsonl)
      r += dq;
      j += dr;
      if (j >= a.d) { j -= a.d; ++r; }
    }
    for (int e = n4 * 4 + threadIdx.x; e < n; e += NW * 64) {  // a ragged last tile's tail
      const int rr = e / a.d, jj = e - rr * a.d;
      a.out[b0 * a.d + e] = fmaf(alpha[rr], tile[e], beta[jj]);
    }
  } else {
    for (int r = 0; r < rows; ++r) {
      float* orow = a.out + (b0 + r) * a.out_stride;
      const float al = alpha[r];
      for (int j = threadIdx.x; j < a.d; j += NW * 64) orow[j] = fmaf(al, tile[r * a.d + j], beta[j]);
    }
  }
  CR_STAMP(6);
}

template <int NT, int NW>
__global__ __launch_bounds__(NW * 64) void cross_mfma(CrossArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tile = smem;                                       // [16][d]
  float* cs = smem + ((16 * a.d + 3) / 4) * 4;              // [NW][16][NT*16+1]
  float* alpha = cs + NW * 16 * (NT * 16 + 1);              // [16]
  const int64_t b0 = (int64_t)blockIdx.x * 16;
  const int rows = (int)((a.batch - b0) < 16 ? (a.batch - b0) : 16);

  // (1) stage the 16 x d tile of x0 (coalesced)
  const int n = rows * a.d;
  if (a.x_stride == a.d && ((uintptr_t)(a.x0 + b0 * a.d) % 16 == 0)) {
    // all of a thread's float4 loads are issued before its LDS stores (a
    // load->store loop would pay one HBM round trip per iteration)
    const float* src = a.x0 + b0 * a.d;
    const int n4 = n / 4;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 8 * NW * 64) {
      floatx4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * NW * 64;
        v[u] = i < n4 ? reinterpret_cast<const floatx4*>(src)[i] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * NW * 64;
        if (i < n4) reinterpret_cast<floatx4*>(tile)[i] = v[u];
      }
    }
    for (int i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) tile[i] = src[i];
  } else {
    for (int r = 0; r < rows; ++r)
      for (int j = threadIdx.x; j < a.d; j += blockDim.x) tile[r * a.d + j] = a.x0[(b0 + r) * a.x_stride + j];
  }
  for (int i = n + threadIdx.x; i < 16 * a.d; i += blockDim.x) tile[i] = 0.f;
  __syncthreads();
  cross_tile<NT, NW>(a, tile, cs, alpha, b0, rows);
}

// Fused DCN input + CrossNet (model/dcn.py:24-27 + CrossLayer): x0 = [dense |
// EmbedLayer(ids)] is assembled straight into the LDS tile (cooperative id
// tile, one sample per wave, every row chunk requested before any LDS store),
// so x0 never round-trips through HBM; then phases (2)-(4).  k % 4 == 0.
struct EmbedCrossArgs {
  const void* ids;
  int64_t id_stride;
  const float* dense;
  int64_t dense_stride;
  int nd, F, k;
  const float* table;
  const int64_t* offs;
  const int64_t* vocab;
  int* err;
};

constexpr int EC_FMAX = 128;

// KA: the field metadata by value (rs_embed_cross_fwd_hm, k = 16, <= 32
// fields): the headline kernel's front end (tile_gather.hpp) instead of the
// cooperative id tile.
// The kernarg front end with the CrossNet contraction done from registers
// (k 16, <= 2 NW fields, <= 16 B columns): wave w gathers fields w and w + NW
// with lane (s = l & 15, q = l >> 4) loading chunk q of sample s's row — the
// MFMA A layout, so the float4 is four MFMAs' A operands (k-slot q of columns
// nd + 16c + 4q + j, j = 0..3) — and contracts them against B fragments read
// per lane from the prepared image (record col / 4, k-slot col % 4) while
// storing them into the tile (row pitch ld, columns [dense nd | fields]); wave
// NW-1-g also contracts dense k-group g (the dense tile columns are the
// caller's).  Rows in two bursts as the headline kernel: the second
// requested once the first is in.  Returns the lane's bad-id flag; `acc` =
// this wave's partial G tile (rows = samples, columns = B columns).
template <int NW, int KIND>
__device__ __forceinline__ bool gather_contract_reg(const CrossArgs& a, const EmbedCrossArgs& e, const FieldMeta* km,
                                                    int64_t b0, int rows, float* tile, int ld, floatx4& acc) {
  typedef Ids<KIND> I;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, q = lane >> 4, F = e.F;
  const int64_t bb = b0 + (s < rows ? s : rows - 1);
  const int c0 = w, c1 = w + NW;
  typename I::raw_t r0{}, r1{};
  if (c0 < F) r0 = I::load(e.ids, bb * e.id_stride + c0);
  if (c1 < F) r1 = I::load(e.ids, bb * e.id_stride + c1);
  auto bimg = [&](int col) -> float { return a.img[(int64_t)(col >> 2) * 64 + (col & 3) * 16 + s]; };
  float bf0[4] = {0.f, 0.f, 0.f, 0.f}, bf1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c0 < F) bf0[j] = bimg(e.nd + 16 * c0 + 4 * q + j);
    if (c1 < F) bf1[j] = bimg(e.nd + 16 * c1 + 4 * q + j);
  }
  floatx4 ac[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ac[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int g = NW - 1 - w; 16 * g < e.nd; g += NW) {  // dense k-groups (nd = 13: wave NW-1 only)
    float xd[4], bd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = 16 * g + 4 * q + j;
      const bool ok = col < e.nd;
      xd[j] = ok && s < rows ? e.dense[bb * e.dense_stride + col] : 0.f;
      bd[j] = ok ? bimg(col) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) ac[j] = mfma16x16x4(xd[j], bd[j], ac[j]);
  }
  bool bad = false;
  auto row = [&](int c, typename I::raw_t r) -> floatx4 {
    int64_t id;
    const bool ok = I::decode(r, km->voc[c], id);
    bad |= !ok && s < rows;
    floatx4 x = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(e.table + (km->off[c] + id) * 16) + q);
    if (!ok || s >= rows) x = floatx4{0.f, 0.f, 0.f, 0.f};
    return x;
  };
  auto put = [&](int c, floatx4 x) {
    float* p = tile + s * ld + e.nd + c * 16 + 4 * q;
    p[0] = x[0];
    p[1] = x[1];
    p[2] = x[2];
    p[3] = x[3];
  };
  floatx4 x0v{0.f, 0.f, 0.f, 0.f}, x1v{0.f, 0.f, 0.f, 0.f};
  if (c0 < F) {
    x0v = row(c0, r0);
    put(c0, x0v);
  }
  if (c1 < F) x1v = row(c1, r1);
  if (c0 < F) {
#pragma unroll
    for (int j = 0; j < 4; ++j) ac[j] = mfma16x16x4(x0v[j], bf0[j], ac[j]);
  }
  if (c1 < F) {
    put(c1, x1v);
#pragma unroll
    for (int j = 0; j < 4; ++j) ac[j] = mfma16x16x4(x1v[j], bf1[j], ac[j]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = (ac[0][i] + ac[1][i]) + (ac[2][i] + ac[3][i]);
  return bad;
}

// REG (RS_OPT_CROSS_KERNEL 0, the default on the kernarg front end, L <= 16):
// gather_contract_reg — each wave's partial G tile goes straight to the
// cross-wave sums: no post-gather tile reads, no contraction phase, one
// barrier fewer.  G's summation order differs from the staged-tile
// contraction (REG false: bit-identical to the cooperative-id-tile kernel),
// so the two forms agree to rounding.
template <int NT, int KIND, bool KA, bool REG = false>
__device__ __forceinline__ void embed_cross_body(const CrossArgs& a, const EmbedCrossArgs& e, const FieldMeta* km) {
  constexpr int NW = 16;
  typedef Ids<KIND> I;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tile = smem;
  float* cs = smem + ((16 * a.d + 3) / 4) * 4;
  float* alpha = cs + NW * 16 * (NT * 16 + 1);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b0 = (int64_t)blockIdx.x * 16;
  const int rows = (int)((a.batch - b0) < 16 ? (a.batch - b0) : 16);
  const int F = e.F;
  if constexpr (KA && REG) {
    static_assert(NT == 1, "register contraction: at most 16 cross layers");
    CR_STAMP(0);
    float* betal = alpha + 16;
    const float bv0 = tid < a.d ? a.beta[tid] : 0.f;
    const float bv1 = tid + NW * 64 < a.d ? a.beta[tid + NW * 64] : 0.f;
    {  // dense columns into the tile (wave w: sample w)
      const int64_t bw = b0 + (w < rows ? w : rows - 1);
      for (int j = lane; j < e.nd; j += 64) tile[w * a.d + j] = w < rows ? e.dense[bw * e.dense_stride + j] : 0.f;
    }
    floatx4 acc[1];
    const bool bad = gather_contract_reg<NW, KIND>(a, e, km, b0, rows, tile, a.d, acc[0]);
    if (__any(bad) && lane == 0) flag_error(e.err);
    if (tid < a.d) betal[tid] = bv0;
    if (tid + NW * 64 < a.d) betal[tid + NW * 64] = bv1;
    CR_STAMP(1);
    CR_STAMP(2);
    cross_finish<1, NW>(a, tile, cs, alpha, b0, rows, acc, a.d <= 2 * NW * 64 ? betal : a.beta);
    return;
  } else if constexpr (KA) {
    CR_STAMP(0);
    CrossB<NT, NW> pre;  // the contraction's first B fragments ride the gather's trips
    pre.load(a, w);
    // beta_L (sample-independent) rides them too: registers now, LDS after the gather
    float* betal = alpha + 16;
    const float bv0 = tid < a.d ? a.beta[tid] : 0.f;
    const float bv1 = tid + NW * 64 < a.d ? a.beta[tid + NW * 64] : 0.f;
    {  // dense columns (wave w: sample w), requested beside the ids
      const int64_t bb = b0 + (w < rows ? w : rows - 1);
      for (int j = lane; j < e.nd; j += 64) tile[w * a.d + j] = w < rows ? e.dense[bb * e.dense_stride + j] : 0.f;
    }
    const bool bad = gather_tile_k16<NW, KIND>(e.ids, e.id_stride, e.table, km, F, b0, rows,
                                               [&](int s, int c, int q, floatx4 x) {
                                                 float* p = tile + s * a.d + e.nd + c * 16 + 4 * q;
                                                 p[0] = x[0];
                                                 p[1] = x[1];
                                                 p[2] = x[2];
                                                 p[3] = x[3];
                                               });
    if (__any(bad) && lane == 0) flag_error(e.err);
    if (tid < a.d) betal[tid] = bv0;
    if (tid + NW * 64 < a.d) betal[tid + NW * 64] = bv1;
    CR_STAMP(1);
    __syncthreads();
    CR_STAMP(2);
    cross_tile<NT, NW>(a, tile, cs, alpha, b0, rows, &pre, a.d <= 2 * NW * 64 ? betal : a.beta);
    return;
  } else {
  __shared__ typename I::raw_t lid[16][EC_FMAX];
  __shared__ int64_t lmeta[2][EC_FMAX];

  for (int t = tid; t < 16 * F; t += NW * 64) {
    const int ss = t / F, c = t - ss * F;
    lid[ss][c] = I::load(e.ids, (b0 + (ss < rows ? ss : rows - 1)) * e.id_stride + c);
  }
  for (int t = tid; t < 2 * F; t += NW * 64) {
    const int c = t < F ? t : t - F;
    lmeta[t < F ? 0 : 1][c] = t < F ? e.offs[c] : e.vocab[c];
  }
  // dense columns (wave w: sample w)
  {
    const int64_t bb = b0 + (w < rows ? w : rows - 1);
    for (int j = lane; j < e.nd; j += 64) tile[w * a.d + j] = w < rows ? e.dense[bb * e.dense_stride + j] : 0.f;
  }
  __syncthreads();

  // rows: wave w gathers sample w's F*k/4 float4 chunks
  bool bad = false;
  {
    const int KQ = e.k >> 2, FKQ = F * KQ;
    const int nit = (FKQ + 63) >> 6;
    // one 64-chunk slice per pass (26 fields x 4 chunks: 2 passes) — as in
    // the headline kernel, requesting the rows in two waves beats one burst
    constexpr int CP = 1;
    for (int base = 0; base < nit; base += CP) {
      floatx4 v[CP];
      int dst[CP];
#pragma unroll
      for (int u = 0; u < CP; ++u) {
        const int ch = (base + u) * 64 + lane;
        dst[u] = -1;
        v[u] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (base + u < nit && ch < FKQ) {
          const int c = ch / KQ, q = ch - c * KQ;
          int64_t id;
          const bool ok = I::decode(lid[w][c], lmeta[1][c], id);
          bad |= !ok && w < rows;
          const floatx4 t =
              __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(e.table + (lmeta[0][c] + id) * e.k + 4 * q));
          v[u] = (ok && w < rows) ? t : floatx4{0.f, 0.f, 0.f, 0.f};
          dst[u] = w * a.d + e.nd + c * e.k + 4 * q;
        }
      }
#pragma unroll
      for (int u = 0; u < CP; ++u)
        if (dst[u] >= 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) tile[dst[u] + q] = v[u][q];
        }
    }
  }
  if (__any(bad) && lane == 0) flag_error(e.err);
  __syncthreads();
  cross_tile<NT, NW>(a, tile, cs, alpha, b0, rows);
  }
}

template <int NT, int KIND>
__global__ __launch_bounds__(16 * 64) void embed_cross(CrossArgs a, EmbedCrossArgs e) {
  embed_cross_body<NT, KIND, false>(a, e, nullptr);
}
template <int NT, int KIND, bool REG = false>
__global__ __launch_bounds__(16 * 64) void embed_cross_ka(CrossArgs a, EmbedCrossArgs e, FieldMeta m) {
  embed_cross_body<NT, KIND, true, REG>(a, e, &m);
}

// Fused DCN forward (model/dcn.py:24-34) in ONE launch: x0 = [dense |
// EmbedLayer(ids)] assembled in the DNN tower's LDS tile (Keras column order,
// row pitch t.rs); CrossNet as the usual G = X0 @ [w_0..w_{L-1}, w_o[:d]]
// contraction (the output Dense's cross half is one more B column: the cross
// branch's logit is alpha_L (x0.w_o) + beta_L.w_o = alpha_L g_L + h_L, x_L is
// never formed); the DNN tower on the same tile with its last layer folded
// with the output Dense's DNN half; head sigmoid(dnn + cross).
template <int NT, int KIND, bool KA, bool TAIL = false, bool REG = false>
__device__ __forceinline__ void dcn_fused_body(const CrossArgs& a, const EmbedCrossArgs& e, const MlpArgs& t,
                                               const FieldMeta* km) {
  constexpr int NW = 16;
  typedef Ids<KIND> I;
  extern __shared__ __attribute__((aligned(16))) float tsm[];
  constexpr int CW = NT * 16 + 1;
  __shared__ float cs[NW * 16 * CW];
  __shared__ float xlog[16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s = lane & 15, kk = lane >> 4;
  const int64_t b0 = (int64_t)blockIdx.x * 16;
  const int rows = (int)((a.batch - b0) < 16 ? (a.batch - b0) : 16);
  const int F = e.F, RS = t.rs, d = a.d;

  // tower weights and biases first (independent of the ids)
  floatx4 ring[MLP_R];
  mlp_first_fill<NW>(t, ring);
  float* par = tsm + 32 * RS + NW * 256;
  for (int i = tid; i < t.ptot; i += NW * 64) par[i] = t.prep[t.wtot + i];
  floatx4 acc[NT];
  if constexpr (KA && REG) {  // RS_OPT_CROSS_KERNEL 0: the contraction from the gathered registers
    static_assert(NT == 1, "register contraction: at most 15 cross layers");
    {  // dense columns + zero padding of the tile row (wave w: sample w)
      const int64_t bb = b0 + (w < rows ? w : rows - 1);
      for (int j = lane; j < e.nd; j += 64) tsm[w * RS + j] = w < rows ? e.dense[bb * e.dense_stride + j] : 0.f;
      for (int j = d + lane; j < t.Kp[0]; j += 64) tsm[w * RS + j] = 0.f;
    }
    const bool bad = gather_contract_reg<NW, KIND>(a, e, km, b0, rows, tsm, RS, acc[0]);
    if (__any(bad) && lane == 0) flag_error(e.err);
  } else {
  CrossB<NT, NW> pre;  // KA: the contraction's first B fragments ride the gather's trips
  if constexpr (KA) pre.load(a, w);
  if constexpr (KA) {
    {  // dense columns + zero padding of the tile row (wave w: sample w)
      const int64_t bb = b0 + (w < rows ? w : rows - 1);
      for (int j = lane; j < e.nd; j += 64) tsm[w * RS + j] = w < rows ? e.dense[bb * e.dense_stride + j] : 0.f;
      for (int j = d + lane; j < t.Kp[0]; j += 64) tsm[w * RS + j] = 0.f;
    }
    const bool bad = gather_tile_k16<NW, KIND>(e.ids, e.id_stride, e.table, km, F, b0, rows,
                                               [&](int sm, int c, int q, floatx4 x) {
                                                 float* p = tsm + sm * RS + e.nd + c * 16 + 4 * q;
                                                 p[0] = x[0];
                                                 p[1] = x[1];
                                                 p[2] = x[2];
                                                 p[3] = x[3];
                                               });
    if (__any(bad) && lane == 0) flag_error(e.err);
    __syncthreads();
  } else {
  __shared__ typename I::raw_t lid[16][EC_FMAX];
  __shared__ int64_t lmeta[2][EC_FMAX];
  for (int t0 = tid; t0 < 16 * F; t0 += NW * 64) {
    const int ss = t0 / F, c = t0 - ss * F;
    lid[ss][c] = I::load(e.ids, (b0 + (ss < rows ? ss : rows - 1)) * e.id_stride + c);
  }
  for (int t0 = tid; t0 < 2 * F; t0 += NW * 64) {
    const int c = t0 < F ? t0 : t0 - F;
    lmeta[t0 < F ? 0 : 1][c] = t0 < F ? e.offs[c] : e.vocab[c];
  }
  {  // dense columns + zero padding of the tile row (wave w: sample w)
    const int64_t bb = b0 + (w < rows ? w : rows - 1);
    for (int j = lane; j < e.nd; j += 64) tsm[w * RS + j] = w < rows ? e.dense[bb * e.dense_stride + j] : 0.f;
    for (int j = d + lane; j < t.Kp[0]; j += 64) tsm[w * RS + j] = 0.f;
  }
  __syncthreads();
  bool bad = false;
  {  // rows: wave w gathers sample w's F*k/4 float4 chunks into its tile row
    const int KQ = e.k >> 2, FKQ = F * KQ;
    const int nit = (FKQ + 63) >> 6;
    // one 64-chunk slice per pass (26 fields x 4 chunks: 2 passes) — as in
    // the headline kernel, requesting the rows in two waves beats one burst
    constexpr int CP = 1;
    for (int base = 0; base < nit; base += CP) {
      floatx4 v[CP];
      int dst[CP];
#pragma unroll
      for (int u = 0; u < CP; ++u) {
        const int ch = (base + u) * 64 + lane;
        dst[u] = -1;
        v[u] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (base + u < nit && ch < FKQ) {
          const int c = ch / KQ, q = ch - c * KQ;
          int64_t id;
          const bool ok = I::decode(lid[w][c], lmeta[1][c], id);
          bad |= !ok && w < rows;
          const floatx4 x =
              __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(e.table + (lmeta[0][c] + id) * e.k + 4 * q));
          v[u] = (ok && w < rows) ? x : floatx4{0.f, 0.f, 0.f, 0.f};
          dst[u] = w * RS + e.nd + c * e.k + 4 * q;
        }
      }
#pragma unroll
      for (int u = 0; u < CP; ++u)
        if (dst[u] >= 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) tsm[dst[u] + q] = v[u][q];
        }
    }
  }
  if (__any(bad) && lane == 0) flag_error(e.err);
  __syncthreads();
  }

  // CrossNet contraction G = X0 @ [w_0 .. w_{L-1}, w_o[:d]] (a.L = L + 1 columns)
  cross_contract<NT, NW>(a, tsm, RS, KA ? &pre : nullptr, acc);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[(w * 16 + kk * 4 + r) * CW + nt * 16 + s] = acc[nt][r];
  __syncthreads();
  if (tid < 16) {  // alpha recurrence over the L real layers, then the cross logit
    const int L = a.L - 1;
    float al = 1.f;
    for (int l = 0; l < L; ++l) {
      float g = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) g += cs[(ww * 16 + tid) * CW + l];
      al = fmaf(al, 1.f + g, a.h[l]);
    }
    float go = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) go += cs[(ww * 16 + tid) * CW + L];
    xlog[tid] = fmaf(al, go, a.h[L]);
  }
  // (the tower's first barrier publishes xlog and the tile)
  if constexpr (TAIL) {
    // layer 0 as usual, layers 1.. as the split-K tail at the DeepFM / DCN
    // widths (256 -> 128 -> 64 -> 1: all 16 waves per layer, mlp_tail_splitk)
    if (t.Np[0] == NW * 16) mlp_layer0_tiles<NW>(t, tsm, ring);
    else mlp_tower_tile<NW>(t, tsm, b0, ring, xlog, 0, 1);
    mlp_tail_run<NW>(t, tsm, b0, xlog);
  } else {
    mlp_tower_tile<NW>(t, tsm, b0, ring, xlog);
  }
}

template <int NT, int KIND>
__global__ __launch_bounds__(16 * 64) void dcn_fused(CrossArgs a, EmbedCrossArgs e, MlpArgs t) {
  dcn_fused_body<NT, KIND, false>(a, e, t, nullptr);
}
template <int NT, int KIND, bool TAIL = false, bool REG = false>
__global__ __launch_bounds__(16 * 64) void dcn_fused_ka(CrossArgs a, EmbedCrossArgs e, MlpArgs t, FieldMeta m) {
  dcn_fused_body<NT, KIND, true, TAIL, REG>(a, e, t, &m);
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_cross_prepared_size(int d, int n_layers) {
  if (d < 1 || n_layers < 0) return -1;
  return cross_geom(d, n_layers < 1 ? 1 : n_layers).size;
}

extern "C" int rs_cross_prepare(const float* w, const float* b, int d, int n_layers, float* prepared,
                                rs_stream_t stream) {
  RS_REQUIRE(d >= 1 && n_layers >= 0 && n_layers <= 32, "rs_cross_prepare: bad shape (d>=1, 0<=L<=32)");
  RS_REQUIRE(prepared && (n_layers == 0 || (w && b)), "rs_cross_prepare: null pointer");
  const int L = n_layers;
  const CrossGeom g = cross_geom(d, L < 1 ? 1 : L);
  hipStream_t st = as_stream(stream);
  (void)hipMemsetAsync(prepared, 0, g.size * sizeof(float), st);
  if (L > 0) {
    int64_t grid = (g.b_img + 255) / 256;
    if (grid > 4096) grid = 4096;
    cross_prepare_img<<<(unsigned)grid, 256, 0, st>>>(w, d, L, g.NT, g.b_img, prepared);
    cross_prepare_bias<<<1, 1024, 0, st>>>(w, b, d, L, prepared + g.h_off, prepared + g.beta_off);
  }
  return launch_status("rs_cross_prepare");
}

extern "C" int rs_cross_fwd(const float* x0, int64_t x_stride, int d, int n_layers, const float* prepared,
                            float* out, int64_t out_stride, int64_t batch, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(x0 && prepared && out, "rs_cross_fwd: null pointer");
  RS_REQUIRE(d >= 1 && n_layers >= 0 && n_layers <= 32 && batch >= 0, "rs_cross_fwd: bad shape");
  RS_REQUIRE(x_stride >= d && out_stride >= d, "rs_cross_fwd: stride < d");
  RS_REQUIRE(d <= 2304, "rs_cross_fwd: d > 2304 not supported (LDS tile)");
  if (batch == 0) return RS_OK;
  const int L = n_layers;
  const CrossGeom g = cross_geom(d, L < 1 ? 1 : L);
  CrossArgs a{x0, x_stride, d, L, g.DB, prepared, prepared + g.h_off, prepared + g.beta_off, out, out_stride, batch,
              g_cross_dbg};
  constexpr int NW = 8;
  const size_t lds = (size_t)(((16 * d + 3) / 4) * 4 + NW * 16 * (g.NT * 16 + 1) + 16) * sizeof(float);
  const unsigned grid = (unsigned)((batch + 15) / 16);
  hipStream_t st = as_stream(stream);
  if (g.NT == 1) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)cross_mfma<1, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    cross_mfma<1, NW><<<grid, NW * 64, lds, st>>>(a);
  } else {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)cross_mfma<2, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    cross_mfma<2, NW><<<grid, NW * 64, lds, st>>>(a);
  }
  return launch_status("rs_cross_fwd");
}

namespace rs {
// host field metadata -> FieldMeta for the kernarg front end (k = 16, <= 32 fields), else null
static const FieldMeta* host_meta(FieldMeta& m, const int64_t* off_h, const int64_t* voc_h, int n_fields, int k) {
  if (!off_h || !voc_h || k != 16 || n_fields < 1 || n_fields > 32) return nullptr;
  for (int c = 0; c < n_fields; ++c) {
    m.off[c] = off_h[c];
    m.voc[c] = voc_h[c];
  }
  return &m;
}

static int embed_cross_run(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                           int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                           const int64_t* field_vocab, int n_fields, int k, int n_layers, const float* prepared,
                           float* out, int64_t out_stride, int64_t batch, int* err_flag, rs_stream_t stream,
                           const FieldMeta* hm) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(ids && table && field_offsets && field_vocab && prepared && out, "rs_embed_cross_fwd: null pointer");
  RS_REQUIRE(nd == 0 || dense, "rs_embed_cross_fwd: dense is null");
  RS_REQUIRE(n_fields >= 1 && n_fields <= EC_FMAX && nd >= 0 && k >= 4 && k % 4 == 0,
             "rs_embed_cross_fwd: need 1..128 fields and k a multiple of 4");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_cross_fwd: bad id_kind");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_embed_cross_fwd: table must be 16-B aligned");
  const int d = nd + n_fields * k;
  RS_REQUIRE(n_layers >= 0 && n_layers <= 32 && batch >= 0, "rs_embed_cross_fwd: bad shape");
  RS_REQUIRE(out_stride >= d, "rs_embed_cross_fwd: out_stride < d");
  RS_REQUIRE(d <= 1600, "rs_embed_cross_fwd: d > 1600 not supported (LDS tile)");
  if (batch == 0) return RS_OK;
  const int L = n_layers;
  const CrossGeom g = cross_geom(d, L < 1 ? 1 : L);
  CrossArgs a{nullptr, d, d, L, g.DB, prepared, prepared + g.h_off, prepared + g.beta_off, out, out_stride, batch,
              g_cross_dbg};
  EmbedCrossArgs e{ids, id_stride, dense, dense_stride, nd, n_fields, k, table, field_offsets, field_vocab, err_flag};
  constexpr int NW = 16;
  // tile | contraction partials | alpha[16] | beta_L copy (the kernarg front end)
  const size_t lds =
      (size_t)(((16 * d + 3) / 4) * 4 + NW * 16 * (g.NT * 16 + 1) + 16 + ((d + 3) / 4) * 4) * sizeof(float);
  const unsigned grid = (unsigned)((batch + 15) / 16);
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KIND = decltype(K)::value;
    if (hm && g.NT == 1 && opt(RS_OPT_CROSS_KERNEL) == 0) {
      static LdsAttr setr;
      lds_attr(setr, (const void*)embed_cross_ka<1, KIND, true>, lds);
      embed_cross_ka<1, KIND, true><<<grid, NW * 64, lds, st>>>(a, e, *hm);
    } else if (hm && g.NT == 1) {
      static LdsAttr setk1;
      lds_attr(setk1, (const void*)embed_cross_ka<1, KIND>, lds);
      embed_cross_ka<1, KIND><<<grid, NW * 64, lds, st>>>(a, e, *hm);
    } else if (hm) {
      static LdsAttr setk2;
      lds_attr(setk2, (const void*)embed_cross_ka<2, KIND>, lds);
      embed_cross_ka<2, KIND><<<grid, NW * 64, lds, st>>>(a, e, *hm);
    } else if (g.NT == 1) {
      static LdsAttr set1;
      lds_attr(set1, (const void*)embed_cross<1, KIND>, lds);
      embed_cross<1, KIND><<<grid, NW * 64, lds, st>>>(a, e);
    } else {
      static LdsAttr set2;
      lds_attr(set2, (const void*)embed_cross<2, KIND>, lds);
      embed_cross<2, KIND><<<grid, NW * 64, lds, st>>>(a, e);
    }
  });
  return launch_status("rs_embed_cross_fwd");
}
}  // namespace rs

extern "C" int rs_embed_cross_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                  int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                                  const int64_t* field_vocab, int n_fields, int k, int n_layers,
                                  const float* prepared, float* out, int64_t out_stride, int64_t batch,
                                  int* err_flag, rs_stream_t stream) {
  return embed_cross_run(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab,
                         n_fields, k, n_layers, prepared, out, out_stride, batch, err_flag, stream, nullptr);
}

extern "C" int rs_embed_cross_fwd_hm(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                     int64_t dense_stride, int nd, const float* table,
                                     const int64_t* field_offsets, const int64_t* field_vocab,
                                     const int64_t* field_offsets_host, const int64_t* field_vocab_host,
                                     int n_fields, int k, int n_layers, const float* prepared, float* out,
                                     int64_t out_stride, int64_t batch, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(field_offsets_host && field_vocab_host, "rs_embed_cross_fwd_hm: host metadata missing");
  FieldMeta m;
  return embed_cross_run(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab,
                         n_fields, k, n_layers, prepared, out, out_stride, batch, err_flag, stream,
                         host_meta(m, field_offsets_host, field_vocab_host, n_fields, k));
}

namespace rs {
static bool dcn_geom(int nd, int n_fields, int k, int n_cross, int n_layers, const int* dims, MlpGeom& mg) {
  if (nd < 0 || n_fields < 1 || n_fields > EC_FMAX || k < 4 || k % 4 != 0 || n_cross < 0 || n_cross > 31) return false;
  if (!mlp_geom(n_layers, dims, mg)) return false;
  const int d = nd + n_fields * k;
  // static LDS: ids (<= 16 KB) + meta 2 KB + partials (<= 33.8 KB) + the tower's dynamic LDS
  return dims[0] == d && dims[n_layers] == 1 && mg.lds <= 100 * 1024;
}
}  // namespace rs

extern "C" int rs_dcn_fused_ok(int nd, int n_fields, int k, int n_cross, int n_layers, const int* dims) {
  MlpGeom mg;
  return dims && dcn_geom(nd, n_fields, k, n_cross, n_layers, dims, mg) ? 1 : 0;
}

namespace rs {
static int dcn_run(const void* ids, int id_kind, int64_t id_stride, const float* dense, int64_t dense_stride,
                   int nd, const float* table, const int64_t* field_offsets, const int64_t* field_vocab,
                   int n_fields, int k, int n_cross, const float* cross_prepared, int n_layers, const int* dims,
                   const int* acts, const float* mlp_prepared, float* out, int64_t batch, int* err_flag,
                   rs_stream_t stream, const FieldMeta* hm) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  MlpGeom mg;
  RS_REQUIRE(dims && acts, "rs_dcn_fwd: null dims/acts");
  RS_REQUIRE(dcn_geom(nd, n_fields, k, n_cross, n_layers, dims, mg), "rs_dcn_fwd: unsupported shape (rs_dcn_fused_ok)");
  RS_REQUIRE(ids && table && field_offsets && field_vocab && cross_prepared && mlp_prepared && out,
             "rs_dcn_fwd: null pointer");
  RS_REQUIRE(nd == 0 || dense, "rs_dcn_fwd: dense is null");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32 && batch >= 0, "rs_dcn_fwd: bad ids");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_dcn_fwd: table must be 16-B aligned");
  MlpArgs t{};
  RS_REQUIRE(mlp_fill_args(mg, acts, mlp_prepared, t), "rs_dcn_fwd: bad activation");
  t.y = out;
  t.ys = 1;
  t.head = 1;
  t.c0 = 1.f;
  t.c1 = 1.f;
  t.M = batch;
  const int d = nd + n_fields * k, Lx = n_cross + 1;  // + the output Dense's cross column
  const CrossGeom g = cross_geom(d, Lx);
  CrossArgs a{nullptr, d, d, Lx, g.DB, cross_prepared, cross_prepared + g.h_off, cross_prepared + g.beta_off,
              nullptr, 0, batch, g_cross_dbg};
  EmbedCrossArgs e{ids, id_stride, dense, dense_stride, nd, n_fields, k, table, field_offsets, field_vocab, err_flag};
  const size_t lds = mg.lds;
  const unsigned grid = (unsigned)((batch + 15) / 16);
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KIND = decltype(K)::value;
    int gwa = 0, gwb = 0;
    const bool reg = opt(RS_OPT_CROSS_KERNEL) == 0;
    if (hm && g.NT == 1 && mlp_tail_ok(t.Np, t.Kp, t.N, t.L, 1, gwa, gwb) && gwa == 8 && gwb == 2) {
      // the split-K tail at the reference's 256-128-64 tower
      if (reg) {
        static LdsAttr setktr;
        lds_attr(setktr, (const void*)dcn_fused_ka<1, KIND, true, true>, lds);
        dcn_fused_ka<1, KIND, true, true><<<grid, 16 * 64, lds, st>>>(a, e, t, *hm);
      } else {
        static LdsAttr setkt;
        lds_attr(setkt, (const void*)dcn_fused_ka<1, KIND, true>, lds);
        dcn_fused_ka<1, KIND, true><<<grid, 16 * 64, lds, st>>>(a, e, t, *hm);
      }
    } else if (hm && g.NT == 1 && reg) {
      static LdsAttr setk1r;
      lds_attr(setk1r, (const void*)dcn_fused_ka<1, KIND, false, true>, lds);
      dcn_fused_ka<1, KIND, false, true><<<grid, 16 * 64, lds, st>>>(a, e, t, *hm);
    } else if (hm && g.NT == 1) {
      static LdsAttr setk1;
      lds_attr(setk1, (const void*)dcn_fused_ka<1, KIND>, lds);
      dcn_fused_ka<1, KIND><<<grid, 16 * 64, lds, st>>>(a, e, t, *hm);
    } else if (hm) {
      static LdsAttr setk2;
      lds_attr(setk2, (const void*)dcn_fused_ka<2, KIND>, lds);
      dcn_fused_ka<2, KIND><<<grid, 16 * 64, lds, st>>>(a, e, t, *hm);
    } else if (g.NT == 1) {
      static LdsAttr set1;
      lds_attr(set1, (const void*)dcn_fused<1, KIND>, lds);
      dcn_fused<1, KIND><<<grid, 16 * 64, lds, st>>>(a, e, t);
    } else {
      static LdsAttr set2;
      lds_attr(set2, (const void*)dcn_fused<2, KIND>, lds);
      dcn_fused<2, KIND><<<grid, 16 * 64, lds, st>>>(a, e, t);
    }
  });
  return launch_status("rs_dcn_fwd");
}
}  // namespace rs

extern "C" int rs_dcn_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense, int64_t dense_stride,
                          int nd, const float* table, const int64_t* field_offsets, const int64_t* field_vocab,
                          int n_fields, int k, int n_cross, const float* cross_prepared, int n_layers,
                          const int* dims, const int* acts, const float* mlp_prepared, float* out, int64_t batch,
                          int* err_flag, rs_stream_t stream) {
  return dcn_run(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab, n_fields, k,
                 n_cross, cross_prepared, n_layers, dims, acts, mlp_prepared, out, batch, err_flag, stream, nullptr);
}

extern "C" int rs_dcn_fwd_hm(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                             int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                             const int64_t* field_vocab, const int64_t* field_offsets_host,
                             const int64_t* field_vocab_host, int n_fields, int k, int n_cross,
                             const float* cross_prepared, int n_layers, const int* dims, const int* acts,
                             const float* mlp_prepared, float* out, int64_t batch, int* err_flag,
                             rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(field_offsets_host && field_vocab_host, "rs_dcn_fwd_hm: host metadata missing");
  FieldMeta m;
  return dcn_run(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab, n_fields, k,
                 n_cross, cross_prepared, n_layers, dims, acts, mlp_prepared, out, batch, err_flag, stream,
                 host_meta(m, field_offsets_host, field_vocab_host, n_fields, k));
}

// diagnostics only: per-wave phase stamps of the CrossNet kernels (null = off)
extern "C" void rs_diag_cross_set_dbg(unsigned long long* p) { rs::g_cross_dbg = p; }
