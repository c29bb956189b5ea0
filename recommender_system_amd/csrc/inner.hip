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
#include "tile_gather.hpp"

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
  int want_inner;  // write the inner products (fast path; the generic kernel always does)
  const float* outer_img;  // OuterProductLayer weights packed by rs_outer_prepare (null: no outer)
  int outer_off;   // column of the first outer product in out
  int contig;      // fast path: out rows are [flat | inner] back to back, 16-B aligned blocks
  int64_t batch;
  int* err;
  unsigned long long* dbg;  // diagnostics only: per-wave phase stamps (rs_diag_inner_set_dbg)
};
// (phase stamps only in the diagnostic build, scripts/build_diag.sh)
#ifdef RS_DIAG_STAMPS
#define IP_STAMP(i)                                                                                   \
  do {                                                                                                \
    if (a.dbg && (threadIdx.x & 63) == 0)                                                             \
      a.dbg[((int64_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define IP_STAMP(i) \
  do {              \
  } while (0)
#endif

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
// k in {4,8,16,32,64}, F <= 64.  Up to 16 samples per 1024-thread workgroup:
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
constexpr int IP_NW = 16, IP_NT = IP_NW * 64;  // 16 waves: one sample per wave in the Gram phase
constexpr int IP_FMAX = 64;

// KA (inner_fast_ka, rs_embed_inner_fwd_hm / rs_embed_product_fwd_hm: K = 16,
// <= 32 fields, 16 samples per workgroup): the rows come in through the
// headline kernel's front end (tile_gather.hpp: field metadata as kernel
// arguments, per-wave field ids, no id tile or barrier before the rows).
template <int K, int KIND, bool KA>
__device__ __forceinline__ void inner_fast_body(const InnerArgs& a, const FieldMeta* km) {
  constexpr int KQ = K / 4;
  typedef Ids<KIND == 3 ? 0 : KIND> I;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int F = a.F, P = F * (F - 1) / 2, S = a.S;
  const int SS = F * K + 4;                    // sample stride: +4 dwords spreads the Gram reads over banks
  const int Pi = a.want_inner ? P : 0, Po = a.outer_img ? P : 0, PP = Pi + Po;
  float* tile = smem;                          // [S][SS]
  float* gram = smem + S * SS;                 // [S][PP]: inner pairs, then outer pairs
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * S;
  const int nvalid = (int)(a.batch - b0 < S ? a.batch - b0 : S);
  IP_STAMP(0);

  if constexpr (KA) {
    static_assert(K == 16 && KIND != 3, "kernarg front end: gathered rows, k = 16");
    const bool bad = gather_tile_k16<IP_NW, KIND>(a.ids, a.id_stride, a.table, km, F, b0, nvalid,
                                                  [&](int s, int c, int q, floatx4 x) {
                                                    *reinterpret_cast<floatx4*>(tile + s * SS + c * 16 + 4 * q) = x;
                                                  });
    IP_STAMP(1);
    if (__any(bad) && (tid & 63) == 0) flag_error(a.err);
    __syncthreads();
    IP_STAMP(2);
  } else {
  __shared__ typename I::raw_t lid[IP_SMAX][IP_FMAX];
  __shared__ int64_t lmeta[2][IP_FMAX];
  if constexpr (KIND != 3) {
    for (int t = tid; t < S * F; t += IP_NT) {
      const int s = t / F, c = t - s * F;
      const int64_t bb = b0 + (s < nvalid ? s : nvalid - 1);
      lid[s][c] = I::load(a.ids, bb * a.id_stride + c);
    }
    for (int t = tid; t < 2 * F; t += IP_NT) {
      const int c = t < F ? t : t - F;
      lmeta[t < F ? 0 : 1][c] = t < F ? a.offs[c] : a.vocab[c];
    }
    __syncthreads();
  }

  bool bad = false;
  const float* src = KIND == 3 ? a.emb : a.table;  // embeddings given vs gathered
  // Row gather: wave w takes samples w, w+4, ...; a sample's F*KQ float4
  // chunks spread over the lanes (chunk = lane + 64*u: field chunk/KQ, quad
  // chunk%KQ), all loads of a pass issued before the LDS stores.
  {
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int FKQ = F * KQ;
    const int per_s = (FKQ + 63) / 64;     // chunks per lane per sample
    const int nit = ((S + IP_NW - 1) / IP_NW) * per_s;  // (sample, chunk-block) steps of this wave
    // one (sample, 64-chunk block) step per pass: the rows go out in two
    // waves at F = 26, k = 16 (as in the headline kernel)
    constexpr int CP = 1;
    for (int base = 0; base < nit; base += CP) {
      floatx4 v[CP];
      int dsti[CP];
#pragma unroll
      for (int u = 0; u < CP; ++u) {
        const int it = base + u;
        const int si = it / per_s, cb = it - si * per_s;  // per_s is 1..2 for F<=64, K<=16
        const int sidx = w + IP_NW * si;
        const int ch = cb * 64 + lane;
        dsti[u] = -1;
        v[u] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (it < nit && sidx < S && ch < FKQ) {
          const int c = ch / KQ, q = ch - c * KQ;
          const int64_t bb = b0 + (sidx < nvalid ? sidx : nvalid - 1);
          int64_t row;
          bool ok = true;
          if constexpr (KIND == 3) {
            row = bb * F + c;
          } else {
            int64_t id;
            ok = I::decode(lid[sidx][c], lmeta[1][c], id);
            row = lmeta[0][c] + id;
            bad |= !ok && sidx < nvalid;
          }
          const floatx4 t = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(src + row * K + 4 * q));
          v[u] = ok ? t : floatx4{0.f, 0.f, 0.f, 0.f};
          dsti[u] = sidx * SS + c * K + 4 * q;
        }
      }
#pragma unroll
      for (int u = 0; u < CP; ++u)
        if (dsti[u] >= 0) *reinterpret_cast<floatx4*>(tile + dsti[u]) = v[u];
    }
  }
  IP_STAMP(1);
  if (bad) flag_error(a.err);
  __syncthreads();
  IP_STAMP(2);
  }

  // Gram matrix per sample on MFMA: G = E E^T with E [F x K] from the LDS
  // tile, 16x16 blocks (bi <= bj) of v_mfma_f32_16x16x4_f32.  Lane l holds
  // float4 E[16b + (l&15)][16grp + 4(l>>4) ..+3] — the A fragment of row block
  // b and, identically, the B fragment of column block b; MFMA j of a group
  // takes component j (k order permuted the same way on both sides).  Only
  // the strict upper triangle i < j < F is stored, at the reference's pair
  // index p(i,j) = i(2F-i-1)/2 + j-i-1 (layer/interaction.py:174-177).
  {
    constexpr int NGRP = (K + 15) / 16;
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int NB = (F + 15) >> 4;
    const int kof = 4 * (lane >> 4);
    for (int si = w; si < S; si += IP_NW) {
      const float* es = tile + si * SS;
      float* gs = gram + si * PP;
      if (!a.want_inner) continue;
      if (NB <= 2) {
        // common case (F <= 32): both row-block fragments read once, the three
        // blocks (0,0) (0,1) (1,1) as independent MFMA chains
        floatx4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c11 = c00;
#pragma unroll
        for (int grp = 0; grp < NGRP; ++grp) {
          const int kk = 16 * grp + kof;
          const int r0 = lane & 15, r1 = 16 + (lane & 15);
          floatx4 f0 = {0.f, 0.f, 0.f, 0.f}, f1 = f0;
          if (kk < K && r0 < F) f0 = *reinterpret_cast<const floatx4*>(es + r0 * K + kk);
          if (kk < K && r1 < F) f1 = *reinterpret_cast<const floatx4*>(es + r1 * K + kk);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            c00 = mfma16x16x4(f0[q], f0[q], c00);
            c01 = mfma16x16x4(f0[q], f1[q], c01);
            c11 = mfma16x16x4(f1[q], f1[q], c11);
          }
        }
        const int jj0 = lane & 15, jj1 = 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i0 = 4 * (lane >> 4) + r, i1 = 16 + i0;
          if (i0 < jj0 && jj0 < F) gs[i0 * (2 * F - i0 - 1) / 2 + jj0 - i0 - 1] = c00[r];
          if (jj1 < F) gs[i0 * (2 * F - i0 - 1) / 2 + jj1 - i0 - 1] = c01[r];
          if (i1 < jj1 && jj1 < F) gs[i1 * (2 * F - i1 - 1) / 2 + jj1 - i1 - 1] = c11[r];
        }
        continue;
      }
      for (int bi = 0; bi < NB; ++bi) {
        for (int bj = bi; bj < NB; ++bj) {
          floatx4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int grp = 0; grp < NGRP; ++grp) {
            const int kk = 16 * grp + kof;
            const int ra = 16 * bi + (lane & 15), rb = 16 * bj + (lane & 15);
            floatx4 fa = {0.f, 0.f, 0.f, 0.f}, fb = {0.f, 0.f, 0.f, 0.f};
            if (kk < K && ra < F) fa = *reinterpret_cast<const floatx4*>(es + ra * K + kk);
            if (kk < K && rb < F) fb = *reinterpret_cast<const floatx4*>(es + rb * K + kk);
#pragma unroll
            for (int q = 0; q < 4; ++q) c = mfma16x16x4(fa[q], fb[q], c);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ii = 16 * bi + 4 * (lane >> 4) + r, jj = 16 * bj + (lane & 15);
            if (ii < jj && jj < F) gs[ii * (2 * F - ii - 1) / 2 + jj - ii - 1] = c[r];
          }
        }
      }
    }
  }
  // OuterProductLayer (layer/interaction.py:186-215): out[b,p] =
  // sum_{a,j} e_row[j] W[a,p,j] e_col[a] — per pair a [16 samples x k] x
  // [k x k] MFMA tile (A = the samples' e_row from the LDS tile, B = W_p^T
  // packed per lane as float4 over 4 k-steps), then the dot with e_col and a
  // DPP row sum over a.  Wave w takes pairs w, w+16, ...
  if (a.outer_img) {
    constexpr int KB = (K + 15) / 16;
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sm = lane & 15, kq = lane >> 4;
    const floatx4* img = reinterpret_cast<const floatx4*>(a.outer_img);
    int i = 0, j = 1;  // (row, col) of the current pair
    // pair index p -> (i, j) in the reference's row-major i<j order, closed
    // form (start(i) = i(2F-i-1)/2) with an integer fix-up: no loops/branches
    // between the pipelined loads
    auto set_pair = [&](int p) {
      const float tf = (float)(2 * F - 1);
      int ii = (int)((tf - sqrtf(tf * tf - 8.f * (float)p)) * 0.5f);
      ii = ii < 0 ? 0 : (ii > F - 2 ? F - 2 : ii);
      if (ii * (2 * F - ii - 1) / 2 > p) --ii;
      if ((ii + 1) * (2 * F - ii - 2) / 2 <= p && ii < F - 2) ++ii;
      i = ii;
      j = p - ii * (2 * F - ii - 1) / 2 + ii + 1;
    };
    // B fragments (L2) of the wave's next pair are requested while the
    // current pair computes (two named register sets, no copies: a copy of
    // an in-flight load makes the compiler drain vmcnt every iteration)
    auto fetch_w = [&](floatx4 (&wv)[KB][KB], int p) {
      const int pc = p < P ? p : P - 1;
#pragma unroll
      for (int ab = 0; ab < KB; ++ab)
#pragma unroll
        for (int jg = 0; jg < KB; ++jg) wv[ab][jg] = img[((int64_t)(pc * KB + ab) * KB + jg) * 64 + lane];
      __builtin_amdgcn_sched_barrier(0);
    };
    auto pair = [&](const floatx4 (&wv)[KB][KB], int p) {
      set_pair(p);
      floatx4 acc[KB];
#pragma unroll
      for (int ab = 0; ab < KB; ++ab) acc[ab] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int jg = 0; jg < KB; ++jg) {
        const int kk = 16 * jg + 4 * kq;
        floatx4 ea = {0.f, 0.f, 0.f, 0.f};
        if (kk < K && sm < S) ea = *reinterpret_cast<const floatx4*>(tile + sm * SS + i * K + kk);
#pragma unroll
        for (int ab = 0; ab < KB; ++ab)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[ab] = mfma16x16x4(ea[q], wv[ab][jg][q], acc[ab]);
      }
      // C[s][a]: lane holds a = 16ab + (lane&15), s = 4kq + r
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ss = 4 * kq + r;
        float v = 0.f;
#pragma unroll
        for (int ab = 0; ab < KB; ++ab) {
          const int aa = 16 * ab + sm;
          const float ec = (aa < K && ss < S) ? tile[ss * SS + j * K + aa] : 0.f;
          v = fmaf(acc[ab][r], ec, v);
        }
        v = row16_sum(v);
        if (sm == 0 && ss < S) gram[ss * PP + Pi + p] = v;
      }
    };
    floatx4 wa[KB][KB], wb[KB][KB];
    fetch_w(wa, w);
    for (int p = w; p < P; p += 2 * IP_NW) {
      fetch_w(wb, p + IP_NW);
      pair(wa, p);
      if (p + IP_NW >= P) break;
      fetch_w(wa, p + 2 * IP_NW);
      pair(wb, p + IP_NW);
    }
  }
  IP_STAMP(5);  // this wave's Gram / outer pairs done (before the barrier)
  __syncthreads();
  IP_STAMP(3);
  // coalesced output rows [flat F*K | inner P | outer P]
  const int FK = a.write_flat ? F * K : 0;
  const int W = FK + PP;
  if (a.contig) {
    // the workgroup's rows are one contiguous, 16-B aligned block: float4
    // stores (scalar stores are issue-bound at ~4 B/clk/CU)
    float* ob = a.out + b0 * a.out_stride;
    const int n = nvalid * W;
    const int dq = 4 * IP_NT / W, dr = 4 * IP_NT - dq * W;
    int f = 4 * tid, s0 = f / W, c0 = f - s0 * W;
    for (; f < n; f += 4 * IP_NT) {
      floatx4 v;
      int ss = s0, cc = c0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = cc < FK ? tile[ss * SS + cc] : gram[ss * PP + (cc - FK)];
        if (++cc == W) { cc = 0; ++ss; }
      }
      if (f + 4 <= n) {
        // streamed: 10.0 -> 8.5 us at B 4096 (profiles/r6_ab_nt_out.jsonl)
        __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(ob + f));
      } else {
        for (int q = 0; q < n - f; ++q) ob[f + q] = v[q];
      }
      s0 += dq;
      c0 += dr;
      if (c0 >= W) { c0 -= W; ++s0; }
    }
  } else {
  for (int s = 0; s < nvalid; ++s) {
    float* orow = a.out + (b0 + s) * a.out_stride;
    for (int col = tid; col < W; col += IP_NT) {
      const float val = col < FK ? tile[s * SS + col] : gram[s * PP + (col - FK)];
      const int cp = col - FK;
      orow[col < FK ? col : (cp < Pi ? a.inner_off + cp : a.outer_off + (cp - Pi))] = val;
    }
  }
  }
  IP_STAMP(4);
}

template <int K, int KIND>
__global__ __launch_bounds__(IP_NT) void inner_fast(InnerArgs a) {
  inner_fast_body<K, KIND, false>(a, nullptr);
}
template <int KIND>
__global__ __launch_bounds__(IP_NT) void inner_fast_ka(InnerArgs a, FieldMeta m) {
  inner_fast_body<16, KIND, true>(a, &m);
}

template <int KIND>
static void launch_inner_fast_k(const InnerArgs& a, size_t lds, unsigned grid, hipStream_t st) {
  switch (a.k) {
    case 4: inner_fast<4, KIND><<<grid, IP_NT, lds, st>>>(a); break;
    case 8: inner_fast<8, KIND><<<grid, IP_NT, lds, st>>>(a); break;
    case 16: inner_fast<16, KIND><<<grid, IP_NT, lds, st>>>(a); break;
    case 32: inner_fast<32, KIND><<<grid, IP_NT, lds, st>>>(a); break;
    default: inner_fast<64, KIND><<<grid, IP_NT, lds, st>>>(a); break;
  }
}

static int launch_inner(InnerArgs a, hipStream_t st, const char* what, const FieldMeta* hm = nullptr) {
  if (a.batch == 0) return RS_OK;
  const bool fast_k = a.k == 4 || a.k == 8 || a.k == 16 || a.k == 32 || a.k == 64;
  if (fast_k && a.F >= 2 && a.F <= IP_FMAX) {
    const int P = a.F * (a.F - 1) / 2;
    const int PP = (a.want_inner ? P : 0) + (a.outer_img ? P : 0);
    const int64_t per = ((int64_t)a.F * a.k + 4 + PP) * sizeof(float);
    int S = IP_SMAX;
    while (S > 1 && S * per > 96 * 1024) --S;
    a.S = S;
    const int FKw = a.write_flat ? a.F * a.k : 0;
    const int W = FKw + PP;
    a.contig = a.out_stride == W && (!a.want_inner || a.inner_off == FKw) &&
               (!a.outer_img || a.outer_off == FKw + (a.want_inner ? P : 0)) && (uintptr_t)a.out % 16 == 0 &&
               ((int64_t)S * W) % 4 == 0;
    const size_t lds = (size_t)S * per;
    const unsigned grid = (unsigned)((a.batch + S - 1) / S);
    if (a.ids == nullptr) {
      launch_inner_fast_k<3>(a, lds, grid, st);
    } else if (hm && a.k == 16 && a.F <= 32 && S == IP_SMAX) {
      with_id_kind(a.id_kind, [&](auto K) {
        constexpr int KIND = decltype(K)::value;
        static LdsAttr set[3];
        lds_attr(set[KIND], (const void*)inner_fast_ka<KIND>, lds);
        inner_fast_ka<KIND><<<grid, IP_NT, lds, st>>>(a, *hm);
      });
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

// OuterProductLayer weights W [k, P, k] (Keras add_weight shape) -> per-lane
// MFMA B fragments: img[((p*KB + ab)*KB + jg)*64 + lane][q] =
// W[a = 16ab + (lane&15)][p][j = 16jg + 4(lane>>4) + q], zero-padded.
__global__ void outer_prepare_kernel(const float* __restrict__ W, int P, int k, int KB, int64_t n,
                                     float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i & 3), lane = (int)((i >> 2) & 63);
    int64_t r = i >> 8;
    const int jg = (int)(r % KB);
    r /= KB;
    const int ab = (int)(r % KB);
    const int p = (int)(r / KB);
    const int aa = 16 * ab + (lane & 15), j = 16 * jg + 4 * (lane >> 4) + q;
    out[i] = (aa < k && j < k) ? W[((int64_t)aa * P + p) * k + j] : 0.f;
  }
}

static int64_t outer_size(int F, int k) {
  const int64_t P = (int64_t)F * (F - 1) / 2, KB = (k + 15) / 16;
  return P * KB * KB * 256;
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_outer_prepared_size(int n_fields, int k) {
  if (n_fields < 2 || n_fields > IP_FMAX || !(k == 4 || k == 8 || k == 16 || k == 32 || k == 64)) return -1;
  return outer_size(n_fields, k);
}

extern "C" int rs_outer_prepare(const float* W, int n_fields, int k, float* prepared, rs_stream_t stream) {
  RS_REQUIRE(rs_outer_prepared_size(n_fields, k) > 0, "rs_outer_prepare: need 2..%d fields, k in {4,8,16,32,64}",
             IP_FMAX);
  RS_REQUIRE(W && prepared, "rs_outer_prepare: null pointer");
  const int64_t n = outer_size(n_fields, k);
  int64_t g = (n + 255) / 256;
  g = g > 8192 ? 8192 : g;
  outer_prepare_kernel<<<(unsigned)g, 256, 0, as_stream(stream)>>>(W, n_fields * (n_fields - 1) / 2, k,
                                                                    (k + 15) / 16, n, prepared);
  return launch_status("rs_outer_prepare");
}

static unsigned long long* g_inner_dbg = nullptr;
extern "C" void rs_diag_inner_set_dbg(unsigned long long* p) { g_inner_dbg = p; }

extern "C" int rs_inner_product_fwd(const float* emb, int n_fields, int k, float* out, int64_t out_stride,
                                    int64_t batch, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(emb && out, "rs_inner_product_fwd: null pointer");
  RS_REQUIRE(n_fields >= 1 && k >= 1 && k <= 64 && batch >= 0, "rs_inner_product_fwd: bad shape (k<=64)");
  RS_REQUIRE(out_stride >= (int64_t)n_fields * (n_fields - 1) / 2, "rs_inner_product_fwd: out_stride too small");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)emb % 16 == 0, "rs_inner_product_fwd: emb must be 16-B aligned");
  InnerArgs a{};
  a.dbg = g_inner_dbg;
  a.emb = emb;
  a.F = n_fields;
  a.k = k;
  a.out = out;
  a.out_stride = out_stride;
  a.inner_off = 0;
  a.write_flat = 0;
  a.want_inner = 1;
  a.batch = batch;
  return launch_inner(a, as_stream(stream), "rs_inner_product_fwd");
}

namespace rs {
static const FieldMeta* inner_host_meta(FieldMeta& m, const int64_t* off_h, const int64_t* voc_h, int n_fields,
                                        int k) {
  if (!off_h || !voc_h || k != 16 || n_fields < 1 || n_fields > 32) return nullptr;
  for (int c = 0; c < n_fields; ++c) {
    m.off[c] = off_h[c];
    m.voc[c] = voc_h[c];
  }
  return &m;
}
}  // namespace rs

extern "C" int rs_embed_inner_fwd_hm(const void* ids, int id_kind, int64_t id_stride, const float* table,
                                     const int64_t* field_offsets, const int64_t* field_vocab,
                                     const int64_t* field_offsets_host, const int64_t* field_vocab_host,
                                     int n_fields, int k, float* out, int64_t out_stride, int64_t batch,
                                     int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(field_offsets_host && field_vocab_host, "rs_embed_inner_fwd_hm: host metadata missing");
  RS_REQUIRE(ids && table && field_offsets && field_vocab && out, "rs_embed_inner_fwd_hm: null pointer");
  RS_REQUIRE(n_fields >= 1 && k >= 1 && k <= 64 && batch >= 0, "rs_embed_inner_fwd_hm: bad shape (k<=64)");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_inner_fwd_hm: bad id_kind");
  RS_REQUIRE(out_stride >= (int64_t)n_fields * k + (int64_t)n_fields * (n_fields - 1) / 2,
             "rs_embed_inner_fwd_hm: out_stride too small");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)table % 16 == 0, "rs_embed_inner_fwd_hm: table must be 16-B aligned");
  InnerArgs a{};
  a.dbg = g_inner_dbg;
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
  a.want_inner = 1;
  a.batch = batch;
  a.err = err_flag;
  FieldMeta m;
  return launch_inner(a, as_stream(stream), "rs_embed_inner_fwd_hm",
                      inner_host_meta(m, field_offsets_host, field_vocab_host, n_fields, k));
}

extern "C" int rs_embed_product_fwd_hm(const void* ids, int id_kind, int64_t id_stride, const float* table,
                                       const int64_t* field_offsets, const int64_t* field_vocab,
                                       const int64_t* field_offsets_host, const int64_t* field_vocab_host,
                                       int n_fields, int k, int inner, const float* outer_prepared, float* out,
                                       int64_t out_stride, int64_t batch, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(field_offsets_host && field_vocab_host, "rs_embed_product_fwd_hm: host metadata missing");
  RS_REQUIRE(ids && table && field_offsets && field_vocab && out, "rs_embed_product_fwd_hm: null pointer");
  RS_REQUIRE(inner || outer_prepared, "rs_embed_product_fwd_hm: nothing to compute (inner=0, no outer weights)");
  RS_REQUIRE(rs_outer_prepared_size(n_fields, k) > 0,
             "rs_embed_product_fwd_hm: need 2..%d fields and k in {4,8,16,32,64}", IP_FMAX);
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32 && batch >= 0, "rs_embed_product_fwd_hm: bad ids");
  const int P = n_fields * (n_fields - 1) / 2;
  RS_REQUIRE(out_stride >= (int64_t)n_fields * k + (inner ? P : 0) + (outer_prepared ? P : 0),
             "rs_embed_product_fwd_hm: out_stride too small");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_embed_product_fwd_hm: table must be 16-B aligned");
  InnerArgs a{};
  a.dbg = g_inner_dbg;
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
  a.write_flat = 1;
  a.want_inner = inner ? 1 : 0;
  a.inner_off = n_fields * k;
  a.outer_img = outer_prepared;
  a.outer_off = n_fields * k + (inner ? P : 0);
  a.batch = batch;
  a.err = err_flag;
  FieldMeta m;
  return launch_inner(a, as_stream(stream), "rs_embed_product_fwd_hm",
                      inner_host_meta(m, field_offsets_host, field_vocab_host, n_fields, k));
}

extern "C" int rs_embed_inner_fwd(const void* ids, int id_kind, int64_t id_stride, const float* table,
                                  const int64_t* field_offsets, const int64_t* field_vocab, int n_fields, int k,
                                  float* out, int64_t out_stride, int64_t batch, int* err_flag,
                                  rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(ids && table && field_offsets && field_vocab && out, "rs_embed_inner_fwd: null pointer");
  RS_REQUIRE(n_fields >= 1 && k >= 1 && k <= 64 && batch >= 0, "rs_embed_inner_fwd: bad shape (k<=64)");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_inner_fwd: bad id_kind");
  RS_REQUIRE(out_stride >= (int64_t)n_fields * k + (int64_t)n_fields * (n_fields - 1) / 2,
             "rs_embed_inner_fwd: out_stride too small");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)table % 16 == 0, "rs_embed_inner_fwd: table must be 16-B aligned");
  InnerArgs a{};
  a.dbg = g_inner_dbg;
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
  a.want_inner = 1;
  a.batch = batch;
  a.err = err_flag;
  return launch_inner(a, as_stream(stream), "rs_embed_inner_fwd");
}

extern "C" int rs_embed_product_fwd(const void* ids, int id_kind, int64_t id_stride, const float* table,
                                    const int64_t* field_offsets, const int64_t* field_vocab, int n_fields, int k,
                                    int inner, const float* outer_prepared, float* out, int64_t out_stride,
                                    int64_t batch, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(ids && table && field_offsets && field_vocab && out, "rs_embed_product_fwd: null pointer");
  RS_REQUIRE(inner || outer_prepared, "rs_embed_product_fwd: nothing to compute (inner=0, no outer weights)");
  RS_REQUIRE(rs_outer_prepared_size(n_fields, k) > 0,
             "rs_embed_product_fwd: need 2..%d fields and k in {4,8,16,32,64}", IP_FMAX);
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32 && batch >= 0, "rs_embed_product_fwd: bad ids");
  const int P = n_fields * (n_fields - 1) / 2;
  RS_REQUIRE(out_stride >= (int64_t)n_fields * k + (inner ? P : 0) + (outer_prepared ? P : 0),
             "rs_embed_product_fwd: out_stride too small");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_embed_product_fwd: table must be 16-B aligned");
  InnerArgs a{};
  a.dbg = g_inner_dbg;
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
  a.write_flat = 1;
  a.want_inner = inner ? 1 : 0;
  a.inner_off = n_fields * k;
  a.outer_img = outer_prepared;
  a.outer_off = n_fields * k + (inner ? P : 0);
  a.batch = batch;
  a.err = err_flag;
  return launch_inner(a, as_stream(stream), "rs_embed_product_fwd");
}

extern "C" int rs_outer_product_fwd(const float* emb, int n_fields, int k, const float* outer_prepared, float* out,
                                    int64_t out_stride, int64_t batch, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(emb && outer_prepared && out, "rs_outer_product_fwd: null pointer");
  RS_REQUIRE(rs_outer_prepared_size(n_fields, k) > 0,
             "rs_outer_product_fwd: need 2..%d fields and k in {4,8,16,32,64}", IP_FMAX);
  RS_REQUIRE(out_stride >= (int64_t)n_fields * (n_fields - 1) / 2 && batch >= 0,
             "rs_outer_product_fwd: out_stride too small");
  RS_REQUIRE((uintptr_t)emb % 16 == 0, "rs_outer_product_fwd: emb must be 16-B aligned");
  InnerArgs a{};
  a.dbg = g_inner_dbg;
  a.emb = emb;
  a.F = n_fields;
  a.k = k;
  a.out = out;
  a.out_stride = out_stride;
  a.want_inner = 0;
  a.outer_img = outer_prepared;
  a.outer_off = 0;
  a.batch = batch;
  return launch_inner(a, as_stream(stream), "rs_outer_product_fwd");
}
