// Diagnostic only (never part of librs_hip.so): the id -> row gather of the
// headline shape (ids [B, F] int32, rows of 64 B in one [F * V, 16] table)
// in several launch structures, to find the fastest skeleton for the fused
// gather + FM kernel.  Each lookup's 16 floats are summed and written to
// out[b * F + c] (so nothing is optimised away).  Built by
// scripts/build_diag_gather.sh into scripts/ab/libdiag_gather.so and timed
// by scripts/diag_gather_shapes.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx4 ldnt(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
}
__device__ __forceinline__ float quad_sum_strided16(float v) {
  // lanes l, l+16, l+32, l+48 hold the 4 chunks of one row
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
__device__ __forceinline__ float quad_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  return v;
}

struct GArgs {
  const int32_t* ids;
  const float* table;
  const int64_t* offs;
  int F;
  int64_t B;
  float* out;
};

// V0: the probe shape — 4 lanes per lookup (adjacent lanes), lookups in
// flattened (b, c) order, 16 per wave, one id load then one row load.
template <int NT>
__global__ __launch_bounds__(NT) void g_flat(GArgs a) {
  const int64_t n = a.B * a.F;
  const int64_t l = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 2;
  const int q = threadIdx.x & 3;
  if (l >= n) return;
  const int c = (int)(l % a.F);
  const int32_t id = a.ids[l];
  const floatx4 r = ldnt(a.table + (a.offs[c] + id) * 16 + 4 * q);
  const float s = quad_sum(r[0] + r[1] + r[2] + r[3]);
  if (q == 0) a.out[l] = s;
}

// V1/V2: the fused kernel's skeleton — 16 samples per workgroup, 16 waves,
// wave w owns fields w and w + 16, lane = sample + 16 * chunk.  TWO_PASS:
// the second field's row is requested after the first one has arrived.
template <bool TWO_PASS>
__global__ __launch_bounds__(1024) void g_tile16(GArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  const int64_t bt = (int64_t)blockIdx.x * 16 + s;
  const int64_t b = bt < a.B ? bt : a.B - 1;
  const int c0 = w, c1 = w + 16;
  const bool h1 = c1 < a.F;
  const int32_t i0 = a.ids[b * a.F + c0];
  const int32_t i1 = a.ids[b * a.F + (h1 ? c1 : c0)];
  const int64_t o0 = a.offs[c0], o1 = a.offs[h1 ? c1 : c0];
  const floatx4 r0 = ldnt(a.table + (o0 + i0) * 16 + 4 * kk);
  float s0 = quad_sum_strided16(r0[0] + r0[1] + r0[2] + r0[3]);
  float s1 = 0.f;
  if (TWO_PASS) {
    asm volatile("" ::"v"(s0));
    if (h1) {
      const floatx4 r1 = ldnt(a.table + (o1 + i1) * 16 + 4 * kk);
      s1 = quad_sum_strided16(r1[0] + r1[1] + r1[2] + r1[3]);
    }
  } else if (h1) {
    const floatx4 r1 = ldnt(a.table + (o1 + i1) * 16 + 4 * kk);
    s1 = quad_sum_strided16(r1[0] + r1[1] + r1[2] + r1[3]);
  }
  if (kk == 0 && bt < a.B) {
    a.out[b * a.F + c0] = s0;
    if (h1) a.out[b * a.F + c1] = s1;
  }
}

// V3: 256-thread workgroups of S samples; wave w of 4 owns fields w, w+4, ...
// (up to 7), every row requested at once; lane = 4 x sample-in-16 + chunk
// (adjacent lanes hold one row).
__global__ __launch_bounds__(256) void g_tile4w(GArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane & 3, s = lane >> 2;
  const int64_t bt = (int64_t)blockIdx.x * 16 + s;
  const int64_t b = bt < a.B ? bt : a.B - 1;
  constexpr int MAXC = 8;
  int32_t id[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = w + 4 * j;
    id[j] = a.ids[b * a.F + (c < a.F ? c : 0)];
  }
  floatx4 r[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = w + 4 * j;
    if (c < a.F) r[j] = ldnt(a.table + (a.offs[c] + id[j]) * 16 + 4 * q);
  }
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = w + 4 * j;
    if (c < a.F) {
      const float sm = quad_sum(r[j][0] + r[j][1] + r[j][2] + r[j][3]);
      if (q == 0 && bt < a.B) a.out[b * a.F + c] = sm;
    }
  }
}

// V4: 16-sample tiles, 16 waves, but lanes in the adjacent (quad) layout and
// the wave's two fields in ONE wave-instruction pair issued at once.
__global__ __launch_bounds__(1024) void g_tile16q(GArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane & 3, s = lane >> 2;
  const int64_t bt = (int64_t)blockIdx.x * 16 + s;
  const int64_t b = bt < a.B ? bt : a.B - 1;
  const int c0 = w, c1 = w + 16;
  const bool h1 = c1 < a.F;
  const int32_t i0 = a.ids[b * a.F + c0];
  const int32_t i1 = a.ids[b * a.F + (h1 ? c1 : c0)];
  const floatx4 r0 = ldnt(a.table + (a.offs[c0] + i0) * 16 + 4 * q);
  floatx4 r1 = {0.f, 0.f, 0.f, 0.f};
  if (h1) r1 = ldnt(a.table + (a.offs[c1] + i1) * 16 + 4 * q);
  const float s0 = quad_sum(r0[0] + r0[1] + r0[2] + r0[3]);
  const float s1 = quad_sum(r1[0] + r1[1] + r1[2] + r1[3]);
  if (q == 0 && bt < a.B) {
    a.out[b * a.F + c0] = s0;
    if (h1) a.out[b * a.F + c1] = s1;
  }
}

extern "C" int diag_gather(int variant, const int32_t* ids, const float* table, const int64_t* offs, int F, int64_t B,
                           float* out, void* stream) {
  GArgs a{ids, table, offs, F, B, out};
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = B * F;
  switch (variant) {
    case 0: g_flat<256><<<(unsigned)((n * 4 + 255) / 256), 256, 0, st>>>(a); break;
    case 1: g_tile16<false><<<(unsigned)((B + 15) / 16), 1024, 0, st>>>(a); break;
    case 2: g_tile16<true><<<(unsigned)((B + 15) / 16), 1024, 0, st>>>(a); break;
    case 3: g_tile4w<<<(unsigned)((B + 15) / 16), 256, 0, st>>>(a); break;
    case 4: g_tile16q<<<(unsigned)((B + 15) / 16), 1024, 0, st>>>(a); break;
    case 5: g_flat<1024><<<(unsigned)((n * 4 + 1023) / 1024), 1024, 0, st>>>(a); break;
    case 6: g_flat<64><<<(unsigned)((n * 4 + 63) / 64), 64, 0, st>>>(a); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------
// Ablations of a 16-sample / 16-wave gather + FM tile (one tile per
// workgroup, the headline shape: int32 ids, k = 16, kfm + 1 <= 16, F <= 32):
// the packed FM image of rs_fm_prepare as B fragments, s = x@v on
// v_mfma_f32_16x16x4_f32, partial tiles combined through LDS.
//   bit 0 ADJ   rows loaded with adjacent lanes (lane = 4 sample + chunk) and
//               moved to the MFMA A layout (lane = sample + 16 chunk) by
//               ds_bpermute; else loaded in the A layout directly
//   bit 1 NOB   no B-fragment / norm loads (constants)
//   bit 2 NOMF  no MFMA (the row chunk is summed instead)
//   bit 3 NOCB  no LDS combine (each wave writes its partial tile)
//   bit 4 BLATE B fragments requested after the rows (else before the ids)
//   bit 5 P2    second field's row requested after the first one's MFMAs
//   bit 6 NDPP  |v_e|^2 from the B fragment by a DPP row sum (no norm loads)
//   bit 7 REP   the FM image replicated 32x, workgroup b reads copy b % 32
struct FArgs {
  const int32_t* ids;
  const float* table;
  const int64_t* offs;
  const int64_t* vocab;
  int F, kfm;
  int64_t B;
  const float* prep;  // rs_fm_prepare image: DB dense records, then F field records
  int64_t dense_rec, field_rec, field_base;
  int nd, DB;
  const float* dense;
  float* out;  // logit [B] (or partial tiles with NOCB)
  int64_t prep_size;  // floats per copy of the image (REP)
};

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float row16(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));
  return x;
}

template <int ABL>
__global__ __launch_bounds__(1024) void fm_abl(FArgs a) {
  constexpr bool ADJ = ABL & 1, NOB = ABL & 2, NOMF = ABL & 4, NOCB = ABL & 8, BLATE = ABL & 16, P2 = ABL & 32;
  constexpr bool NDPP = ABL & 64, REP = ABL & 128;
  const float* prep = a.prep + (REP ? (int64_t)(blockIdx.x % 32) * a.prep_size : 0);
  __shared__ float cs[16][16][17];
  __shared__ float qs[16][16];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;       // A layout: sample, chunk
  const int qa = lane & 3, sa = lane >> 2;       // adjacent layout: chunk, sample
  const int ls = ADJ ? sa : s, lq = ADJ ? qa : kk;  // the row this lane loads
  const int64_t b0 = (int64_t)blockIdx.x * 16;
  const int64_t bl = b0 + ls < a.B ? b0 + ls : a.B - 1;
  const int c0 = w, c1 = w + 16;
  const bool h1 = c1 < a.F;
  const int cf1 = h1 ? c1 : c0;
  const int32_t i0 = a.ids[bl * a.F + c0];
  const int32_t i1 = a.ids[bl * a.F + cf1];
  floatx4 bw0 = {1.f, 1.f, 1.f, 1.f}, bw1 = bw0, n0 = bw0, n1 = bw0;
  auto loadb = [&]() {
    if constexpr (!NOB) {
      const float* r0 = prep + a.field_base + (int64_t)c0 * a.field_rec;
      const float* r1 = prep + a.field_base + (int64_t)cf1 * a.field_rec;
      if (s <= a.kfm) {
        bw0 = *reinterpret_cast<const floatx4*>(r0 + lane * 4);
        bw1 = *reinterpret_cast<const floatx4*>(r1 + lane * 4);
      } else {
        bw0 = bw1 = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (NDPP) {
#pragma unroll
        for (int tp = 0; tp < 4; ++tp) {
          const float b0v = s < a.kfm ? bw0[tp] : 0.f, b1v = s < a.kfm ? bw1[tp] : 0.f;
          n0[tp] = row16(b0v * b0v);
          n1[tp] = row16(b1v * b1v);
        }
      } else {
        n0 = *reinterpret_cast<const floatx4*>(r0 + 256 + kk * 4);
        n1 = *reinterpret_cast<const floatx4*>(r1 + 256 + kk * 4);
      }
    }
  };
  if (!BLATE) loadb();
  const int64_t o0 = a.offs[c0], o1 = a.offs[cf1];
  floatx4 x0 = ldnt(a.table + (o0 + i0) * 16 + 4 * lq);
  floatx4 x1 = {0.f, 0.f, 0.f, 0.f};
  if (!P2 && h1) x1 = ldnt(a.table + (o1 + i1) * 16 + 4 * lq);
  if (BLATE) loadb();
  // dense k-step of the last 4 waves
  const int dw = 15 - w;
  const bool hd = dw < a.DB;
  float dx = 0.f, drec = 0.f, dn = 0.f;
  if (hd) {
    const int e = 4 * dw + kk;
    dx = e < a.nd ? a.dense[(b0 + s < a.B ? b0 + s : a.B - 1) * a.nd + e] : 0.f;
    drec = prep[(int64_t)dw * a.dense_rec + lane];
    if constexpr (NDPP) {
      const float dv = s < a.kfm ? drec : 0.f;
      dn = row16(dv * dv);
    } else {
      dn = prep[(int64_t)dw * a.dense_rec + 64 + kk];
    }
  }
  auto to_a = [&](floatx4 v) -> floatx4 {
    if constexpr (!ADJ) return v;
    // lane L' = s + 16 q takes chunk q of row s from lane 4 s + q
    const int src = (4 * s + kk) << 2;
    floatx4 r;
    r[0] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[0])));
    r[1] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[1])));
    r[2] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[2])));
    r[3] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[3])));
    return r;
  };
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  float qn = 0.f;
  auto field = [&](floatx4 xv, floatx4 bw, floatx4 nn) {
    const floatx4 xa = to_a(xv);
#pragma unroll
    for (int tp = 0; tp < 4; ++tp) {
      if constexpr (NOMF) acc[tp] += xa[tp] * bw[tp];
      else acc = mfma4(xa[tp], bw[tp], acc);
      qn = fmaf(xa[tp] * xa[tp], nn[tp], qn);
    }
  };
  field(x0, bw0, n0);
  if (P2 && h1) x1 = ldnt(a.table + (o1 + i1) * 16 + 4 * lq);
  if (h1) field(x1, bw1, n1);
  if (hd) {
    if constexpr (NOMF) acc[0] += dx * drec;
    else acc = mfma4(dx, drec, acc);
    qn = fmaf(dx * dx, dn, qn);
  }
  if constexpr (NOCB) {
    const int64_t bb = b0 + kk * 4;
    if (bb < a.B) a.out[bb] = acc[0] + acc[1] + acc[2] + acc[3] + qn;
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) cs[w][kk * 4 + r][s] = acc[r];
  qn += __shfl_xor(qn, 16);
  qn += __shfl_xor(qn, 32);
  if (lane < 16) qs[w][lane] = qn;
  __syncthreads();
  if (threadIdx.x < 256) {
    const int smp = threadIdx.x >> 4, col = threadIdx.x & 15;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 16; ++ww) v += cs[ww][smp][col];
    float t = col < a.kfm ? v * v : 0.f;
    t -= qs[col][smp];
    float lin = col == a.kfm ? v : 0.f;
    t = row16(t);
    lin = row16(lin);
    const int64_t bb = b0 + smp;
    if (col == 0 && bb < a.B) a.out[bb] = lin + 0.5f * t;
  }
}

extern "C" int diag_fm_abl(int abl, const int32_t* ids, const float* table, const int64_t* offs, const int64_t* vocab,
                           int F, int kfm, int64_t B, const float* prep, int64_t dense_rec, int64_t field_rec,
                           int64_t field_base, int nd, int DB, const float* dense, float* out, int64_t prep_size,
                           void* stream) {
  FArgs a{ids, table, offs, vocab, F, kfm, B, prep, dense_rec, field_rec, field_base, nd, DB, dense, out, prep_size};
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = (unsigned)((B + 15) / 16);
#define ABL_CASE(x) \
  case x: fm_abl<x><<<g, 1024, 0, st>>>(a); break;
  switch (abl) {
    ABL_CASE(0) ABL_CASE(1) ABL_CASE(3) ABL_CASE(17) ABL_CASE(33) ABL_CASE(65) ABL_CASE(129) ABL_CASE(193)
    ABL_CASE(81) ABL_CASE(209) ABL_CASE(225) ABL_CASE(97) ABL_CASE(64) ABL_CASE(192)
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
