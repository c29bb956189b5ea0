// embed_fm_tiles.hip — the headline kernel of rs_embed_fm_fwd in two
// persistent, tile-pipelined forms (one launch: ids -> rows -> FM logit).
//
// Reference: EmbedLayer.call (layer/core.py:273-280), the DeepFM concat
// x = [dense | emb] (model/deepFM.py:24-26) and FMLayer.call
// (layer/interaction.py:106-114):
//   logit = x@w1 + w0 + 0.5 * sum_f [ (x@v)_f^2 - (x^2 @ v^2)_f ]
// computed as (x@w1 + w0) + 0.5 (sum_f s_f^2 - sum_i x_i^2 |v_i|^2), the
// regrouping every FM kernel here uses.
//
// Both kernels keep a workgroup resident for several sample tiles (grid =
// min(tiles, a per-CU share)) and hold every sample-independent operand in
// registers for the whole launch, so per tile only ids and rows move:
//   * each wave owns a fixed set of fields: their row offsets / vocabularies
//     are wave-uniform scalars, their FM weights are loaded once;
//   * ids of tile t + G are requested while tile t's rows are in flight, and
//     tile t + G's rows are requested before tile t's partial sums are
//     combined, so the id -> row chain of one tile overlaps the previous
//     tile's arithmetic and combine;
//   * the combine goes through a double-buffered LDS slab: one barrier per
//     tile.
//
//  fm_tiles_mfma (RS_OPT_EMBED_FM_KERNEL = 2): 16 waves, 16-sample tiles,
//    wave w owns fields w and w + 16; s = x@v and x@w1 on
//    v_mfma_f32_16x16x4_f32 with the B fragments (the packed FM image of
//    rs_fm_prepare) held in registers.
//  fm_tiles_valu (RS_OPT_EMBED_FM_KERNEL = 1): the north-star VALU form —
//    8-sample tiles, 4 lanes x float4 per 64-B row (k = 16), wave w owns
//    fields 2w and 2w + 1 (lane bit 5 picks one), one more wave for the
//    dense block; each lane keeps its 4 elements' [v | w1 | |v|^2] rows
//    (kfm + 2 floats each, staged once through LDS) in registers, FMAs its
//    row chunk against them and the partial sums are reduced by DPP quad
//    permutes (the row's 4 lanes) and a cross-half swap (the wave's 2 fields)
//    — no matrix core.
#include "embed_fm.hpp"

namespace rs {

// ---------------------------------------------------------------- MFMA form
constexpr int TM_NW = 16;  // waves per workgroup (fields w, w + 16)

template <int KV, int NT, int KIND>
__global__ __launch_bounds__(TM_NW * 64, NT == 1 ? 8 : 4) void fm_tiles_mfma(EmbedFmArgs a, int ntiles) {
  typedef Ids<KIND> I;
  constexpr int NW = TM_NW, NC = NT * 16;
  __shared__ float cs[2][NW][16][NC + 1];
  __shared__ float qs[2][NW][16];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  const int F = a.F;
  const int c0 = w, c1 = w + NW;            // wave-uniform field slots
  const bool h0 = c0 < F, h1 = c1 < F;      // wave-uniform
  const int cf0 = h0 ? c0 : 0, cf1 = h1 ? c1 : 0;
  const int dw = NW - 1 - w;                // dense k-step of this wave
  const bool hd = dw < a.DB;                // wave-uniform (DB <= NW checked on the host)

  int tile = blockIdx.x;
  auto sample = [&](int t) -> int64_t {
    const int64_t bt = (int64_t)t * 16 + s;
    return bt < a.batch ? bt : a.batch - 1;  // padded lanes recompute the last sample
  };
  // ---- the first tile's ids go out before anything else: the id -> row
  // chain is the launch's critical path, everything below overlaps it
  typename I::raw_t id0, id1;
  {
    const int64_t b = sample(tile);
    id0 = I::load(a.ids, b * a.id_stride + cf0);
    id1 = I::load(a.ids, b * a.id_stride + cf1);
  }
  // ---- launch-constant operands: field metadata, B fragments, norms
  const int64_t off0 = a.offs[cf0], voc0 = h0 ? a.vocab[cf0] : 0;
  const int64_t off1 = a.offs[cf1], voc1 = h1 ? a.vocab[cf1] : 0;
  Chunk<KV> bw0[NT], bw1[NT], nr0, nr1;
  {
    const float* r0 = a.prep + a.field_base + (int64_t)cf0 * a.field_rec;
    const float* r1 = a.prep + a.field_base + (int64_t)cf1 * a.field_rec;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (nt * 16 + s <= a.kfm) {
        bw0[nt].load(r0 + (int64_t)(nt * 64 + lane) * KV);
        bw1[nt].load(r1 + (int64_t)(nt * 64 + lane) * KV);
      } else {
        bw0[nt].zero();
        bw1[nt].zero();
      }
    }
    nr0.load(r0 + NT * 64 * KV + kk * KV);
    nr1.load(r1 + NT * 64 * KV + kk * KV);
  }
  float drec[NT], dn = 0.f;
  const int de = 4 * dw + kk;  // dense element of this lane
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) drec[nt] = 0.f;
  if (hd) {
    const float* rec = a.prep + (int64_t)dw * a.dense_rec;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) drec[nt] = rec[nt * 64 + lane];
    dn = de < a.nd ? rec[NT * 64 + kk] : 0.f;
  }

  Chunk<KV> x0, x1;
  bool ok0, ok1;
  float dx = 0.f;
  // rows of tile t (and the dense features of the waves with a dense k-step)
  auto issue_rows = [&](int t, typename I::raw_t r0, typename I::raw_t r1) {
    int64_t i0, i1;
    ok0 = I::decode(r0, voc0, i0);
    ok1 = I::decode(r1, voc1, i1);
    x0.load_nt(a.table + (off0 + i0) * a.k + KV * kk);
    if (h1) x1.load_nt(a.table + (off1 + i1) * a.k + KV * kk);
    else x1.zero();
    if (hd) dx = a.dense[sample(t) * a.dense_stride + (de < a.nd ? de : 0)];
  };
  issue_rows(tile, id0, id1);
  int nxt = tile + gridDim.x;
  if (nxt < ntiles) {
    const int64_t b = sample(nxt);
    id0 = I::load(a.ids, b * a.id_stride + cf0);
    id1 = I::load(a.ids, b * a.id_stride + cf1);
  }
  bool bad = false;
  int buf = 0;
  while (true) {
    const bool valid = (int64_t)tile * 16 + s < a.batch;
    // ---- MFMAs of this tile (waits on its rows)
    floatx4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    float qn = 0.f;
    bad |= (h0 && !ok0) || (h1 && !ok1);
    const bool u0 = h0 && ok0, u1 = h1 && ok1;
#pragma unroll
    for (int tp = 0; tp < KV; ++tp) {
      const float xv0 = u0 ? x0.v[tp] : 0.f;
      const float xv1 = u1 ? x1.v[tp] : 0.f;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16x16x4(xv0, bw0[nt].v[tp], acc[nt]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16x16x4(xv1, bw1[nt].v[tp], acc[nt]);
      qn = fmaf(xv0 * xv0, nr0.v[tp], qn);
      qn = fmaf(xv1 * xv1, nr1.v[tp], qn);
    }
    if (hd) {
      const float xd = de < a.nd ? dx : 0.f;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16x16x4(xd, drec[nt], acc[nt]);
      qn = fmaf(xd * xd, dn, qn);
    }
    // ---- next tile's rows go out before this tile's combine
    const int cur = tile;
    tile = nxt;
    const bool more = tile < ntiles;
    if (more) {
      issue_rows(tile, id0, id1);
      nxt = tile + gridDim.x;
      if (nxt < ntiles) {
        const int64_t bn = sample(nxt);
        id0 = I::load(a.ids, bn * a.id_stride + cf0);
        id1 = I::load(a.ids, bn * a.id_stride + cf1);
      }
    }
    // ---- combine the 16 waves' partial tiles (double-buffered slab)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[buf][w][kk * 4 + r][nt * 16 + s] = acc[nt][r];
    qn += __shfl_xor(qn, 16);
    qn += __shfl_xor(qn, 32);
    if (lane < 16) qs[buf][w][lane] = qn;
    __syncthreads();
    if (threadIdx.x < 16 * NC) {
      const int smp = threadIdx.x / NC, col = threadIdx.x % NC;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) v += cs[buf][ww][smp][col];
      float t = col < a.kfm ? v * v : 0.f;  // s_f^2
      if (col < NW) t -= qs[buf][col][smp];  // - sum_i x_i^2 |v_i|^2 (wave partials)
      float lin = col == a.kfm ? v : 0.f;   // x@w1
      t = row16_sum(t);
      lin = row16_sum(lin);
      if constexpr (NT == 2) {
        t += __shfl_xor(t, 16);
        lin += __shfl_xor(lin, 16);
      }
      const int64_t bb = (int64_t)cur * 16 + smp;
      if (col == 0 && bb < a.batch) a.logit[bb] = (lin + a.w0[0]) + 0.5f * t;
    }
    if (__any(bad && valid) && lane == 0) flag_error(a.err);
    bad = false;
    if (!more) break;
    buf ^= 1;
  }
}

// ---------------------------------------------------------------- VALU form
// 8-sample tiles; lane = q + 4 s + 32 h: row quarter q (float4 of the 64-B
// row), sample s, field half h (field 2w + h of wave w).
template <int NF, int KIND>
__global__ __launch_bounds__(1024) void fm_tiles_valu(EmbedFmArgs a, int ntiles) {
  typedef Ids<KIND> I;
  constexpr int NV = NF + 2;  // per element: v[0..NF-1], w1, |v|^2
  extern __shared__ float4 vsm[];  // the packed FM image (rs_fm_prepare), staged once
  __shared__ float part[2][16][8][NV + 1];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nfw = (a.F + 1) >> 1;  // field waves; wave nfw (if nd > 0) = dense wave
  const int q = lane & 3, s = (lane >> 2) & 7, h = lane >> 5;
  const bool fwave = w < nfw;       // wave-uniform
  const int c = 2 * w + h;          // this lane's field (field waves)
  const bool hc = fwave && c < a.F;
  const int cc = hc ? c : 0;

  // ---- stage the FM image (16-B aligned, size % 4 == 0) through LDS
  const int n4 = (int)(a.field_base + (int64_t)a.F * a.field_rec) >> 2;
  const float4* prep4 = reinterpret_cast<const float4*>(a.prep);
  for (int i = threadIdx.x; i < n4; i += blockDim.x) vsm[i] = prep4[i];
  // field metadata: the wave's two fields (scalar), picked per lane by h
  const int cw0 = fwave ? min(2 * w, a.F - 1) : 0, cw1 = fwave ? min(2 * w + 1, a.F - 1) : 0;
  const int64_t o0 = a.offs[cw0], o1 = a.offs[cw1];
  const int64_t v0 = a.vocab[cw0], v1 = a.vocab[cw1];
  const int64_t off = h ? o1 : o0, voc = h ? v1 : v0;
  int tile = blockIdx.x;
  auto sample = [&](int t) -> int64_t {
    const int64_t bt = (int64_t)t * 8 + s;
    return bt < a.batch ? bt : a.batch - 1;
  };
  // ids of the first tile go out with the staging loads
  typename I::raw_t rid = I::load(a.ids, sample(tile) * a.id_stride + cc);
  __syncthreads();
  // ---- this lane's weights, kept for the whole launch
  float vr[4][NV];  // field lanes: elements e = nd + c k + 4q + j; dense lanes: see below
  const float* vf = reinterpret_cast<const float*>(vsm);
  if (fwave) {
    const float* rec = vf + a.field_base + (int64_t)cc * a.field_rec;
#pragma unroll
    for (int f = 0; f < NF + 1; ++f) {  // columns 0..NF-1 = v, NF = w1 (f <= kfm < 16)
      const float4 t4 = *reinterpret_cast<const float4*>(rec + (q * 16 + f) * 4);
      vr[0][f] = t4.x;
      vr[1][f] = t4.y;
      vr[2][f] = t4.z;
      vr[3][f] = t4.w;
    }
    const float4 n4v = *reinterpret_cast<const float4*>(rec + 64 * 4 + q * 4);
    vr[0][NF + 1] = n4v.x;
    vr[1][NF + 1] = n4v.y;
    vr[2][NF + 1] = n4v.z;
    vr[3][NF + 1] = n4v.w;
  } else {
    // dense wave: lane element e_j = 4 (2 j + h) + q, j < 4 (nd <= 32)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 2 * j + h;
      const bool he = t < a.DB && 4 * t + q < a.nd;
      const float* rec = vf + (int64_t)(t < a.DB ? t : 0) * a.dense_rec;
#pragma unroll
      for (int f = 0; f < NF + 1; ++f) vr[j][f] = he ? rec[q * 16 + f] : 0.f;
      vr[j][NF + 1] = he ? rec[64 + q] : 0.f;
    }
  }
  float4 x;
  bool ok = true;
  auto issue_row = [&](typename I::raw_t r, float4& y, bool& k) {
    int64_t id;
    k = I::decode(r, voc, id);
    const floatx4 t4 = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + (off + id) * 16 + 4 * q));
    y = float4{t4[0], t4[1], t4[2], t4[3]};
  };
  auto dense_x = [&](int64_t b, float4& y) {
    float e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int el = 4 * (2 * j + h) + q;
      e[j] = a.dense[b * a.dense_stride + (el < a.nd ? el : 0)];
      e[j] = el < a.nd ? e[j] : 0.f;
    }
    y = float4{e[0], e[1], e[2], e[3]};
  };
  if (fwave) issue_row(rid, x, ok);
  else x = float4{0.f, 0.f, 0.f, 0.f};
  int nxt = tile + gridDim.x;
  if (fwave && nxt < ntiles) rid = I::load(a.ids, sample(nxt) * a.id_stride + cc);
  if (!fwave) dense_x(sample(tile), x);
  bool bad = false;
  int buf = 0;
  while (true) {
    const bool valid = (int64_t)tile * 8 + s < a.batch;
    // ---- the lane's partial [s_0..s_{NF-1}, x@w1, sum x^2 |v|^2] over its 4 elements
    const bool use = fwave ? (hc && ok) : true;
    bad |= hc && !ok;
    const float xe[4] = {use ? x.x : 0.f, use ? x.y : 0.f, use ? x.z : 0.f, use ? x.w : 0.f};
    float acc[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) acc[f] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int f = 0; f < NF + 1; ++f) acc[f] = fmaf(xe[j], vr[j][f], acc[f]);
      acc[NF + 1] = fmaf(xe[j] * xe[j], vr[j][NF + 1], acc[NF + 1]);
    }
    // ---- next tile's row goes out before this tile's reduction
    const int cur = tile;
    tile = nxt;
    const bool more = tile < ntiles;
    if (more) {
      if (fwave) {
        issue_row(rid, x, ok);
        nxt = tile + gridDim.x;
        if (nxt < ntiles) rid = I::load(a.ids, sample(nxt) * a.id_stride + cc);
      } else {
        nxt = tile + gridDim.x;
        dense_x(sample(tile), x);
      }
    }
    // ---- reduce over the row's 4 lanes (DPP quad permutes) and the wave's
    // two fields (lanes 32 apart), then the waves through LDS
#pragma unroll
    for (int f = 0; f < NV; ++f) {
      float t = acc[f];
      t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
      t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
      t += __shfl_xor(t, 32);
      acc[f] = t;
    }
    if (h == 0) {
#pragma unroll
      for (int f = 0; f < NV; ++f)
        if ((f & 3) == q) part[buf][w][s][f] = acc[f];
    }
    __syncthreads();
    const int nwv = blockDim.x >> 6;
    if (threadIdx.x < 128) {
      const int smp = threadIdx.x >> 4, col = threadIdx.x & 15;
      float v = 0.f;
      if (col < NV)
        for (int ww = 0; ww < nwv; ++ww) v += part[buf][ww][smp][col];
      float t = col < NF ? v * v : 0.f;
      if (col == NF + 1) t = -v;
      float lin = col == NF ? v : 0.f;
      t = row16_sum(t);
      lin = row16_sum(lin);
      const int64_t bb = (int64_t)cur * 8 + smp;
      if (col == 0 && bb < a.batch) a.logit[bb] = (lin + a.w0[0]) + 0.5f * t;
    }
    if (__any(bad && valid) && lane == 0) flag_error(a.err);
    bad = false;
    if (!more) break;
    buf ^= 1;
  }
}

// ------------------------------------------------------------------ launch
template <int KIND>
static bool launch_kind(const EmbedFmArgs& a, const FmGeom& g, int variant, hipStream_t st) {
  if (variant == 1) {
    // VALU form: k = 16, kfm in {8, 10, 16 - 2 = 14}, <= 30 fields, nd <= 32
    if (g.k != 16 || a.F < 1 || a.F > 30 || a.nd > 32 || g.NT != 1) return false;
    const int ntiles = (int)((a.batch + 7) / 8);
    const int waves = (a.F + 1) / 2 + (a.nd > 0 ? 1 : 0);
    const size_t lds = (size_t)(g.field_base + (int64_t)a.F * g.field_rec) * sizeof(float);
    if (lds > 64 * 1024) return false;
    const int grid = ntiles < 256 ? ntiles : 256;
    switch (a.kfm) {
      case 8: fm_tiles_valu<8, KIND><<<grid, waves * 64, lds, st>>>(a, ntiles); return true;
      case 10: fm_tiles_valu<10, KIND><<<grid, waves * 64, lds, st>>>(a, ntiles); return true;
      default: return false;
    }
  }
  if (variant == 2 || variant == 3) {
    if (a.F < 1 || a.F > 2 * TM_NW || g.DB > TM_NW) return false;
    const int ntiles = (int)((a.batch + 15) / 16);
    const int cap = variant == 2 ? 512 : 256;  // 2 or 1 resident workgroups per CU
    const int grid = ntiles < cap ? ntiles : cap;
    if (g.KV == 4 && g.NT == 1) fm_tiles_mfma<4, 1, KIND><<<grid, TM_NW * 64, 0, st>>>(a, ntiles);
    else if (g.KV == 2 && g.NT == 1) fm_tiles_mfma<2, 1, KIND><<<grid, TM_NW * 64, 0, st>>>(a, ntiles);
    else if (g.KV == 4 && g.NT == 2) fm_tiles_mfma<4, 2, KIND><<<grid, TM_NW * 64, 0, st>>>(a, ntiles);
    else return false;
    return true;
  }
  return false;
}

bool launch_embed_fm_tiles(const EmbedFmArgs& a, const FmGeom& g, int kind, int variant, hipStream_t st) {
  if (!g.mfma || a.F == 0 || a.x_out || variant == 0) return false;
  if (a.batch > ((int64_t)1 << 30)) return false;
  switch (kind) {
    case RS_ID_I32: return launch_kind<0>(a, g, variant, st);
    case RS_ID_I64: return launch_kind<1>(a, g, variant, st);
    case RS_ID_F32: return launch_kind<2>(a, g, variant, st);
    default: return false;
  }
}

}  // namespace rs
