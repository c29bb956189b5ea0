// embed_fm.hip — embedding lookup (EmbedLayer) and FM second-order kernels.
//
// Reference semantics:
//   EmbedLayer.call            algorithm/deep_learning/layer/core.py:273-280
//   DeepFM x = [dense | emb]   algorithm/deep_learning/model/deepFM.py:24-26
//   FMLayer.call               algorithm/deep_learning/layer/interaction.py:106-114
//   FM model (one-hot input)   algorithm/deep_learning/model/fm.py:19-23,
//                              utils/dataset.py:47-48 (get_dummies layout)
//
// Headline kernel: embed_fm_mfma — one launch does ids -> rows -> FM logit.
//   * A workgroup owns 16 samples (one MFMA row tile) and NW waves split the
//     contraction dimension d = nd + F*k round-robin by field (K-split).
//   * Lane l of a wave is sample s = l&15 and k-slot kk = l>>4: for field c it
//     loads k/4 consecutive floats of the sample's row (k=16: one float4, so a
//     wave-instruction reads 16 whole 64-B rows), which are its A-operand
//     values for the field's k/4 MFMA k-steps (k order permuted per field;
//     the packed B image from rs_fm_prepare uses the same permutation).
//   * s = x@v and the linear term x@w1 come out of v_mfma_f32_16x16x4_f32
//     (B columns 0..kfm-1 = v, column kfm = w1); the second-order correction
//     sum_f (x^2@v^2)_f = sum_i x_i^2 * |v_i|^2 is a per-lane FMA with the row
//     norms packed beside B, reduced across the 4 k-slots by wave shuffles.
//   * Partial tiles of the NW waves are summed through LDS; wave 0 finishes
//     logit = (x@w1 + w0) + 0.5*(sum_f s_f^2 - sum_i x_i^2 |v_i|^2).
#include <stdlib.h>

#include <type_traits>

#include "embed_fm.hpp"
#include "mlp_tower.hpp"
#include "peer.hpp"
#include "rs_common.hpp"
#include "shard_route.hpp"

namespace rs {

__device__ __forceinline__ float fm_bval(const float* w1, const float* v, int d, int kfm, int e, int colg) {
  if (e >= d) return 0.f;
  if (colg < kfm) return v[(int64_t)e * kfm + colg];
  if (colg == kfm) return w1[e];
  return 0.f;
}

__device__ __forceinline__ float fm_rownorm(const float* v, int d, int kfm, int e) {
  if (e >= d) return 0.f;
  float n = 0.f;
  for (int f = 0; f < kfm; ++f) {
    const float t = v[(int64_t)e * kfm + f];
    n = fmaf(t, t, n);
  }
  return n;
}

__global__ void fm_prepare_mfma(const float* __restrict__ w1, const float* __restrict__ v, int nd, int F,
                                int k, int kfm, int KV, int NT, int DB, int64_t dense_rec,
                                int64_t field_rec, int64_t field_base, int64_t size,
                                float* __restrict__ out) {
  const int d = nd + F * k;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < size;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float val;
    if (idx < field_base) {
      const int t = (int)(idx / dense_rec);
      const int r = (int)(idx % dense_rec);
      if (r < NT * 64) {
        const int nt = r / 64, lane = r % 64;
        const int e = 4 * t + (lane >> 4);
        val = (e < nd) ? fm_bval(w1, v, d, kfm, e, nt * 16 + (lane & 15)) : 0.f;
      } else {
        const int e = 4 * t + (r - NT * 64);
        val = (e < nd) ? fm_rownorm(v, d, kfm, e) : 0.f;
      }
    } else {
      const int64_t j = idx - field_base;
      const int c = (int)(j / field_rec);
      const int r = (int)(j % field_rec);
      if (r < NT * 64 * KV) {
        const int nt = r / (64 * KV), rem = r % (64 * KV);
        const int lane = rem / KV, tp = rem % KV;
        const int e = nd + c * k + KV * (lane >> 4) + tp;
        val = fm_bval(w1, v, d, kfm, e, nt * 16 + (lane & 15));
      } else {
        const int r2 = r - NT * 64 * KV;
        const int e = nd + c * k + KV * (r2 / KV) + (r2 % KV);
        val = fm_rownorm(v, d, kfm, e);
      }
    }
    out[idx] = val;
  }
}

__global__ void fm_prepare_generic(const float* __restrict__ w1, const float* __restrict__ v, int d, int kfm,
                                   float* __restrict__ out) {
  const int64_t n = (int64_t)d * (kfm + 2);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float val;
    if (idx < d) val = w1[idx];
    else if (idx < (int64_t)d * (kfm + 1)) val = v[idx - d];
    else val = fm_rownorm(v, d, kfm, (int)(idx - (int64_t)d * (kfm + 1)));
    out[idx] = val;
  }
}

// Phase stamps (s_memrealtime, 100 MHz) for the diagnostic library built by
// scripts/build_diag.sh; compiled out of librs_hip.so.
#ifdef RS_DIAG_STAMPS
#define RS_STAMP(i)                                                                          \
  do {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    if (a.dbg && lane == 0)                                                                  \
      a.dbg[((int64_t)blockIdx.x * NW + w) * 16 + (i)] = __builtin_amdgcn_s_memrealtime();  \
    __builtin_amdgcn_sched_barrier(0);                                                       \
  } while (0)
#define RS_USE(x) asm volatile("" ::"v"(x))
#else
#define RS_STAMP(i) \
  do {              \
  } while (0)
#define RS_USE(x) \
  do {            \
  } while (0)
#endif

// KIND: 0 i32, 1 i64, 2 f32 ids; 3 = rows already gathered (row(b,c) = b*F+c);
// 4 = owner side of the sharded FM (sharded.py, partial protocol): ids are
// int32 LOCAL rows of the owner's shard (-1 = lookup not owned here: a zero
// contribution, not an error), no dense block, and instead of the logit the
// workgroup writes each sample's partial record
//   [s_0 .. s_{kfm-1}, x@w1, sum_i x_i^2 |v_i|^2, 0-pad]   (a.pw floats)
// over the fields it was given; rs_shard_fm_combine finishes the FM.
// TW: fused DeepFM — x goes to an LDS tile ([emb F*k | dense nd | 0-pad],
// row stride tw->rs) instead of x_out, and the DNN tower of mlp_tower.hpp runs
// on it, closed by sigmoid(c0*dnn + c1*fm) (model/deepFM.py:24-30).
// A workgroup owns one 16-sample MFMA row tile.
// FC / KFMC / NDC: the field count, FM width and dense width as compile-time
// constants (0 / 0 / -1: the kernel arguments' run-time values) — the
// headline shape's kernarg and streamed kernels take 26 / 10 / 13
template <int KV, int NT, int NW, int KIND, bool TW, int MC = 0, bool PF = false, bool KA = false, int FC = 0,
          int KFMC = 0, int NDC = -1>
__device__ __forceinline__ void embed_fm_body(const EmbedFmArgs& a, const MlpArgs* tw, const int tile,
                                              const FieldMeta* km = nullptr) {
  const int aF = FC > 0 ? FC : a.F;        // (compile-time at the specialised shapes)
  const int akfm = KFMC > 0 ? KFMC : a.kfm;
  const int and_ = NDC >= 0 ? NDC : a.nd;
  // MC > 0: field slots per wave and pass (owner kernels with few fields)
  constexpr int MAXC0 = MC > 0 ? MC : 128 / (NW * KV);
  constexpr int MAXC = MAXC0 < 1 ? 1 : (MAXC0 > 8 ? 8 : MAXC0);
  typedef Ids<(KIND >= 3) ? 0 : KIND> I;
  constexpr bool OWNER = KIND == 4;
  __shared__ float cs[NW][16][NT * 16 + 1];
  __shared__ float qs[NW][16];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15;   // A: sample row of the tile; B/C: column
  const int kk = lane >> 4;  // k-slot
  const int64_t bt = (int64_t)tile * 16 + s;
  const bool valid = bt < a.batch;
  // Padded lanes of the last tile recompute the last sample: an MFMA output
  // row depends only on its own A row, so they never touch valid outputs.
  const int64_t b = bt < a.batch ? bt : a.batch - 1;
  const int d = and_ + aF * a.k;
  // w0 is requested now, not behind the rows (a dependent load at the end)
  const float w0v = OWNER ? 0.f : a.w0[0];

  // four accumulation chains: MFMA tp of a field slot into chain tp & 3,
  // summed below.  Fixed at compile time: the runtime switch this replaced
  // put a scalar branch beside every MFMA and cost 6.01 vs 5.74 us per
  // headline launch (cold instruction cache, profiles/r4_ab_ka_chains_compile_time.json)
  floatx4 ac[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int c = 0; c < 4; ++c) ac[nt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  float qn = 0.f;
  bool bad = false;

  // ---- prologue: everything that does not depend on the ids is issued first
  // (dense features, packed weights, field offsets/vocab), so the kernel's
  // critical path is exactly two dependent memory trips: ids -> rows.
  // A dense block of at most NW k-steps (DeepFM: 13 features = 4 k-steps) is
  // one k-step per wave; wider dense inputs (FMLayer on a plain x) stream.
  // Materialise every kernel argument at entry: one batched s_load instead
  // of lazy per-use kernarg loads (each a dependent K$ round trip).
  asm volatile("" ::"s"(a.ids), "s"(a.id_stride), "s"(a.dense), "s"(a.dense_stride), "s"(a.nd), "s"(a.table),
               "s"(a.offs), "s"(a.vocab), "s"(aF), "s"(a.k), "s"(a.prep), "s"(akfm));
  asm volatile("" ::"s"(a.batch), "s"(a.DB), "s"(a.dense_rec), "s"(a.field_rec), "s"(a.field_base), "s"(a.x_out),
               "s"(a.logit), "s"(a.w0), "s"(a.err));
  RS_STAMP(0);
  RS_USE(b);
  RS_STAMP(5);
  if constexpr (TW) {
    const MlpArgs& a = *tw;  // MLP_STAMP reads a.dbg
    MLP_STAMP(0);
  }
  // fused tower: its layer-0 weights, the bias/alpha block and the x tile's
  // zero padding do not depend on the ids; issue them first
  extern __shared__ float tsm[];
  __shared__ float fmlog[TW ? 16 : 1];
  floatx4 ring[TW ? MLP_R : 1];
  const int xrs = TW ? tw->rs : 0;
  if constexpr (TW) {
    mlp_first_fill<NW>(*tw, ring);
    float* par = tsm + 32 * tw->rs + NW * 256;
    for (int i = threadIdx.x; i < tw->ptot; i += NW * 64) par[i] = tw->prep[tw->wtot + i];
    const int d0 = aF * a.k + and_, padw = tw->Kp[0] - d0;
    for (int i = threadIdx.x; i < 16 * padw; i += NW * 64) {
      const int r = i / padw;
      tsm[r * xrs + d0 + (i - r * padw)] = 0.f;
    }
  }
  const bool dense_small = KA || a.DB <= NW;  // (the kernarg kernel is launched for DB <= 16 only)
  // Dense k-steps go to the LAST waves: with F = 26 fields over 16 waves the
  // first F - NW waves already carry two fields.
  const int dw = NW - 1 - w;                        // dense k-step of this wave
  const bool has_dense = dense_small && dw < a.DB;  // wave-uniform
  float dx = 0.f, dn = 0.f, drec[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) drec[nt] = 0.f;
  auto load_dense = [&]() {
    if (has_dense) {
      const int e = 4 * dw + kk;
      dx = a.dense[b * a.dense_stride + (e < and_ ? e : 0)];  // masked at use
      const float* rec = a.prep + (int64_t)dw * a.dense_rec;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) drec[nt] = rec[nt * 64 + lane];
      dn = rec[NT * 64 + kk];
    }
  };
  // ---- cooperative id tile: the workgroup's 16 x F ids and the F field
  // (offset, vocab) pairs arrive through coalesced loads into LDS, once per
  // workgroup (instead of 4 redundant lanes per id and one metadata load per
  // wave and field), then one barrier.  Fields beyond FMAX use direct loads.
  constexpr int FMAX = 128;
  __shared__ typename I::raw_t lid[16][FMAX];
  __shared__ int64_t lmeta[2][FMAX];
  // (owner side, KIND 4: the local rows need no field metadata, so every
  // wave loads its own ids — no id tile, no barrier before the rows)
#ifdef RS_DIAG_STAMPS
  const bool coop = !KA && !OWNER && (KIND != 3) && aF <= FMAX && !(a.ablate & 16);  // bit 16: per-wave id loads
#else
  const bool coop = !KA && !OWNER && (KIND != 3) && aF <= FMAX;
#endif
  if (coop) {
    const int64_t b0 = (int64_t)tile * 16;
    for (int t = threadIdx.x; t < 16 * aF; t += NW * 64) {
      const int ss = t / aF, c = t - ss * aF;
      const int64_t bb = b0 + ss < a.batch ? b0 + ss : a.batch - 1;
      const auto idv = I::load(a.ids, bb * a.id_stride + c);
#ifdef RS_DIAG_STAMPS
      RS_USE(idv);
      RS_STAMP(8);
#endif
      lid[ss][c] = idv;
    }
    if constexpr (!OWNER) {
      for (int t = threadIdx.x; t < 2 * aF; t += NW * 64) {
        const int c = t < aF ? t : t - aF;
        lmeta[t < aF ? 0 : 1][c] = t < aF ? a.offs[c] : a.vocab[c];
      }
    }
  }
  // ---- fields c = cg + j*NW + w; slots past F re-read field F-1 and add 0.
  // A pass = its B fragments and |v_e|^2 (launch constants), then its rows,
  // then the MFMAs.  The first two passes' B fragments are requested here,
  // inside the id trip (L2 hits, done before the ids arrive), and their norms
  // computed while the first rows are in flight, so a pass's work after its
  // rows arrive is its MFMAs and one FMA per element.
  struct Pass {
    int cj[MAXC];
    bool ok[MAXC];
    typename I::raw_t rid[MAXC];
    int64_t off[MAXC], voc[MAXC];
    int64_t row[MAXC];  // decoded table rows (decode_rows)
    Chunk<KV> xs[MAXC];
    Chunk<KV> bw[MAXC][NT];
    float nrm[MAXC][KV];
  };
  auto issue_b = [&](int cg, Pass& P) {
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = cg + j * NW + w;
      P.cj[j] = c < aF ? c : aF - 1;
      const float* rec = a.prep + a.field_base + (int64_t)P.cj[j] * a.field_rec;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
#ifdef RS_DIAG_STAMPS
        if (a.ablate & 2) { P.bw[j][nt].zero(); P.bw[j][nt].v[0] = (float)P.cj[j]; continue; }
#endif
        // lanes of the zero-padded columns (> kfm) load nothing
        if (nt * 16 + s <= akfm) P.bw[j][nt].load(rec + (int64_t)(nt * 64 + lane) * KV);
        else P.bw[j][nt].zero();
      }
    }
  };
  auto norms = [&](Pass& P) {
    // |v_e|^2 for this lane's element e: the B lanes of DPP row kk hold
    // v[e][0..15] — the same row as the A lane that holds x_e.
#pragma unroll
    for (int j = 0; j < MAXC; ++j)
#pragma unroll
      for (int tp = 0; tp < KV; ++tp) {
        float sq = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const float bv = nt * 16 + s < akfm ? P.bw[j][nt].v[tp] : 0.f;
          sq = fmaf(bv, bv, sq);
        }
        P.nrm[j][tp] = row16_sum(sq);
      }
  };
  const int wv = threadIdx.x >> 6;
  // a pass's ids and field metadata (issue_rows takes them from here)
  auto fetch_ids = [&](int cg, Pass& P) {
    int64_t* offc = P.off;
    int64_t* vocc = P.voc;
    // Field metadata through the VECTOR path (wave index taken from the raw
    // thread id, not readfirstlane, so these are not scalar loads): issued
    // with the ids, no dependent K$-miss round trip on the critical path.
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      if constexpr (KIND != 3) {
        if (OWNER) {
          offc[j] = 0;
          vocc[j] = a.owner_rows;
          P.rid[j] = coop ? lid[s][P.cj[j]] : I::load(a.ids, b * a.id_stride + P.cj[j]);
        } else if (coop) {
          offc[j] = lmeta[0][P.cj[j]];
          vocc[j] = lmeta[1][P.cj[j]];
          P.rid[j] = lid[s][P.cj[j]];
        } else if constexpr (KA) {  // kernarg metadata: scalar loads, wave-uniform field
          offc[j] = km->off[P.cj[j]];
          vocc[j] = km->voc[P.cj[j]];
          P.rid[j] = I::load(a.ids, b * a.id_stride + P.cj[j]);
        } else {
          const int cv = min(cg + j * NW + wv, aF - 1);
          offc[j] = a.offs[cv];
          vocc[j] = a.vocab[cv];
          P.rid[j] = I::load(a.ids, b * a.id_stride + P.cj[j]);
        }
      }
    }
    if (cg == 0 && !coop && aF > 0) load_dense();
  };
  // id -> table row (the ids must have arrived)
  auto decode_rows = [&](int cg, Pass& P) {
    if (cg == 0) RS_STAMP(6);
    else RS_STAMP(10);
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      if constexpr (KIND == 3) {
        P.row[j] = b * aF + P.cj[j];
        P.ok[j] = true;
      } else {
        int64_t id;
        P.ok[j] = I::decode(P.rid[j], P.voc[j], id);
        P.row[j] = P.off[j] + id;
      }
    }
    RS_USE(P.row[MAXC - 1]);
    if (cg == 0) RS_STAMP(1);
    else RS_STAMP(11);
  };
  // row gather: KV consecutive floats of the sample's row per lane
  auto load_rows = [&](int cg, Pass& P) {
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
#ifdef RS_DIAG_STAMPS
      if ((a.ablate & 8) && cg + j * NW + w >= aF) { P.xs[j].zero(); continue; }
#endif
      P.xs[j].load_nt(a.table + P.row[j] * a.k + KV * kk);
    }
  };
  auto issue_rows = [&](int cg, Pass& P, bool fetched) {
    if (!fetched) fetch_ids(cg, P);
    decode_rows(cg, P);
    load_rows(cg, P);
  };
  auto consume = [&](int cg, Pass& P) {
    RS_USE(P.xs[MAXC - 1].v[KV - 1]);
    RS_USE(P.bw[MAXC - 1][0].v[KV - 1]);
    if (cg == 0) RS_STAMP(2);
    else RS_STAMP(12);
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const bool live = cg + j * NW + w < aF;
      if constexpr (OWNER) bad |= live && !P.ok[j] && P.rid[j] != -1;
      else bad |= live && !P.ok[j];
      const bool use = live && P.ok[j];
#pragma unroll
      for (int tp = 0; tp < KV; ++tp) {
        const float xv = use ? P.xs[j].v[tp] : 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
#ifdef RS_DIAG_STAMPS
          if (a.ablate & 1) { ac[nt][0][0] += xv * P.bw[j][nt].v[tp]; continue; }
#endif
          ac[nt][tp & 3] = mfma16x16x4(xv, P.bw[j][nt].v[tp], ac[nt][tp & 3]);
        }
        qn = fmaf(xv * xv, P.nrm[j][tp], qn);
      }
      if constexpr (TW) {
        if (live) {
          float* xo = tsm + s * xrs + P.cj[j] * a.k + KV * kk;
#pragma unroll
          for (int tp = 0; tp < KV; ++tp) xo[tp] = P.ok[j] ? P.xs[j].v[tp] : 0.f;
        }
      } else if (!KA && a.x_out && live && valid) {  // (the kernarg kernel never emits x)
        float* xo = a.x_out + b * d + and_ + P.cj[j] * a.k + KV * kk;
#pragma unroll
        for (int tp = 0; tp < KV; ++tp) xo[tp] = P.ok[j] ? P.xs[j].v[tp] : 0.f;
      }
    }
    RS_USE(ac[0][0][0]);
    if (cg == 0) RS_STAMP(13);
    else RS_STAMP(14);
  };
  // one slot per wave: a wave with no field left in a pass stops there (a
  // wave-uniform exit; nothing after the loop needs its slot)
  auto has_pass = [&](int cg) { return cg < aF && !(MAXC == 1 && cg + w >= aF); };
  constexpr int PS = NW * MAXC;  // fields per pass
  // PF: B fragments of the first two passes ride the id trip (registers: two
  // passes only where they are few; larger rows load theirs per pass).
  // Measured (scripts/ab, profiles/r3_ab_prefetch_*.json): 14.51 vs 15.30 us
  // at batch 16384 (4 tiles per CU), 6.15 vs 6.13 at 4096 (1 tile per CU)
  constexpr bool PRE = PF && KV * MAXC * NT <= 8;
  Pass P0, P1;
  if (PRE) {
    if (has_pass(0)) issue_b(0, P0);
    if (has_pass(PS)) issue_b(PS, P1);
  }
  if (aF == 0 || coop) load_dense();
  if (coop) __syncthreads();
  RS_STAMP(9);
  if (PRE) {
    const bool one = has_pass(0), two = one && has_pass(PS);
    if (one) {
      // both passes' ids requested together: the second pass's id trip is
      // not serialised behind the first pass's rows and MFMAs (after the B
      // fragments: ids first was slower, 5.95 vs 5.75 us at 4096)
      fetch_ids(0, P0);
      if (two) fetch_ids(PS, P1);
    } else if (!coop && aF > 0) {
      load_dense();  // a wave with no field (F < NW) may still own a dense k-step
    }
    if (one) {
      // (the second pass's rows stay behind the first pass's MFMAs: issuing
      // them with the first pass's was slower, 6.19 vs 5.82 us at 4096 —
      // the r1 finding that two row bursts beat one, again)
      issue_rows(0, P0, true);
      norms(P0);
      if (two) norms(P1);
      // the second pass's ids arrive with the first's: its row addresses are
      // worked out while the first rows are in flight, so only the loads
      // themselves sit between the first pass's MFMAs and the second trip
      if (two) decode_rows(PS, P1);
      consume(0, P0);
      if (two) {
        load_rows(PS, P1);
        consume(PS, P1);
        // (a third pass: more than 2 x NW fields — never in the kernarg kernel, F <= 32)
        for (int cg = 2 * PS; !KA && has_pass(cg); cg += PS) {
          issue_b(cg, P0);
          issue_rows(cg, P0, false);
          norms(P0);
          consume(cg, P0);
        }
      }
    }
  } else {
    for (int cg = 0; has_pass(cg); cg += PS) {
      issue_b(cg, P0);
      issue_rows(cg, P0, false);
      norms(P0);
      consume(cg, P0);
    }
  }

  // ---- dense MFMAs (their loads were issued in the prologue)
  if (has_dense) {
    const int e = 4 * dw + kk;
    dx = e < and_ ? dx : 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ac[nt][0] = mfma16x16x4(dx, drec[nt], ac[nt][0]);
    qn = fmaf(dx * dx, dn, qn);
    if constexpr (TW) {
      if (e < and_) tsm[s * xrs + aF * a.k + e] = dx;
    } else if (!KA && a.x_out && valid && e < and_) {
      a.x_out[b * d + e] = dx;
    }
  }
  if (!dense_small) {
    for (int t = w; t < a.DB; t += NW) {
      const int e = 4 * t + kk;
      const float xv = a.dense[b * a.dense_stride + (e < and_ ? e : 0)];
      const float x = e < and_ ? xv : 0.f;
      const float* rec = a.prep + (int64_t)t * a.dense_rec;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) ac[nt][0] = mfma16x16x4(x, rec[nt * 64 + lane], ac[nt][0]);
      qn = fmaf(x * x, rec[NT * 64 + kk], qn);
      if constexpr (TW) {
        if (e < and_) tsm[s * xrs + aF * a.k + e] = x;
      } else if (a.x_out && valid && e < and_) {
        a.x_out[b * d + e] = x;
      }
    }
  }
  floatx4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[nt][i] = (ac[nt][0][i] + ac[nt][1][i]) + (ac[nt][2][i] + ac[nt][3][i]);
  RS_USE(acc[0][0]);
  RS_STAMP(3);
  if (__any(bad && valid) && lane == 0) flag_error(a.err);

#ifdef RS_DIAG_STAMPS
  if (a.ablate & 4) {
    if (w == 0 && kk == 0 && b < a.batch) a.logit[b] = acc[0][0] + acc[0][1] + qn;
    return;
  }
#endif
  // ---- combine the NW partial tiles: thread (sample, column) sums the waves'
  // partials; the per-sample reductions over columns are DPP row sums.
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[w][kk * 4 + r][nt * 16 + s] = acc[nt][r];
  qn += __shfl_xor(qn, 16);
  qn += __shfl_xor(qn, 32);
  if (lane < 16) qs[w][lane] = qn;
  __syncthreads();
  RS_STAMP(7);
  constexpr int NC = NT * 16;  // columns per sample
  if (threadIdx.x < 16 * NC) {
    const int smp = threadIdx.x / NC, col = threadIdx.x % NC;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += cs[ww][smp][col];
    float t = col < akfm ? v * v : 0.f;       // s_f^2
    if (col < NW) t -= qs[col][smp];           // - sum_i x_i^2 |v_i|^2 (wave partials)
    float lin = col == akfm ? v : 0.f;        // x@w1
    t = row16_sum(t);
    lin = row16_sum(lin);
    if constexpr (NT == 2) {
      t += __shfl_xor(t, 16);
      lin += __shfl_xor(lin, 16);
    }
    const int64_t bb = (int64_t)tile * 16 + smp;
    if constexpr (OWNER) {
      // partial record: column sums as they stand, the q term row-summed
      float q = col < NW ? qs[col][smp] : 0.f;
      q = row16_sum(q);
      if constexpr (NT == 2) q += __shfl_xor(q, 16);
      if (bb < a.batch) {
        float* rec = a.logit + bb * a.pstride;
        if (col <= akfm) rec[col] = v;
        if (col == 0) rec[akfm + 1] = q;
        else if (akfm + 1 + col < a.pw) rec[akfm + 1 + col] = 0.f;
      }
      return;
    }
    const float fm = (lin + w0v) + 0.5f * t;
    if (col == 0 && bb < a.batch && a.logit) a.logit[bb] = fm;
    if constexpr (TW) {
      if (col == 0) fmlog[smp] = fm;
    }
  }
  RS_STAMP(4);
  if constexpr (TW) {
    {
      const MlpArgs& a = *tw;
      MLP_STAMP(1);
    }
    mlp_tower_tile<NW>(*tw, tsm, (int64_t)tile * 16, ring, fmlog);
  }
}

template <int KV, int NT, int NW, int KIND, int MC, bool PF = false>
__global__ __launch_bounds__(NW * 64) void embed_fm_mfma(EmbedFmArgs a) {
  embed_fm_body<KV, NT, NW, KIND, false, MC, PF>(a, nullptr, blockIdx.x);
}

// the field metadata by value (rs_embed_fm_fwd_hm): each wave loads its own
// fields' ids and reads (offset, vocab) through scalar kernarg loads — no LDS
// id tile, no barrier, no per-wave metadata loads from one hot L2 line
template <int KV, int NT, int NW, int KIND, bool PF, int FC = 0, int KFMC = 0, int NDC = -1>
__global__ __launch_bounds__(NW * 64) void embed_fm_mfma_ka(EmbedFmArgs a, FieldMeta m) {
  embed_fm_body<KV, NT, NW, KIND, false, 1, PF, true, FC, KFMC, NDC>(a, nullptr, blockIdx.x, &m);
}

// S consecutive batches in ONE launch (rs_embed_fm_fwd_hm_stream): workgroup
// g runs the kernarg kernel's body on tile g % tpb of batch g / tpb (batch-
// major dispatch order) — the same instantiation and tile arithmetic as the
// per-batch launch, so every batch's logits are bit-identical to
// rs_embed_fm_fwd_hm's; batch s's ids / dense / logit start at the given
// per-batch strides; the last batch may be shorter (its own tile count).
// MINB = 2 asks for two resident workgroups per CU (<= 64 VGPRs), so one
// tile's id trip runs under another's rows and combine.
struct StreamArgs {
  int tpb, S;
  int64_t ids_bstride_bytes, dense_bstride, logit_bstride, last_batch;
};
template <int KV, int NT, int KIND, int MINB, int FC = 0, int KFMC = 0, int NDC = -1>
__global__ __launch_bounds__(16 * 64, MINB) void embed_fm_stream_ka(EmbedFmArgs a, FieldMeta m, StreamArgs sa) {
  const int s = blockIdx.x / sa.tpb, tile = blockIdx.x - s * sa.tpb;
  EmbedFmArgs b = a;
  b.ids = static_cast<const char*>(a.ids) + s * sa.ids_bstride_bytes;
  b.dense = a.dense + s * sa.dense_bstride;
  b.logit = a.logit + s * sa.logit_bstride;
  if (s == sa.S - 1) b.batch = sa.last_batch;
  if ((int64_t)tile * 16 >= b.batch) return;  // a shorter last batch: fewer tiles (uniform exit)
  embed_fm_body<KV, NT, 16, KIND, false, 1, true, true, FC, KFMC, NDC>(b, nullptr, tile, &m);
}

// ---- sharded FM, partial protocol: combine (requester side) as a block part
struct CombineArgs {
  const float* part;  // partial records [world][batch], pst floats apart
  int64_t pst;
  int world;
  int64_t batch;
  const float* dense;
  int64_t ds;
  int nd;
  const float* prep;  // the packed FM image (dense records at its start)
  int64_t dense_rec;
  int NT;
  const float* w0;
  int kfm;
  float* logit;
  // training (rs_shard_fm_combine_grad): [s_0..s_{kfm-1} | g] records gst
  // floats apart, g = (sigmoid(logit) - label) * gscale; per-sample BCE
  const float* labels;
  float gscale;
  float* gs;
  int64_t gst;
  float* loss;
};

// 16 lanes per sample (lane = partial column, strided by 16), DPP row sums;
// blocks blk of nblk, NTH threads each, grid-stride over batch*16 lanes.
template <int NTH>
__device__ __forceinline__ void fm_combine_part(const CombineArgs& c, int blk, int nblk) {
  for (int64_t idx = (int64_t)blk * NTH + threadIdx.x; idx < c.batch * 16; idx += (int64_t)nblk * NTH) {
    const int64_t b = idx >> 4;
    const int cl = threadIdx.x & 15;
    float t = 0.f, lin = 0.f, q = 0.f;
    for (int col = cl; col < c.kfm + 2; col += 16) {
      float acc = 0.f;
      for (int o = 0; o < c.world; ++o) acc += c.part[((int64_t)o * c.batch + b) * c.pst + col];
      for (int e = 0; e < c.nd; ++e) {
        const float x = c.dense[b * c.ds + e];
        const float* rec = c.prep + (int64_t)(e >> 2) * c.dense_rec;
        if (col <= c.kfm) acc = fmaf(x, rec[(col >> 4) * 64 + (e & 3) * 16 + (col & 15)], acc);
        else acc = fmaf(x * x, rec[c.NT * 64 + (e & 3)], acc);
      }
      if (col < c.kfm) {
        t = fmaf(acc, acc, t);
        if (c.gs) c.gs[b * c.gst + col] = acc;
      } else if (col == c.kfm) lin = acc;
      else q = acc;
    }
    t = row16_sum(t);
    lin = row16_sum(lin);
    q = row16_sum(q);
    if (cl == 0) {
      const float z = (lin + c.w0[0]) + 0.5f * (t - q);
      c.logit[b] = z;
      if (c.gs) {
        const float y = c.labels[b];
        c.gs[b * c.gst + c.kfm] = (sigmoidf_(z) - y) * c.gscale;
        if (c.loss) c.loss[b] = fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)));
      }
    }
  }
}

// One launch per pipelined step (sharded.py pipe_step): blocks
// [0, owner_blocks) are the owner side of batch t (KIND 4, 16 pairs each),
// then route_blocks of batch t+1's field route, then combine_blocks of batch
// t-1's combine — three independent parts, so a step is ONE kernel + ONE
// all-to-all.  Any part may be empty.
struct PipeArgs {
  int owner_blocks, route_blocks, combine_blocks;
  RouteArgs r;
  CombineArgs c;
  // two-deep peer step (rs_shard_fm_pipe_peer, XCHG): the exchange of the
  // NEXT batch's records (x.chunks x x.world workgroups, first in dispatch
  // order) rides in this launch beside the pipe parts of this batch
  int xchg_blocks;
  PeerArgs x;
};

template <int KV, int NT, int NW, int MC, bool XCHG = false, int FC = 0, int KFMC = 0>
__global__ __launch_bounds__(NW * 64) void shard_fm_pipe(EmbedFmArgs a, PipeArgs p) {
  // the short route / combine blocks come first in dispatch order, the owner
  // blocks (the headline kernel's body) after them: dispatched last, the
  // owner tiles spread over the CUs the short blocks leave instead of
  // doubling up behind them.  XCHG: the exchange workgroups before all of
  // them (workgroup 0 publishes this rank's mailbox readiness at once; they
  // wait on peers, never on the other parts of this launch, and those never
  // wait, so the launch drains whatever the dispatch order)
  int bid = blockIdx.x;
  if constexpr (XCHG) {
    if (bid < p.xchg_blocks) {
      peer_a2a_part<false>(p.x, bid / p.x.world, bid % p.x.world);
      return;
    }
    bid -= p.xchg_blocks;
  }
  if (bid < p.route_blocks) {
    field_route_part<NW * 64>(p.r, bid, p.route_blocks);
  } else if (bid < p.route_blocks + p.combine_blocks) {
    fm_combine_part<NW * 64>(p.c, bid - p.route_blocks, p.combine_blocks);
  } else {
    // the headline kernel's schedule: B fragments of the first two passes and
    // both passes' ids issued before the first rows (PF)
    embed_fm_body<KV, NT, NW, 4, false, MC, true, false, FC, KFMC, (FC > 0 ? 0 : -1)>(
        a, nullptr, bid - p.route_blocks - p.combine_blocks);
  }
}

// Fused DeepFM forward: gather + FM + DNN tower + head, one launch.
template <int KV, int KIND>
__global__ __launch_bounds__(16 * 64) void deepfm_fused(EmbedFmArgs a, MlpArgs t) {
  embed_fm_body<KV, 1, 16, KIND, true, 1>(a, &t, blockIdx.x);
}
// ... with the field metadata by value (rs_deepfm_fwd_hm; see embed_fm_mfma_ka)
template <int KV, int KIND>
__global__ __launch_bounds__(16 * 64) void deepfm_fused_ka(EmbedFmArgs a, MlpArgs t, FieldMeta m) {
  embed_fm_body<KV, 1, 16, KIND, true, 1, false, true>(a, &t, blockIdx.x, &m);
}

// ---- Fused DeepFM with split wave roles (deepfm_ws; rs_deepfm_fwd_hm at the
// Criteo shape: k = 16, 26 fields, 1..16 dense features, a first hidden layer
// of 241..256 units).  The tower's first layer is the bulk of the MFMA work
// and only needs each field's 16 columns of the tile, so it need not wait for
// the whole gather: waves 0..7 LOAD — ids, then the rows in two bursts
// (fields 0..15, 16..25) into the LDS tile, the FM partial tiles on the way,
// the dense block — and count each burst in an LDS counter; waves 8..15
// COMPUTE layer 0 (two 16-column output tiles each, k-groups in arrival
// order: the dense group first, then the fields) with their weight ring
// streaming from the start and waiting only on the counters.  Their vector
// memory queue holds weights only, so no row load sits in front of a weight
// wait.  The FM partials of the loaders meet by the last-wave finish; layers
// 1.. run as mlp_tower_tile on all 16 waves.  Every spin is bounded.
constexpr int WS_NL = 8;

// A logic error must neither hang the kernel nor pass silently: a wait that
// gives up raises RS_FLAG_TIMEOUT in the launch's error flag (the host layer
// then raises RSError instead of returning the outputs) and the kernel runs
// on to its end, so every wave still reaches every barrier and the grid drains.
__device__ __forceinline__ void lds_wait_ge(int* p, int v, int* err) {
  for (int spins = 0; __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v; ++spins) {
    if (spins > (1 << 22)) {
      if ((threadIdx.x & 63) == 0) flag_error(err, RS_FLAG_TIMEOUT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ void lds_signal(int* p) {
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int KIND, int G, int GWA = 0, int GWB = 0>
__global__ __launch_bounds__(16 * 64) void deepfm_ws(EmbedFmArgs a, MlpArgs t, FieldMeta m) {
  typedef Ids<KIND> I;
  constexpr int NW = 16, F = G - 1, MF = (F + WS_NL - 1) / WS_NL;
  static_assert(F <= 32 && MF <= 4, "deepfm_ws: <= 32 fields");
  extern __shared__ float tsm[];
  __shared__ floatx4 lf_acc[WS_NL][64];
  __shared__ floatx4 lf_q[WS_NL][4];
  __shared__ float fmlog[16];
  __shared__ int cnt[4];  // dense k-steps written | loaders past burst 0 | past burst 1 | FM partials in
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  const int64_t bt = (int64_t)blockIdx.x * 16 + s;
  const bool valid = bt < a.batch;
  const int64_t b = valid ? bt : a.batch - 1;
  const int RS = t.rs;
  float* par = tsm + 32 * RS + NW * 256;
  floatx4 ring[MLP_R];
  {
    const MlpArgs& a = t;  // MLP_STAMP reads a.dbg (diagnostic hook)
    MLP_STAMP(0);
  }
  if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
  if (w < WS_NL) {
    // ================================ loader
    const int l = w;
    const float w0v = a.w0[0];
    const int dw = l - (WS_NL - a.DB);  // dense k-steps on the last DB loaders (fewest fields)
    const bool has_dense = dw >= 0;
    float dx = 0.f, drec = 0.f, dn = 0.f;
    if (has_dense) {
      const int e = 4 * dw + kk;
      dx = a.dense[b * a.dense_stride + (e < a.nd ? e : 0)];
      const float* rec = a.prep + (int64_t)dw * a.dense_rec;
      drec = rec[lane];
      dn = rec[64 + kk];
    }
    typename I::raw_t rid[MF];
    floatx4 bw[MF];
#pragma unroll
    for (int p = 0; p < MF; ++p) {
      const int c = l + WS_NL * p;
      bw[p] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (c < F) {
        rid[p] = I::load(a.ids, b * a.id_stride + c);
        if (s <= a.kfm) bw[p] = *reinterpret_cast<const floatx4*>(a.prep + a.field_base + (int64_t)c * a.field_rec + lane * 4);
      }
    }
    // burst 0's rows go out before the barrier (round 5: the bias-block copy
    // that used to sit here — two dependent L2 trips — moved to the compute
    // waves, which wait for the rows anyway)
    floatx4 xs0[2];
    bool ok0[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = l + WS_NL * q;
      ok0[q] = false;
      if (q < MF && c < F) {
        int64_t id;
        ok0[q] = I::decode(rid[q], m.voc[c], id);
        xs0[q] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + (m.off[c] + id) * 16) + kk);
      }
    }
    __syncthreads();  // the counters start at 0 (the compute waves pass the same barrier)
    floatx4 ac[4];  // four accumulation chains (MFMA tp into chain tp)
#pragma unroll
    for (int c = 0; c < 4; ++c) ac[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    float qn = 0.f;
    if (has_dense) {  // the dense group of the tile: dense columns + the zero padding up to 16
      const int e = 4 * dw + kk;
      const float x = e < a.nd ? dx : 0.f;
      ac[0] = mfma16x16x4(x, drec, ac[0]);
      qn = fmaf(x * x, dn, qn);
      tsm[s * RS + F * 16 + e] = x;
      lds_signal(&cnt[0]);
    }
    float nrm[MF][4];
#pragma unroll
    for (int p = 0; p < MF; ++p)
#pragma unroll
      for (int tp = 0; tp < 4; ++tp) nrm[p][tp] = row16_sum(s < a.kfm ? bw[p][tp] * bw[p][tp] : 0.f);
    bool bad = false;
#pragma unroll
    for (int burst = 0; burst < 2; ++burst) {
      floatx4 xs[2];
      bool ok[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int p = 2 * burst + q, c = l + WS_NL * p;
        if (burst == 0) {
          xs[q] = xs0[q];
          ok[q] = ok0[q];
          continue;
        }
        ok[q] = false;
        if (p < MF && c < F) {
          int64_t id;
          ok[q] = I::decode(rid[p], m.voc[c], id);
          xs[q] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + (m.off[c] + id) * 16) + kk);
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int p = 2 * burst + q, c = l + WS_NL * p;
        if (p < MF && c < F) {
          bad |= !ok[q];
          const floatx4 x = ok[q] ? xs[q] : floatx4{0.f, 0.f, 0.f, 0.f};
          *reinterpret_cast<floatx4*>(tsm + s * RS + c * 16 + 4 * kk) = x;
#pragma unroll
          for (int tp = 0; tp < 4; ++tp) {
            ac[tp] = mfma16x16x4(x[tp], bw[p][tp], ac[tp]);
            qn = fmaf(x[tp] * x[tp], nrm[p][tp], qn);
          }
        }
      }
#ifdef RS_DIAG_STAMPS
      if (!(burst == 1 && (a.ablate & 32)))  // diagnostic knob: burst 1 never signalled (the timeout test)
#endif
      lds_signal(&cnt[1 + burst]);
      {
        const MlpArgs& a = t;
        MLP_STAMP(2 + burst);  // diagnostic hook: this loader's burst in
      }
    }
    if (__any(bad && valid) && lane == 0) flag_error(a.err);
    // FM: last-wave finish over the loaders' partial tiles (wave order)
    floatx4 acc;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (ac[0][i] + ac[1][i]) + (ac[2][i] + ac[3][i]);
    lf_acc[l][lane] = acc;
    qn += __shfl_xor(qn, 16);
    qn += __shfl_xor(qn, 32);
    if (lane < 16) reinterpret_cast<float*>(&lf_q[l][0])[lane] = qn;
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&cnt[3], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old == WS_NL - 1) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ww = 0; ww < WS_NL; ++ww) {
        const floatx4 pv = lf_acc[ww][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += pv[i];
      }
      const floatx4 q4 = lf_q[s < WS_NL ? s : 0][kk];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float tt = s < a.kfm ? v[i] * v[i] : 0.f;
        if (s < WS_NL) tt -= q4[i];
        float ll = s == a.kfm ? v[i] : 0.f;
        tt = row16_sum(tt);
        ll = row16_sum(ll);
        const float fm = (ll + w0v) + 0.5f * tt;
        const int64_t bb = (int64_t)blockIdx.x * 16 + 4 * kk + i;
        if (s == 0) {
          fmlog[4 * kk + i] = fm;
          if (bb < a.batch && a.logit) a.logit[bb] = fm;
        }
      }
    }
  } else {
    // ================================ layer 0 compute
    const int c8 = w - WS_NL;
    const floatx4* W0 = reinterpret_cast<const floatx4*>(t.prep + t.off[0]) + lane + (int64_t)c8 * G * 64;
    const floatx4* W1 = W0 + (int64_t)WS_NL * G * 64;  // output tile c8 + 8
    // k-group order: the dense group (G - 1) first, then fields 0 .. F-1
    auto grp = [](int i) { return i == 0 ? G - 1 : i - 1; };
    floatx4 r0[3], r1[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      r0[u] = W0[(int64_t)grp(u) * 64];
      r1[u] = W1[(int64_t)grp(u) * 64];
    }
    __syncthreads();  // the counters start at 0
    // the bias / alpha block -> LDS for the layers after the first (visible
    // at the tail's first barrier); this layer's epilogue reads its 4 values
    // per lane from global memory, so no hand-off among the compute waves
    for (int i = threadIdx.x - WS_NL * 64; i < t.ptot; i += (NW - WS_NL) * 64) par[i] = t.prep[t.wtot + i];
    const int ecol0 = 16 * c8 + s, ecol1 = ecol0 + 16 * WS_NL;
    const float* pb = t.prep + t.wtot + t.poff[0];
    const float eb0 = pb[ecol0], eb1 = pb[ecol1], ea0 = pb[t.Np[0] + ecol0], ea1 = pb[t.Np[0] + ecol1];
    const float* ap = tsm + s * RS + 4 * kk;
    // two output tiles, two chains each (MFMA j of a group into chain j & 1)
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc0b = acc0, acc1b = acc0;
    lds_wait_ge(&cnt[0], a.DB, a.err);
    // one k-group: MFMAs of ring slot U, then the slot refilled 3 groups ahead
    auto step = [&](int i, auto U) {
      constexpr int u = decltype(U)::value;
      const floatx4 av = *reinterpret_cast<const floatx4*>(ap + 16 * grp(i));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        acc0 = mfma16x16x4(av[j], r0[u][j], acc0);
        acc1 = mfma16x16x4(av[j], r1[u][j], acc1);
        acc0b = mfma16x16x4(av[j + 1], r0[u][j + 1], acc0b);
        acc1b = mfma16x16x4(av[j + 1], r1[u][j + 1], acc1b);
      }
      const int nx = i + 3 < G ? i + 3 : G - 1;
      r0[u] = W0[(int64_t)grp(nx) * 64];
      r1[u] = W1[(int64_t)grp(nx) * 64];
      __builtin_amdgcn_sched_barrier(0);
    };
    using U0 = std::integral_constant<int, 0>;
    using U1 = std::integral_constant<int, 1>;
    using U2 = std::integral_constant<int, 2>;
    auto wait_burst = [&](int which) {
      lds_wait_ge(&cnt[1 + which], WS_NL, a.err);  // fields 0..15 / 16.. in the tile
      const MlpArgs& a = t;
      MLP_STAMP(2 + which);  // diagnostic hook: burst seen
    };
    constexpr int B1 = 1 + 2 * WS_NL;  // first group of the second burst
    if (t.unroll) {
      // straight-line (RS_OPT_MLP_UNROLL 1)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        if (i == 1) wait_burst(0);
        if (i == B1) wait_burst(1);
        if (i % 3 == 0) step(i, U0{});
        else if (i % 3 == 1) step(i, U1{});
        else step(i, U2{});
      }
    } else {
      // compact loops (three groups a trip, ring slots fixed per position):
      // straight-line code of this length runs at instruction-fetch speed
      // (every 64-B line a miss, the cache is cold each launch: DESIGN 10)
      static_assert((B1 - 2) % 3 == 0 && (G - 1 - B1) % 3 == 0, "deepfm_ws: group / ring phase");
      step(0, U0{});
      wait_burst(0);
      int i = 1;
#pragma unroll 1
      for (; i + 2 < B1; i += 3) {
        step(i, U1{});
        step(i + 1, U2{});
        step(i + 2, U0{});
      }
      step(i, U1{});  // i = B1 - 1
      wait_burst(1);
#pragma unroll 1
      for (i = B1; i + 2 < G; i += 3) {
        step(i, U2{});
        step(i + 1, U0{});
        step(i + 2, U1{});
      }
      step(i, U2{});  // i = G - 1
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc0[i] += acc0b[i];
      acc1[i] += acc1b[i];
    }
    float* out = tsm + 16 * RS;  // layer 0 -> buf1
    with_act(t.act[0], [&](auto A) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * kk + r;
        out[row * RS + ecol0] = mlp_act_c<decltype(A)::value>(acc0[r] + eb0, ea0);
        out[row * RS + ecol1] = mlp_act_c<decltype(A)::value>(acc1[r] + eb1, ea1);
      }
    });
  }
  {
    const MlpArgs& a = t;
    MLP_STAMP(1);  // loader: rows + FM done; compute wave: layer 0 done
  }
  if constexpr (GWA > 0) {
    // the split-K tail (mlp_tail_splitk) at the DeepFM widths: layer 1's whole slice of this wave
    if constexpr (GWA == 8 && GWB == 2) {
      mlp_tail_run<NW>(t, tsm, (int64_t)blockIdx.x * 16, fmlog);
    } else {
      floatx4 wr[GWA];
      mlp_tail_fetch<GWA>(t, 1, wr);
      mlp_tail_splitk<NW, GWA, GWB>(t, tsm, (int64_t)blockIdx.x * 16, wr, fmlog, 1);
    }
  } else {
    {  // layer 1's first weights (this wave's first item of it, if any)
      const int T1 = t.Np[1] >> 4, G1 = t.Kp[1] >> 4;
      const int S1 = mlp_slices(T1, G1, NW);
      if (w < T1 * S1) {
        const MlpItem it = mlp_item(w, T1, G1, S1);
        mlp_ring_fill(ring, reinterpret_cast<const floatx4*>(t.prep + t.off[1]) + lane + (int64_t)it.t * G1 * 64,
                      it.g0, it.g1);
      }
    }
    mlp_tower_tile<NW>(t, tsm, (int64_t)blockIdx.x * 16, ring, fmlog, 1);
  }
}

// ---- Fused DeepFM, every wave on layer 0 (deepfm_all; RS_OPT_DEEPFM_KERNEL 2
// / 3 = weight ring 3 / 4 k-groups deep) at the Criteo shape (k 16, 26 fields,
// 1..16 dense features, a 256-unit first layer).  deepfm_ws ran layer 0 on 8
// of the 16 waves (2 per SIMD, ~48 cycles per MFMA per SIMD) while the other
// 8 gathered; here all 16 waves both gather and compute, one 16-column output
// tile of layer 0 each (4 waves per SIMD share the matrix pipe), and nothing
// spins (two workgroup barriers publish the two row bursts):
//   * front end (the headline kernel's recipe): only the ids of the wave's
//     fields c0 = w, c1 = w + 16 (< 26) and the dense features of waves
//     12..15 go out before the first burst (row c0 of every wave); weights,
//     FM fragments and the bias block follow it;
//   * row c0 -> LDS tile + its FM partial (MFMA against the packed [v | w1]
//     image, q = sum x^2 |v|^2 on the VALU), the dense group written by waves
//     12..15 -> barrier A -> the second burst (row c1) requested, layer 0
//     over the dense group and fields 0..15 with row c1 stored under them ->
//     barrier B -> fields 16..25 (every load unconditional, every wait the
//     compiler's counted one).  Requesting c1 only after barrier A: barrier A
//     waits for 8.4 MB of row lines instead of 13.6 (7.5k vs 11.4k cycles);
//   * the 16 FM partial tiles meet in LDS (fixed wave order); every wave then
//     finishes one sample's FM logit; layers 1.. run as the split-K tail
//     (mlp_tail_splitk) at the DeepFM widths, else as mlp_tower_tile.
// Reference: model/deepFM.py:23-31, layer/interaction.py:40-46 (DNN),
// :106-114 (FM), layer/core.py:273-280 (lookup).
template <int KIND, int G, int RD, int GWA = 0, int GWB = 0>
__global__ __launch_bounds__(16 * 64) void deepfm_all(EmbedFmArgs a, MlpArgs t, FieldMeta m) {
  typedef Ids<KIND> I;
  constexpr int NW = 16, F = G - 1;
  static_assert(F > 16 && F <= 32, "deepfm_all: 17..32 fields (two per wave at most)");
  static_assert(RD == 3 || RD == 4, "deepfm_all: weight ring 3 or 4 k-groups deep");
  extern __shared__ float tsm[];
  __shared__ floatx4 fm_acc[NW][64];  // FM partial tile of each wave
  __shared__ float fm_q[NW][16];      // sum_i x_i^2 |v_i|^2 partial of each wave, per sample
  __shared__ float fmlog[16];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int s = lane & 15, kk = lane >> 4;
  const int64_t bt = (int64_t)blockIdx.x * 16 + s;
  const bool valid = bt < a.batch;
  const int64_t b = valid ? bt : a.batch - 1;  // padded lanes recompute the last sample
  const int RS = t.rs;
  float* par = tsm + 32 * RS + NW * 256;
  {
    const MlpArgs& a = t;
    MLP_STAMP(0);
  }
  // ---- front end: ids (+ the dense features of waves 12..15), then row c0
  const int c0 = w, c1 = w + 16 < F ? w + 16 : w;  // (waves past F-16: c1 re-reads c0, unused)
  const bool two = w + 16 < F;                     // wave-uniform
  const typename I::raw_t rid0 = I::load(a.ids, b * a.id_stride + c0);
  const typename I::raw_t rid1 = I::load(a.ids, b * a.id_stride + c1);
  const int dw = w - (NW - 4);                  // FM dense k-step of waves 12..15 (they also write the dense group)
  const bool has_dense = dw >= 0 && dw < a.DB;  // wave-uniform
  const int dwc = dw < 0 ? 0 : (dw < a.DB ? dw : 0);
  const int de = 4 * dwc + kk;
  const float dxv = a.dense[b * a.dense_stride + (de < a.nd ? de : 0)];
  int64_t id0, id1;
  const bool ok0 = I::decode(rid0, m.voc[c0], id0);
  const bool ok1 = I::decode(rid1, m.voc[c1], id1);
  const floatx4 x0 = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + (m.off[c0] + id0) * 16) + kk);
  const floatx4* x1p = reinterpret_cast<const floatx4*>(a.table + (m.off[c1] + id1) * 16) + kk;
  // ---- behind the first burst: layer-0 weights of output tile w (k-groups in
  // the order dense (G-1), 0, 1, ..), the FM fragments, the bias / alpha block
  const floatx4* W0 = reinterpret_cast<const floatx4*>(t.prep + t.off[0]) + lane + (int64_t)w * G * 64;
  auto grp = [](int i) { return i == 0 ? G - 1 : i - 1; };
  floatx4 ring[RD];
#pragma unroll
  for (int u = 0; u < RD; ++u) ring[u] = W0[(int64_t)grp(u) * 64];
  const float* drec = a.prep + (int64_t)dwc * a.dense_rec;
  const float drv = drec[lane], dnv = drec[64 + kk];
  const floatx4 bw0 = *reinterpret_cast<const floatx4*>(a.prep + a.field_base + (int64_t)c0 * a.field_rec + lane * 4);
  const floatx4 bw1 = *reinterpret_cast<const floatx4*>(a.prep + a.field_base + (int64_t)c1 * a.field_rec + lane * 4);
  const float w0v = a.w0[0];
  const int npar = t.ptot;
  const int pi = threadIdx.x < npar ? threadIdx.x : 0;
  const float pv = t.prep[t.wtot + pi];
  bool bad = !ok0 || (two && !ok1);
  // ---- layer 0, four chains (MFMA j of a k-group into chain j), ring slot i % RD
  MacAcc<4> L0;
  const float* ap = tsm + s * RS + 4 * kk;
  // A fragments one k-group ahead inside a segment (the LDS latency hides
  // behind the previous group's MFMAs); a segment's first read is issued
  // after its barrier (seg_start)
  floatx4 an = {0.f, 0.f, 0.f, 0.f};
  auto seg_start = [&](int i) { an = *reinterpret_cast<const floatx4*>(ap + 16 * grp(i)); };
  auto step = [&](int i, auto U) {
    constexpr int u = decltype(U)::value;
    const floatx4 av = an;
    if (i != 16 && i + 1 < G) an = *reinterpret_cast<const floatx4*>(ap + 16 * grp(i + 1));  // 16: last before barrier B
    __builtin_amdgcn_sched_barrier(0);
    L0.mac4(av, ring[u]);
    if (i + RD < G) ring[u] = W0[(int64_t)grp(i + RD) * 64];
    __builtin_amdgcn_sched_barrier(0);
  };
  auto step_i = [&](int i) {
    switch (i % RD) {
      case 0: step(i, std::integral_constant<int, 0>{}); break;
      case 1: step(i, std::integral_constant<int, 1>{}); break;
      case 2: step(i, std::integral_constant<int, 2>{}); break;
      default: step(i, std::integral_constant<int, (RD > 3 ? 3 : 0)>{}); break;
    }
  };
  // ---- FM partials: the dense k-step, then each field as its row lands
  floatx4 fa = {0.f, 0.f, 0.f, 0.f};
  float qn = 0.f;
  if (dw >= 0) {
    // the tile's dense group (columns F*16 .. F*16+15, zero past nd), and the FM's dense k-step
    const int e = 4 * dw + kk;
    const float x = e < a.nd ? dxv : 0.f;
    tsm[s * RS + F * 16 + e] = x;
    if (has_dense) {
      fa = mfma16x16x4(x, drv, fa);
      qn = fmaf(x * x, dnv, qn);
    }
  }
  float n0[4], n1[4];
#pragma unroll
  for (int tp = 0; tp < 4; ++tp) {
    n0[tp] = row16_sum(s < a.kfm ? bw0[tp] * bw0[tp] : 0.f);
    n1[tp] = row16_sum(s < a.kfm ? bw1[tp] * bw1[tp] : 0.f);
  }
  if (threadIdx.x < npar) par[pi] = pv;
  auto put_row = [&](int c, const floatx4& xr, bool ok, const floatx4& bw, const float (&nr)[4]) {
    const floatx4 x = ok ? xr : floatx4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<floatx4*>(tsm + s * RS + c * 16 + 4 * kk) = x;
#pragma unroll
    for (int tp = 0; tp < 4; ++tp) {
      fa = mfma16x16x4(x[tp], bw[tp], fa);
      qn = fmaf(x[tp] * x[tp], nr[tp], qn);
    }
  };
  put_row(c0, x0, ok0, bw0, n0);
  __syncthreads();  // A: fields 0..15 (one per wave), the dense group, the bias / alpha block in LDS
  {
    const MlpArgs& a = t;
    MLP_STAMP(2);
  }
  // the second burst (unconditional: waves past F-16 re-read their first row)
  const floatx4 x1 = __builtin_nontemporal_load(x1p);
  __builtin_amdgcn_sched_barrier(0);
  // the dense group and fields 0..15: k-groups 0..16; row c1 lands under the first nine
  seg_start(0);
#pragma unroll
  for (int i = 0; i <= 16; ++i) {
    step_i(i);
    if (i == 8) {
      if (two) put_row(c1, x1, ok1, bw1, n1);
      // the wave's FM partial tile (its fields + dense k-step) for the combine
      fm_acc[w][lane] = fa;
      qn += __shfl_xor(qn, 16);
      qn += __shfl_xor(qn, 32);
      if (lane < 16) fm_q[w][lane] = qn;
      if (__any(bad && valid) && lane == 0) flag_error(a.err);
    }
  }
  __syncthreads();  // B: fields 16..F-1 in the tile, the FM partials in LDS
  {
    const MlpArgs& a = t;
    MLP_STAMP(3);
  }
  // FM logit of sample w (wave = sample, lane = column < 16): its 16 wave
  // partials added in wave order — the reads go out before the last layer-0
  // groups and are summed after them; wave index ww doubles as the q column.
  float fmv[NW];
  {
    const int ln = (w >> 2) * 16 + s, r = w & 3;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) fmv[ww] = fm_acc[ww][ln][r];
  }
  const float fq = fm_q[s][w];
  seg_start(17);
#pragma unroll
  for (int i = 17; i < G; ++i) step_i(i);
  const floatx4 acc0 = L0.sum();
  // layer 1's weights: the split-K tail's whole slice, or the ring's first groups
  constexpr bool TAIL = GWA > 0;
  floatx4 wr[TAIL ? GWA : 1];
  floatx4 tring[MLP_R];
  if constexpr (TAIL) {
    mlp_tail_fetch<GWA>(t, 1, wr);
  } else {
    const int T1 = t.Np[1] >> 4, G1 = t.Kp[1] >> 4;
    const int S1 = mlp_slices(T1, G1, NW);
    if (w < T1 * S1) {
      const MlpItem it = mlp_item(w, T1, G1, S1);
      mlp_ring_fill(tring, reinterpret_cast<const floatx4*>(t.prep + t.off[1]) + lane + (int64_t)it.t * G1 * 64,
                    it.g0, it.g1);
    }
  }
  {
    float* out = tsm + 16 * RS;  // layer 0 -> buf1
    const int col = 16 * w + s;
    const float bc = par[t.poff[0] + col], ac = par[t.poff[0] + t.Np[0] + col];  // registers before the stores
    with_act(t.act[0], [&](auto A) {
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(4 * kk + r) * RS + col] = mlp_act_c<decltype(A)::value>(acc0[r] + bc, ac);
    });
  }
  {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += fmv[ww];
    float tq = (s < a.kfm ? v * v : 0.f) - fq;
    float lin = s == a.kfm ? v : 0.f;
    tq = row16_sum(tq);
    lin = row16_sum(lin);
    const float fm = (lin + w0v) + 0.5f * tq;
    if (lane == 0) {
      fmlog[w] = fm;
      const int64_t bb = (int64_t)blockIdx.x * 16 + w;
      if (bb < a.batch && a.logit) a.logit[bb] = fm;
    }
  }
  {
    const MlpArgs& a = t;
    MLP_STAMP(1);
  }
  if constexpr (TAIL) {
    if constexpr (GWA == 8 && GWB == 2) mlp_tail_dispatch<NW>(t, tsm, (int64_t)blockIdx.x * 16, wr, fmlog, 1);
    else mlp_tail_splitk<NW, GWA, GWB>(t, tsm, (int64_t)blockIdx.x * 16, wr, fmlog, 1);
  }
  else mlp_tower_tile<NW>(t, tsm, (int64_t)blockIdx.x * 16, tring, fmlog, 1);
}

// Generic fallback (any k / kfm): one 256-thread workgroup per sample.
__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

template <int KIND>
__global__ __launch_bounds__(256) void embed_fm_generic(EmbedFmArgs a) {
  typedef Ids<KIND == 3 ? 0 : KIND> I;
  __shared__ int64_t rows[1024];
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const int d = a.nd + a.F * a.k;
  const float* w1 = a.prep;
  const float* v = a.prep + d;
  const float* nsq = a.prep + (int64_t)d * (a.kfm + 1);
  for (int c = threadIdx.x; c < a.F; c += blockDim.x) {
    int64_t row = b * a.F + c;
    if constexpr (KIND != 3) {
      int64_t id;
      if (I::decode(I::load(a.ids, b * a.id_stride + c), a.vocab[c], id)) row = a.offs[c] + id;
      else { row = -1; flag_error(a.err); }
    }
    rows[c] = row;
  }
  __syncthreads();
  auto xval = [&](int e) -> float {
    if (e < a.nd) return a.dense[b * a.dense_stride + e];
    const int c = (e - a.nd) / a.k, j = (e - a.nd) % a.k;
    const int64_t r = rows[c];
    return r >= 0 ? a.table[r * a.k + j] : 0.f;
  };
  float lin = 0.f, q = 0.f;
  for (int e = threadIdx.x; e < d; e += blockDim.x) {
    const float x = xval(e);
    lin = fmaf(x, w1[e], lin);
    q = fmaf(x * x, nsq[e], q);
    if (a.x_out) a.x_out[b * d + e] = x;
  }
  lin = block_sum(lin, red);
  q = block_sum(q, red);
  float ss = 0.f;
  for (int f = 0; f < a.kfm; ++f) {
    float p = 0.f;
    for (int e = threadIdx.x; e < d; e += blockDim.x) p = fmaf(xval(e), v[(int64_t)e * a.kfm + f], p);
    p = block_sum(p, red);
    ss = fmaf(p, p, ss);
  }
  if (threadIdx.x == 0) a.logit[b] = (lin + a.w0[0]) + 0.5f * (ss - q);
}

// -------------------------------------------------------------- gather
struct GatherArgs {
  const void* ids;
  int64_t id_stride;
  const float* dense;
  int64_t dense_stride;
  int nd;
  const float* table;
  const int64_t* offs;
  const int64_t* vocab;
  int F, k;
  float* out;
  int64_t out_stride;
  int64_t batch;
  int* err;
  int vec_store;
};

// Thread t handles chunk q of field c of sample b (VW floats); consecutive
// threads walk a row then the next field, so 4 threads read one 64-B row.
template <int VW, int KIND>
__global__ __launch_bounds__(256) void embed_gather_kernel(GatherArgs a) {
  typedef Ids<KIND> I;
  const uint32_t KQ = a.k / VW;
  const uint32_t per_row = (uint32_t)a.F * KQ;
  const uint32_t total = (uint32_t)a.batch * per_row;
  bool bad = false;
  for (uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const uint32_t bb = idx / per_row, r = idx - bb * per_row;
    const uint32_t c = r / KQ, q = r - c * KQ;
    const int64_t b = bb;
    int64_t id;
    const bool ok = I::decode(I::load(a.ids, b * a.id_stride + c), a.vocab[c], id);
    bad |= !ok;
    Chunk<VW> x;
    x.load(a.table + (a.offs[c] + id) * a.k + q * VW);
    float* dst = a.out + b * a.out_stride + a.nd + c * a.k + q * VW;
    if constexpr (VW == 4) {
      if (a.vec_store) {
        *reinterpret_cast<floatx4*>(dst) =
            ok ? floatx4{x.v[0], x.v[1], x.v[2], x.v[3]} : floatx4{0.f, 0.f, 0.f, 0.f};
        continue;
      }
    }
#pragma unroll
    for (int t = 0; t < VW; ++t) dst[t] = ok ? x.v[t] : 0.f;
  }
  if (bad) flag_error(a.err);
  if (a.nd > 0) {
    const uint32_t tot = (uint32_t)a.batch * a.nd;
    for (uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += gridDim.x * blockDim.x) {
      const uint32_t bb = idx / a.nd, e = idx - bb * a.nd;
      a.out[(int64_t)bb * a.out_stride + e] = a.dense[(int64_t)bb * a.dense_stride + e];
    }
  }
}

// ------------------------------------------------------ FM one-hot gather
struct OnehotArgs {
  const void* ids;
  int64_t id_stride;
  const float* dense;
  int64_t dense_stride;
  int nd;
  const int64_t* offs;
  const int64_t* vocab;
  int F;
  const float* w1;
  const float* w0;
  const float* v;
  int kfm;
  float* logit;
  int64_t batch;
  int* err;
};

// G lanes per sample (lane f owns latent factor f); 256/G samples per block.
template <int G, int KIND>
__global__ __launch_bounds__(256) void fm_onehot_kernel(OnehotArgs a) {
  typedef Ids<KIND> I;
  const int f = threadIdx.x % G;
  const int64_t bt = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  const bool valid = bt < a.batch;
  const int64_t b = valid ? bt : a.batch - 1;
  const int fc = f < a.kfm ? f : 0;
  float s = 0.f, q = 0.f, lin = 0.f;
  bool bad = false;
  for (int i = 0; i < a.nd; ++i) {
    const float x = a.dense[b * a.dense_stride + i];
    const float vf = f < a.kfm ? a.v[(int64_t)i * a.kfm + fc] : 0.f;
    s = fmaf(x, vf, s);
    q = fmaf(x * x, vf * vf, q);
    lin = fmaf(x, a.w1[i], lin);
  }
  for (int c = 0; c < a.F; ++c) {
    int64_t id;
    const bool ok = I::decode(I::load(a.ids, b * a.id_stride + c), a.vocab[c], id);
    bad |= !ok;
    const int64_t row = a.nd + a.offs[c] + id;
    const float vr = a.v[row * a.kfm + fc];
    const float wr = a.w1[row];
    const float vf = (ok && f < a.kfm) ? vr : 0.f;
    s += vf;
    q = fmaf(vf, vf, q);
    lin += ok ? wr : 0.f;
  }
  float term = (f < a.kfm) ? (s * s - q) : 0.f;
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) term += __shfl_xor(term, o, G);
  if (bad && valid && f == 0) flag_error(a.err);
  if (valid && f == 0) a.logit[b] = (lin + a.w0[0]) + 0.5f * term;
}

// ------------------------------------------------------- launch helpers
static int grid_for(int64_t work, int block, int cap = 2048) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <int KV, int NT, int KIND>
static void launch_embed_fm3(const EmbedFmArgs& a, hipStream_t st, const FieldMeta* hm) {
  // 16 waves per 16-sample tile (measured against 4, 8 and 13 waves), one
  // field slot per wave and pass: the headline's 26 fields take two passes
  // (16 + 10), 6.05 us per launch against 6.54 with both in one pass (2 slots
  // per wave) — the second pass's row requests queue behind a shorter first
  // wave of 256 rows per CU.  More than 32 fields: 2 slots per pass.
  const int grid = (int)((a.batch + 15) / 16);
  // several tiles per CU: prefetch the first passes' B fragments (PF) and
  // use fewer waves per tile, so more tiles share a CU (one field slot per
  // wave and pass): 8 waves up to 1024 tiles, 4 beyond (scripts/ab A/B,
  // graph slots: 13.0 -> 11.4 us at B 12288, 14.5 -> 13.5 at 16384, 27.0 ->
  // 22.9 at 32768, 50.7 -> 42.7 at 65536; profiles/r3_ab_nw*.json)
  // host field metadata given (rs_embed_fm_fwd_hm), up to 2 tiles per CU:
  // the kernarg-metadata kernel (6.92 -> 6.50 us at B 4096, 6.10 -> 5.78 at
  // 2048; profiles/r3_ab_kernarg_meta_{4096,2048}.json)
  // with the ids loaded per wave, the first passes' B fragments beside them
  // pay at 4096 too (6.61 -> 6.39 us, profiles/r3_ab_kernarg_pf_4096.json);
  // above 512 tiles the device-metadata kernels stay faster (14.26 vs 13.48
  // us at 16384, 47.5 vs 42.6 at 65536, still 14.34 vs 13.54 / 47.8 vs 42.6
  // with both passes' ids requested together; profiles/r3_ab_kernarg_*)
  // 16 waves (13: 6.20 us, 9: 6.78 vs 5.76 at 4096; profiles/r3_ab_kernarg_waves_4096.json)
  // (the kernarg kernel is built lean: at most 2 x 16 fields, 16 dense k-steps,
  // no x output — its straight-line code runs from a cold instruction cache)
  if (hm && a.F <= 32 && KIND != 3 && grid <= 512 && a.DB <= 16 && !a.x_out) {
    // (round 5: the ids through 16 scalar loads per wave and a lane select
    // chain, off the vector memory queue, ran 7.08 vs 6.12 us per launch,
    // bit-identical — profiles/r5_ab_scalar_ids.json; not kept)
    if constexpr (KV == 4 && NT == 1 && KIND != 2) {
      if (a.F == 26 && a.kfm == 10 && a.nd == 13) {  // the Criteo / headline shape
        embed_fm_mfma_ka<KV, NT, 16, KIND, true, 26, 10, 13><<<grid, 16 * 64, 0, st>>>(a, *hm);
        return;
      }
    }
    embed_fm_mfma_ka<KV, NT, 16, KIND, true><<<grid, 16 * 64, 0, st>>>(a, *hm);
    return;
  }
  if (a.F <= 32 && grid > 1024) embed_fm_mfma<KV, NT, 4, KIND, 1, true><<<grid, 4 * 64, 0, st>>>(a);
  else if (a.F <= 32 && grid > 512) embed_fm_mfma<KV, NT, 8, KIND, 1, true><<<grid, 8 * 64, 0, st>>>(a);
  else if (a.F <= 32) embed_fm_mfma<KV, NT, 16, KIND, 1><<<grid, 16 * 64, 0, st>>>(a);
  else embed_fm_mfma<KV, NT, 16, KIND, 0><<<grid, 16 * 64, 0, st>>>(a);
}

template <int KIND>
static void launch_embed_fm_k(const EmbedFmArgs& a, int KV, int NT, hipStream_t st,
                              const FieldMeta* hm = nullptr) {
  if (NT == 1) {
    switch (KV) {
      case 1: launch_embed_fm3<1, 1, KIND>(a, st, hm); break;
      case 2: launch_embed_fm3<2, 1, KIND>(a, st, hm); break;
      case 4: launch_embed_fm3<4, 1, KIND>(a, st, hm); break;
      case 8: launch_embed_fm3<8, 1, KIND>(a, st, hm); break;
      default: launch_embed_fm3<16, 1, KIND>(a, st, hm); break;
    }
  } else {
    switch (KV) {
      case 1: launch_embed_fm3<1, 2, KIND>(a, st, hm); break;
      case 2: launch_embed_fm3<2, 2, KIND>(a, st, hm); break;
      case 4: launch_embed_fm3<4, 2, KIND>(a, st, hm); break;
      case 8: launch_embed_fm3<8, 2, KIND>(a, st, hm); break;
      default: launch_embed_fm3<16, 2, KIND>(a, st, hm); break;
    }
  }
}

// kind: RS_ID_* or 3 (rows already gathered)
static int run_embed_fm(EmbedFmArgs a, const FmGeom& g, int kind, hipStream_t st, const char* what,
                        const FieldMeta* hm = nullptr) {
  if (a.batch == 0) return RS_OK;
  if (g.mfma) {
    a.DB = g.DB;
    a.dense_rec = g.dense_rec;
    a.field_rec = g.field_rec;
    a.field_base = g.field_base;
    if (a.F == 0) {
      // dense-only (FMLayer on x): no field loop runs, any instantiation works
      launch_embed_fm_k<3>(a, 4, g.NT, st);
    } else if (kind == 3) {
      launch_embed_fm_k<3>(a, g.KV, g.NT, st);
    } else if (launch_embed_fm_tiles(a, g, kind, opt(RS_OPT_EMBED_FM_KERNEL), st)) {
      // the persistent tile kernels (embed_fm_tiles.hip), when selected and the shape fits
    } else {
      with_id_kind(kind, [&](auto K) { launch_embed_fm_k<decltype(K)::value>(a, g.KV, g.NT, st, hm); });
    }
  } else {
    if (a.F > 1024) {
      set_error("%s: generic FM path supports at most 1024 fields", what);
      return RS_ERR_UNSUPPORTED;
    }
    if (kind == 3 || a.F == 0) embed_fm_generic<3><<<(unsigned)a.batch, 256, 0, st>>>(a);
    else with_id_kind(kind, [&](auto K) {
      embed_fm_generic<decltype(K)::value><<<(unsigned)a.batch, 256, 0, st>>>(a);
    });
  }
  return launch_status(what);
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_fm_prepared_size(int nd, int n_fields, int k, int kfm) {
  if (nd < 0 || n_fields < 0 || kfm < 1 || (n_fields > 0 && k < 1)) return -1;
  return fm_geom(nd, n_fields, k, kfm).size;
}

extern "C" int rs_fm_prepare(const float* w1, const float* v, int nd, int n_fields, int k, int kfm,
                             float* prepared, rs_stream_t stream) {
  RS_REQUIRE(w1 && v && prepared, "rs_fm_prepare: null pointer");
  RS_REQUIRE(nd >= 0 && n_fields >= 0 && kfm >= 1 && (n_fields == 0 || k >= 1), "rs_fm_prepare: bad shape");
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);
  RS_REQUIRE(g.d > 0, "rs_fm_prepare: empty feature vector");
  hipStream_t st = as_stream(stream);
  if (g.mfma) {
    fm_prepare_mfma<<<grid_for(g.size, 256), 256, 0, st>>>(w1, v, nd, n_fields, k, kfm, g.KV, g.NT, g.DB,
                                                           g.dense_rec, g.field_rec, g.field_base, g.size,
                                                           prepared);
  } else {
    fm_prepare_generic<<<grid_for(g.size, 256), 256, 0, st>>>(w1, v, g.d, kfm, prepared);
  }
  return launch_status("rs_fm_prepare");
}

extern "C" int rs_embed_fm_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                               int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                               const int64_t* field_vocab, int n_fields, int k, const float* prepared,
                               const float* w0, int kfm, float* logit, float* x_out, int64_t batch,
                               int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(batch >= 0 && nd >= 0 && n_fields >= 0 && kfm >= 1, "rs_embed_fm_fwd: bad shape");
  RS_REQUIRE(prepared && w0 && logit, "rs_embed_fm_fwd: null pointer");
  RS_REQUIRE(nd == 0 || dense, "rs_embed_fm_fwd: dense is null");
  RS_REQUIRE(n_fields == 0 || (ids && table && field_offsets && field_vocab && k >= 1),
             "rs_embed_fm_fwd: sparse inputs missing");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_fm_fwd: bad id_kind");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)table % 16 == 0, "rs_embed_fm_fwd: table must be 16-B aligned");
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);
  EmbedFmArgs a{};
  a.ids = ids;
  a.id_stride = id_stride;
  a.dense = dense;
  a.dense_stride = dense_stride;
  a.nd = nd;
  a.table = table;
  a.offs = field_offsets;
  a.vocab = field_vocab;
  a.F = n_fields;
  a.k = k;
  a.prep = prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = logit;
  a.x_out = x_out;
  a.batch = batch;
  a.err = err_flag;
  return run_embed_fm(a, g, id_kind, as_stream(stream), "rs_embed_fm_fwd");
}

extern "C" int rs_embed_fm_fwd_hm(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                  int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                                  const int64_t* field_vocab, const int64_t* field_offsets_host,
                                  const int64_t* field_vocab_host, int n_fields, int k, const float* prepared,
                                  const float* w0, int kfm, float* logit, float* x_out, int64_t batch,
                                  int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(field_offsets_host && field_vocab_host, "rs_embed_fm_fwd_hm: host metadata missing");
  const int variant = opt(RS_OPT_EMBED_FM_KERNEL);
  if (n_fields > 32 || (variant >= 1 && variant <= 3))
    return rs_embed_fm_fwd(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab,
                           n_fields, k, prepared, w0, kfm, logit, x_out, batch, err_flag, stream);
  RS_REQUIRE(batch >= 0 && nd >= 0 && n_fields >= 0 && kfm >= 1, "rs_embed_fm_fwd_hm: bad shape");
  RS_REQUIRE(prepared && w0 && logit, "rs_embed_fm_fwd_hm: null pointer");
  RS_REQUIRE(nd == 0 || dense, "rs_embed_fm_fwd_hm: dense is null");
  RS_REQUIRE(n_fields == 0 || (ids && table && field_offsets && field_vocab && k >= 1),
             "rs_embed_fm_fwd_hm: sparse inputs missing");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_fm_fwd_hm: bad id_kind");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)table % 16 == 0, "rs_embed_fm_fwd_hm: table must be 16-B aligned");
  FieldMeta m{};
  for (int c = 0; c < n_fields; ++c) {
    m.off[c] = field_offsets_host[c];
    m.voc[c] = field_vocab_host[c];
  }
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);
  EmbedFmArgs a{};
  a.ids = ids;
  a.id_stride = id_stride;
  a.dense = dense;
  a.dense_stride = dense_stride;
  a.nd = nd;
  a.table = table;
  a.offs = field_offsets;
  a.vocab = field_vocab;
  a.F = n_fields;
  a.k = k;
  a.prep = prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = logit;
  a.x_out = x_out;
  a.batch = batch;
  a.err = err_flag;
  return run_embed_fm(a, g, id_kind, as_stream(stream), "rs_embed_fm_fwd_hm", &m);
}

// S consecutive batch requests of `batch` samples each (the last one
// `last_batch`), batch s's ids at ids + s * ids_batch_stride elements, dense
// at dense + s * dense_batch_stride, logits at logit + s * logit_batch_stride:
// one launch, each batch's logits bit-identical to rs_embed_fm_fwd_hm's on
// that batch alone.  The kernarg-metadata kernel's shapes only (k 16 / 8 / 4,
// kfm <= 15, <= 32 fields, <= 16 dense k-steps, int32 / int64 ids, batch <=
// 8192, no x output); min_blocks: 1 or 2 resident workgroups per CU.
extern "C" int rs_embed_fm_fwd_hm_stream(const void* ids, int id_kind, int64_t id_stride, int64_t ids_batch_stride,
                                         const float* dense, int64_t dense_stride, int64_t dense_batch_stride,
                                         int nd, const float* table, const int64_t* field_offsets_host,
                                         const int64_t* field_vocab_host, int n_fields, int k,
                                         const float* prepared, const float* w0, int kfm, float* logit,
                                         int64_t logit_batch_stride, int64_t batch, int n_batches,
                                         int64_t last_batch, int min_blocks, int* err_flag, rs_stream_t stream) {
  if (n_batches == 0 || batch == 0) return RS_OK;
  RS_REQUIRE(n_batches > 0 && batch > 0 && last_batch > 0 && last_batch <= batch && batch <= 8192 && nd >= 0 &&
                 nd <= 64 && n_fields >= 1 && n_fields <= 32 && kfm >= 1 && kfm <= 15 &&
                 (k == 4 || k == 8 || k == 16) && (min_blocks == 1 || min_blocks == 2),
             "rs_embed_fm_fwd_hm_stream: unsupported shape");
  RS_REQUIRE(id_kind == RS_ID_I32 || id_kind == RS_ID_I64, "rs_embed_fm_fwd_hm_stream: int32 / int64 ids only");
  RS_REQUIRE(ids && table && prepared && w0 && logit && (nd == 0 || dense) && field_offsets_host &&
                 field_vocab_host,
             "rs_embed_fm_fwd_hm_stream: null pointer");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_embed_fm_fwd_hm_stream: table must be 16-B aligned");
  RS_REQUIRE(ids_batch_stride >= batch * id_stride && dense_batch_stride >= (nd ? batch * dense_stride : 0) &&
                 logit_batch_stride >= batch,
             "rs_embed_fm_fwd_hm_stream: batches overlap");
  const int64_t tpb = (batch + 15) / 16;
  RS_REQUIRE(tpb * n_batches < (1ll << 31), "rs_embed_fm_fwd_hm_stream: too many tiles");
  FieldMeta m{};
  for (int c = 0; c < n_fields; ++c) {
    m.off[c] = field_offsets_host[c];
    m.voc[c] = field_vocab_host[c];
  }
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);
  EmbedFmArgs a{};
  a.ids = ids;
  a.id_stride = id_stride;
  a.dense = dense;
  a.dense_stride = dense_stride;
  a.nd = nd;
  a.table = table;
  a.F = n_fields;
  a.k = k;
  a.prep = prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = logit;
  a.batch = batch;
  a.err = err_flag;
  a.DB = g.DB;
  a.dense_rec = g.dense_rec;
  a.field_rec = g.field_rec;
  a.field_base = g.field_base;
  StreamArgs sa{(int)tpb, n_batches, ids_batch_stride * (id_kind == RS_ID_I64 ? 8 : 4), dense_batch_stride,
                logit_batch_stride, last_batch};
  const unsigned grid = (unsigned)(tpb * n_batches);
  hipStream_t st = as_stream(stream);
  auto go = [&](auto kv, auto kind) {
    constexpr int KV = decltype(kv)::value, KIND = decltype(kind)::value;
    if constexpr (KV == 4) {
      if (n_fields == 26 && kfm == 10 && nd == 13) {  // the headline shape, as the single launch
        if (min_blocks == 2) embed_fm_stream_ka<KV, 1, KIND, 2, 26, 10, 13><<<grid, 16 * 64, 0, st>>>(a, m, sa);
        else embed_fm_stream_ka<KV, 1, KIND, 1, 26, 10, 13><<<grid, 16 * 64, 0, st>>>(a, m, sa);
        return;
      }
    }
    if (min_blocks == 2) embed_fm_stream_ka<KV, 1, KIND, 2><<<grid, 16 * 64, 0, st>>>(a, m, sa);
    else embed_fm_stream_ka<KV, 1, KIND, 1><<<grid, 16 * 64, 0, st>>>(a, m, sa);
  };
  auto by_kind = [&](auto kv) {
    if (id_kind == RS_ID_I64) go(kv, std::integral_constant<int, 1>());
    else go(kv, std::integral_constant<int, 0>());
  };
  if (k == 16) by_kind(std::integral_constant<int, 4>());
  else if (k == 8) by_kind(std::integral_constant<int, 2>());
  else by_kind(std::integral_constant<int, 1>());
  return launch_status("rs_embed_fm_fwd_hm_stream");
}

#ifdef RS_DIAG_STAMPS
// Ceiling probe: sum 64-B rows at given row indices (4 lanes per row, one
// float4 each) with different cache-policy bits on the row load.
template <int MODE>
__device__ __forceinline__ floatx4 probe_load(const float* p) {
  if constexpr (MODE == 0) {
    return *reinterpret_cast<const floatx4*>(p);
  } else if constexpr (MODE == 1) {
    return __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
  } else {
    floatx4 v;
    if constexpr (MODE == 2) asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (MODE == 3) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx4 %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
  }
}
template <int MODE>
__global__ __launch_bounds__(256) void diag_gather_sum(const float* __restrict__ table,
                                                      const int64_t* __restrict__ rows, int64_t n, float* out) {
  float acc = 0.f;
  // MODE 5: nontemporal with the MFMA A-operand lane layout of embed_fm_mfma
  // (lane l reads chunk l>>4 of row l&15: the 4 lanes of a row are 16 apart)
  const int lane = threadIdx.x & 63;
  const int q = MODE == 5 ? lane >> 4 : threadIdx.x & 3;
  const int64_t quad = MODE == 5 ? (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 16 + (lane & 15)
                                 : ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int64_t nquads = ((int64_t)gridDim.x * blockDim.x) >> 2;
  for (int64_t i = quad; i < n; i += nquads) {
    const floatx4 v = probe_load<MODE == 5 ? 1 : MODE>(table + rows[i] * 16 + 4 * q);
    acc += v[0] + v[1] + v[2] + v[3];
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;  // keep the loads live, never true
}
extern "C" int rs_diag_gather_sum(const float* table, const int64_t* rows, int64_t n, int grid, float* out,
                                  int mode, rs_stream_t stream) {
  hipStream_t st = as_stream(stream);
  switch (mode) {
    case 0: diag_gather_sum<0><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 1: diag_gather_sum<1><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 2: diag_gather_sum<2><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 3: diag_gather_sum<3><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 5: diag_gather_sum<5><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    default: diag_gather_sum<4><<<grid, 256, 0, st>>>(table, rows, n, out); break;
  }
  return launch_status("rs_diag_gather_sum");
}

// Cache-policy probe: U unrolled 16-B loads per lane in flight (4 lanes per
// 64-B row), issued by inline asm with the given policy bits and waited for
// together; POL 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc0 sc1 nt, 5 sc1 nt, 6 sc0,
// 7 sc0 nt.
#define RS_PROBE_ASM(bits) asm volatile("global_load_dwordx4 %0, %1, off " bits : "=v"(v[u]) : "v"(p[u]) : "memory")
template <int POL>
__global__ __launch_bounds__(256) void diag_policy_sum(const float* __restrict__ table, const int64_t* __restrict__ rows,
                                                       int64_t n, float* out) {
  constexpr int U = 4;
  float acc = 0.f;
  const int q = threadIdx.x & 3;
  const int64_t quad = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int64_t nquads = ((int64_t)gridDim.x * blockDim.x) >> 2;
  for (int64_t i0 = quad; i0 < n; i0 += U * nquads) {
    const float* p[U];
    floatx4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * nquads < n ? i0 + u * nquads : i0;
      p[u] = table + rows[i] * 16 + 4 * q;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (POL == 0) RS_PROBE_ASM("");
      else if constexpr (POL == 1) RS_PROBE_ASM("nt");
      else if constexpr (POL == 2) RS_PROBE_ASM("sc1");
      else if constexpr (POL == 3) RS_PROBE_ASM("sc0 sc1");
      else if constexpr (POL == 4) RS_PROBE_ASM("sc0 sc1 nt");
      else if constexpr (POL == 5) RS_PROBE_ASM("sc1 nt");
      else if constexpr (POL == 6) RS_PROBE_ASM("sc0");
      else RS_PROBE_ASM("sc0 nt");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u][0] + v[u][1] + v[u][2] + v[u][3];
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;  // keep the loads live, never true
}
extern "C" int rs_diag_policy_sum(const float* table, const int64_t* rows, int64_t n, int grid, float* out, int pol,
                                  rs_stream_t stream) {
  hipStream_t st = as_stream(stream);
  switch (pol) {
    case 0: diag_policy_sum<0><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 1: diag_policy_sum<1><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 2: diag_policy_sum<2><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 3: diag_policy_sum<3><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 4: diag_policy_sum<4><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 5: diag_policy_sum<5><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    case 6: diag_policy_sum<6><<<grid, 256, 0, st>>>(table, rows, n, out); break;
    default: diag_policy_sum<7><<<grid, 256, 0, st>>>(table, rows, n, out); break;
  }
  return launch_status("rs_diag_policy_sum");
}

extern "C" int rs_diag_embed_fm_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                    int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                                    const int64_t* field_vocab, int n_fields, int k, const float* prepared,
                                    const float* w0, int kfm, float* logit, int64_t batch,
                                    unsigned long long* dbg, rs_stream_t stream) {
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);
  EmbedFmArgs a{};
  a.ids = ids;
  a.id_stride = id_stride;
  a.dense = dense;
  a.dense_stride = dense_stride;
  a.nd = nd;
  a.table = table;
  a.offs = field_offsets;
  a.vocab = field_vocab;
  a.F = n_fields;
  a.k = k;
  a.prep = prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = logit;
  a.batch = batch;
  a.dbg = dbg;
  a.ablate = getenv("RS_ABLATE") ? atoi(getenv("RS_ABLATE")) : 0;
  if (getenv("RS_DIAG_HM") && n_fields <= 32) {  // the kernarg-metadata kernel (rs_embed_fm_fwd_hm)
    FieldMeta m{};
    (void)hipMemcpy(m.off, field_offsets, n_fields * sizeof(int64_t), hipMemcpyDeviceToHost);
    (void)hipMemcpy(m.voc, field_vocab, n_fields * sizeof(int64_t), hipMemcpyDeviceToHost);
    return run_embed_fm(a, g, id_kind, as_stream(stream), "rs_diag_embed_fm_fwd", &m);
  }
  return run_embed_fm(a, g, id_kind, as_stream(stream), "rs_diag_embed_fm_fwd");
}
#endif

// ------------------------------------------------ sharded FM, partial protocol
// Owner side: rs_shard_owner_fm runs embed_fm_body in KIND 4 on the local rows
// every requester asked of this owner (pairs = requester-major samples), over
// the owner's contiguous field range; requester side: rs_shard_fm_combine sums
// the world partial records of each sample in owner order, adds the dense
// block and finishes logit = (lin + w0) + 0.5 (sum_f S_f^2 - q)
// (layer/interaction.py:106-114 regrouped; same reassociation as the headline).
namespace rs {

template <int KV, int NT, int NW, int MC, bool XCHG = false>
static void launch_pipe4(const EmbedFmArgs& a, PipeArgs p, hipStream_t st) {
  const int T = NW * 64;
  p.owner_blocks = a.F > 0 ? (int)((a.batch + 15) / 16) : 0;
  if (p.route_blocks) p.route_blocks = (int)std::min<int64_t>((p.r.total + T - 1) / T, 4096);
  if (p.combine_blocks) p.combine_blocks = (int)std::min<int64_t>((p.c.batch * 16 + T - 1) / T, 4096);
  if (!XCHG) p.xchg_blocks = 0;
  const int grid = p.xchg_blocks + p.owner_blocks + p.route_blocks + p.combine_blocks;
  if (!grid) return;
  if constexpr (KV == 4 && NT == 1 && NW == 16 && MC == 1) {
    // the world-1 owner of the Criteo table (all 26 fields, kfm 10, no dense
    // block): field count and FM width as constants (as the headline kernel)
    if (a.F == 26 && a.kfm == 10 && a.nd == 0) {
      shard_fm_pipe<KV, NT, NW, MC, XCHG, 26, 10><<<grid, T, 0, st>>>(a, p);
      return;
    }
  }
  shard_fm_pipe<KV, NT, NW, MC, XCHG><<<grid, T, 0, st>>>(a, p);
}

// the two-deep peer step: 1-tile (kfm <= 15) owner part with <= 32 fields
template <int KV>
static void launch_pipe_xchg_kv(const EmbedFmArgs& a, const PipeArgs& p, hipStream_t st) {
  if (a.F <= 4) launch_pipe4<KV, 1, 4, 1, true>(a, p, st);
  else if (a.F <= 8) launch_pipe4<KV, 1, 8, 1, true>(a, p, st);
  else launch_pipe4<KV, 1, 16, 1, true>(a, p, st);
}
static void launch_pipe_xchg(const EmbedFmArgs& a, const PipeArgs& p, const FmGeom& g, hipStream_t st) {
  switch (g.KV) {
    case 1: launch_pipe_xchg_kv<1>(a, p, st); break;
    case 2: launch_pipe_xchg_kv<2>(a, p, st); break;
    case 4: launch_pipe_xchg_kv<4>(a, p, st); break;
    case 8: launch_pipe_xchg_kv<8>(a, p, st); break;
    default: launch_pipe_xchg_kv<16>(a, p, st); break;
  }
}

// NW / MC by the owner's field count: 4 waves x 1 slot for <= 4 fields (the
// 8-rank shape), 8 waves for <= 8 (4 ranks), 16 waves x 1 slot per pass up
// to 32 fields (as the headline kernel), 2 slots per pass beyond.
template <int KV>
static void launch_pipe_kv(const EmbedFmArgs& a, const PipeArgs& p, int NT, hipStream_t st) {
  if (NT == 1 && a.F <= 4) launch_pipe4<KV, 1, 4, 1>(a, p, st);
  else if (NT == 1 && a.F <= 8) launch_pipe4<KV, 1, 8, 1>(a, p, st);
  else if (NT == 1 && a.F <= 32) launch_pipe4<KV, 1, 16, 1>(a, p, st);
  else if (NT == 1) launch_pipe4<KV, 1, 16, 0>(a, p, st);
  else if (a.F <= 32) launch_pipe4<KV, 2, 16, 1>(a, p, st);
  else launch_pipe4<KV, 2, 16, 0>(a, p, st);
}

static void launch_pipe(const EmbedFmArgs& a0, const PipeArgs& p, const FmGeom& g, hipStream_t st) {
  EmbedFmArgs a = a0;
  switch (g.KV) {
    case 1: launch_pipe_kv<1>(a, p, g.NT, st); break;
    case 2: launch_pipe_kv<2>(a, p, g.NT, st); break;
    case 4: launch_pipe_kv<4>(a, p, g.NT, st); break;
    case 8: launch_pipe_kv<8>(a, p, g.NT, st); break;
    default: launch_pipe_kv<16>(a, p, g.NT, st); break;
  }
}

}  // namespace rs

extern "C" int rs_fm_partial_width(int kfm) { return kfm < 1 ? -1 : (kfm + 2 + 3) / 4 * 4; }

namespace rs {
// owner part (KIND 4) of a pipe launch over the received row-id records
static EmbedFmArgs owner_args(const FmGeom& g, const int32_t* local_rows, int64_t rec_stride, int field_lo,
                              int n_owned, const float* shard, int64_t shard_rows, int k, const float* prepared,
                              int kfm, float* partial, int64_t partial_stride, int64_t n_pairs, int* err_flag) {
  EmbedFmArgs a{};
  a.ids = local_rows;
  a.id_stride = rec_stride;
  a.nd = 0;
  a.table = shard;
  a.F = n_owned;
  a.k = k;
  a.prep = prepared + (int64_t)field_lo * g.field_rec;  // weights of the owner's first field
  a.kfm = kfm;
  a.logit = partial;
  a.batch = n_pairs;
  a.err = err_flag;
  a.DB = 0;  // dense block: added by the requester (combine part)
  a.dense_rec = g.dense_rec;
  a.field_rec = g.field_rec;
  a.field_base = g.field_base;
  a.owner_rows = shard_rows;
  a.pw = (kfm + 2 + 3) / 4 * 4;
  a.pstride = partial_stride;
  return a;
}
}  // namespace rs

#define RS_PIPE_GEOM(what)                                                                   \
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);                                            \
  if (!g.mfma) {                                                                             \
    set_error("%s: needs the packed FM image (k in {4,8,16,32,64}, kfm <= 31)", what);       \
    return RS_ERR_UNSUPPORTED;                                                               \
  }                                                                                          \
  const int pw = (kfm + 2 + 3) / 4 * 4;                                                      \
  (void)pw

extern "C" int rs_shard_owner_fm(const int32_t* local_rows, int64_t rec_stride, int field_lo, int n_owned,
                                 const float* shard, int64_t shard_rows, int nd, int n_fields, int k,
                                 const float* prepared, int kfm, float* partial, int64_t partial_stride,
                                 int64_t n_pairs, int* err_flag, rs_stream_t stream) {
  if (n_pairs == 0) return RS_OK;  // empty batch: nothing to launch
  RS_REQUIRE(n_pairs > 0 && kfm >= 1 && nd >= 0 && k >= 1 && field_lo >= 0 && n_owned >= 0 &&
                 field_lo + n_owned <= n_fields && n_owned <= rec_stride && shard_rows >= 0,
             "rs_shard_owner_fm: bad shape");
  RS_REQUIRE(prepared && partial && (n_owned == 0 || (local_rows && (shard || shard_rows == 0))),
             "rs_shard_owner_fm: null pointer");
  RS_REQUIRE((uintptr_t)shard % 16 == 0, "rs_shard_owner_fm: shard must be 16-B aligned");
  RS_PIPE_GEOM("rs_shard_owner_fm");
  RS_REQUIRE(partial_stride >= pw, "rs_shard_owner_fm: partial_stride < rs_fm_partial_width");
  hipStream_t st = as_stream(stream);
  if (n_owned == 0) {  // this owner holds no rows: every partial is zero
    (void)hipMemset2DAsync(partial, partial_stride * sizeof(float), 0, pw * sizeof(float), n_pairs, st);
    return launch_status("rs_shard_owner_fm");
  }
  PipeArgs p{};
  launch_pipe(owner_args(g, local_rows, rec_stride, field_lo, n_owned, shard, shard_rows, k, prepared, kfm, partial,
                         partial_stride, n_pairs, err_flag),
              p, g, st);
  return launch_status("rs_shard_owner_fm");
}

extern "C" int rs_shard_fm_combine(const float* partials, int64_t partial_stride, int world, int64_t batch,
                                   const float* dense, int64_t dense_stride, int nd, int n_fields, int k,
                                   const float* prepared, const float* w0, int kfm, float* logit,
                                   rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch
  RS_REQUIRE(batch > 0 && world >= 1 && nd >= 0 && n_fields >= 0 && kfm >= 1, "rs_shard_fm_combine: bad shape");
  RS_REQUIRE(partials && prepared && w0 && logit && (nd == 0 || dense), "rs_shard_fm_combine: null pointer");
  RS_PIPE_GEOM("rs_shard_fm_combine");
  RS_REQUIRE(partial_stride >= pw, "rs_shard_fm_combine: partial_stride < rs_fm_partial_width");
  EmbedFmArgs a{};  // no owner part
  PipeArgs p{};
  p.combine_blocks = 1;
  p.c = CombineArgs{partials, partial_stride, world, batch, dense, dense_stride, nd, prepared, g.dense_rec, g.NT,
                    w0, kfm, logit};
  launch_pipe(a, p, g, as_stream(stream));
  return launch_status("rs_shard_fm_combine");
}

extern "C" int rs_shard_fm_combine_grad(const float* partials, int64_t partial_stride, int world, int64_t batch,
                                        const float* dense, int64_t dense_stride, int nd, int n_fields, int k,
                                        const float* prepared, const float* w0, int kfm, const float* labels,
                                        float grad_scale, float* logit, float* gs, int64_t gs_stride, float* loss,
                                        rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(batch > 0 && world >= 1 && nd >= 0 && n_fields >= 0 && kfm >= 1 && gs_stride >= kfm + 1,
             "rs_shard_fm_combine_grad: bad shape");
  RS_REQUIRE(partials && prepared && w0 && logit && labels && gs && (nd == 0 || dense),
             "rs_shard_fm_combine_grad: null pointer");
  RS_PIPE_GEOM("rs_shard_fm_combine_grad");
  RS_REQUIRE(partial_stride >= pw, "rs_shard_fm_combine_grad: partial_stride < rs_fm_partial_width");
  EmbedFmArgs a{};
  PipeArgs p{};
  p.combine_blocks = 1;
  p.c = CombineArgs{partials, partial_stride, world, batch, dense, dense_stride, nd, prepared, g.dense_rec, g.NT,
                    w0, kfm, logit, labels, grad_scale, gs, gs_stride, loss};
  launch_pipe(a, p, g, as_stream(stream));
  return launch_status("rs_shard_fm_combine_grad");
}

extern "C" int rs_shard_fm_pipe(const int32_t* recv, int field_lo, int n_owned, const float* shard,
                                int64_t shard_rows, const float* dense_prev, int64_t dense_stride, float* logit_prev,
                                const void* ids_next, int id_kind, int64_t id_stride, const int64_t* field_offsets,
                                const int64_t* field_vocab, int64_t rows_per_rank, const int32_t* owner_fields,
                                int slot_stride, int32_t* send, int world, int64_t batch, int nd, int n_fields,
                                int k, const float* prepared, const float* w0, int kfm, int* err_flag,
                                rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch
  RS_REQUIRE(batch > 0 && world >= 1 && world <= 64 && nd >= 0 && n_fields >= 1 && k >= 1 && kfm >= 1 &&
                 slot_stride >= 1 && slot_stride <= n_fields && field_lo >= 0 && n_owned >= 0 &&
                 field_lo + n_owned <= n_fields && n_owned <= slot_stride && shard_rows >= 0 && rows_per_rank >= 1,
             "rs_shard_fm_pipe: bad shape");
  RS_REQUIRE(recv && send && prepared && w0 && (n_owned == 0 || shard || shard_rows == 0),
             "rs_shard_fm_pipe: null pointer");
  RS_REQUIRE(!ids_next || (field_offsets && field_vocab && owner_fields), "rs_shard_fm_pipe: route inputs missing");
  RS_REQUIRE(!logit_prev || nd == 0 || dense_prev, "rs_shard_fm_pipe: dense_prev is null");
  RS_REQUIRE((uintptr_t)shard % 16 == 0, "rs_shard_fm_pipe: shard must be 16-B aligned");
  RS_REQUIRE((int64_t)world * batch * (slot_stride + 32) < ((int64_t)1 << 31) && rows_per_rank < ((int64_t)1 << 31),
             "rs_shard_fm_pipe: too many slots / shard rows must fit int32");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_shard_fm_pipe: bad id_kind");
  RS_PIPE_GEOM("rs_shard_fm_pipe");
  const int64_t R = slot_stride + pw;  // words per fused record: [row ids | partial]
  hipStream_t st = as_stream(stream);
  const int64_t n_pairs = (int64_t)world * batch;
  float* pout = reinterpret_cast<float*>(send + slot_stride);
  const float* pin = reinterpret_cast<const float*>(recv + slot_stride);
  EmbedFmArgs a{};
  if (n_owned > 0) {
    a = owner_args(g, recv, R, field_lo, n_owned, shard, shard_rows, k, prepared, kfm, pout, R, n_pairs, err_flag);
  } else {  // no rows here: zero partials for every requester
    (void)hipMemset2DAsync(pout, R * sizeof(float), 0, pw * sizeof(float), n_pairs, st);
  }
  PipeArgs p{};
  if (ids_next) {
    p.route_blocks = 1;
    p.r = RouteArgs{ids_next, id_kind, id_stride, field_offsets, field_vocab, rows_per_rank, owner_fields,
                    slot_stride, (int)batch, R, send, err_flag, (int64_t)world * batch * slot_stride};
  }
  if (logit_prev) {
    p.combine_blocks = 1;
    p.c = CombineArgs{pin, R, world, batch, dense_prev, dense_stride, nd, prepared, g.dense_rec, g.NT, w0, kfm,
                      logit_prev};
  }
  launch_pipe(a, p, g, st);
  return launch_status("rs_shard_fm_pipe");
}

// The two-deep pipelined step with the peer exchange inside the launch:
// launch t = exchange of batch t+1's records [row ids of t+1 | partials of
// t-1] (send slot xslot -> every peer's mailbox slot xslot) | combine of t-2 |
// owner partials of t | route of t+2, the pipe parts reading this rank's
// mailbox slot (recv) and writing send slot t % 2 (send).  Host contract in
// sharded.py (ShardedEmbeddingFM.pipe2_step); protocol in peer.hip.
extern "C" int rs_shard_fm_pipe_peer(const int32_t* recv, int32_t* send, const int32_t* xsend, int xslot,
                                     int exchange, int field_lo, int n_owned, const float* shard, int64_t shard_rows,
                                     const float* dense_prev, int64_t dense_stride, float* logit_prev,
                                     const void* ids_next, int id_kind, int64_t id_stride,
                                     const int64_t* field_offsets, const int64_t* field_vocab, int64_t rows_per_rank,
                                     const int32_t* owner_fields, int slot_stride, int world, int64_t batch, int nd,
                                     int n_fields, int k, const float* prepared, const float* w0, int kfm,
                                     int* err_flag, void* const* mailboxes, int rank, void* peer_state, int chunks,
                                     int64_t spin_limit, int* xerr, rs_stream_t stream) {
  if (batch == 0) return RS_OK;
  RS_REQUIRE(batch > 0 && world >= 1 && world <= PEER_MAXW && rank >= 0 && rank < world && nd >= 0 &&
                 n_fields >= 1 && k >= 1 && kfm >= 1 && slot_stride >= 1 && slot_stride <= n_fields &&
                 field_lo >= 0 && n_owned >= 0 && field_lo + n_owned <= n_fields && n_owned <= slot_stride &&
                 shard_rows >= 0 && rows_per_rank >= 1 && (xslot == 0 || xslot == 1),
             "rs_shard_fm_pipe_peer: bad shape");
  RS_REQUIRE(recv && send && prepared && w0 && (n_owned == 0 || shard || shard_rows == 0),
             "rs_shard_fm_pipe_peer: null pointer");
  RS_REQUIRE(!exchange || (xsend && mailboxes && peer_state && xerr), "rs_shard_fm_pipe_peer: exchange inputs missing");
  RS_REQUIRE(!exchange || (chunks >= 1 && (int64_t)chunks * world <= 1024 && spin_limit >= 1),
             "rs_shard_fm_pipe_peer: bad chunks / limit");
  RS_REQUIRE(!ids_next || (field_offsets && field_vocab && owner_fields),
             "rs_shard_fm_pipe_peer: route inputs missing");
  RS_REQUIRE(!logit_prev || nd == 0 || dense_prev, "rs_shard_fm_pipe_peer: dense_prev is null");
  RS_REQUIRE((uintptr_t)shard % 16 == 0, "rs_shard_fm_pipe_peer: shard must be 16-B aligned");
  RS_REQUIRE((int64_t)world * batch * (slot_stride + 32) < ((int64_t)1 << 31) && rows_per_rank < ((int64_t)1 << 31),
             "rs_shard_fm_pipe_peer: too many slots / shard rows must fit int32");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_shard_fm_pipe_peer: bad id_kind");
  RS_PIPE_GEOM("rs_shard_fm_pipe_peer");
  if (g.NT != 1 || n_owned > 32) {
    set_error("rs_shard_fm_pipe_peer: needs kfm <= 15 and <= 32 owned fields");
    return RS_ERR_UNSUPPORTED;
  }
  const int64_t R = slot_stride + pw;
  hipStream_t st = as_stream(stream);
  const int64_t n_pairs = (int64_t)world * batch;
  float* pout = reinterpret_cast<float*>(send + slot_stride);
  const float* pin = reinterpret_cast<const float*>(recv + slot_stride);
  EmbedFmArgs a{};
  if (n_owned > 0) {
    a = owner_args(g, recv, R, field_lo, n_owned, shard, shard_rows, k, prepared, kfm, pout, R, n_pairs, err_flag);
  } else {
    (void)hipMemset2DAsync(pout, R * sizeof(float), 0, pw * sizeof(float), n_pairs, st);
  }
  PipeArgs p{};
  if (ids_next) {
    p.route_blocks = 1;
    p.r = RouteArgs{ids_next, id_kind, id_stride, field_offsets, field_vocab, rows_per_rank, owner_fields,
                    slot_stride, (int)batch, R, send, err_flag, (int64_t)world * batch * slot_stride};
  }
  if (logit_prev) {
    p.combine_blocks = 1;
    p.c = CombineArgs{pin, R, world, batch, dense_prev, dense_stride, nd, prepared, g.dense_rec, g.NT, w0, kfm,
                      logit_prev};
  }
  if (exchange) {
    const int64_t blk = batch * R * 4;  // bytes of one rank's records for one peer
    if (blk % 16) {
      set_error("rs_shard_fm_pipe_peer: batch * record bytes must be a multiple of 16");
      return RS_ERR_ARG;
    }
    p.xchg_blocks = chunks * world;
    p.x = PeerArgs{reinterpret_cast<const char*>(xsend), blk, reinterpret_cast<char* const*>(mailboxes),
                   (2 * (int64_t)world * blk + 255) / 256 * 256, static_cast<PeerState*>(peer_state), rank, world,
                   chunks, spin_limit, xerr, nullptr, 0, nullptr, 0, (int64_t)xslot * world * blk,
                   opt(RS_OPT_PEER_FENCES) == 0};
  }
  launch_pipe_xchg(a, p, g, st);
  return launch_status("rs_shard_fm_pipe_peer");
}

extern "C" int rs_rows_fm_fwd(const float* emb, const float* dense, int64_t dense_stride, int nd, int n_fields,
                              int k, const float* prepared, const float* w0, int kfm, float* logit, int64_t batch,
                              rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(batch >= 0 && nd >= 0 && n_fields >= 0 && kfm >= 1, "rs_rows_fm_fwd: bad shape");
  RS_REQUIRE(prepared && w0 && logit && (n_fields == 0 || emb) && (nd == 0 || dense),
             "rs_rows_fm_fwd: null pointer");
  RS_REQUIRE(k % 4 != 0 || (uintptr_t)emb % 16 == 0, "rs_rows_fm_fwd: emb must be 16-B aligned");
  const FmGeom g = fm_geom(nd, n_fields, k, kfm);
  EmbedFmArgs a{};
  a.dense = dense;
  a.dense_stride = dense_stride;
  a.nd = nd;
  a.table = emb;
  a.F = n_fields;
  a.k = k;
  a.prep = prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = logit;
  a.batch = batch;
  return run_embed_fm(a, g, 3, as_stream(stream), "rs_rows_fm_fwd");
}

extern "C" int rs_fm_fwd(const float* x, int64_t x_stride, int n, const float* prepared, const float* w0, int kfm,
                         float* logit, int64_t batch, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(x && prepared && w0 && logit, "rs_fm_fwd: null pointer");
  RS_REQUIRE(n >= 1 && kfm >= 1 && batch >= 0, "rs_fm_fwd: bad shape");
  const FmGeom g = fm_geom(n, 0, 0, kfm);
  EmbedFmArgs a{};
  a.dense = x;
  a.dense_stride = x_stride;
  a.nd = n;
  a.F = 0;
  a.k = 0;
  a.prep = prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = logit;
  a.batch = batch;
  return run_embed_fm(a, g, 3, as_stream(stream), "rs_fm_fwd");
}

extern "C" int rs_embed_gather(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                               int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                               const int64_t* field_vocab, int n_fields, int k, float* out, int64_t out_stride,
                               int64_t batch, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(batch >= 0 && nd >= 0 && n_fields >= 0, "rs_embed_gather: bad shape");
  RS_REQUIRE(out && (nd == 0 || dense), "rs_embed_gather: null pointer");
  RS_REQUIRE(n_fields == 0 || (ids && table && field_offsets && field_vocab && k >= 1),
             "rs_embed_gather: sparse inputs missing");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_embed_gather: bad id_kind");
  RS_REQUIRE(out_stride >= nd + (int64_t)n_fields * k, "rs_embed_gather: out_stride too small");
  RS_REQUIRE(batch * (int64_t)(n_fields * (int64_t)k + nd) < (int64_t)1 << 31,
             "rs_embed_gather: batch*row too large for one launch");
  if (batch == 0) return RS_OK;
  GatherArgs a{ids, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab,
               n_fields, k, out, out_stride, batch, err_flag, 0};
  hipStream_t st = as_stream(stream);
  const bool vec_src = (k % 4 == 0) && ((uintptr_t)table % 16 == 0);
  if (n_fields == 0) {
    a.F = 0;
    a.k = 4;
    embed_gather_kernel<4, 0><<<grid_for(batch * nd, 256, 8192), 256, 0, st>>>(a);
  } else if (vec_src) {
    a.vec_store = ((uintptr_t)out % 16 == 0) && (out_stride % 4 == 0) && (nd % 4 == 0);
    const int64_t work = batch * n_fields * (k / 4);
    with_id_kind(id_kind, [&](auto K) {
      embed_gather_kernel<4, decltype(K)::value>
          <<<grid_for(work > batch * nd ? work : batch * nd, 256, 8192), 256, 0, st>>>(a);
    });
  } else {
    const int64_t work = batch * n_fields * k;
    with_id_kind(id_kind, [&](auto K) {
      embed_gather_kernel<1, decltype(K)::value>
          <<<grid_for(work > batch * nd ? work : batch * nd, 256, 8192), 256, 0, st>>>(a);
    });
  }
  return launch_status("rs_embed_gather");
}

extern "C" int rs_fm_onehot_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                int64_t dense_stride, int nd, const int64_t* field_offsets,
                                const int64_t* field_vocab, int n_fields, const float* w1, const float* w0,
                                const float* v, int kfm, float* logit, int64_t batch, int* err_flag,
                                rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(batch >= 0 && nd >= 0 && n_fields >= 0 && kfm >= 1 && kfm <= 64, "rs_fm_onehot_fwd: bad shape");
  RS_REQUIRE(w1 && w0 && v && logit && (nd == 0 || dense), "rs_fm_onehot_fwd: null pointer");
  RS_REQUIRE(n_fields == 0 || (ids && field_offsets && field_vocab), "rs_fm_onehot_fwd: sparse inputs missing");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_fm_onehot_fwd: bad id_kind");
  if (batch == 0) return RS_OK;
  OnehotArgs a{ids, id_stride, dense, dense_stride, nd, field_offsets, field_vocab, n_fields,
               w1, w0, v, kfm, logit, batch, err_flag};
  hipStream_t st = as_stream(stream);
  int G = 4;
  while (G < kfm) G *= 2;
  const int spb = 256 / G;
  const unsigned grid = (unsigned)((batch + spb - 1) / spb);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KI = decltype(K)::value;
    switch (G) {
      case 4: fm_onehot_kernel<4, KI><<<grid, 256, 0, st>>>(a); break;
      case 8: fm_onehot_kernel<8, KI><<<grid, 256, 0, st>>>(a); break;
      case 16: fm_onehot_kernel<16, KI><<<grid, 256, 0, st>>>(a); break;
      case 32: fm_onehot_kernel<32, KI><<<grid, 256, 0, st>>>(a); break;
      default: fm_onehot_kernel<64, KI><<<grid, 256, 0, st>>>(a); break;
    }
  });
  return launch_status("rs_fm_onehot_fwd");
}

// ------------------------------------------------------- fused DeepFM forward
namespace rs {
static bool deepfm_geom(int nd, int n_fields, int k, int kfm, int n_layers, const int* dims, FmGeom& fg,
                        MlpGeom& mg) {
  if (nd < 0 || n_fields < 1 || n_fields > 128 || kfm < 1 || (k != 8 && k != 16)) return false;
  fg = fm_geom(nd, n_fields, k, kfm);
  if (!fg.mfma || fg.NT != 1) return false;
  if (!mlp_geom(n_layers, dims, mg)) return false;
  // static LDS of the embed part (<= 37 KB) + the tower's dynamic LDS
  return dims[0] == nd + n_fields * k && dims[n_layers] == 1 && mg.lds <= 120 * 1024;
}

// deepfm_ws covers: kernel-argument metadata, k = 16, 26 fields, 13..16 dense
// features (one k-group of dense + padding, written whole by the 4 dense
// loaders), a first hidden layer of 241..256
// units (16 output tiles: two per compute wave), >= 2 layers whose second has
// >= 8 output tiles (its items start on the loader waves)
static bool deepfm_ws_ok(const EmbedFmArgs& a, const MlpArgs& t, const FieldMeta* hm, int KV) {
  return hm && KV == 4 && a.F == 26 && a.nd >= 13 && a.nd <= 16 && a.DB == 4 && t.L >= 2 &&
         t.Np[0] == 256 && t.Kp[0] == 16 * (a.F + 1) && (t.Np[1] >> 4) >= WS_NL &&
         opt(RS_OPT_DEEPFM_KERNEL) == 0;
}

// deepfm_all covers the same shapes as deepfm_ws (every wave owns one of the
// 16 output tiles of the 256-unit first layer and at most two of the fields)
static bool deepfm_all_ok(const EmbedFmArgs& a, const MlpArgs& t, const FieldMeta* hm, int KV) {
  return hm && KV == 4 && a.F == 26 && a.nd >= 1 && a.nd <= 16 && a.DB <= 4 && t.L >= 2 && t.Np[0] == 256 &&
         t.Kp[0] == 16 * (a.F + 1) && t.ptot <= 1024 && opt(RS_OPT_DEEPFM_KERNEL) >= 2;
}

template <int KV, int KIND>
static void launch_deepfm(const EmbedFmArgs& a, const MlpArgs& t, size_t lds, hipStream_t st,
                          const FieldMeta* hm) {
  const unsigned grid = (unsigned)((a.batch + 15) / 16);
  if constexpr (KV == 4) {
    if (deepfm_all_ok(a, t, hm, KV)) {
      // the split-K tail at the DeepFM widths (256 -> 128 -> 64 -> 1: 8 + 2
      // k-groups per wave), the one-role tail for other towers
      int gwa = 0, gwb = 0;
      const bool tail = mlp_tail_ok(t.Np, t.Kp, t.N, t.L, 1, gwa, gwb) && gwa == 8 && gwb == 2;
      const bool ring4 = opt(RS_OPT_DEEPFM_KERNEL) == 3;
      static LdsAttr all_set[3];
      auto go = [&](const void* k, LdsAttr& set, auto launch) {
        lds_attr(set, k, lds);
        launch();
      };
      if (tail && ring4)
        go((const void*)deepfm_all<KIND, 27, 4, 8, 2>, all_set[0],
           [&] { deepfm_all<KIND, 27, 4, 8, 2><<<grid, 16 * 64, lds, st>>>(a, t, *hm); });
      else if (tail)
        go((const void*)deepfm_all<KIND, 27, 3, 8, 2>, all_set[1],
           [&] { deepfm_all<KIND, 27, 3, 8, 2><<<grid, 16 * 64, lds, st>>>(a, t, *hm); });
      else
        go((const void*)deepfm_all<KIND, 27, 3>, all_set[2],
           [&] { deepfm_all<KIND, 27, 3><<<grid, 16 * 64, lds, st>>>(a, t, *hm); });
      return;
    }
    if (deepfm_ws_ok(a, t, hm, KV)) {
      // layers 1.. as the split-K tail at the DeepFM widths (256 -> 128 -> 64 -> 1), else mlp_tower_tile
      int gwa = 0, gwb = 0;
      static LdsAttr ws_set[2];
      if (mlp_tail_ok(t.Np, t.Kp, t.N, t.L, 1, gwa, gwb) && gwa == 8 && gwb == 2) {
        lds_attr(ws_set[0], (const void*)deepfm_ws<KIND, 27, 8, 2>, lds);
        deepfm_ws<KIND, 27, 8, 2><<<grid, 16 * 64, lds, st>>>(a, t, *hm);
      } else {
        lds_attr(ws_set[1], (const void*)deepfm_ws<KIND, 27>, lds);
        deepfm_ws<KIND, 27><<<grid, 16 * 64, lds, st>>>(a, t, *hm);
      }
      return;
    }
  }
  static LdsAttr lds_set[2];  // opt in to exactly what is needed beyond the default
  // the kernarg body is built lean for at most 16 dense k-steps (nd <= 64):
  // its dense loop is compiled out (embed_fm_body: dense_small = KA || ...)
  const int ka = hm && a.F <= 32 && a.DB <= 16 ? 1 : 0;
  lds_attr(lds_set[ka], ka ? (const void*)deepfm_fused_ka<KV, KIND> : (const void*)deepfm_fused<KV, KIND>, lds);
  if (ka) deepfm_fused_ka<KV, KIND><<<grid, 16 * 64, lds, st>>>(a, t, *hm);
  else deepfm_fused<KV, KIND><<<grid, 16 * 64, lds, st>>>(a, t);
}
}  // namespace rs

extern "C" int rs_deepfm_fused_ok(int nd, int n_fields, int k, int kfm, int n_layers, const int* dims) {
  FmGeom fg;
  MlpGeom mg;
  return dims && deepfm_geom(nd, n_fields, k, kfm, n_layers, dims, fg, mg) ? 1 : 0;
}

static int deepfm_run(const void* ids, int id_kind, int64_t id_stride, const float* dense, int64_t dense_stride,
                      int nd, const float* table, const int64_t* field_offsets, const int64_t* field_vocab,
                      int n_fields, int k, const float* fm_prepared, const float* w0, int kfm, int n_layers,
                      const int* dims, const int* acts, const float* mlp_prepared, float c0, float c1, float* out,
                      float* fm_logit, int64_t batch, int* err_flag, rs_stream_t stream, const FieldMeta* hm) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  FmGeom fg;
  MlpGeom mg;
  RS_REQUIRE(dims && acts, "rs_deepfm_fwd: null dims/acts");
  RS_REQUIRE(deepfm_geom(nd, n_fields, k, kfm, n_layers, dims, fg, mg),
             "rs_deepfm_fwd: unsupported shape (see rs_deepfm_fused_ok)");
  RS_REQUIRE(batch >= 0 && ids && table && field_offsets && field_vocab && fm_prepared && w0 && mlp_prepared && out,
             "rs_deepfm_fwd: null pointer");
  RS_REQUIRE(nd == 0 || dense, "rs_deepfm_fwd: dense is null");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_deepfm_fwd: bad id_kind");
  RS_REQUIRE((uintptr_t)table % 16 == 0, "rs_deepfm_fwd: table must be 16-B aligned");
  MlpArgs t{};
  RS_REQUIRE(mlp_fill_args(mg, acts, mlp_prepared, t), "rs_deepfm_fwd: bad activation");
  if (batch == 0) return RS_OK;
  t.y = out;
  t.ys = 1;
  t.head = 1;
  t.c0 = c0;
  t.c1 = c1;
  t.M = batch;
  t.dbg = mlp_diag_dbg();
  EmbedFmArgs a{};
  a.ids = ids;
  a.id_stride = id_stride;
  a.dense = dense;
  a.dense_stride = dense_stride;
  a.nd = nd;
  a.table = table;
  a.offs = field_offsets;
  a.vocab = field_vocab;
  a.F = n_fields;
  a.k = k;
  a.prep = fm_prepared;
  a.w0 = w0;
  a.kfm = kfm;
  a.logit = fm_logit;
  a.batch = batch;
  a.err = err_flag;
  a.DB = fg.DB;
  a.dense_rec = fg.dense_rec;
  a.field_rec = fg.field_rec;
  a.field_base = fg.field_base;
#ifdef RS_DIAG_STAMPS
  a.ablate = getenv("RS_ABLATE") ? atoi(getenv("RS_ABLATE")) : 0;  // 32: deepfm_ws never signals burst 1
#endif
  hipStream_t st = as_stream(stream);
  with_id_kind(id_kind, [&](auto K) {
    constexpr int KIND = decltype(K)::value;
    if (fg.KV == 2) launch_deepfm<2, KIND>(a, t, mg.lds, st, hm);
    else launch_deepfm<4, KIND>(a, t, mg.lds, st, hm);
  });
  return launch_status("rs_deepfm_fwd");
}

extern "C" int rs_deepfm_fwd(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                             int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                             const int64_t* field_vocab, int n_fields, int k, const float* fm_prepared,
                             const float* w0, int kfm, int n_layers, const int* dims, const int* acts,
                             const float* mlp_prepared, float c0, float c1, float* out, float* fm_logit,
                             int64_t batch, int* err_flag, rs_stream_t stream) {
  return deepfm_run(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab, n_fields, k,
                    fm_prepared, w0, kfm, n_layers, dims, acts, mlp_prepared, c0, c1, out, fm_logit, batch, err_flag,
                    stream, nullptr);
}

extern "C" int rs_deepfm_fwd_hm(const void* ids, int id_kind, int64_t id_stride, const float* dense,
                                int64_t dense_stride, int nd, const float* table, const int64_t* field_offsets,
                                const int64_t* field_vocab, const int64_t* field_offsets_host,
                                const int64_t* field_vocab_host, int n_fields, int k, const float* fm_prepared,
                                const float* w0, int kfm, int n_layers, const int* dims, const int* acts,
                                const float* mlp_prepared, float c0, float c1, float* out, float* fm_logit,
                                int64_t batch, int* err_flag, rs_stream_t stream) {
  RS_REQUIRE(batch == 0 || (field_offsets_host && field_vocab_host), "rs_deepfm_fwd_hm: host metadata missing");
  FieldMeta m{};
  const bool use = n_fields <= 32 && batch > 0;
  for (int c = 0; use && c < n_fields; ++c) {
    m.off[c] = field_offsets_host[c];
    m.voc[c] = field_vocab_host[c];
  }
  return deepfm_run(ids, id_kind, id_stride, dense, dense_stride, nd, table, field_offsets, field_vocab, n_fields, k,
                    fm_prepared, w0, kfm, n_layers, dims, acts, mlp_prepared, c0, c1, out, fm_logit, batch, err_flag,
                    stream, use ? &m : nullptr);
}
