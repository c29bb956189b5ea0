// embed_fm.hpp — shared declarations of the fused gather + FM kernels
// (embed_fm.hip: MFMA K-split kernel, sharded owner / pipe parts, DeepFM;
// embed_fm_tiles.hip: the pipelined MFMA and VALU/DPP kernels of
// rs_embed_fm_fwd).  Reference: FMLayer.call, layer/interaction.py:106-114.
#pragma once
#include "rs_common.hpp"

namespace rs {

// ----------------------------------------------------------- packed layout
struct FmGeom {
  int nd, F, k, kfm, d;
  bool mfma;
  int KV, NT, DB;
  int64_t dense_rec, field_rec, field_base, size;
};

static inline FmGeom fm_geom(int nd, int F, int k, int kfm) {
  FmGeom g{};
  g.nd = nd;
  g.F = F;
  g.k = k;
  g.kfm = kfm;
  g.d = nd + F * k;
  const bool kv_ok = (F == 0) || (k % 4 == 0 && (k == 4 || k == 8 || k == 16 || k == 32 || k == 64));
  g.mfma = kv_ok && kfm >= 1 && kfm + 1 <= 32;
  if (g.mfma) {
    g.KV = (F == 0) ? 4 : k / 4;
    g.NT = (kfm + 1 + 15) / 16;
    g.DB = (nd + 3) / 4;
    g.dense_rec = (int64_t)g.NT * 64 + 4;
    g.field_rec = (int64_t)g.NT * 64 * g.KV + 4 * g.KV;
    g.field_base = (int64_t)g.DB * g.dense_rec;
    g.size = g.field_base + (int64_t)F * g.field_rec;
  } else {
    // generic path: [w1 (d) | v (d*kfm) | |v_i|^2 (d)]
    g.size = (int64_t)g.d * (kfm + 2);
  }
  return g;
}

// ----------------------------------------------------------- arguments
struct EmbedFmArgs {
  const void* ids;
  int64_t id_stride;
  const float* dense;
  int64_t dense_stride;
  int nd;
  const float* table;
  const int64_t* offs;
  const int64_t* vocab;
  int F;
  int k;
  const float* prep;
  const float* w0;
  int kfm;
  float* logit;
  float* x_out;
  int64_t batch;
  int* err;
  int DB;
  int64_t dense_rec, field_rec, field_base;
  int64_t owner_rows;       // KIND 4: rows of the owner's shard (ids are local rows, -1 = absent)
  int pw;                   // KIND 4: floats per partial record (logit -> partial records)
  int64_t pstride;          // KIND 4: floats between consecutive samples' partial records
  unsigned long long* dbg;  // diagnostic builds only (RS_DIAG_STAMPS): phase stamps
  int ablate;               // diagnostic builds only: bit0 no MFMA, bit1 no B loads, bit2 no combine
};

// Field metadata by value in the kernarg (diagnostic build -DRS_DIAG_KARG:
// the per-wave id path reads it through scalar loads, no LDS id tile)
struct FieldMeta {
  int64_t off[32];
  int64_t voc[32];
};

// Launches of embed_fm_tiles.hip (rs_embed_fm_fwd, id kinds 0..2): returns
// false when the shape / option has no kernel there (the caller then runs the
// K-split kernel of embed_fm.hip).
bool launch_embed_fm_tiles(const EmbedFmArgs& a, const FmGeom& g, int kind, int variant, hipStream_t st);

}  // namespace rs
