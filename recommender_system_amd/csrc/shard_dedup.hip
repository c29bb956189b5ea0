// shard_dedup.hip — row-id deduplication before the sharded row exchange
// ("id dedup before the all-to-all").
//
// ShardedDeepFM(dedup=...) sends each owner only the DISTINCT rows a rank
// needs from it instead of one word per (sample, owned field):
//   * every valid lookup j = b*F + c gets its global row
//     field_offsets[c] + id(b,c) as a sort key (bad ids: 0xffffffff, last);
//   * one stable radix sort of (row, j) groups the lookups by owner (owners
//     hold contiguous row blocks) and, inside an owner, by row;
//   * an inclusive scan of the segment heads numbers the distinct rows; the
//     distinct row u of owner o goes to word o*cap + u of the send buffer
//     (words past the owner's count stay -1: served as zero rows), and every
//     lookup of that row gets slot_of[j] = o*cap + u — the reply row it will
//     read after the row all-to-all (rs_deepfm_fwd with ids = slot_of, as
//     in the non-deduplicated protocol);
//   * u >= cap raises *overflow (the caller falls back, collectively, to the
//     field-range protocol) and that lookup's slot_of is -1.
// Backward: rs_shard_dedup_grad sums each distinct row's gradient rows over
// its lookups (stable sort order = lookup order: deterministic) into its
// send slot, so the reverse all-to-all carries one gradient row per distinct
// row and owner.
#include "radix_sort.hpp"
#include "rs_common.hpp"

namespace rs {

struct DedupWs {
  int64_t key_in, key_out, val_in, val_out, head, incl, ustart, strad, fmeta, sort, scan, total;
  size_t sort_bytes, scan_bytes;
};

// Fields per route on the per-field path (its cnt / base slab).
constexpr int DD_MAXF = 1024;

static int64_t dd_al(int64_t x) { return (x + 255) / 256 * 256; }

static DedupWs dedup_ws(int64_t n, int world) {
  DedupWs w{};
  const int64_t sb = sort_pairs_ws_bytes(n), cb = scan_ws_bytes(n);
  w.sort_bytes = (size_t)sb;
  w.scan_bytes = (size_t)cb;
  int64_t o = 0;
  w.key_in = o; o = dd_al(o + n * 4);
  w.key_out = o; o = dd_al(o + n * 4);
  w.val_in = o; o = dd_al(o + n * 4);
  w.val_out = o; o = dd_al(o + n * 4);
  w.head = o; o = dd_al(o + n * 4);
  w.incl = o; o = dd_al(o + n * 4);
  w.ustart = o; o = dd_al(o + ((int64_t)world + 1) * 4);
  w.strad = o; o = dd_al(o + ((int64_t)world + 1) * 4);
  w.fmeta = o; o = dd_al(o + DD_MAXF * 4);  // cnt
  w.sort = o; o = dd_al(o + (int64_t)sb);
  w.scan = o; o = dd_al(o + (int64_t)cb);
  w.total = o;
  return w;
}

template <int KIND>
__global__ __launch_bounds__(256) void dedup_keys(const void* ids, int64_t id_stride, const int64_t* __restrict__ offs,
                                                  const int64_t* __restrict__ vocab, int F, int64_t n,
                                                  uint32_t* __restrict__ key, int32_t* __restrict__ val, int* err) {
  typedef Ids<KIND> I;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int64_t b = j / F;
  const int c = (int)(j - b * F);
  int64_t id;
  const bool ok = I::decode(I::load(ids, b * id_stride + c), vocab[c], id);
  if (!ok) flag_error(err);
  key[j] = ok ? (uint32_t)(offs[c] + id) : 0xffffffffu;
  val[j] = (int32_t)j;
}

__global__ __launch_bounds__(256) void dedup_heads(const uint32_t* __restrict__ key, int64_t n,
                                                   int32_t* __restrict__ head) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const uint32_t r = key[p];
  head[p] = (r != 0xffffffffu && (p == 0 || key[p - 1] != r)) ? 1 : 0;
}

// ustart[o] = distinct rows of owners < o: incl at the last position before
// owner o's first row (binary search over the sorted keys)
__global__ void dedup_owner_start(const uint32_t* __restrict__ key, const int32_t* __restrict__ incl, int64_t n,
                                  int64_t rpr, int world, int32_t* __restrict__ ustart) {
  const int o = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (o >= world) return;
  const uint64_t lo_row = (uint64_t)o * (uint64_t)rpr;
  int64_t lo = 0, hi = n;  // first p with key[p] >= lo_row
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((uint64_t)key[mid] < lo_row) lo = mid + 1;
    else hi = mid;
  }
  ustart[o] = lo == 0 ? 0 : incl[lo - 1];
}

__device__ __forceinline__ int dd_owner(uint32_t r, int64_t rpr, int world) {
  const int64_t o = (int64_t)r / rpr;
  return (int)(o < world - 1 ? o : world - 1);
}

__global__ __launch_bounds__(256) void dedup_scatter(const uint32_t* __restrict__ key, const int32_t* __restrict__ val,
                                                     const int32_t* __restrict__ head,
                                                     const int32_t* __restrict__ incl,
                                                     const int32_t* __restrict__ ustart, int64_t n, int64_t rpr,
                                                     int world, int64_t cap, int32_t* __restrict__ send,
                                                     int32_t* __restrict__ slot_of, int* overflow) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const uint32_t r = key[p];
  const int32_t j = val[p];
  if (r == 0xffffffffu) {
    slot_of[j] = -1;
    return;
  }
  const int o = dd_owner(r, rpr, world);
  const int64_t u = (int64_t)incl[p] - 1 - ustart[o];
  if (u >= cap) {
    slot_of[j] = -1;
    if (head[p] && u == cap && overflow) __hip_atomic_store(overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  slot_of[j] = (int32_t)(o * cap + u);
  if (head[p]) send[o * cap + u] = (int32_t)((int64_t)r - (int64_t)o * rpr);
}

// one thread per (sorted position, column): each row's gradient summed over
// its segment (lookup order) into dst[slot of the segment head], in chunk
// pieces (seg_piece / seg_cross, rs_common.hpp) so a Zipf-hot row stays
// parallel; the pieces' partials reuse the route's head / scan slabs
__global__ __launch_bounds__(256) void dedup_grad_piece(const uint32_t* __restrict__ key,
                                                        const int32_t* __restrict__ val, int64_t n, int F, int k,
                                                        const float* __restrict__ grad, int64_t ldg,
                                                        const int32_t* __restrict__ slot_of, int64_t C,
                                                        float* __restrict__ part_first, float* __restrict__ part_last,
                                                        float* __restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t p = t / k;
  const int f = (int)(t - p * k);
  if (p >= n) return;
  uint32_t r;
  float s;
  if (!seg_piece(key, n, C, p, k, f, [&](int64_t q) {
        const int64_t j = val[q];
        const int64_t b = j / F;
        const int c = (int)(j - b * F);
        return grad[b * ldg + (int64_t)c * k + f];
      }, part_first, part_last, r, s))
    return;
  const int32_t slot = slot_of[val[p]];
  if (slot >= 0) dst[(int64_t)slot * k + f] = s;
}

__global__ __launch_bounds__(256) void dedup_grad_cross(const uint32_t* __restrict__ key,
                                                        const int32_t* __restrict__ val, int64_t n, int k,
                                                        const int32_t* __restrict__ slot_of, int64_t C,
                                                        const float* __restrict__ part_first,
                                                        const float* __restrict__ part_last, float* __restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t p = t / k;
  const int f = (int)(t - p * k);
  if (p >= n) return;
  uint32_t r;
  float s;
  if (!seg_cross(key, n, C, p, k, f, part_first, part_last, r, s)) return;
  const int32_t slot = slot_of[val[p]];
  if (slot >= 0) dst[(int64_t)slot * k + f] = s;
}

// ---- hand-written route (batch <= 4096, world <= 4096): one workgroup per
// field + one scatter launch, no sort.  Field c's rows are [off_c, off_c +
// vocab_c) and the concatenated table's offsets increase with c, so an
// owner's distinct rows, taken field by field, are contiguous per field;
// inside a field they are numbered in order of FIRST OCCURRENCE (lookup
// order), separately for each owner the field's rows fall into ("parts": a
// field straddling an owner boundary has two).
//   dedup_field_hash: the field's lookups go into an LDS hash table (linear
//     probing, 4 slots per lookup) that also keeps each row's first lookup
//     (atomic min); heads (first lookups) are numbered per part by ballot
//     prefix sums in lookup order -> fu, the row's index in the field's
//     owner-major distinct order, published through the table.  Outputs:
//     per lookup its global row and fu | head << 30 (field-major, coalesced);
//     cnt[c]; strad[o] = the field's distinct rows below owner o where o's
//     first row falls inside it.
//   dedup_scatter_f: every workgroup first rebuilds base[c] (distinct rows
//     of the fields before c) and ustart[o] (distinct rows below owner o) in
//     LDS from cnt / strad; then slot_of = o*cap + base[c] + fu - ustart[o]
//     (-1 past cap: *overflow), heads write send, words past each owner's
//     count = -1.
//   dedup_group_f (the backward's first launch, rs_shard_dedup_grad): the
//     lookups grouped by row — segments in fu order, lookup order inside,
//     bad ids last — as the sorted key / val the segment sums read.  Every
//     wave owns a contiguous block of lookups; 64 at a time it finds the
//     lanes with the same fu (ballots on its bits) and counts per wave and
//     fu, so a lookup's occurrence index = earlier waves' counts + its
//     wave's; segment starts = a scan of the rows' lookup counts.
// Deterministic: no result depends on the order of LDS atomics (the table
// slot of a row may, but only as a name).
// Phase stamps (s_memrealtime, 100 MHz) of thread 0 per workgroup into the
// workspace's incl slab, for a diagnostic build (-DRS_DH_STAMPS) only.
#ifdef RS_DH_STAMPS
#define DH_STAMP(i)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0)                                                                    \
      reinterpret_cast<uint64_t*>(stamps)[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define DH_STAMP(i) \
  do {              \
  } while (0)
#endif
constexpr int DH_KPL = 16;                // lookups per lane
constexpr int DH_MAXB = 64 * DH_KPL * 4;  // 4096: 4 waves
constexpr int DH_MAXW = 4096;             // owners (the scatter's LDS ustart)
constexpr uint32_t DH_EMPTY = 0xffffffffu;

__device__ __forceinline__ int dh_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// exclusive prefix of v over the workgroup (thread order) and its total;
// red: >= 16 ints of LDS; every thread calls it (two barriers)
__device__ __forceinline__ int dd_block_excl(int v, int* red, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) red[wv] = inc;
  __syncthreads();
  int wb = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    const int x = red[w];
    wb += w < wv ? x : 0;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return wb + inc - v;
}

// the hand-written path's domain (else: the device-wide radix sort)
inline bool dh_per_field(int64_t batch, int n_fields, int world) {
  return batch <= DH_MAXB && n_fields <= DD_MAXF && world <= DH_MAXW;
}
inline int dh_n2(int64_t batch) {
  int N2 = 1024;
  while (N2 < batch) N2 <<= 1;
  return N2;
}

// LW = log2(waves): N2 = 1024 << LW lookups at most, HS = 4 N2 slots;
// LDS: keys[HS] (later the slot's fu), first lookup[HS], 64 ints
template <int KIND, int LW>
__global__ __launch_bounds__(256) void dedup_field_hash(const void* ids, int64_t id_stride,
                                                        const int64_t* __restrict__ offs,
                                                        const int64_t* __restrict__ vocab, int F, int64_t B,
                                                        int64_t rpr, int world, uint32_t* __restrict__ rowg,
                                                        int32_t* __restrict__ fuh, int32_t* __restrict__ cnt,
                                                        int32_t* __restrict__ strad, int* err, void* stamps) {
  typedef Ids<KIND> I;
  extern __shared__ uint32_t sm[];
  DH_STAMP(0);
  constexpr int W = 1 << LW, T = 64 * W, N2 = 1024 << LW, HS = 4 * N2, LH = 12 + LW;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t* tk = sm;                             // [HS] keys; later the slot's fu
  int* first = reinterpret_cast<int*>(sm + HS);  // [HS] the row's first lookup
  int* red = reinterpret_cast<int*>(sm + 2 * HS);
  const int c = blockIdx.x;
  const int64_t off = offs[c], voc = vocab[c];
  // lookup b = (w DH_KPL + r) 64 + lane
  uint32_t row[DH_KPL];
  int hh[DH_KPL];
  bool bad = false;
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int b = (w * DH_KPL + r) * 64 + lane;
    row[r] = 0;
    hh[r] = HS;  // not a lookup / bad id
    if (b < B) {
      int64_t id;
      if (I::decode(I::load(ids, (int64_t)b * id_stride + c), voc, id)) {
        row[r] = (uint32_t)id;
        hh[r] = (int)((row[r] * 0x9E3779B1u) >> (32 - LH));
      } else {
        bad = true;
      }
    }
  }
  {
    uint4* t4 = reinterpret_cast<uint4*>(tk);
    for (int i = t; i < HS / 4; i += T) t4[i] = make_uint4(DH_EMPTY, DH_EMPTY, DH_EMPTY, DH_EMPTY);
    int4* f4 = reinterpret_cast<int4*>(first);
    for (int i = t; i < HS / 4; i += T) f4[i] = make_int4(INT_MAX, INT_MAX, INT_MAX, INT_MAX);
  }
  if (bad) flag_error(err);
  if (t == 0 && c + 1 < F && off + voc > offs[c + 1]) flag_error(err, RS_FLAG_LAYOUT);
  __syncthreads();
  DH_STAMP(1);
  // insert (linear probing, the table at most a quarter full): every
  // lookup's first probe at once, then the collisions; then the row's first
  // lookup by atomic min (order-free)
  uint32_t pend = 0;
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    if (hh[r] < HS) {
      const uint32_t prev = atomicCAS(&tk[hh[r]], DH_EMPTY, row[r]);
      if (prev != DH_EMPTY && prev != row[r]) pend |= 1u << r;
    }
  }
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    if (pend & (1u << r)) {
      uint32_t h = (uint32_t)hh[r];
      while (true) {
        h = (h + 1) & (uint32_t)(HS - 1);
        const uint32_t prev = atomicCAS(&tk[h], DH_EMPTY, row[r]);
        if (prev == DH_EMPTY || prev == row[r]) break;
      }
      hh[r] = (int)h;
    }
  }
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r)
    if (hh[r] < HS) atomicMin(&first[hh[r]], (w * DH_KPL + r) * 64 + lane);
  __syncthreads();
  DH_STAMP(2);
  // the owner part of each head (-1: not a head)
  const int o0 = dd_owner((uint32_t)off, rpr, world);
  const int S = dd_owner((uint32_t)(off + voc - 1), rpr, world) - o0 + 1;
  int part[DH_KPL];
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int b = (w * DH_KPL + r) * 64 + lane;
    const bool head = hh[r] < HS && first[hh[r]] == b;
    part[r] = !head ? -1 : (S == 1 ? 0 : dd_owner((uint32_t)(off + row[r]), rpr, world) - o0);
  }
  // heads numbered per part in lookup order: fu = the part's offset + rank
  int fu[DH_KPL];
  int pbase = 0;
  for (int p = 0; p < S; ++p) {
    int wrun = 0;
#pragma unroll
    for (int r = 0; r < DH_KPL; ++r) {
      const bool hp = part[r] == p;
      const uint64_t m = __builtin_amdgcn_ballot_w64(hp);
      if (hp) fu[r] = wrun + dh_below(m);
      wrun += __popcll(m);
    }
    if (lane == 0) red[w] = wrun;
    __syncthreads();
    int wo = 0, sum = 0;
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const int x = red[v];
      wo += v < w ? x : 0;
      sum += x;
    }
#pragma unroll
    for (int r = 0; r < DH_KPL; ++r)
      if (part[r] == p) fu[r] += pbase + wo;
    if (p > 0 && t == 0) strad[o0 + p] = pbase;
    pbase += sum;
    __syncthreads();
  }
  DH_STAMP(3);
  // heads publish their fu through the table (keys are no longer needed)
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r)
    if (part[r] >= 0) tk[hh[r]] = (uint32_t)fu[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int b = (w * DH_KPL + r) * 64 + lane;
    if (b < B) {
      const bool ok = hh[r] < HS;
      rowg[(int64_t)c * B + b] = ok ? (uint32_t)(off + row[r]) : DH_EMPTY;
      fuh[(int64_t)c * B + b] = ok ? (int)tk[hh[r]] | (part[r] >= 0 ? (1 << 30) : 0) : 0;
    }
  }
  if (t == 0) cnt[c] = pbase;
  DH_STAMP(4);
}

// the backward's grouping (see above); LW as in dedup_field_hash; LDS:
// [W][N2] per-wave counts (u16), then seg / grouped keys / grouped vals
// ([N2] each), 64 ints
__host__ __device__ inline int dg_words(int N2) {
  const int W = N2 / DH_KPL / 64;
  return (W * N2 / 2 > 3 * N2 ? W * N2 / 2 : 3 * N2) + 64;
}

template <int LW>
__global__ __launch_bounds__(256) void dedup_group_f(const uint32_t* __restrict__ rowg,
                                                     const int32_t* __restrict__ fuh, int F, int64_t B,
                                                     const int32_t* __restrict__ cnt,
                                                     uint32_t* __restrict__ key_out, int32_t* __restrict__ val_out) {
  extern __shared__ uint32_t sm[];
  constexpr int W = 1 << LW, N2 = 1024 << LW, LU = 10 + LW;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint16_t* cw = reinterpret_cast<uint16_t*>(sm);  // [W][N2]
  int* seg = reinterpret_cast<int*>(sm);           // later: [N2]
  uint32_t* gk = sm + N2;
  int* gv = reinterpret_cast<int*>(sm + 2 * N2);
  int* red = reinterpret_cast<int*>(sm + dg_words(N2) - 64);
  const int c = blockIdx.x;
  const int D = cnt[c];
  int uu[DH_KPL];  // the lookup's fu, N2 = not a lookup / bad id
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int b = (w * DH_KPL + r) * 64 + lane;
    uu[r] = N2;
    if (b < B && rowg[(int64_t)c * B + b] != DH_EMPTY) uu[r] = fuh[(int64_t)c * B + b] & ((1 << 30) - 1);
  }
  {
    uint4* c4 = reinterpret_cast<uint4*>(cw);
    for (int i = t; i < W * N2 / 8; i += 64 * W) c4[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  // lanes with the same fu, all batches at once
  uint32_t mlo[DH_KPL], mhi[DH_KPL];
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) mlo[r] = mhi[r] = ~0u;
#pragma unroll 1
  for (int i = 0; i <= LU; ++i) {  // fu bits + the sentinel's
#pragma unroll
    for (int r = 0; r < DH_KPL; ++r) {
      const uint32_t v = ((uint32_t)uu[r] >> i) & 1u;
      const uint64_t bl = __builtin_amdgcn_ballot_w64(v != 0);
      const uint32_t flip = v - 1u;  // 0 where the bit is set, ~0 where clear
      mlo[r] &= (uint32_t)bl ^ flip;
      mhi[r] &= (uint32_t)(bl >> 32) ^ flip;
    }
  }
  // occurrence index inside the wave (wave-private counters, lookup order)
  int occ[DH_KPL];
  uint16_t* mine = cw + w * N2;
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int u = uu[r];
    const int below = (int)__builtin_amdgcn_mbcnt_hi(mhi[r], __builtin_amdgcn_mbcnt_lo(mlo[r], 0u));
    const int prior = u < N2 ? (int)mine[u] : 0;
    occ[r] = u < N2 ? prior + below : 0;
    __builtin_amdgcn_wave_barrier();
    if (u < N2 && below == 0) mine[u] = (uint16_t)(prior + __popc(mlo[r]) + __popc(mhi[r]));
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // global occurrence index (+ earlier waves' counts) and the row's count
  int tot[DH_KPL];
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int u = uu[r];
    int before = 0, all = 0;
    if (u < N2) {
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const int x = cw[v * N2 + u];
        before += v < w ? x : 0;
        all += x;
      }
    }
    occ[r] += before;
    tot[r] = all;
  }
  // bad ids: ranked in lookup order after the valid lookups
  int pos[DH_KPL];
  {
    int wrun = 0;
#pragma unroll
    for (int r = 0; r < DH_KPL; ++r) {
      const int b = (w * DH_KPL + r) * 64 + lane;
      const bool isbad = b < B && uu[r] >= N2;
      const uint64_t m = __builtin_amdgcn_ballot_w64(isbad);
      pos[r] = wrun + dh_below(m);
      wrun += __popcll(m);
    }
    int nbad;
    const int wo = dd_block_excl(lane == 0 ? wrun : 0, red, nbad);  // barriers: cw reads are done
    const int wb = __shfl(wo, 0);
#pragma unroll
    for (int r = 0; r < DH_KPL; ++r) pos[r] += wb + (int)B - nbad;
  }
  // rows' counts by fu, then segment starts (16 consecutive entries a thread)
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r)
    if (uu[r] < N2 && occ[r] == 0) seg[uu[r]] = tot[r];
  __syncthreads();
  {
    int4* s4 = reinterpret_cast<int4*>(seg) + 4 * t;
    int v[DH_KPL];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 x = s4[q];
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
    int sum = 0;
#pragma unroll
    for (int e = 0; e < DH_KPL; ++e) {
      v[e] = DH_KPL * t + e < D ? v[e] : 0;
      sum += v[e];
    }
    int all;
    int acc = dd_block_excl(sum, red, all);
#pragma unroll
    for (int e = 0; e < DH_KPL; ++e) {
      const int x = v[e];
      v[e] = acc;
      acc += x;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) s4[q] = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r)
    if (uu[r] < N2) pos[r] = seg[uu[r]] + occ[r];
#pragma unroll
  for (int r = 0; r < DH_KPL; ++r) {
    const int b = (w * DH_KPL + r) * 64 + lane;
    if (b < B) {
      gk[pos[r]] = uu[r] < N2 ? rowg[(int64_t)c * B + b] : DH_EMPTY;
      gv[pos[r]] = b * F + c;
    }
  }
  __syncthreads();
  for (int i = t; i < B; i += 64 * W) {
    key_out[(int64_t)c * B + i] = gk[i];
    val_out[(int64_t)c * B + i] = gv[i];
  }
}

// every workgroup: base[c] and ustart[o] in LDS from cnt / strad, then one
// thread per lookup (field-major p = c*B + b: slot_of, head -> send word)
// and per send word q < world * cap (-1 past its owner's distinct count)
__global__ __launch_bounds__(256) void dedup_scatter_f(const uint32_t* __restrict__ rowg,
                                                       const int32_t* __restrict__ fuh,
                                                       const int32_t* __restrict__ cnt,
                                                       const int32_t* __restrict__ strad,
                                                       const int64_t* __restrict__ offs,
                                                       const int64_t* __restrict__ vocab, int F, int64_t B,
                                                       int64_t n, int64_t rpr, int world, int64_t cap,
                                                       int32_t* __restrict__ send, int32_t* __restrict__ slot_of,
                                                       int* overflow) {
  __shared__ int sb[DD_MAXF + 1];
  __shared__ int su[DH_MAXW + 1];
  __shared__ int64_t sf[DD_MAXF];
  __shared__ int red[16];
  const int t = threadIdx.x;
  const int chunk = (F + 255) / 256;
  int v[4] = {0, 0, 0, 0}, mine = 0;  // chunk <= 4 (F <= 1024)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int f = t * chunk + e;
    if (e < chunk && f < F) {
      v[e] = cnt[f];
      sf[f] = offs[f] + vocab[f];
      mine += v[e];
    }
  }
  int all;
  int acc = dd_block_excl(mine, red, all);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int f = t * chunk + e;
    if (e < chunk && f < F) {
      sb[f] = acc;
      acc += v[e];
    }
  }
  if (t == 0) {
    sb[F] = all;
    su[world] = all;
  }
  __syncthreads();
  for (int o = t; o < world; o += 256) {
    const uint64_t lo_row = (uint64_t)o * (uint64_t)rpr;
    int lo = 0, hi = F;  // first field whose rows end past lo_row
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((uint64_t)sf[mid] <= lo_row) lo = mid + 1;
      else hi = mid;
    }
    int u = sb[lo];
    if (lo < F && (uint64_t)offs[lo] < lo_row) u += strad[o];
    su[o] = u;
  }
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * 256 + t;
  if (p < (int64_t)world * cap) {
    const int o = (int)(p / cap);
    if (p - (int64_t)o * cap >= (int64_t)su[o + 1] - su[o]) send[p] = -1;
  }
  if (p >= n) return;
  const int c = (int)(p / B);
  const int64_t b = p - (int64_t)c * B, j = b * F + c;
  const uint32_t r = rowg[p];
  if (r == DH_EMPTY) {
    slot_of[j] = -1;
    return;
  }
  const int32_t fh = fuh[p];
  const bool head = (fh >> 30) & 1;
  const int o = dd_owner(r, rpr, world);
  const int64_t u = (int64_t)sb[c] + (fh & ((1 << 30) - 1)) - su[o];
  if (u >= cap) {
    slot_of[j] = -1;
    if (head && u == cap && overflow) __hip_atomic_store(overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  slot_of[j] = (int32_t)(o * cap + u);
  if (head) send[o * cap + u] = (int32_t)((int64_t)r - (int64_t)o * rpr);
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_shard_dedup_workspace_size(int64_t n_lookups, int world) {
  if (n_lookups < 0 || world < 1) return -1;
  return dedup_ws(n_lookups, world).total;
}

extern "C" int rs_shard_dedup_route(const void* ids, int id_kind, int64_t id_stride, const int64_t* field_offsets,
                                    const int64_t* field_vocab, int n_fields, int64_t batch, int64_t rows_per_rank,
                                    int world, int64_t cap, int32_t* send, int32_t* slot_of, void* workspace,
                                    int* err_flag, int* overflow_flag, rs_stream_t stream) {
  const int64_t n = batch * n_fields;
  RS_REQUIRE(world >= 1 && rows_per_rank >= 1 && cap >= 1 && batch >= 0 && n_fields >= 0,
             "rs_shard_dedup_route: bad shape");
  RS_REQUIRE(send && workspace, "rs_shard_dedup_route: null pointer");
  RS_REQUIRE((int64_t)world * rows_per_rank <= 0xfffffffell && n < (1ll << 31) && (int64_t)world * cap < (1ll << 31),
             "rs_shard_dedup_route: rows must fit uint32, lookups and slots int32");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_shard_dedup_route: bad id_kind");
  hipStream_t st = as_stream(stream);
  const bool per_field = dh_per_field(batch, n_fields, world);
  hipError_t e = hipSuccess;
  if (!per_field || n == 0) {
    // words past each owner's count ask for row -1 (a zero row)
    e = hipMemsetAsync(send, 0xff, (size_t)world * cap * 4, st);
    if (e != hipSuccess) {
      set_error("rs_shard_dedup_route: memset failed: %s", hipGetErrorString(e));
      return RS_ERR_HIP;
    }
  }
  if (n == 0) return RS_OK;
  RS_REQUIRE(ids && field_offsets && field_vocab && slot_of, "rs_shard_dedup_route: null pointer");
  const DedupWs w = dedup_ws(n, world);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  uint32_t* key_in = reinterpret_cast<uint32_t*>(ws + w.key_in);
  uint32_t* key_out = reinterpret_cast<uint32_t*>(ws + w.key_out);
  int32_t* val_in = reinterpret_cast<int32_t*>(ws + w.val_in);
  int32_t* val_out = reinterpret_cast<int32_t*>(ws + w.val_out);
  int32_t* head = reinterpret_cast<int32_t*>(ws + w.head);
  int32_t* incl = reinterpret_cast<int32_t*>(ws + w.incl);
  int32_t* ustart = reinterpret_cast<int32_t*>(ws + w.ustart);
  const unsigned g = (unsigned)((n + 255) / 256);
  if (per_field) {
    // hand-written path: one hash workgroup per field + one scatter, no sort
    int N2 = 1024;
    while (N2 < batch) N2 <<= 1;
    const int T = N2 / DH_KPL;
    const size_t lds = (size_t)(8 * N2 + 64) * 4;
    const int LW = N2 == 1024 ? 0 : (N2 == 2048 ? 1 : 2);
    int32_t* cnt = reinterpret_cast<int32_t*>(ws + w.fmeta);
    int32_t* strad = reinterpret_cast<int32_t*>(ws + w.strad);
    with_id_kind(id_kind, [&](auto K) {
      constexpr int KI = decltype(K)::value;
      auto go = [&](auto kern) {
        static LdsAttr lds_set[3][3];
        lds_attr(lds_set[KI][LW], (const void*)kern, lds);
        kern<<<n_fields, T, lds, st>>>(ids, id_stride, field_offsets, field_vocab, n_fields, batch, rows_per_rank,
                                       world, key_in, val_in, cnt, strad, err_flag, ws + w.incl);
      };
      if (LW == 0) go(dedup_field_hash<KI, 0>);
      else if (LW == 1) go(dedup_field_hash<KI, 1>);
      else go(dedup_field_hash<KI, 2>);
    });
    const int64_t work = n > (int64_t)world * cap ? n : (int64_t)world * cap;
    dedup_scatter_f<<<(unsigned)((work + 255) / 256), 256, 0, st>>>(key_in, val_in, cnt, strad, field_offsets,
                                                                    field_vocab, n_fields, batch, n, rows_per_rank,
                                                                    world, cap, send, slot_of, overflow_flag);
    return launch_status("rs_shard_dedup_route");
  }
  with_id_kind(id_kind, [&](auto K) {
    dedup_keys<decltype(K)::value><<<g, 256, 0, st>>>(ids, id_stride, field_offsets, field_vocab, n_fields, n,
                                                      key_in, val_in, err_flag);
  });
  // 2^bits > every valid row: a bad key (0xffffffff) still sorts last
  const uint64_t rows = (uint64_t)world * (uint64_t)rows_per_rank;
  int bits = 1;
  while (bits < 32 && ((uint64_t)1 << bits) <= rows) ++bits;
  e = sort_pairs_u32(key_in, reinterpret_cast<const uint32_t*>(val_in), key_out, reinterpret_cast<uint32_t*>(val_out),
                     n, bits, ws + w.sort, st);
  if (e == hipSuccess) {
    dedup_heads<<<g, 256, 0, st>>>(key_out, n, head);
    e = inclusive_sum_i32(head, incl, n, ws + w.scan, st);
  }
  if (e != hipSuccess) {
    set_error("rs_shard_dedup_route: sort/scan failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  dedup_owner_start<<<(world + 63) / 64, 64, 0, st>>>(key_out, incl, n, rows_per_rank, world, ustart);
  dedup_scatter<<<g, 256, 0, st>>>(key_out, val_out, head, incl, ustart, n, rows_per_rank, world, cap, send, slot_of,
                                   overflow_flag);
  return launch_status("rs_shard_dedup_route");
}

extern "C" int rs_shard_dedup_grad(const float* grad, int64_t grad_stride, int n_fields, int k, int64_t batch,
                                   int world, const int32_t* slot_of, void* workspace, float* dst,
                                   rs_stream_t stream) {
  const int64_t n = batch * n_fields;
  if (n == 0) return RS_OK;
  RS_REQUIRE(grad && slot_of && workspace && dst && k >= 1 && world >= 1 && grad_stride >= (int64_t)n_fields * k,
             "rs_shard_dedup_grad: bad arguments");
  const DedupWs w = dedup_ws(n, world);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  const uint32_t* key = reinterpret_cast<const uint32_t*>(ws + w.key_out);
  const int32_t* val = reinterpret_cast<const int32_t*>(ws + w.val_out);
  // piece partials (2 k floats per chunk, <= n floats when n > C) in the
  // route's head + scan slabs (2n floats), which the route no longer needs
  const int64_t C = seg_chunk(k);
  const int64_t nch = (n + C - 1) / C;
  float* part_first = reinterpret_cast<float*>(ws + w.head);
  float* part_last = part_first + nch * k;
  hipStream_t st = as_stream(stream);
  if (dh_per_field(batch, n_fields, world)) {
    // the hand-written route leaves no grouped order: build it
    const int N2 = dh_n2(batch), LW = N2 == 1024 ? 0 : (N2 == 2048 ? 1 : 2);
    const size_t lds = (size_t)dg_words(N2) * 4;
    const uint32_t* rowg = reinterpret_cast<const uint32_t*>(ws + w.key_in);
    const int32_t* fuh = reinterpret_cast<const int32_t*>(ws + w.val_in);
    const int32_t* cnt = reinterpret_cast<const int32_t*>(ws + w.fmeta);
    uint32_t* ko = reinterpret_cast<uint32_t*>(ws + w.key_out);
    int32_t* vo = reinterpret_cast<int32_t*>(ws + w.val_out);
    auto go = [&](auto kern) {
      static LdsAttr lds_set[3];
      lds_attr(lds_set[LW], (const void*)kern, lds);
      kern<<<n_fields, N2 / DH_KPL, lds, st>>>(rowg, fuh, n_fields, batch, cnt, ko, vo);
    };
    if (LW == 0) go(dedup_group_f<0>);
    else if (LW == 1) go(dedup_group_f<1>);
    else go(dedup_group_f<2>);
  }
  const unsigned g = (unsigned)((n * k + 255) / 256);
  dedup_grad_piece<<<g, 256, 0, st>>>(key, val, n, n_fields, k, grad, grad_stride, slot_of, C, part_first, part_last,
                                      dst);
  if (nch > 1) dedup_grad_cross<<<g, 256, 0, st>>>(key, val, n, k, slot_of, C, part_first, part_last, dst);
  return launch_status("rs_shard_dedup_grad");
}
