// shard.hip — row-sharded embedding lookup support.
//
// The reference has no distributed code; this is the MI355X-native exchange
// for one concatenated table split by row blocks across the ranks of a node:
//   global row of lookup i = b*F + c is field_offsets[c] + id(b,c)
//   owner = row / rows_per_rank,  local row = row - owner*rows_per_rank.
// rs_shard_bucketize produces, deterministically and without float atomics,
// the per-owner counts, the owner-major (stable) position of every lookup and
// the local row ids to send; RCCL all-to-all (host side) moves ids and rows;
// rs_gather_rows serves the owner's rows; rs_unpermute_rows puts the returned
// rows back in sample order for the FM kernel (rs_rows_fm_fwd).
#include "rs_common.hpp"
#include "shard_route.hpp"

namespace rs {

constexpr int SH_CHUNK = 256;  // lookups per workgroup (one per thread)
constexpr int SH_THREADS = 256;
constexpr int SH_MAXW = 64;

struct ShardArgs {
  const void* ids;
  int id_kind;
  int64_t id_stride;
  const int64_t* offs;
  const int64_t* vocab;
  int F;
  int64_t n;  // batch * F
  int64_t rpr;
  int world;
  int* err;
  double inv_rpr;
};

__device__ __forceinline__ int shard_owner(const ShardArgs& a, int64_t i, int64_t& local) {
  const int64_t b = (int64_t)((uint32_t)i / (uint32_t)a.F);  // n < 2^31
  const int c = (int)(i - b * a.F);
  const int64_t off = b * a.id_stride + c;
  int64_t id;
  bool ok;
  if (a.id_kind == RS_ID_F32) {
    const float f = static_cast<const float*>(a.ids)[off];
    ok = f > -1.0f && static_cast<double>(f) < static_cast<double>(a.vocab[c]);
    id = ok ? static_cast<int64_t>(f) : 0;
  } else {
    id = (a.id_kind == RS_ID_I64) ? static_cast<const int64_t*>(a.ids)[off]
                                  : static_cast<const int32_t*>(a.ids)[off];
    ok = id >= 0 && id < a.vocab[c];
  }
  if (!ok) {
    flag_error(a.err);
    local = -1;
    return 0;
  }
  const int64_t row = a.offs[c] + id;
  // owner = row / rpr without a 64-bit integer division: an fp64 quotient
  // (exact to < 1 for rows < 2^52) and a +-1 fix-up
  int o = (int)((double)row * a.inv_rpr);
  if ((int64_t)o * a.rpr > row) --o;
  else if ((int64_t)(o + 1) * a.rpr <= row) ++o;
  if (o >= a.world) o = a.world - 1;
  local = row - (int64_t)o * a.rpr;
  return o;
}

__global__ __launch_bounds__(SH_THREADS) void shard_hist(ShardArgs a, int32_t* hist) {
  __shared__ int h[SH_MAXW];
  for (int o = threadIdx.x; o < a.world; o += blockDim.x) h[o] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * SH_CHUNK;
  for (int r = threadIdx.x; r < SH_CHUNK; r += blockDim.x) {
    const int64_t i = base + r;
    if (i < a.n) {
      int64_t local;
      atomicAdd(&h[shard_owner(a, i, local)], 1);
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < a.world; o += blockDim.x) hist[(int64_t)blockIdx.x * a.world + o] = h[o];
}

// counts[o] = sum_b hist[b][o]; hist[b][o] <- base(o) + sum_{b'<b} hist[b'][o]
// base(o) = sum_{p<o} counts[p] (packed) or o * cap (slotted, cap > 0).
// One 256-thread workgroup: wave w owns owners w, w+4, ...; each owner's
// column is reduced / scanned 64 blocks at a time (independent loads, a
// wave-level inclusive scan, a running carry) — no serial per-block chain.
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(256) void shard_scan(int32_t* hist, int nblocks, int world, int32_t* counts, int cap) {
  __shared__ int tot[SH_MAXW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int o = w; o < world; o += 4) {
    int s = 0;
    for (int b = lane; b < nblocks; b += 64) s += hist[(int64_t)b * world + o];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d);
    if (lane == 0) {
      tot[o] = s;
      counts[o] = s;
    }
  }
  __syncthreads();
  for (int o = w; o < world; o += 4) {
    int carry = 0;
    if (cap > 0) carry = o * cap;
    else
      for (int p = 0; p < o; ++p) carry += tot[p];
    for (int b0 = 0; b0 < nblocks; b0 += 64) {
      const int b = b0 + lane;
      const int v = b < nblocks ? hist[(int64_t)b * world + o] : 0;
      const int inc = wave_incl_scan(v, lane);
      if (b < nblocks) hist[(int64_t)b * world + o] = carry + inc - v;
      carry += __shfl(inc, 63);
    }
  }
}

// cap > 0 (slotted): lookup i goes to slot o*cap + rank-within-owner; ranks
// >= cap (and out-of-range ids) get perm[i] = -1 and raise *overflow / *err.
__global__ __launch_bounds__(SH_THREADS) void shard_place(ShardArgs a, const int32_t* hist, int32_t* perm,
                                                          int32_t* send_rows, int cap, int* overflow) {
  __shared__ int running[SH_MAXW];
  __shared__ int wcnt[SH_THREADS / 64][SH_MAXW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int o = threadIdx.x; o < a.world; o += blockDim.x) running[o] = hist[(int64_t)blockIdx.x * a.world + o];
  const int64_t base = (int64_t)blockIdx.x * SH_CHUNK;
  for (int r0 = 0; r0 < SH_CHUNK; r0 += SH_THREADS) {
    for (int o = threadIdx.x; o < (SH_THREADS / 64) * SH_MAXW; o += blockDim.x) (&wcnt[0][0])[o] = 0;
    __syncthreads();
    const int64_t i = base + r0 + threadIdx.x;
    const bool act = i < a.n;
    int64_t local = -1;
    const int o = act ? shard_owner(a, i, local) : -1;
    // stable in-wave rank: peel one owner at a time
    int rank = 0;
    uint64_t todo = __ballot(act);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const int lo = __shfl(o, leader);
      const uint64_t m = __ballot(act && o == lo);
      if (act && o == lo) rank = __popcll(m & ((1ull << lane) - 1));
      if (lane == 0) wcnt[w][lo] = __popcll(m);
      todo &= ~m;
    }
    __syncthreads();
    if (act) {
      int pos = running[o] + rank;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][o];
      if (cap > 0 && (pos - o * cap >= cap || local < 0)) {
        if (local >= 0) flag_error(overflow);
        perm[i] = -1;
      } else {
        perm[i] = pos;
        send_rows[pos] = (int32_t)local;
      }
    }
    __syncthreads();
    for (int oo = threadIdx.x; oo < a.world; oo += blockDim.x) {
      int s = 0;
      for (int ww = 0; ww < SH_THREADS / 64; ++ww) s += wcnt[ww][oo];
      running[oo] += s;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- one pass
// Slotted bucketize in ONE launch (replaces hist -> scan -> place when cap > 0):
// a workgroup takes SP_PER consecutive lookups (one per thread per round),
// ranks them stably per owner in LDS (wave ballots), and gets the number of
// earlier lookups of every owner by a decoupled look-back over its
// predecessors' published per-owner totals (single-pass chained scan).  The
// result is identical to the three-kernel form: stable slot order.
//   status[b][o] (u64): [63:62] 1 = aggregate of block b, 2 = inclusive prefix
//   through block b; [61:32] launch epoch; [31:0] value.
//   ctrl (u64): [63:32] epoch, [31:0] block ticket.  Blocks take dynamic ids
//   (a block only ever waits on blocks that have already started); the block
//   that draws the launch's last ticket re-arms ctrl to (epoch + 1, 0) — every
//   ticket of this launch is drawn by then — so the next launch needs no
//   memset (graph-replay safe).  The ids of block blockIdx.x are loaded while
//   the ticket is in flight and kept when the ticket matches (in-order
//   dispatch, the common case).
constexpr int SP_THREADS = 1024;
constexpr int SP_PER = SP_THREADS;

__device__ __forceinline__ uint64_t sp_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sp_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(SP_THREADS) void shard_slot_onepass(ShardArgs a, uint64_t* status, uint64_t* ctrl,
                                                                 int nb, int32_t* counts, int32_t* slot_of,
                                                                 int32_t* send, int cap, int* overflow, int mode) {
  constexpr int NW = SP_THREADS / 64;
  __shared__ int wcnt[NW][SH_MAXW];
  __shared__ int excl[SH_MAXW];
  __shared__ uint64_t sh_tk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    if (mode & 1) {
      sh_tk = blockIdx.x;
    } else {
      // relaxed: an agent-scope release/acquire would write back / invalidate L2
      const uint64_t t = __hip_atomic_fetch_add(ctrl, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)t == (uint32_t)nb - 1)
        __hip_atomic_store(ctrl, ((t >> 32) + 1) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sh_tk = t;
    }
  }
  for (int i = threadIdx.x; i < NW * SH_MAXW; i += SP_THREADS) (&wcnt[0][0])[i] = 0;
  // speculative: this block's lookups as if the ticket equals blockIdx.x
  int64_t i = (int64_t)blockIdx.x * SP_PER + threadIdx.x;
  int64_t loc = -1;
  int o = i < a.n ? shard_owner(a, i, loc) : -1;
  __syncthreads();
  const int bid = (int)(uint32_t)sh_tk;
  const uint64_t ep = ((sh_tk >> 32) & 0x3fffffffull) << 32;
  if (bid != (int)blockIdx.x) {  // out-of-order dispatch: redo for the ticket
    i = (int64_t)bid * SP_PER + threadIdx.x;
    loc = -1;
    o = i < a.n ? shard_owner(a, i, loc) : -1;
  }
  // stable in-block rank: peel one owner at a time per wave
  const bool act = o >= 0;
  int rank = 0;
  uint64_t todo = __ballot(act);
  while (todo) {
    const int leader = __ffsll((unsigned long long)todo) - 1;
    const int lo = __shfl(o, leader);
    const uint64_t m = __ballot(act && o == lo);
    if (act && o == lo) rank = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wcnt[w][lo] = __popcll(m);
    todo &= ~m;
  }
  __syncthreads();
  // per owner (wave o, o + NW, ...): this block's total, published at once,
  // then a look-back over 128 predecessors per step (two per lane) that stops
  // at the nearest published inclusive prefix
  for (int oo = w; oo < a.world; oo += NW) {
    int agg = 0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) agg += wcnt[ww][oo];
    uint64_t* st_o = status + oo;
    if (lane == 0) sp_store(st_o + (int64_t)bid * a.world, ((bid == 0 ? 2ull : 1ull) << 62) | ep | (uint32_t)agg);
    int before = 0;
    for (int hi = (mode & 2) ? -1 : bid - 1; hi >= 0; hi -= 128) {
      const int p0 = hi - lane, p1 = hi - 64 - lane;
      uint64_t v0 = 0, v1 = 0;
      bool r0 = p0 < 0, r1 = p1 < 0;
      while (!__all(r0 && r1)) {
        if (!r0) v0 = sp_load(st_o + (int64_t)p0 * a.world);
        if (!r1) v1 = sp_load(st_o + (int64_t)p1 * a.world);
        r0 = r0 || ((v0 & 0x3fffffff00000000ull) == ep && (v0 >> 62) != 0);
        r1 = r1 || ((v1 & 0x3fffffff00000000ull) == ep && (v1 >> 62) != 0);
      }
      const uint64_t pm0 = __ballot(p0 >= 0 && (v0 >> 62) == 2);
      const uint64_t pm1 = __ballot(p1 >= 0 && (v1 >> 62) == 2);
      // nearest inclusive prefix: lowest lane of window 0, else of window 1
      const int stop = pm0 ? __ffsll((unsigned long long)pm0) - 1
                           : (pm1 ? 64 + __ffsll((unsigned long long)pm1) - 1 : 127);
      int val = (p0 >= 0 && lane <= stop ? (int)(uint32_t)v0 : 0) +
                (p1 >= 0 && 64 + lane <= stop ? (int)(uint32_t)v1 : 0);
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) val += __shfl_xor(val, d);
      before += val;
      if (pm0 | pm1) break;
    }
    if (lane == 0) {
      if (bid > 0) sp_store(st_o + (int64_t)bid * a.world, (2ull << 62) | ep | (uint32_t)(before + agg));
      excl[oo] = before;
      if (bid == nb - 1) counts[oo] = before + agg;
    }
  }
  __syncthreads();
  if (i < a.n) {
    if (o < 0 || loc < 0) {  // out-of-range id (shard_owner raised *err)
      slot_of[i] = -1;
    } else {
      int pos = excl[o] + rank;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][o];
      if (pos >= cap) {
        flag_error(overflow);
        slot_of[i] = -1;
      } else {
        slot_of[i] = o * cap + pos;
        send[(int64_t)o * cap + pos] = (int32_t)loc;
      }
    }
  }
}

// field route of the partial protocol: shard_route.hpp
__global__ __launch_bounds__(256) void shard_field_route(RouteArgs a) {
  field_route_part<256>(a, blockIdx.x, gridDim.x);
}


template <int VW>
__global__ void gather_rows_kernel(const float* __restrict__ table, int64_t n_rows, int k,
                                   const int32_t* __restrict__ rows, int64_t n, float* __restrict__ out, int* err) {
  const int KQ = k / VW;
  const int64_t total = n * KQ;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx / KQ;
    const int q = (int)(idx - i * KQ);
    const int64_t r = rows[i];
    Chunk<VW> x;
    x.zero();
    if (r >= 0 && r < n_rows) x.load(table + r * k + q * VW);
    else if (r != -1) flag_error(err);
    float* d = out + i * k + q * VW;
    if constexpr (VW == 4) {
      *reinterpret_cast<floatx4*>(d) = floatx4{x.v[0], x.v[1], x.v[2], x.v[3]};
    } else {
      d[0] = x.v[0];
    }
  }
}

template <int VW>
__global__ void unpermute_rows_kernel(const float* __restrict__ src, const int32_t* __restrict__ perm, int k,
                                      int64_t n, float* __restrict__ dst) {
  const int KQ = k / VW;
  const int64_t total = n * KQ;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx / KQ;
    const int q = (int)(idx - i * KQ);
    const int64_t p = perm[i];
    if constexpr (VW == 4) {
      *reinterpret_cast<floatx4*>(dst + i * k + q * 4) = *reinterpret_cast<const floatx4*>(src + p * k + q * 4);
    } else {
      dst[i * k + q] = src[p * k + q];
    }
  }
}

// k = 16 fast path (the configs' dim): 4 lanes per row, one float4 each,
// 32-bit indexing, every load issued before any store
__global__ __launch_bounds__(256) void gather_rows_k16(const float* __restrict__ table, int64_t n_rows,
                                                       const int32_t* __restrict__ rows, int n,
                                                       float* __restrict__ out, int* err) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int i = idx >> 2, q = idx & 3;
  if (i >= n) return;
  const int64_t r = rows[i];
  floatx4 x = floatx4{0.f, 0.f, 0.f, 0.f};
  if (r >= 0 && r < n_rows) x = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(table + r * 16) + q);
  else if (r != -1 && q == 0) flag_error(err);
  reinterpret_cast<floatx4*>(out)[idx] = x;  // a non-temporal store: 5.66 -> 5.78 us (profiles/r6_ab_nt_out.jsonl)
}

static unsigned sh_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace rs

using namespace rs;

// diagnostic timing modes of shard_slot_onepass (scripts only; 0 = product):
// bit0 blockIdx instead of the ticket, bit1 no look-back (wrong slots: timing only)
static int g_sp_mode = 0;
extern "C" void rs_diag_shard_set_mode(int m) { g_sp_mode = m; }

// workspace = [256 B control word (fixed offset: it must survive calls with a
// different n or world, and the exact protocol's hist) | hist (int32 per
// 256-lookup block and owner) and status (u64 per 1024-lookup block and owner)
// share one region]
constexpr int64_t SH_CTRL_BYTES = 256;
static int64_t sh_region_bytes(int64_t n_lookups, int world) {
  const int64_t hist = (n_lookups + SH_CHUNK - 1) / SH_CHUNK * world * 4;
  const int64_t stat = (n_lookups + SP_PER - 1) / SP_PER * world * 8;
  return (((hist > stat ? hist : stat) + 255) / 256) * 256;
}

extern "C" int64_t rs_shard_workspace_size(int64_t n_lookups, int world) {
  if (n_lookups < 0 || world < 1 || world > SH_MAXW) return -1;
  return SH_CTRL_BYTES + sh_region_bytes(n_lookups, world);
}

extern "C" int rs_shard_bucketize(const void* ids, int id_kind, int64_t id_stride, const int64_t* field_offsets,
                                  const int64_t* field_vocab, int n_fields, int64_t batch, int64_t rows_per_rank,
                                  int world, int32_t* counts, int32_t* perm, int32_t* send_rows, void* workspace,
                                  int* err_flag, rs_stream_t stream) {
  RS_REQUIRE(ids && field_offsets && field_vocab && counts && perm && send_rows && workspace,
             "rs_shard_bucketize: null pointer");
  RS_REQUIRE(world >= 1 && world <= SH_MAXW && rows_per_rank >= 1 && n_fields >= 1 && batch >= 0,
             "rs_shard_bucketize: bad shape (1 <= world <= %d)", SH_MAXW);
  RS_REQUIRE(batch * n_fields < ((int64_t)1 << 31), "rs_shard_bucketize: too many lookups");
  RS_REQUIRE(rows_per_rank < ((int64_t)1 << 31), "rs_shard_bucketize: shard rows must fit int32");
  hipStream_t st = as_stream(stream);
  ShardArgs a{ids, id_kind, id_stride, field_offsets, field_vocab, n_fields, batch * n_fields, rows_per_rank, world,
              err_flag, 1.0 / (double)rows_per_rank};
  const int nb = (int)((a.n + SH_CHUNK - 1) / SH_CHUNK);
  int32_t* hist = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(workspace) + SH_CTRL_BYTES);
  if (a.n == 0) {
    (void)hipMemsetAsync(counts, 0, world * sizeof(int32_t), st);
    return launch_status("rs_shard_bucketize");
  }
  shard_hist<<<nb, SH_THREADS, 0, st>>>(a, hist);
  shard_scan<<<1, 256, 0, st>>>(hist, nb, world, counts, 0);
  shard_place<<<nb, SH_THREADS, 0, st>>>(a, hist, perm, send_rows, 0, nullptr);
  return launch_status("rs_shard_bucketize");
}

extern "C" int rs_shard_slot_bucketize(const void* ids, int id_kind, int64_t id_stride,
                                       const int64_t* field_offsets, const int64_t* field_vocab, int n_fields,
                                       int64_t batch, int64_t rows_per_rank, int world, int cap, int32_t* counts,
                                       int32_t* slot_of, int32_t* send_slots, void* workspace, int* err_flag,
                                       int* overflow_flag, rs_stream_t stream) {
  RS_REQUIRE(ids && field_offsets && field_vocab && counts && slot_of && send_slots && workspace && overflow_flag,
             "rs_shard_slot_bucketize: null pointer");
  RS_REQUIRE(world >= 1 && world <= SH_MAXW && rows_per_rank >= 1 && n_fields >= 1 && batch >= 0 && cap >= 1,
             "rs_shard_slot_bucketize: bad shape (1 <= world <= %d, cap >= 1)", SH_MAXW);
  RS_REQUIRE(batch * n_fields < ((int64_t)1 << 31) && (int64_t)world * cap < ((int64_t)1 << 31),
             "rs_shard_slot_bucketize: too many lookups / slots");
  RS_REQUIRE(rows_per_rank < ((int64_t)1 << 31), "rs_shard_slot_bucketize: shard rows must fit int32");
  hipStream_t st = as_stream(stream);
  ShardArgs a{ids, id_kind, id_stride, field_offsets, field_vocab, n_fields, batch * n_fields, rows_per_rank, world,
              err_flag, 1.0 / (double)rows_per_rank};
  const int nb = (int)((a.n + SH_CHUNK - 1) / SH_CHUNK);
  int32_t* hist = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(workspace) + SH_CTRL_BYTES);
  if (a.n == 0) {
    (void)hipMemsetAsync(counts, 0, world * sizeof(int32_t), st);
    return launch_status("rs_shard_slot_bucketize");
  }
  (void)hist;
  const int nbp = (int)((a.n + SP_PER - 1) / SP_PER);
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  shard_slot_onepass<<<nbp, SP_THREADS, 0, st>>>(a, reinterpret_cast<uint64_t*>(ws + SH_CTRL_BYTES),
                                                 reinterpret_cast<uint64_t*>(ws), nbp,
                                                 counts, slot_of, send_slots, cap, overflow_flag, g_sp_mode);
  return launch_status("rs_shard_slot_bucketize");
}

extern "C" int rs_shard_field_route(const void* ids, int id_kind, int64_t id_stride, const int64_t* field_offsets,
                                    const int64_t* field_vocab, int n_fields, int64_t batch, int64_t rows_per_rank,
                                    int world, const int32_t* owner_fields, int slot_stride, int64_t rec_stride,
                                    int32_t* send, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(ids && field_offsets && field_vocab && owner_fields && send, "rs_shard_field_route: null pointer");
  RS_REQUIRE(world >= 1 && world <= SH_MAXW && rows_per_rank >= 1 && n_fields >= 1 && batch > 0 &&
                 slot_stride >= 1 && slot_stride <= n_fields && rec_stride >= slot_stride,
             "rs_shard_field_route: bad shape (1 <= world <= %d, 1 <= slot_stride <= n_fields)", SH_MAXW);
  RS_REQUIRE((int64_t)world * batch * slot_stride < ((int64_t)1 << 31) && rows_per_rank < ((int64_t)1 << 31),
             "rs_shard_field_route: too many slots / shard rows must fit int32");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_shard_field_route: bad id_kind");
  const int64_t total = (int64_t)world * batch * slot_stride;
  RouteArgs a{ids, id_kind, id_stride, field_offsets, field_vocab, rows_per_rank, owner_fields, slot_stride,
              (int)batch, rec_stride, send, err_flag, total};
  shard_field_route<<<sh_grid(total), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_shard_field_route");
}

extern "C" int rs_shard_row_route(const void* ids, int id_kind, int64_t id_stride, const int64_t* field_offsets,
                                  const int64_t* field_vocab, int n_fields, int64_t batch, int64_t rows_per_rank,
                                  int world, const int32_t* owner_fields, int slot_stride, int32_t* send,
                                  int32_t* slot_of, int* err_flag, rs_stream_t stream) {
  if (batch == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(ids && field_offsets && field_vocab && owner_fields && send && slot_of,
             "rs_shard_row_route: null pointer");
  RS_REQUIRE(world >= 1 && world <= SH_MAXW && rows_per_rank >= 1 && n_fields >= 1 && batch > 0 &&
                 slot_stride >= 1 && slot_stride <= n_fields,
             "rs_shard_row_route: bad shape (1 <= world <= %d, 1 <= slot_stride <= n_fields)", SH_MAXW);
  RS_REQUIRE((int64_t)world * batch * slot_stride < ((int64_t)1 << 31) && rows_per_rank < ((int64_t)1 << 31) &&
                 batch * n_fields < ((int64_t)1 << 31),
             "rs_shard_row_route: too many slots / shard rows must fit int32");
  RS_REQUIRE(id_kind >= RS_ID_I32 && id_kind <= RS_ID_F32, "rs_shard_row_route: bad id_kind");
  const int64_t total = (int64_t)world * batch * slot_stride;
  RouteArgs a{ids, id_kind, id_stride, field_offsets, field_vocab, rows_per_rank, owner_fields, slot_stride,
              (int)batch, slot_stride, send, err_flag, total, slot_of, n_fields};
  shard_field_route<<<sh_grid(total), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_shard_row_route");
}

extern "C" int rs_gather_rows(const float* table, int64_t n_rows, int k, const int32_t* rows, int64_t n, float* out,
                              int* err_flag, rs_stream_t stream) {
  if (n == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(rows && out && (n == 0 || table || n_rows == 0), "rs_gather_rows: null pointer");
  RS_REQUIRE(k >= 1 && n >= 0 && n_rows >= 0, "rs_gather_rows: bad shape");
  if (n == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  if (k == 16 && n < (1 << 29) && (uintptr_t)table % 16 == 0 && (uintptr_t)out % 16 == 0)
    gather_rows_k16<<<(unsigned)((n * 4 + 255) / 256), 256, 0, st>>>(table, n_rows, rows, (int)n, out, err_flag);
  else if (k % 4 == 0 && (uintptr_t)table % 16 == 0 && (uintptr_t)out % 16 == 0)
    gather_rows_kernel<4><<<sh_grid(n * (k / 4)), 256, 0, st>>>(table, n_rows, k, rows, n, out, err_flag);
  else
    gather_rows_kernel<1><<<sh_grid(n * k), 256, 0, st>>>(table, n_rows, k, rows, n, out, err_flag);
  return launch_status("rs_gather_rows");
}

extern "C" int rs_unpermute_rows(const float* src, const int32_t* perm, int k, int64_t n, float* dst,
                                 rs_stream_t stream) {
  if (n == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(src && perm && dst && k >= 1 && n >= 0, "rs_unpermute_rows: bad arguments");
  if (n == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  if (k % 4 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0)
    unpermute_rows_kernel<4><<<sh_grid(n * (k / 4)), 256, 0, st>>>(src, perm, k, n, dst);
  else
    unpermute_rows_kernel<1><<<sh_grid(n * k), 256, 0, st>>>(src, perm, k, n, dst);
  return launch_status("rs_unpermute_rows");
}

// ------------------------------------- row-gradient scatter (sharded backward)
// dst[slot_of[j]] = src[b*src_stride + c*k : +k] for lookup j = b*n_fields + c
// (slot_of < 0: skipped).  The sharded DeepFM backward writes each lookup's
// dL/drow into its slot of the row-exchange layout, so the reverse
// all-to-all hands every owner the gradients aligned with the row ids it
// served.  One thread per (lookup, column).
namespace rs {
__global__ __launch_bounds__(256) void scatter_rows_kernel(const float* __restrict__ src, int64_t src_stride,
                                                           int n_fields, int k, const int32_t* __restrict__ slot_of,
                                                           int64_t n, float* __restrict__ dst) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n * k; t += (int64_t)gridDim.x * 256) {
    const int64_t j = t / k;
    const int f = (int)(t - j * k);
    const int64_t slot = slot_of[j];
    if (slot < 0) continue;
    const int64_t b = j / n_fields;
    const int c = (int)(j - b * n_fields);
    dst[slot * k + f] = src[b * src_stride + (int64_t)c * k + f];
  }
}
}  // namespace rs

extern "C" int rs_scatter_rows(const float* src, int64_t src_stride, int n_fields, int k, const int32_t* slot_of,
                               int64_t batch, float* dst, rs_stream_t stream) {
  if (batch == 0 || n_fields == 0) return RS_OK;
  RS_REQUIRE(src && slot_of && dst && k >= 1 && batch > 0 && n_fields > 0 && src_stride >= (int64_t)n_fields * k,
             "rs_scatter_rows: bad arguments");
  const int64_t n = batch * n_fields;
  scatter_rows_kernel<<<sh_grid(n * k), 256, 0, as_stream(stream)>>>(src, src_stride, n_fields, k, slot_of, n, dst);
  return launch_status("rs_scatter_rows");
}
