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

static unsigned sh_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_shard_workspace_size(int64_t n_lookups, int world) {
  if (n_lookups < 0 || world < 1 || world > SH_MAXW) return -1;
  const int64_t nb = (n_lookups + SH_CHUNK - 1) / SH_CHUNK;
  return ((nb * world * 4 + 255) / 256) * 256 + 256;
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
  int32_t* hist = static_cast<int32_t*>(workspace);
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
  int32_t* hist = static_cast<int32_t*>(workspace);
  if (a.n == 0) {
    (void)hipMemsetAsync(counts, 0, world * sizeof(int32_t), st);
    return launch_status("rs_shard_slot_bucketize");
  }
  shard_hist<<<nb, SH_THREADS, 0, st>>>(a, hist);
  shard_scan<<<1, 256, 0, st>>>(hist, nb, world, counts, cap);
  shard_place<<<nb, SH_THREADS, 0, st>>>(a, hist, slot_of, send_slots, cap, overflow_flag);
  return launch_status("rs_shard_slot_bucketize");
}

extern "C" int rs_gather_rows(const float* table, int64_t n_rows, int k, const int32_t* rows, int64_t n, float* out,
                              int* err_flag, rs_stream_t stream) {
  if (n == 0) return RS_OK;  // empty batch: nothing to launch (null data pointers allowed)
  RS_REQUIRE(rows && out && (n == 0 || table || n_rows == 0), "rs_gather_rows: null pointer");
  RS_REQUIRE(k >= 1 && n >= 0 && n_rows >= 0, "rs_gather_rows: bad shape");
  if (n == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  if (k % 4 == 0 && (uintptr_t)table % 16 == 0 && (uintptr_t)out % 16 == 0)
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
