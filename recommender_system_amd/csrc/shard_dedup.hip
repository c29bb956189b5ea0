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
#include <hipcub/hipcub.hpp>

#include "rs_common.hpp"

namespace rs {

struct DedupWs {
  int64_t key_in, key_out, val_in, val_out, head, incl, ustart, fmeta, sort, scan, total;
  size_t sort_bytes, scan_bytes;
};

// Fields per route on the per-field path (its cnt / base slab) and the
// largest batch whose field fits one workgroup's LDS sort (8-B keys).
constexpr int DD_MAXF = 1024;
constexpr int64_t DD_MAXB = 16384;

static int64_t dd_al(int64_t x) { return (x + 255) / 256 * 256; }

static DedupWs dedup_ws(int64_t n, int world) {
  DedupWs w{};
  const int nn = (int)(n > 0 ? n : 1);
  size_t sb = 0, cb = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sb, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                           (int32_t*)nullptr, nn);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, cb, (int32_t*)nullptr, (int32_t*)nullptr, nn);
  w.sort_bytes = sb;
  w.scan_bytes = cb;
  int64_t o = 0;
  w.key_in = o; o = dd_al(o + n * 4);
  w.key_out = o; o = dd_al(o + n * 4);
  w.val_in = o; o = dd_al(o + n * 4);
  w.val_out = o; o = dd_al(o + n * 4);
  w.head = o; o = dd_al(o + n * 4);
  w.incl = o; o = dd_al(o + n * 4);
  w.ustart = o; o = dd_al(o + (int64_t)world * 4);
  w.fmeta = o; o = dd_al(o + 2 * DD_MAXF * 4);
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

// ---- hand-written route: one workgroup per field sorts that field's B
// lookups in LDS.  Field c's rows are [off_c, off_c + vocab_c) and the
// concatenated table's offsets increase with c, so the field-ordered
// concatenation of the per-field sorted segments IS the global (row, lookup)
// order — no device-wide sort.  Each segment's keys end with its bad ids
// (0xffffffff), which are never heads.
//   dedup_field_sort: composite 64-bit key (row << 32 | b) — unique, so the
//     bitonic network gives the stable order; heads + an in-LDS inclusive
//     scan number the field's distinct rows (incl_w), cnt[c] = their count.
//   dedup_field_meta: base[c] = distinct rows of the fields before c,
//     ustart[o] = distinct rows below owner o's first row (whole fields
//     below it + a binary search inside the straddling one).
//   dedup_scatter_f: as dedup_scatter with u = base + incl_w - 1 - ustart.
template <int KIND>
__global__ __launch_bounds__(1024) void dedup_field_sort(const void* ids, int64_t id_stride,
                                                         const int64_t* __restrict__ offs,
                                                         const int64_t* __restrict__ vocab, int F, int64_t B, int N2,
                                                         uint32_t* __restrict__ key_out, int32_t* __restrict__ val_out,
                                                         int32_t* __restrict__ incl_w, int32_t* __restrict__ cnt,
                                                         int* err) {
  typedef Ids<KIND> I;
  extern __shared__ uint64_t kv[];  // N2 composite keys, then 1024 + 32 ints of scan scratch
  int* part = reinterpret_cast<int*>(kv + N2);
  const int c = blockIdx.x;
  const int64_t off = offs[c], voc = vocab[c];
  bool bad = false;
  for (int p = threadIdx.x; p < N2; p += 1024) {
    uint64_t key = ~0ull;
    if (p < B) {
      int64_t id;
      const bool ok = I::decode(I::load(ids, (int64_t)p * id_stride + c), voc, id);
      bad |= !ok;
      key = ((uint64_t)(ok ? (uint32_t)(off + id) : 0xffffffffu) << 32) | (uint32_t)p;
    }
    kv[p] = key;
  }
  if (bad) flag_error(err);
  // the layout this path relies on: field c's rows end where field c+1's begin (or before)
  if (threadIdx.x == 0 && c + 1 < F && off + voc > offs[c + 1]) flag_error(err, RS_FLAG_LAYOUT);
  __syncthreads();
  // bitonic sort, ascending
  for (int kk = 2; kk <= N2; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < N2 / 2; t += 1024) {
        const int lo = 2 * j * (t / j) + (t % j), hi = lo + j;
        const bool up = (lo & kk) == 0;
        const uint64_t x = kv[lo], y = kv[hi];
        if ((x > y) == up) {
          kv[lo] = y;
          kv[hi] = x;
        }
      }
      __syncthreads();
    }
  }
  // heads and the field's inclusive scan of them: E = N2 / 1024 consecutive
  // positions per thread, thread totals scanned through LDS
  const int E = N2 >= 1024 ? N2 / 1024 : 1;
  const int p0 = threadIdx.x * E;
  int h[16];
  int tot = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    h[e] = 0;
    const int p = p0 + e;
    if (e < E && p < N2 && p < B) {
      const uint32_t r = (uint32_t)(kv[p] >> 32);
      h[e] = (r != 0xffffffffu && (p == 0 || (uint32_t)(kv[p - 1] >> 32) != r)) ? 1 : 0;
    }
    tot += h[e];
  }
  part[threadIdx.x] = tot;
  __syncthreads();
  if (threadIdx.x < 32) {  // 32 lanes scan 32 chunks of 32 thread totals
    int sum = 0;
    for (int i = 0; i < 32; ++i) sum += part[threadIdx.x * 32 + i];
    part[1024 + threadIdx.x] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int i = 0; i < 32; ++i) {
      const int v = part[1024 + i];
      part[1024 + i] = run;
      run += v;
    }
    cnt[c] = run;
  }
  __syncthreads();
  int run = part[1024 + threadIdx.x / 32];
  for (int i = (threadIdx.x / 32) * 32; i < (int)threadIdx.x; ++i) run += part[i];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int p = p0 + e;
    if (e < E && p < B) {
      run += h[e];
      const uint64_t key = kv[p];
      key_out[(int64_t)c * B + p] = (uint32_t)(key >> 32);
      val_out[(int64_t)c * B + p] = (int32_t)((int64_t)(uint32_t)key * F + c);
      incl_w[(int64_t)c * B + p] = run;
    }
  }
}

__global__ void dedup_field_meta(const uint32_t* __restrict__ key, const int32_t* __restrict__ incl_w,
                                 const int32_t* __restrict__ cnt, const int64_t* __restrict__ offs,
                                 const int64_t* __restrict__ vocab, int F, int64_t B, int64_t rpr, int world,
                                 int32_t* __restrict__ ustart, int32_t* __restrict__ base) {
  const int o = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (o == world) {
    int run = 0;
    for (int c = 0; c < F; ++c) {
      base[c] = run;
      run += cnt[c];
    }
  }
  if (o >= world) return;
  const uint64_t lo_row = (uint64_t)o * (uint64_t)rpr;
  int u = 0;
  for (int c = 0; c < F; ++c) {
    const uint64_t f0 = (uint64_t)offs[c], f1 = f0 + (uint64_t)vocab[c];
    if (f1 <= lo_row) {
      u += cnt[c];
    } else if (f0 < lo_row) {  // the straddling field: first position with row >= lo_row
      const uint32_t* k = key + (int64_t)c * B;
      int64_t lo = 0, hi = B;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((uint64_t)k[mid] < lo_row) lo = mid + 1;
        else hi = mid;
      }
      if (lo > 0) u += incl_w[(int64_t)c * B + lo - 1];
    }
  }
  ustart[o] = u;
}

__global__ __launch_bounds__(256) void dedup_scatter_f(const uint32_t* __restrict__ key,
                                                       const int32_t* __restrict__ val,
                                                       const int32_t* __restrict__ incl_w,
                                                       const int32_t* __restrict__ base,
                                                       const int32_t* __restrict__ ustart, int64_t B, int64_t n,
                                                       int64_t rpr, int world, int64_t cap,
                                                       int32_t* __restrict__ send, int32_t* __restrict__ slot_of,
                                                       int* overflow) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const uint32_t r = key[p];
  const int32_t j = val[p];
  if (r == 0xffffffffu) {
    slot_of[j] = -1;
    return;
  }
  const int64_t c = p / B, pp = p - c * B;
  const bool head = pp == 0 || key[p - 1] != r;
  const int o = dd_owner(r, rpr, world);
  const int64_t u = (int64_t)base[c] + incl_w[p] - 1 - ustart[o];
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
  // words past each owner's count ask for row -1 (a zero row)
  hipError_t e = hipMemsetAsync(send, 0xff, (size_t)world * cap * 4, st);
  if (e != hipSuccess) {
    set_error("rs_shard_dedup_route: memset failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
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
  if (batch <= DD_MAXB && n_fields <= DD_MAXF) {
    // hand-written path: per-field LDS sorts (no device-wide radix sort)
    int N2 = 1;
    while (N2 < batch) N2 <<= 1;
    const size_t lds = (size_t)N2 * 8 + (1024 + 32) * 4;
    int32_t* cnt = reinterpret_cast<int32_t*>(ws + w.fmeta);
    int32_t* base = cnt + DD_MAXF;
    with_id_kind(id_kind, [&](auto K) {
      constexpr int KI = decltype(K)::value;
      static size_t lds_set[3] = {64 * 1024, 64 * 1024, 64 * 1024};
      if (lds > lds_set[KI]) {
        (void)hipFuncSetAttribute((const void*)dedup_field_sort<KI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        lds_set[KI] = lds;
      }
      dedup_field_sort<KI><<<n_fields, 1024, lds, st>>>(ids, id_stride, field_offsets, field_vocab, n_fields, batch,
                                                         N2, key_out, val_out, head, cnt, err_flag);
    });
    dedup_field_meta<<<(world + 1 + 63) / 64, 64, 0, st>>>(key_out, head, cnt, field_offsets, field_vocab, n_fields,
                                                         batch, rows_per_rank, world, ustart, base);
    dedup_scatter_f<<<g, 256, 0, st>>>(key_out, val_out, head, base, ustart, batch, n, rows_per_rank, world, cap,
                                       send, slot_of, overflow_flag);
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
  size_t sb = w.sort_bytes, cb = w.scan_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(ws + w.sort, sb, key_in, key_out, val_in, val_out, (int)n, 0, bits, st);
  if (e == hipSuccess) {
    dedup_heads<<<g, 256, 0, st>>>(key_out, n, head);
    e = hipcub::DeviceScan::InclusiveSum(ws + w.scan, cb, head, incl, (int)n, st);
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
  const unsigned g = (unsigned)((n * k + 255) / 256);
  dedup_grad_piece<<<g, 256, 0, st>>>(key, val, n, n_fields, k, grad, grad_stride, slot_of, C, part_first, part_last,
                                      dst);
  if (nch > 1) dedup_grad_cross<<<g, 256, 0, st>>>(key, val, n, k, slot_of, C, part_first, part_last, dst);
  return launch_status("rs_shard_dedup_grad");
}
