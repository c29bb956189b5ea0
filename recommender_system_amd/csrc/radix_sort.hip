// radix_sort.hip — stable LSD radix sort of (uint32 key, uint32 val) pairs and
// an int32 inclusive scan, written for the row-sparse scatter-adds: the
// embedding SGD and FM training group every lookup's gradient by table row
// (seg_piece / seg_cross, rs_common.hpp, sum a row's segment in lookup order,
// so the sort must be stable), and the dedup route's large-batch path numbers
// distinct rows by a scan of segment heads.
//
// One pass per 8 key bits, over tiles of 256 threads x RX_ITEMS pairs, three
// launches a pass:
//   radix_hist      the tile's digit counts in LDS (order-free atomics),
//                   written digit-major hist[d][tile];
//   radix_row_scan  one workgroup per digit scans its row in place (tiles in
//                   order) and writes the row total;
//   radix_scatter   the tile's start for each digit (the row totals scanned
//                   over the 256 digits in the workgroup + the tile's row
//                   prefix), then each pair's rank among equal digits in tile
//                   order: per 64-lane batch the lanes with the same digit are
//                   found by 8 ballots (no LDS atomics, so the rank is the
//                   pair's position, not an arrival order), wave-private digit
//                   counters carry the rank across a wave's batches and a sum
//                   over the earlier waves' counters across waves.
// Tile order inside a workgroup: pair e = (wave * RX_ITEMS + r) * 64 + lane,
// a wave's batches consecutive, so loads are coalesced and the rank order is
// the input order.  Bytes per pass: 8 B read twice + 8 B written per pair
// (HBM-bound integer work; ~2.6 MB a pass for the 106,496 lookups of a B 4096
// x 26 batch).  Tile size and the row-scan split were chosen by
// scripts/ab_sort.py against hipCUB on one box (profiles/r3_ab_sort.jsonl):
// 52 vs 51 us at 106,496 pairs, 134 vs 143 us at 1,703,936.
#include "radix_sort.hpp"
#include "rs_common.hpp"

namespace rs {

constexpr int RX_T = 256;              // threads per workgroup
#ifndef RX_ITEMS
#define RX_ITEMS 8
#endif
constexpr int RX_R = RX_ITEMS;         // pairs per lane
constexpr int RX_TILE = RX_T * RX_R;   // pairs per tile
constexpr int RX_D = 8;                // digit bits
constexpr int RX_ND = 1 << RX_D;       // digits

static int64_t rx_al(int64_t x) { return (x + 255) / 256 * 256; }

__device__ __forceinline__ int64_t rx_elem(int64_t tile, int w, int r, int lane) {
  return tile * RX_TILE + (int64_t)(w * RX_R + r) * 64 + lane;
}

__global__ __launch_bounds__(RX_T) void radix_hist(const uint32_t* __restrict__ key, int64_t n, int shift,
                                                   uint32_t* __restrict__ hist, int64_t ntile) {
  __shared__ uint32_t h[RX_ND];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int d = t; d < RX_ND; d += RX_T) h[d] = 0;
  __syncthreads();
  uint32_t k[RX_R];
#pragma unroll
  for (int r = 0; r < RX_R; ++r) {
    const int64_t e = rx_elem(blockIdx.x, w, r, lane);
    k[r] = e < n ? key[e] : 0u;
  }
#pragma unroll
  for (int r = 0; r < RX_R; ++r)
    if (rx_elem(blockIdx.x, w, r, lane) < n) atomicAdd(&h[(k[r] >> shift) & (RX_ND - 1)], 1u);
  __syncthreads();
  for (int d = t; d < RX_ND; d += RX_T) hist[(int64_t)d * ntile + blockIdx.x] = h[d];
}

// exclusive scan of v over one 1024-thread workgroup (thread order)
__device__ __forceinline__ uint32_t rx_block_excl(uint32_t v, uint32_t* red, uint32_t& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) red[wv] = inc;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    const uint32_t x = red[w];
    wb += w < wv ? x : 0u;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return wb + inc - v;
}

// in-place exclusive (EXCL) or inclusive scan of m values by one workgroup:
// thread t owns a contiguous chunk, chunk sums scanned across the workgroup
template <bool EXCL, class T>
__global__ __launch_bounds__(1024) void rx_scan_one(T* __restrict__ a, const T* __restrict__ src, int64_t m,
                                                    T* __restrict__ carry_out) {
  __shared__ uint32_t red[16];
  const int64_t per = (m + 1023) / 1024;
  const int64_t lo = (int64_t)threadIdx.x * per, hi = lo + per < m ? lo + per : m;
  uint32_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += (uint32_t)src[i];
  uint32_t total;
  uint32_t run = rx_block_excl(s, red, total);
  for (int64_t i = lo; i < hi; ++i) {
    const uint32_t x = (uint32_t)src[i];
    if (EXCL) {
      a[i] = (T)run;
      run += x;
    } else {
      run += x;
      a[i] = (T)run;
    }
  }
  if (carry_out && threadIdx.x == 0) carry_out[0] = (T)total;
}

// many tiles: one workgroup per digit scans its row of the count table in
// place (exclusive, tiles in order) and writes the row total; the scatter
// then adds the totals of the digits below (its own 256-entry scan)
__global__ __launch_bounds__(RX_T) void radix_row_scan(uint32_t* __restrict__ hist, int64_t ntile,
                                                       uint32_t* __restrict__ rowsum) {
  __shared__ uint32_t red[RX_T / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t* row = hist + (int64_t)blockIdx.x * ntile;
  const int64_t per = (ntile + RX_T - 1) / RX_T;
  const int64_t lo = (int64_t)t * per, hi = lo + per < ntile ? lo + per : ntile;
  uint32_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += row[i];
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) red[w] = inc;
  __syncthreads();
  uint32_t run = inc - s;
  for (int ww = 0; ww < w; ++ww) run += red[ww];
  for (int64_t i = lo; i < hi; ++i) {
    const uint32_t x = row[i];
    row[i] = run;
    run += x;
  }
  if (t == RX_T - 1) rowsum[blockIdx.x] = run;
}

__global__ __launch_bounds__(RX_T) void radix_scatter(const uint32_t* __restrict__ kin,
                                                      const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
                                                      uint32_t* __restrict__ vout, int64_t n, int shift,
                                                      const uint32_t* __restrict__ hist, int64_t ntile,
                                                      const uint32_t* __restrict__ rowsum) {
  __shared__ uint32_t cnt[RX_T / 64][RX_ND];
  __shared__ uint32_t gb[RX_ND];
  __shared__ uint32_t red[RX_T / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t k[RX_R], v[RX_R];
  int dg[RX_R];
#pragma unroll
  for (int r = 0; r < RX_R; ++r) {
    const int64_t e = rx_elem(blockIdx.x, w, r, lane);
    const bool ok = e < n;
    k[r] = ok ? kin[e] : 0u;
    v[r] = ok ? vin[e] : 0u;
    dg[r] = ok ? (int)((k[r] >> shift) & (RX_ND - 1)) : RX_ND;
  }
  for (int i = t; i < (RX_T / 64) * RX_ND; i += RX_T) (&cnt[0][0])[i] = 0;
  {
    // thread d: digit d's total over all tiles (rowsum) and its count over
    // the tiles before this one (the scanned row); the tile's start = (totals
    // of the digits below d) + that prefix
    static_assert(RX_T == RX_ND, "one thread per digit");
    const uint32_t tot = rowsum[t];
    const uint32_t pre = hist[(int64_t)t * ntile + blockIdx.x];
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == 63) red[w] = inc;
    __syncthreads();
    uint32_t below = inc - tot;
    for (int ww = 0; ww < w; ++ww) below += red[ww];
    gb[t] = below + pre;
  }
  __syncthreads();
  // rank inside the wave: lanes with the same digit (and present) in batch r
  int occ[RX_R];
  uint32_t* mine = cnt[w];
#pragma unroll
  for (int r = 0; r < RX_R; ++r) {
    const uint32_t d = (uint32_t)dg[r];
    uint64_t m = __builtin_amdgcn_ballot_w64(d < RX_ND);
#pragma unroll
    for (int i = 0; i < RX_D; ++i) {
      const uint64_t bl = __builtin_amdgcn_ballot_w64(((d >> i) & 1u) != 0);
      m &= ((d >> i) & 1u) ? bl : ~bl;
    }
    const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const uint32_t prior = d < RX_ND ? mine[d] : 0u;
    occ[r] = (int)prior + below;
    __builtin_amdgcn_wave_barrier();
    if (d < RX_ND && below == 0) mine[d] = prior + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RX_R; ++r) {
    const int d = dg[r];
    if (d < RX_ND) {
      uint32_t pos = gb[d] + (uint32_t)occ[r];
      for (int ww = 0; ww < w; ++ww) pos += cnt[ww][d];
      kout[pos] = k[r];
      vout[pos] = v[r];
    }
  }
}

struct RxWs {
  int64_t hist, rowsum, tk, tv, total;
};
static RxWs rx_ws(int64_t n) {
  RxWs w{};
  const int64_t ntile = (n + RX_TILE - 1) / RX_TILE;
  int64_t o = 0;
  w.hist = o; o = rx_al(o + ntile * RX_ND * 4);
  w.rowsum = o; o = rx_al(o + RX_ND * 4);
  w.tk = o; o = rx_al(o + n * 4);
  w.tv = o; o = rx_al(o + n * 4);
  w.total = o;
  return w;
}

int64_t sort_pairs_ws_bytes(int64_t n) { return rx_ws(n > 0 ? n : 1).total; }

hipError_t sort_pairs_u32(const uint32_t* key_in, const uint32_t* val_in, uint32_t* key_out, uint32_t* val_out,
                          int64_t n, int bits, void* ws, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (bits < 1) bits = 1;
  if (bits > 32) bits = 32;
  const RxWs w = rx_ws(n);
  uint8_t* base = static_cast<uint8_t*>(ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + w.hist);
  uint32_t* rowsum = reinterpret_cast<uint32_t*>(base + w.rowsum);
  uint32_t* tk = reinterpret_cast<uint32_t*>(base + w.tk);
  uint32_t* tv = reinterpret_cast<uint32_t*>(base + w.tv);
  const int64_t ntile = (n + RX_TILE - 1) / RX_TILE;
  const int P = (bits + RX_D - 1) / RX_D;
  const uint32_t* sk = key_in;
  const uint32_t* sv = val_in;
  for (int p = 0; p < P; ++p) {
    // the last pass lands in key_out / val_out; earlier ones alternate so a
    // pass never reads the buffer it writes
    const bool to_out = ((P - 1 - p) & 1) == 0;
    uint32_t* dk = to_out ? key_out : tk;
    uint32_t* dv = to_out ? val_out : tv;
    radix_hist<<<(unsigned)ntile, RX_T, 0, st>>>(sk, n, p * RX_D, hist, ntile);
    radix_row_scan<<<RX_ND, RX_T, 0, st>>>(hist, ntile, rowsum);
    radix_scatter<<<(unsigned)ntile, RX_T, 0, st>>>(sk, sv, dk, dv, n, p * RX_D, hist, ntile, rowsum);
    sk = dk;
    sv = dv;
  }
  return hipGetLastError();
}

// ---- inclusive scan: per-tile sums, one-workgroup scan of the sums, per-tile
// scan from its carry (tile = RX_TILE values: RX_T threads x RX_R per thread)
__global__ __launch_bounds__(RX_T) void scan_tile_sums(const int32_t* __restrict__ in, int64_t n,
                                                       int32_t* __restrict__ sums) {
  __shared__ int32_t red[RX_T / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int32_t s = 0;
  const int64_t lo = (int64_t)blockIdx.x * RX_TILE + (int64_t)t * RX_R;
#pragma unroll
  for (int r = 0; r < RX_R; ++r) s += lo + r < n ? in[lo + r] : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) red[w] = s;
  __syncthreads();
  if (t == 0) sums[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(RX_T) void scan_tiles(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                   int64_t n, const int32_t* __restrict__ carry) {
  __shared__ int32_t red[RX_T / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t lo = (int64_t)blockIdx.x * RX_TILE + (int64_t)t * RX_R;
  int32_t x[RX_R];
  int32_t s = 0;
#pragma unroll
  for (int r = 0; r < RX_R; ++r) {
    x[r] = lo + r < n ? in[lo + r] : 0;
    s += x[r];
  }
  int32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) red[w] = inc;
  __syncthreads();
  int32_t run = carry[blockIdx.x] + inc - s;
  for (int ww = 0; ww < w; ++ww) run += red[ww];
#pragma unroll
  for (int r = 0; r < RX_R; ++r) {
    run += x[r];
    if (lo + r < n) out[lo + r] = run;
  }
}

int64_t scan_ws_bytes(int64_t n) {
  const int64_t ntile = (n > 0 ? n + RX_TILE - 1 : RX_TILE) / RX_TILE;
  return rx_al(ntile * 4);
}

hipError_t inclusive_sum_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t ntile = (n + RX_TILE - 1) / RX_TILE;
  int32_t* sums = static_cast<int32_t*>(ws);
  scan_tile_sums<<<(unsigned)ntile, RX_T, 0, st>>>(in, n, sums);
  rx_scan_one<true, int32_t><<<1, 1024, 0, st>>>(sums, sums, ntile, nullptr);  // tile carries
  scan_tiles<<<(unsigned)ntile, RX_T, 0, st>>>(in, out, n, sums);
  return hipGetLastError();
}

}  // namespace rs

using namespace rs;

// C-ABI of the two primitives (tests/test_gpu_sort.py checks them against a
// stable numpy argsort / cumsum; the product calls them internally)
extern "C" int64_t rs_sort_pairs_workspace_size(int64_t n) { return n < 0 ? -1 : sort_pairs_ws_bytes(n); }

extern "C" int rs_sort_pairs_u32(const uint32_t* key_in, const uint32_t* val_in, uint32_t* key_out,
                                 uint32_t* val_out, int64_t n, int bits, void* workspace, rs_stream_t stream) {
  if (n == 0) return RS_OK;
  RS_REQUIRE(n > 0 && n < (1ll << 31) && bits >= 1 && bits <= 32, "rs_sort_pairs_u32: bad shape");
  RS_REQUIRE(key_in && val_in && key_out && val_out && workspace, "rs_sort_pairs_u32: null pointer");
  RS_REQUIRE(key_in != key_out && val_in != val_out, "rs_sort_pairs_u32: in and out must differ");
  (void)sort_pairs_u32(key_in, val_in, key_out, val_out, n, bits, workspace, as_stream(stream));
  return launch_status("rs_sort_pairs_u32");
}

extern "C" int64_t rs_inclusive_sum_workspace_size(int64_t n) { return n < 0 ? -1 : scan_ws_bytes(n); }

extern "C" int rs_inclusive_sum_i32(const int32_t* in, int32_t* out, int64_t n, void* workspace,
                                    rs_stream_t stream) {
  if (n == 0) return RS_OK;
  RS_REQUIRE(n > 0 && n < (1ll << 31) && in && out && workspace, "rs_inclusive_sum_i32: bad arguments");
  (void)inclusive_sum_i32(in, out, n, workspace, as_stream(stream));
  return launch_status("rs_inclusive_sum_i32");
}
