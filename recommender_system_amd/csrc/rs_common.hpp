// rs_common.hpp — shared device/host helpers for librs_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rs_capi.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

namespace rs {

// Thread-local last-error message (rs_last_error_string).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Map the status of the launch just issued to an rs_status.
int launch_status(const char* what);

inline hipStream_t as_stream(rs_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// A kernel's dynamic-LDS opt-in (hipFuncSetAttribute) beyond the 64 KiB
// default, per device: set[d] = the largest size set so far on device d (only
// successful calls are recorded; a failure is retried at the next launch,
// whose own launch status then reports it).
struct LdsAttr {
  size_t set[64] = {};
};
inline void lds_attr(LdsAttr& s, const void* kern, size_t lds) {
  if (lds <= 64 * 1024) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds <= s.set[dev]) return;
  if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess) s.set[dev] = lds;
}

#define RS_REQUIRE(cond, ...)            \
  do {                                   \
    if (!(cond)) {                       \
      ::rs::set_error(__VA_ARGS__);      \
      return RS_ERR_ARG;                 \
    }                                    \
  } while (0)

// ------------------------------------------------------------ device side
// Compile-time id plumbing for the hot kernels (no per-lane branches):
// KIND 0 = int32, 1 = int64, 2 = float32 (Keras int32 truncation), 3 = no ids
// (rows already gathered).  decode() returns validity and a clamped id (0 when
// invalid) so the caller can issue the row load unconditionally and zero it.
template <int KIND>
struct Ids {
  typedef typename std::conditional<KIND == 1, int64_t,
                                    typename std::conditional<KIND == 2, float, int32_t>::type>::type raw_t;
  static __device__ __forceinline__ raw_t load(const void* p, int64_t off) {
    return static_cast<const raw_t*>(p)[off];  // a non-temporal id load: +0.05 / +0.1 us (profiles/r6_ab_nt_ids_rejected.jsonl)
  }
  static __device__ __forceinline__ bool decode(raw_t r, int64_t vocab, int64_t& id) {
    if constexpr (KIND == 2) {
      const bool ok = (r > -1.0f) && (static_cast<double>(r) < static_cast<double>(vocab));
      id = ok ? static_cast<int64_t>(r) : 0;
      return ok;
    } else {
      const int64_t v = static_cast<int64_t>(r);
      const bool ok = (v >= 0) && (v < vocab);
      id = ok ? v : 0;
      return ok;
    }
  }
};

// Host helper: call f(std::integral_constant<int, KIND>) for a runtime id kind.
template <class Fn>
inline void with_id_kind(int kind, Fn&& f) {
  switch (kind) {
    case RS_ID_I32: f(std::integral_constant<int, 0>()); break;
    case RS_ID_I64: f(std::integral_constant<int, 1>()); break;
    default: f(std::integral_constant<int, 2>()); break;
  }
}

// Device error flag: RS_FLAG_BAD_ID (an id outside [0, vocab)) unless another
// code is given; codes are or-ed, so one flag carries every kind seen.
__device__ __forceinline__ void flag_error(int* err_flag, int code = RS_FLAG_BAD_ID) {
  if (err_flag) __hip_atomic_fetch_or(err_flag, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Runtime tuning options (rs_set_option); read on the host at launch time.
int opt(int option);

template <int N>
struct VecF;
template <>
struct VecF<1> {
  typedef float T;
  static __device__ __forceinline__ float get(const T& v, int) { return v; }
};
template <>
struct VecF<2> {
  typedef floatx2 T;
  static __device__ __forceinline__ float get(const T& v, int i) { return v[i]; }
};
template <>
struct VecF<4> {
  typedef floatx4 T;
  static __device__ __forceinline__ float get(const T& v, int i) { return v[i]; }
};

// Load N consecutive floats (N in {1,2,4,8,16}) as vectors; p must be aligned
// to min(16, 4N) bytes.
template <int N>
struct Chunk {
  float v[N];
  __device__ __forceinline__ void load(const float* p) {
    if constexpr (N == 1) {
      v[0] = p[0];
    } else if constexpr (N == 2) {
      floatx2 t = *reinterpret_cast<const floatx2*>(p);
      v[0] = t[0];
      v[1] = t[1];
    } else {
#pragma unroll
      for (int q = 0; q < N / 4; ++q) {
        floatx4 t = *reinterpret_cast<const floatx4*>(p + 4 * q);
        v[4 * q + 0] = t[0];
        v[4 * q + 1] = t[1];
        v[4 * q + 2] = t[2];
        v[4 * q + 3] = t[3];
      }
    }
  }
  // Non-temporal variant for once-read gathered rows: measured +16% on
  // random 64-B rows (scripts/diag_gather_bw.py, 2.85 -> 3.3 TB/s).
  __device__ __forceinline__ void load_nt(const float* p) {
    if constexpr (N == 1) {
      v[0] = __builtin_nontemporal_load(p);
    } else if constexpr (N == 2) {
      floatx2 t = __builtin_nontemporal_load(reinterpret_cast<const floatx2*>(p));
      v[0] = t[0];
      v[1] = t[1];
    } else {
#pragma unroll
      for (int q = 0; q < N / 4; ++q) {
        floatx4 t = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p + 4 * q));
        v[4 * q + 0] = t[0];
        v[4 * q + 1] = t[1];
        v[4 * q + 2] = t[2];
        v[4 * q + 3] = t[3];
      }
    }
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = 0.f;
  }
};

// Sorted-segment helpers for the deterministic scatter-adds (embedding SGD,
// FM training, dedup gradients): the end of key r's segment starting at p
// (binary search: keys are sorted), and the segment's sum of get(q) with 8
// independent partial sums (q mod 8 in segment order) combined in a fixed
// tree — a hot row's thousands of duplicates keep 8 loads in flight instead
// of one, and the result is the same on every run.
__device__ __forceinline__ int64_t seg_end(const uint32_t* __restrict__ key, int64_t p, int64_t n, uint32_t r) {
  int64_t lo = p + 1, hi = n;  // first q > p with key[q] != r
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key[mid] == r) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
template <class G>
__device__ __forceinline__ float seg_sum8(int64_t p, int64_t e, G get) {
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t q = p;
  for (; q + 8 <= e; q += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += get(q + u);
  }
  for (int u = 0; q < e; ++q, ++u) a[u] += get(q);
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}
// The same with U (a power of two >= 8) partial sums: U loads in flight per
// round for sums whose every term is a dependent gather (index, then value);
// the partials combined in a fixed pairwise tree.
template <int U, class G>
__device__ __forceinline__ float seg_sum_u(int64_t p, int64_t e, G get) {
  if constexpr (U == 8) {
    return seg_sum8(p, e, get);
  } else {
    float a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = 0.f;
    int64_t q = p;
    for (; q + U <= e; q += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = get(q + u);
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] += v[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q + u < e) a[u] += get(q + u);
#pragma unroll
    for (int w = U / 2; w >= 1; w >>= 1)
#pragma unroll
      for (int u = 0; u < w; ++u) a[u] = a[u] + a[u + w];
    return a[0];
  }
}

// Chunked segment sums over sorted keys (row-sparse SGD with hot rows): a
// segment is cut into PIECES at the fixed chunk boundaries (multiples of C
// sorted positions); each piece is summed in position order (seg_sum8) and a
// segment's pieces are added in chunk order, so the sum is bitwise
// reproducible and a row with 10^5 duplicates costs C/8 + (#chunks)/8
// dependent steps instead of 10^5/8.  One lane per (position p, column f) of
// W columns; key 0xffffffff = skip.
//  seg_piece: true (with r and the whole sum) when p heads a segment inside
//   one chunk; a piece of a crossing segment goes to part_last[chunk] (its
//   head piece) or part_first[chunk] (the piece starting at the chunk start);
//  seg_cross (after every seg_piece): true (with r and the sum) when p heads a
//   crossing segment.
__device__ __forceinline__ int64_t seg_end_in(const uint32_t* __restrict__ key, int64_t p, int64_t hi, uint32_t r) {
  int64_t lo = p + 1;  // first q in (p, hi) with key[q] != r, else hi
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key[mid] == r) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
template <int U = 8, class G>
__device__ __forceinline__ bool seg_piece(const uint32_t* __restrict__ key, int64_t n, int64_t C, int64_t p, int W,
                                          int f, G get, float* __restrict__ part_first,
                                          float* __restrict__ part_last, uint32_t& r, float& sum) {
  r = key[p];
  if (r == 0xffffffffu) return false;
  const bool head = p == 0 || key[p - 1] != r;
  const int64_t c = p / C;
  if (!head && p != c * C) return false;
  const int64_t cend = (c + 1) * C < n ? (c + 1) * C : n;
  const int64_t e = seg_end_in(key, p, cend, r);
  const float s = seg_sum_u<U>(p, e, get);
  const bool crosses = e == cend && cend < n && key[cend] == r;
  if (head && !crosses) {
    sum = s;
    return true;
  }
  (head ? part_last : part_first)[c * W + f] = s;
  return false;
}
__device__ __forceinline__ bool seg_cross(const uint32_t* __restrict__ key, int64_t n, int64_t C, int64_t p, int W,
                                          int f, const float* __restrict__ part_first,
                                          const float* __restrict__ part_last, uint32_t& r, float& sum) {
  r = key[p];
  if (r == 0xffffffffu || (p > 0 && key[p - 1] == r)) return false;
  const int64_t c0 = p / C, cend = (c0 + 1) * C;
  if (cend >= n || key[cend] != r) return false;  // ends inside its chunk (keys are sorted)
  const int64_t c1 = (seg_end(key, cend, n, r) - 1) / C;
  sum = part_last[c0 * W + f] + seg_sum8(c0 + 1, c1 + 1, [&](int64_t c) { return part_first[c * W + f]; });
  return true;
}
// chunk length for W columns: >= 4W so the partials (2W floats per chunk,
// only when n > C) fit in n floats
inline int64_t seg_chunk(int W) {
  int64_t C = 256;
  while (C < 4 * (int64_t)W) C <<= 1;
  return C;
}

// Sum over the 16 lanes of a DPP row (lanes 16r..16r+15); every lane of the
// row receives the total.  Four row_ror steps, VALU only.
__device__ __forceinline__ float row16_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));
  return x;
}

__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

}  // namespace rs
