// Diagnostic only (never linked into librs_hip.so): the library radix sort the
// product used before round 3, for a same-box timing comparison with
// rs_sort_pairs_u32 (scripts/ab_sort.py).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

extern "C" int64_t diag_hipcub_sort_bytes(int64_t n) {
  size_t sb = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sb, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)n);
  return (int64_t)sb;
}

extern "C" int diag_hipcub_sort(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout, int64_t n,
                                int bits, void* ws, int64_t ws_bytes, void* stream) {
  size_t sb = (size_t)ws_bytes;
  return (int)hipcub::DeviceRadixSort::SortPairs(ws, sb, kin, kout, vin, vout, (int)n, 0, bits,
                                                 (hipStream_t)stream);
}
