// diag.hip — measurement helpers of the C-ABI (rs_capi.h "Diagnostic").
#include "rs_common.hpp"

namespace rs {
__global__ void diag_empty_kernel() {}

// Each wave's lane 0 records the HW_ID register (wave slot, SIMD, CU, SE ...):
// which SIMD each wave of a workgroup lands on.
__global__ void diag_wave_slots_kernel(uint32_t* out) {
  extern __shared__ float lds_hold[];
  const int w = threadIdx.x >> 6;
  // s_getreg HW_REG_HW_ID (id 4), all 32 bits
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  if ((threadIdx.x & 63) == 0) {
    lds_hold[w] = 0.f;
    out[(int64_t)blockIdx.x * (blockDim.x >> 6) + w] = hw;
  }
}

// MFMA issue timing: every wave runs n v_mfma_f32_16x16x4_f32 as `chains`
// independent accumulation chains (1, 2 or 4); lane 0 records its start and
// end s_memtime and its HW_ID, cyc[3 wave + {0, 1, 2}] — the host groups the
// waves by (workgroup, SIMD) and divides each SIMD's window (first start to
// last end) by the MFMAs issued on it.  (Round 4 divided one wave's own
// window by the waves per SIMD, which assumed the waves ran in perfect
// overlap and read faster than the 32-cycle issue rate.)
__global__ void diag_mfma_chain_kernel(int n, int chains, unsigned long long* cyc, float* sink) {
  const int lane = threadIdx.x & 63;
  float a = 1.0f + lane * 1e-3f, b = 0.5f - lane * 1e-3f;
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_REG_HW_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (chains == 4) {
    for (int i = 0; i < n; i += 4) {
      c0 = mfma16x16x4(a, b, c0);
      c1 = mfma16x16x4(a, b, c1);
      c2 = mfma16x16x4(a, b, c2);
      c3 = mfma16x16x4(a, b, c3);
    }
  } else if (chains == 2) {
    for (int i = 0; i < n; i += 2) {
      c0 = mfma16x16x4(a, b, c0);
      c1 = mfma16x16x4(a, b, c1);
    }
  } else {
    for (int i = 0; i < n; ++i) c0 = mfma16x16x4(a, b, c0);
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) r += c0[i] + c1[i] + c2[i] + c3[i];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (lane == 0) {
    const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    cyc[3 * wv] = t0;
    cyc[3 * wv + 1] = t1;
    cyc[3 * wv + 2] = hw;
  }
}

// Instruction-fetch cost: 2048 FMAs on 8 independent accumulators as a loop
// (8 per iteration, the body stays in the instruction cache) or straight-line
// (fully unrolled, ~8 KB of code); cyc[wave] = {first pass, second pass} of
// the same code in one launch.
template <bool UNROLL>
__global__ void diag_icache_kernel(float x, float y, unsigned long long* cyc, float* sink) {
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = x + i;
  unsigned long long t[3];
  for (int pass = 0; pass < 2; ++pass) {
    t[pass] = __builtin_amdgcn_s_memtime();
    if constexpr (UNROLL) {
#pragma unroll
      for (int i = 0; i < 2048; ++i) acc[i & 7] = fmaf(acc[i & 7], x, y);
    } else {
#pragma unroll 1
      for (int i = 0; i < 2048; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(acc[j], x, y);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  t[2] = __builtin_amdgcn_s_memtime();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += acc[i];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) {
    const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    cyc[2 * wv] = t[1] - t[0];
    cyc[2 * wv + 1] = t[2] - t[1];
  }
}
}  // namespace rs

extern "C" int rs_diag_icache(int grid, int block, int unroll, unsigned long long* cyc, float* sink,
                              rs_stream_t stream) {
  if (grid < 1 || block < 64 || block > 1024 || block % 64 || !cyc || !sink) {
    rs::set_error("rs_diag_icache: bad arguments");
    return RS_ERR_ARG;
  }
  if (unroll) rs::diag_icache_kernel<true><<<grid, block, 0, (hipStream_t)stream>>>(1.0001f, 1e-4f, cyc, sink);
  else rs::diag_icache_kernel<false><<<grid, block, 0, (hipStream_t)stream>>>(1.0001f, 1e-4f, cyc, sink);
  return rs::launch_status("rs_diag_icache");
}

extern "C" int rs_diag_mfma_chain(int grid, int block, int n, int chains, unsigned long long* cyc, float* sink,
                                  rs_stream_t stream) {
  if (grid < 1 || block < 64 || block > 1024 || block % 64 || n < 4 || n % 4 || !cyc || !sink ||
      (chains != 1 && chains != 2 && chains != 4)) {
    rs::set_error("rs_diag_mfma_chain: bad arguments");
    return RS_ERR_ARG;
  }
  rs::diag_mfma_chain_kernel<<<grid, block, 0, (hipStream_t)stream>>>(n, chains, cyc, sink);
  return rs::launch_status("rs_diag_mfma_chain");
}

// An empty launch: replayed back to back from a hipGraph it measures the
// dependent-launch slot (dispatch + end-of-kernel + barrier) of the box.
extern "C" int rs_diag_empty(int grid, int block, rs_stream_t stream) {
  if (grid < 1 || block < 1 || block > 1024) {
    rs::set_error("rs_diag_empty: grid %d / block %d out of range", grid, block);
    return RS_ERR_ARG;
  }
  rs::diag_empty_kernel<<<grid, block, 0, (hipStream_t)stream>>>();
  return rs::launch_status("rs_diag_empty");
}

// Where the waves of a `block`-thread workgroup run: HW_ID per wave into
// out[grid * block / 64] (lds_bytes of dynamic LDS pins the occupancy).
extern "C" int rs_diag_wave_slots(int grid, int block, int lds_bytes, uint32_t* out, rs_stream_t stream) {
  if (grid < 1 || block < 64 || block > 1024 || block % 64 || lds_bytes < 256 || lds_bytes > 160 * 1024 || !out) {
    rs::set_error("rs_diag_wave_slots: bad arguments");
    return RS_ERR_ARG;
  }
  if (lds_bytes > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)rs::diag_wave_slots_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds_bytes);
  rs::diag_wave_slots_kernel<<<grid, block, lds_bytes, (hipStream_t)stream>>>(out);
  return rs::launch_status("rs_diag_wave_slots");
}
