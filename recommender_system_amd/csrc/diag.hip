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
}  // namespace rs

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
