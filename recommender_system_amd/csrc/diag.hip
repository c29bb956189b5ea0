// diag.hip — measurement helpers of the C-ABI (rs_capi.h "Diagnostic").
#include "rs_common.hpp"

namespace rs {
__global__ void diag_empty_kernel() {}
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
