// capi.cpp — version / error plumbing of the C-ABI (rs_capi.h).
#include <stdarg.h>
#include <stdio.h>

#include "rs_common.hpp"

namespace rs {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  return RS_OK;
}
}  // namespace rs

extern "C" const char* rs_version(void) { return "recommender_system_amd 0.1.0 (gfx950)"; }
extern "C" const char* rs_last_error_string(void) { return rs::g_err; }
