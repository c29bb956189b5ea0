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

// option values and their valid ranges [lo, hi]
// Per host thread (rs_capi.h): a thread's setting changes only the launches
// that thread makes, so concurrent callers never see each other's choices.
// defaults: K-split headline kernel, unrolled towers, split-role DeepFM, one-launch DIN attention,
// lean peer-exchange ordering, register contraction in embed_cross
static thread_local int g_opt[RS_OPT_COUNT] = {0, 1, 0, 0, 0, 0};
static const int g_opt_hi[RS_OPT_COUNT] = {3, 1, 3, 1, 1, 1};
int opt(int option) { return (option >= 0 && option < RS_OPT_COUNT) ? g_opt[option] : 0; }
}  // namespace rs

extern "C" int rs_set_option(int option, int value) {
  if (option < 0 || option >= RS_OPT_COUNT || value < 0 || value > rs::g_opt_hi[option]) {
    rs::set_error("rs_set_option: unknown option %d or value %d out of range", option, value);
    return -1;
  }
  const int prev = rs::g_opt[option];
  rs::g_opt[option] = value;
  return prev;
}

extern "C" int rs_get_option(int option) {
  return (option >= 0 && option < RS_OPT_COUNT) ? rs::g_opt[option] : -1;
}

extern "C" const char* rs_version(void) { return "recommender_system_amd 0.1.0 (gfx950)"; }
extern "C" const char* rs_last_error_string(void) { return rs::g_err; }
