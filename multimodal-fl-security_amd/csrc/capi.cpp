// Library-level C ABI: version, status strings, last-error text.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../include/flr.h"

namespace flr {
static thread_local char g_last_error[256] = "";

void set_last_error(const char* where, hipError_t e) {
  std::snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, hipGetErrorString(e));
}
}  // namespace flr

extern "C" const char* flr_version(void) { return "flr 0.1.0 gfx950"; }

extern "C" const char* flr_last_error(void) { return flr::g_last_error; }

extern "C" const char* flr_status_string(int status) {
  switch (status) {
    case FLR_OK: return "ok";
    case FLR_ERR_ARG: return "invalid argument";
    case FLR_ERR_HIP: return "HIP runtime error";
    case FLR_ERR_UNSUPPORTED: return "unsupported shape";
    case FLR_ERR_WORKSPACE: return "workspace too small or misaligned";
    case FLR_ERR_KRUM_N: return "Krum requires n >= 2f + 3";
    default: return "unknown status";
  }
}
