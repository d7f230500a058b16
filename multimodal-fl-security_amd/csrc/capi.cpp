// Library-level C ABI: version, build flags, status strings, last-error text,
// and the A/B switch registry.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

#include <unistd.h>

#include "../../include/flr.h"

namespace flr {
static thread_local char g_last_error[256] = "";

void set_last_error(const char* where, hipError_t e) {
  std::snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, hipGetErrorString(e));
}
// The A/B switches (FLR_* names): the process environment's FLR_*
// variables are read ONCE, when the library is loaded; afterwards only
// flr_set_knob changes them (an in-process A/B, e.g. a test comparing two
// bit-identical forms).  Kernels and launchers call knob(), never getenv.
namespace {
std::mutex g_knob_mu;
std::unordered_map<std::string, std::string>& knob_table() {
  static std::unordered_map<std::string, std::string> t;
  return t;
}
__attribute__((constructor)) void knobs_from_environment() {
  std::lock_guard<std::mutex> lock(g_knob_mu);
  for (char** e = environ; e && *e; ++e) {
    if (std::strncmp(*e, "FLR_", 4) != 0) continue;
    const char* eq = std::strchr(*e, '=');
    if (eq) knob_table()[std::string(*e, eq - *e)] = std::string(eq + 1);
  }
}
}  // namespace

// The value is copied under the lock into this thread's own table (ADVICE r5:
// a pointer into the shared table dangled when another thread's
// flr_set_knob replaced the entry).  The returned pointer stays valid until
// this thread asks for the same name again.
const char* knob(const char* name) {
  thread_local std::unordered_map<std::string, std::string> copies;
  std::string v;
  {
    std::lock_guard<std::mutex> lock(g_knob_mu);
    auto& t = knob_table();
    auto it = t.find(name);
    if (it == t.end()) return nullptr;
    v = it->second;
  }
  std::string& c = copies[name];
  c = std::move(v);
  return c.c_str();
}
}  // namespace flr

extern "C" int flr_set_knob(const char* name, const char* value) {
  if (!name || std::strncmp(name, "FLR_", 4) != 0) return FLR_ERR_ARG;
  std::lock_guard<std::mutex> lock(flr::g_knob_mu);
  if (value)
    flr::knob_table()[name] = value;
  else
    flr::knob_table().erase(name);
  return FLR_OK;
}

extern "C" const char* flr_version(void) { return "flr 0.1.0 gfx950"; }

extern "C" const char* flr_build_info(void) {
#ifdef FLR_ABLATION
  return "gfx950 ablation";
#else
  return "gfx950";
#endif
}

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
