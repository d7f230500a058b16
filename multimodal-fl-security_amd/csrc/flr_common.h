// Internal helpers shared by the flr HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/flr.h"

namespace flr {

// Records the last HIP error text for flr_last_error().
void set_last_error(const char* where, hipError_t e);

// An A/B switch's value (the FLR_* environment read once at library load, or
// flr_set_knob since), nullptr when unset (capi.cpp).
const char* knob(const char* name);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Checks the launch that was just enqueued.
inline int launch_status(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_last_error(where, e);
    return FLR_ERR_HIP;
  }
  return FLR_OK;
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// fp32 add/mul/div with no contraction (the reference computes each op as a
// separate rounded torch op, so FMA contraction would break bit parity).
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float div_rn(float a, float b) { return __fdiv_rn(a, b); }

// Correctly rounded fp32 sqrt (std::sqrt / torch's sqrt on the CPU).  HIP's
// __fsqrt_rn is the native v_sqrt_f32 (up to 1 ulp off) unless the OCML
// rounded operations are enabled, so the candidate is checked against the
// rounding midpoints in fp64 (exact: a midpoint has 25 significant bits, its
// square at most 50) and moved by one ulp when needed.
__device__ __forceinline__ float sqrt_rn(float s) {
  float r = __builtin_sqrtf(s);
  if (!(s > 0.f) || !(r < __builtin_huge_valf())) return r;  // 0, negative, NaN, inf
  const uint32_t u = __float_as_uint(r);
  const float up = __uint_as_float(u + 1), dn = __uint_as_float(u - 1);
  const double sd = (double)s, rd = (double)r;
  const double hi = 0.5 * (rd + (double)up);
  if (sd > hi * hi) return up;
  const double lo = 0.5 * (rd + (double)dn);
  if (sd < lo * lo) return dn;
  return r;
}

}  // namespace flr
