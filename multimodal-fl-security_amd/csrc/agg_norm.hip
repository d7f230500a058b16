// §8(f) rows 1-2 — per-client norms and general weighted row combinations:
// the building blocks of the norm-based defenses and the geometric median.
//
// Reference call sites:
//   GradientClippingDefense._compute_norm / clip_update
//       (src/defenses/differential_privacy.py:223-256): ||u||_2 or ||u||_inf,
//       u *= clip/norm when norm > clip, then sum(n_i * u_i) / sum(n)
//   NormBoundingDefense.aggregate (:299-334): ||u||_2 in [min, max] filter,
//       then the weighted mean over the kept clients (client order)
//   DPSGDDefense.clip_gradient / aggregate (:74-164): as clipping (+ noise)
//   GeometricMedianDefense.aggregate (src/defenses/trimmed_mean.py:216-251):
//       distances ||u_i - current|| and (w * U).sum(0) / w.sum()
//
// flr_row_norms: ||X_i - v|| per row (v optional), differences rounded to
// fp32 as the reference's `flat - current`, squares summed in fp64 in a fixed
// two-stage order (deterministic, and exact to fp32 output precision; the
// reference's fp32 torch.norm itself drifts ~1e-5..3e-4 relative at 1e6..1e7
// coordinates).  linf is exact.
//
// flr_row_dots: X_i . v per row, exact products summed in fp64 (FLTrust's
// torch.dot, src/defenses/fltrust.py:176).
//
// flr_weighted_rows: out = (sum_j fl(fl(X[r_j] * s_j) * w_j)) / divisor,
// sequential in j from +0 (Python sum() order, each op rounded separately).
#include "flr_common.h"

namespace flr {
namespace norm {

constexpr int THREADS = 256;
constexpr int NBLK = 64;  // partial blocks per row
constexpr int MAXROWS = 4096;

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int TYPE, bool CENTER, bool VEC>
__global__ __launch_bounds__(THREADS) void partial_kernel(const float* __restrict__ X, int64_t P, int64_t ldx,
                                                          const float* __restrict__ v, double* __restrict__ part) {
  __shared__ double red[THREADS / 64];
  const int i = blockIdx.y, b = blockIdx.x;
  const float* x = X + (int64_t)i * ldx;
  double acc = 0.0;
  auto one = [&](float xv, float cv) {
    if constexpr (TYPE == 2) {  // dot with v (exact products, fp64 sum)
      acc += (double)xv * (double)cv;
    } else {
      const float d = CENTER ? xv - cv : xv;
      if constexpr (TYPE == 0) acc += (double)d * (double)d;
      else acc = fmax(acc, (double)fabsf(d));
    }
  };
  if constexpr (VEC) {  // block b: 4-float vectors [nv*b/NBLK, nv*(b+1)/NBLK); last block also the tail
    const int64_t nv = P / 4, q0 = nv * b / NBLK, q1 = nv * (b + 1) / NBLK;
    for (int64_t q = q0 + threadIdx.x; q < q1; q += THREADS) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + 4 * q);
      f32x4 cv = {0.f, 0.f, 0.f, 0.f};
      if constexpr (CENTER) cv = *reinterpret_cast<const f32x4*>(v + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) one(xv[e], cv[e]);
    }
    if (b == NBLK - 1)
      for (int64_t p = 4 * nv + threadIdx.x; p < P; p += THREADS) one(x[p], CENTER ? v[p] : 0.f);
  } else {
    const int64_t p0 = P * b / NBLK, p1 = P * (b + 1) / NBLK;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += THREADS) one(x[p], CENTER ? v[p] : 0.f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double w = __shfl_xor(acc, o, 64);
    acc = TYPE == 1 ? fmax(acc, w) : acc + w;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = red[0];
    for (int w = 1; w < THREADS / 64; ++w) s = TYPE == 1 ? fmax(s, red[w]) : s + red[w];
    part[(int64_t)i * NBLK + b] = s;
  }
}

template <int TYPE>
__global__ void finish_kernel(const double* __restrict__ part, int K, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  double s = part[(int64_t)i * NBLK];
  for (int b = 1; b < NBLK; ++b) s = TYPE == 1 ? fmax(s, part[(int64_t)i * NBLK + b]) : s + part[(int64_t)i * NBLK + b];
  out[i] = TYPE == 0 ? sqrt(s) : s;
}

template <bool ROWS, bool SCALE, bool VEC>
__global__ __launch_bounds__(THREADS) void weighted_rows_kernel(const float* __restrict__ X, int64_t P, int64_t ldx,
                                                                const int32_t* __restrict__ rows, int m,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ s, float divisor,
                                                                float* __restrict__ out) {
  __shared__ int32_t rs[MAXROWS];
  __shared__ float ws[MAXROWS];
  __shared__ float ss[SCALE ? MAXROWS : 1];
  for (int t = threadIdx.x; t < m; t += THREADS) {
    rs[t] = ROWS ? rows[t] : t;
    ws[t] = w[t];
    if constexpr (SCALE) ss[t] = s[t];
  }
  __syncthreads();
  auto term = [&](int t, float x) {
    if constexpr (SCALE) x = mul_rn(x, ss[t]);
    return mul_rn(x, ws[t]);
  };
  if constexpr (VEC) {
    const int64_t nv = P / 4;
    for (int64_t q = (int64_t)blockIdx.x * THREADS + threadIdx.x; q < nv; q += (int64_t)gridDim.x * THREADS) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int t = 0; t < m; ++t) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(X + (int64_t)rs[t] * ldx + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = add_rn(acc[e], term(t, x[e]));
      }
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = div_rn(acc[e], divisor);
      *reinterpret_cast<f32x4*>(out + 4 * q) = o;
    }
    if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {
      const int64_t p = nv * 4 + threadIdx.x;
      float acc = 0.f;
      for (int t = 0; t < m; ++t) acc = add_rn(acc, term(t, X[(int64_t)rs[t] * ldx + p]));
      out[p] = div_rn(acc, divisor);
    }
  } else {
    for (int64_t p = (int64_t)blockIdx.x * THREADS + threadIdx.x; p < P; p += (int64_t)gridDim.x * THREADS) {
      float acc = 0.f;
      for (int t = 0; t < m; ++t) acc = add_rn(acc, term(t, X[(int64_t)rs[t] * ldx + p]));
      out[p] = div_rn(acc, divisor);
    }
  }
}

inline int grid_for(int64_t work) {
  int64_t g = (work + THREADS - 1) / THREADS;
  if (g > 256 * 16) g = 256 * 16;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace norm
}  // namespace flr

using namespace flr;

extern "C" size_t flr_row_norms_workspace(int64_t K) {
  return K < 1 ? 0 : (size_t)K * norm::NBLK * sizeof(double);
}

extern "C" int flr_row_norms(const float* X, int64_t K, int64_t P, int64_t ldx, const float* center, int type,
                             double* out, void* ws, size_t ws_bytes, void* stream) {
  if (K < 1 || P < 0 || ldx < P || !X || !out || (type != 0 && type != 1)) return FLR_ERR_ARG;
  if (!ws || ws_bytes < flr_row_norms_workspace(K)) return FLR_ERR_WORKSPACE;
  if (K > 65535) return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  const dim3 grid(norm::NBLK, (unsigned)K);
  const bool vec = ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(center)) & 15) == 0 && ldx % 4 == 0;
#define FLR_NORM_LAUNCH(T, C, V)                                                                          \
  hipLaunchKernelGGL((norm::partial_kernel<T, C, V>), grid, dim3(norm::THREADS), 0, st, X, P, ldx, center, \
                     part)
  if (type == 0) {
    if (center) { if (vec) FLR_NORM_LAUNCH(0, true, true); else FLR_NORM_LAUNCH(0, true, false); }
    else { if (vec) FLR_NORM_LAUNCH(0, false, true); else FLR_NORM_LAUNCH(0, false, false); }
  } else {
    if (center) { if (vec) FLR_NORM_LAUNCH(1, true, true); else FLR_NORM_LAUNCH(1, true, false); }
    else { if (vec) FLR_NORM_LAUNCH(1, false, true); else FLR_NORM_LAUNCH(1, false, false); }
  }
#undef FLR_NORM_LAUNCH
  int rc = launch_status("row_norms partial");
  if (rc != FLR_OK) return rc;
  const unsigned g = (unsigned)((K + 255) / 256);
  if (type == 0) hipLaunchKernelGGL(norm::finish_kernel<0>, dim3(g), dim3(256), 0, st, part, (int)K, out);
  else hipLaunchKernelGGL(norm::finish_kernel<1>, dim3(g), dim3(256), 0, st, part, (int)K, out);
  return launch_status("row_norms finish");
}

extern "C" int flr_row_dots(const float* X, int64_t K, int64_t P, int64_t ldx, const float* v, double* out,
                            void* ws, size_t ws_bytes, void* stream) {
  if (K < 1 || P < 0 || ldx < P || !X || !v || !out) return FLR_ERR_ARG;
  if (!ws || ws_bytes < flr_row_norms_workspace(K)) return FLR_ERR_WORKSPACE;
  if (K > 65535) return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  const dim3 grid(norm::NBLK, (unsigned)K);
  const bool vec = ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(v)) & 15) == 0 && ldx % 4 == 0;
  if (vec) hipLaunchKernelGGL((norm::partial_kernel<2, true, true>), grid, dim3(norm::THREADS), 0, st, X, P, ldx, v, part);
  else hipLaunchKernelGGL((norm::partial_kernel<2, true, false>), grid, dim3(norm::THREADS), 0, st, X, P, ldx, v, part);
  int rc = launch_status("row_dots partial");
  if (rc != FLR_OK) return rc;
  hipLaunchKernelGGL(norm::finish_kernel<2>, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st, part, (int)K, out);
  return launch_status("row_dots finish");
}

extern "C" int flr_weighted_rows(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows, int64_t m,
                                 const float* weights, const float* scales, float divisor, float* out,
                                 void* stream) {
  if (K < 1 || P < 0 || ldx < P || m < 1 || (!rows && m != K) || m > K || !X || !weights || !out) return FLR_ERR_ARG;
  if (m > norm::MAXROWS) return FLR_ERR_UNSUPPORTED;
  if (P == 0) return FLR_OK;
  hipStream_t st = as_stream(stream);
  const bool vec = ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(out)) & 15) == 0 && ldx % 4 == 0;
  const dim3 grid(norm::grid_for(vec ? P / 4 : P));
#define FLR_WR_LAUNCH(R, S, V)                                                                                  \
  hipLaunchKernelGGL((norm::weighted_rows_kernel<R, S, V>), grid, dim3(norm::THREADS), 0, st, X, P, ldx, rows, \
                     (int)m, weights, scales, divisor, out)
  const bool r = rows != nullptr, s = scales != nullptr;
  if (vec) {
    if (r && s) FLR_WR_LAUNCH(true, true, true);
    else if (r) FLR_WR_LAUNCH(true, false, true);
    else if (s) FLR_WR_LAUNCH(false, true, true);
    else FLR_WR_LAUNCH(false, false, true);
  } else {
    if (r && s) FLR_WR_LAUNCH(true, true, false);
    else if (r) FLR_WR_LAUNCH(true, false, false);
    else if (s) FLR_WR_LAUNCH(false, true, false);
    else FLR_WR_LAUNCH(false, false, false);
  }
#undef FLR_WR_LAUNCH
  return launch_status("weighted_rows_kernel");
}
