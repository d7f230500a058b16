// a11 / a14 — row-subset mean (Multi-Krum) and example-weighted FedAvg.
//
// Both are one pass over the client matrix: HBM-bound, 16-B loads per lane.
// Summation order and rounding restate the reference exactly:
//   Multi-Krum (src/defenses/krum.py:186-190):
//     param_sum = sum(u[param_idx] for u in selected_updates)  # 0 + u0 + u1 ...
//     param_sum / multi_k                                     # IEEE fp32 div
//   FedAvg (src/defenses/base_defense.py:90-95, run_experiments.py:246-254):
//     sum(n_i * u_i for i in clients) / total                 # fp32 mul, add, div
// Python's sum() starts from int 0, so the first add is 0 + u0 (turns -0 into
// +0); that is kept.  Every op is a separately rounded fp32 op (no FMA).
#include "flr_common.h"

#include <algorithm>

namespace flr {
namespace mean {

constexpr int THREADS = 256;
constexpr int MAXROWS = 4096;

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool VEC>
__global__ __launch_bounds__(THREADS) void rows_mean_kernel(const float* __restrict__ X, int64_t P,
                                                            int64_t ldx, const int32_t* __restrict__ rows,
                                                            int m, float fm, float* __restrict__ out,
                                                            uint32_t rmax) {
  __shared__ int32_t rs[MAXROWS];
  // an index outside [0, K) is clamped into range: no out-of-bounds read (flr.h)
  for (int t = threadIdx.x; t < m; t += THREADS) rs[t] = (int32_t)min((uint32_t)rows[t], rmax);
  __syncthreads();
  if constexpr (VEC) {
    const int64_t nv = P / 4;
    for (int64_t v = (int64_t)blockIdx.x * THREADS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * THREADS) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int t = 0; t < m; ++t) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(X + (int64_t)rs[t] * ldx + 4 * v);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = add_rn(acc[e], x[e]);
      }
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = div_rn(acc[e], fm);
      *reinterpret_cast<f32x4*>(out + 4 * v) = o;
    }
    if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {  // scalar tail
      const int64_t p = nv * 4 + threadIdx.x;
      float acc = 0.f;
      for (int t = 0; t < m; ++t) acc = add_rn(acc, X[(int64_t)rs[t] * ldx + p]);
      out[p] = div_rn(acc, fm);
    }
  } else {
    for (int64_t p = (int64_t)blockIdx.x * THREADS + threadIdx.x; p < P; p += (int64_t)gridDim.x * THREADS) {
      float acc = 0.f;
      for (int t = 0; t < m; ++t) acc = add_rn(acc, X[(int64_t)rs[t] * ldx + p]);
      out[p] = div_rn(acc, fm);
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(THREADS) void fedavg_kernel(const float* __restrict__ X, int K, int64_t P,
                                                         int64_t ldx, const int64_t* __restrict__ n,
                                                         float* __restrict__ out) {
  __shared__ float wts[MAXROWS];
  __shared__ float total_f;
  for (int i = threadIdx.x; i < K; i += THREADS) wts[i] = (float)n[i];
  if (threadIdx.x == 0) {
    int64_t tot = 0;
    for (int i = 0; i < K; ++i) tot += n[i];
    total_f = (float)tot;
  }
  __syncthreads();
  const float tf = total_f;
  if constexpr (VEC) {
    const int64_t nv = P / 4;
    for (int64_t v = (int64_t)blockIdx.x * THREADS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * THREADS) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int i = 0; i < K; ++i) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(X + (int64_t)i * ldx + 4 * v);
        const float w = wts[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = add_rn(acc[e], mul_rn(w, x[e]));
      }
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = div_rn(acc[e], tf);
      *reinterpret_cast<f32x4*>(out + 4 * v) = o;
    }
    if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {  // scalar tail
      const int64_t p = nv * 4 + threadIdx.x;
      float acc = 0.f;
      for (int i = 0; i < K; ++i) acc = add_rn(acc, mul_rn(wts[i], X[(int64_t)i * ldx + p]));
      out[p] = div_rn(acc, tf);
    }
  } else {
    for (int64_t p = (int64_t)blockIdx.x * THREADS + threadIdx.x; p < P; p += (int64_t)gridDim.x * THREADS) {
      float acc = 0.f;
      for (int i = 0; i < K; ++i) acc = add_rn(acc, mul_rn(wts[i], X[(int64_t)i * ldx + p]));
      out[p] = div_rn(acc, tf);
    }
  }
}

// rows_mean over a matrix whose dead-tap ranges are not written (the round
// engine's FLR_DEFER_DEAD=2): float4 groups wholly inside a dead range are
// skipped (their rows are never read), then dead_mean_kernel writes those
// coordinates from the global vector — row k's value there is gdead (negated
// for k < nneg), summed in the same order as rows_mean_kernel's: bit-identical
// to the mean of the filled rows.
constexpr int MAXDEAD = 96;
struct DeadRanges {
  int64_t off[MAXDEAD], end[MAXDEAD];
  int n;
};
__global__ __launch_bounds__(THREADS) void rows_mean_live_kernel(const float* __restrict__ X, int64_t P, int64_t ldx,
                                                                 const int32_t* __restrict__ rows, int m, float fm,
                                                                 float* __restrict__ out, uint32_t rmax,
                                                                 const DeadRanges dr) {
  __shared__ int32_t rs[MAXROWS];
  for (int t = threadIdx.x; t < m; t += THREADS) rs[t] = (int32_t)min((uint32_t)rows[t], rmax);
  __syncthreads();
  const int64_t nv = P / 4;
  for (int64_t v = (int64_t)blockIdx.x * THREADS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * THREADS) {
    bool skip = false;
    for (int r = 0; r < dr.n; ++r) skip |= 4 * v >= dr.off[r] && 4 * v + 4 <= dr.end[r];
    if (skip) continue;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < m; ++t) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(X + (int64_t)rs[t] * ldx + 4 * v);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = add_rn(acc[e], x[e]);
    }
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = div_rn(acc[e], fm);
    *reinterpret_cast<f32x4*>(out + 4 * v) = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {  // scalar tail (a dead tail is rewritten below)
    const int64_t p = nv * 4 + threadIdx.x;
    float acc = 0.f;
    for (int t = 0; t < m; ++t) acc = add_rn(acc, X[(int64_t)rs[t] * ldx + p]);
    out[p] = div_rn(acc, fm);
  }
}
// grid (slices, ranges): out[p] of dead range r from gdead[p] and the rows' signs
__global__ __launch_bounds__(THREADS) void dead_mean_kernel(const float* __restrict__ g,
                                                            const int32_t* __restrict__ rows, int m, float fm,
                                                            uint32_t rmax, int nneg, float* __restrict__ out,
                                                            const DeadRanges dr) {
  __shared__ float sg[MAXROWS];
  for (int t = threadIdx.x; t < m; t += THREADS) sg[t] = (int)min((uint32_t)rows[t], rmax) < nneg ? -1.f : 1.f;
  __syncthreads();
  const int r = blockIdx.y;
  for (int64_t p = dr.off[r] + (int64_t)blockIdx.x * THREADS + threadIdx.x; p < dr.end[r];
       p += (int64_t)gridDim.x * THREADS) {
    const float gv = g[p];
    float acc = 0.f;
    for (int t = 0; t < m; ++t) acc = add_rn(acc, gv * sg[t]);  // the row's value: exactly +-gv
    out[p] = div_rn(acc, fm);
  }
}

inline int grid_for(int64_t work) {
  int64_t g = (work + THREADS - 1) / THREADS;
  if (g > 256 * 16) g = 256 * 16;
  return (int)(g < 1 ? 1 : g);
}

inline bool vec_ok(const void* X, int64_t ldx, int64_t P, const void* out) {
  return ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(out)) & 15) == 0 && ldx % 4 == 0;
}

}  // namespace mean
}  // namespace flr

using namespace flr;

extern "C" int flr_rows_mean(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows,
                             int64_t m, int64_t divisor, float* out, void* stream) {
  if (K < 1 || P < 0 || ldx < P || m < 1 || m > K || divisor < 1 || !X || !rows || !out) return FLR_ERR_ARG;
  const float fdiv = (float)divisor;
  if (m > mean::MAXROWS) return FLR_ERR_UNSUPPORTED;
  if (P == 0) return FLR_OK;
  hipStream_t st = as_stream(stream);
  if (mean::vec_ok(X, ldx, P, out)) {
    hipLaunchKernelGGL(mean::rows_mean_kernel<true>, dim3(mean::grid_for(P / 4)), dim3(mean::THREADS), 0, st,
                       X, P, ldx, rows, (int)m, fdiv, out, (uint32_t)(K - 1));
  } else {
    hipLaunchKernelGGL(mean::rows_mean_kernel<false>, dim3(mean::grid_for(P)), dim3(mean::THREADS), 0, st, X,
                       P, ldx, rows, (int)m, fdiv, out, (uint32_t)(K - 1));
  }
  return launch_status("rows_mean_kernel");
}

extern "C" int flr_rows_mean_dead(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows,
                                  int64_t m, int64_t divisor, const int64_t* dead_off, const int64_t* dead_n,
                                  int64_t ndead, const float* gdead, int64_t nneg, float* out, void* stream) {
  if (K < 1 || P < 0 || ldx < P || m < 1 || m > K || divisor < 1 || !X || !rows || !out || ndead < 0 || nneg < 0 ||
      (ndead > 0 && (!dead_off || !dead_n || !gdead)))
    return FLR_ERR_ARG;
  if (m > mean::MAXROWS || ndead > mean::MAXDEAD) return FLR_ERR_UNSUPPORTED;
  mean::DeadRanges dr;
  dr.n = (int)ndead;
  int64_t longest = 0;
  for (int64_t r = 0; r < ndead; ++r) {
    if (dead_off[r] < 0 || dead_n[r] < 0 || dead_off[r] + dead_n[r] > P) return FLR_ERR_ARG;
    dr.off[r] = dead_off[r];
    dr.end[r] = dead_off[r] + dead_n[r];
    longest = std::max(longest, dead_n[r]);
  }
  if (P == 0) return FLR_OK;
  if (!mean::vec_ok(X, ldx, P, out)) return FLR_ERR_ARG;  // the engine's matrix: 16-B rows
  hipStream_t st = as_stream(stream);
  const float fdiv = (float)divisor;
  hipLaunchKernelGGL(mean::rows_mean_live_kernel, dim3(mean::grid_for(P / 4)), dim3(mean::THREADS), 0, st, X, P, ldx,
                     rows, (int)m, fdiv, out, (uint32_t)(K - 1), dr);
  int rc = launch_status("rows_mean_live_kernel");
  if (rc != FLR_OK || ndead == 0 || longest == 0) return rc;
  const int gx = (int)std::min<int64_t>(256, (longest + mean::THREADS - 1) / mean::THREADS);
  hipLaunchKernelGGL(mean::dead_mean_kernel, dim3((unsigned)gx, (unsigned)ndead), dim3(mean::THREADS), 0, st, gdead,
                     rows, (int)m, fdiv, (uint32_t)(K - 1), (int)std::min<int64_t>(nneg, K), out, dr);
  return launch_status("dead_mean_kernel");
}

extern "C" int flr_fedavg(const float* X, int64_t K, int64_t P, int64_t ldx, const int64_t* num_examples,
                          float* out, void* stream) {
  if (K < 1 || P < 0 || ldx < P || !X || !num_examples || !out) return FLR_ERR_ARG;
  if (K > mean::MAXROWS) return FLR_ERR_UNSUPPORTED;
  if (P == 0) return FLR_OK;
  hipStream_t st = as_stream(stream);
  if (mean::vec_ok(X, ldx, P, out)) {
    hipLaunchKernelGGL(mean::fedavg_kernel<true>, dim3(mean::grid_for(P / 4)), dim3(mean::THREADS), 0, st, X,
                       (int)K, P, ldx, num_examples, out);
  } else {
    hipLaunchKernelGGL(mean::fedavg_kernel<false>, dim3(mean::grid_for(P)), dim3(mean::THREADS), 0, st, X,
                       (int)K, P, ldx, num_examples, out);
  }
  return launch_status("fedavg_kernel");
}
