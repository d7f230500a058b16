// §8(f) rank 3 — per-round evaluation of the global model and the backdoor
// attack-success rate, forward-only on the training kernels.
//
// Reference: evaluate_model (src/utils/metrics.py:14-59: model.eval(), mean
// cross-entropy per test batch, predicted = torch.max(outputs, 1)),
// compute_attack_success_rate (:62-98: share of triggered samples predicted as
// the target class) and compute_label_flip_asr (:101-157), called after every
// round and at the end of run_simulation (run_experiments.py:262, 281-291).
// Two pieces are new relative to training:
//   * BatchNorm in eval mode: running statistics instead of batch statistics
//     (alpha = gamma / sqrt(running_var + eps), y = x*alpha + (beta -
//     running_mean*alpha), the formulas of torch's inference path), with the
//     block's residual add and ReLU fused as in the training kernel;
//   * a row classifier: the first index of the maximum logit (NaN counts as
//     the maximum, as torch.max) and the row's cross-entropy, plus integer
//     tallies (atomics on integers: exact and order-independent).
#include "flr_common.h"

#include <algorithm>

namespace flr {
namespace evalk {

constexpr int THREADS = 256;

// grid (chunks, KC): plane kc = n contiguous values.
template <bool RELU, bool RES>
__global__ __launch_bounds__(THREADS) void bn_infer_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ rmean,
                                                           const float* __restrict__ rvar, const float* __restrict__ res,
                                                           float* __restrict__ y, int64_t n, float eps) {
  const int64_t kc = blockIdx.y;
  const float invstd = 1.0f / sqrtf(rvar[kc] + eps);
  const float alpha = invstd * gamma[kc];
  const float shift = beta[kc] - rmean[kc] * alpha;
  const int64_t base = kc * n;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS) {
    float v = x[base + i] * alpha + shift;
    if constexpr (RES) v = v + res[base + i];
    if constexpr (RELU) v = fmaxf(v, 0.f);
    y[base + i] = v;
  }
}

// torch.max's order on (value, index): NaN beats every number, ties go to the
// lower index.
__device__ __forceinline__ bool beats(float v, int i, float b, int bi) {
  const bool vn = v != v, bn = b != b;
  if (vn || bn) return vn && (!bn || i < bi);
  return v > b || (v == b && i < bi);
}

// One wave per row of logits [R][C].
__global__ __launch_bounds__(THREADS) void classify_kernel(const float* __restrict__ logits,
                                                           const int64_t* __restrict__ labels, int R, int C,
                                                           int64_t target, int64_t source, int32_t* __restrict__ pred,
                                                           float* __restrict__ loss_rows,
                                                           unsigned long long* __restrict__ counts) {
  const int r = blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float* z = logits + (int64_t)r * C;
  float best = -__builtin_huge_valf();
  int bi = C;
  for (int c = lane; c < C; c += 64) {
    const float v = z[c];
    if (beats(v, c, best, bi)) {
      best = v;
      bi = c;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (beats(ov, oi, best, bi)) {
      best = ov;
      bi = oi;
    }
  }
  if (bi >= C) bi = 0;  // a row of -inf: torch returns index 0
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += expf(z[c] - best);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
  if (lane != 0) return;
  pred[r] = bi;
  atomicAdd(&counts[1], (unsigned long long)(bi == target));
  if (labels) {
    const int64_t y = labels[r];
    loss_rows[r] = best + logf(se) - z[y];
    atomicAdd(&counts[0], (unsigned long long)(bi == y));
    atomicAdd(&counts[2], (unsigned long long)(y == source));
    atomicAdd(&counts[3], (unsigned long long)(y == source && bi == y));
    atomicAdd(&counts[4], (unsigned long long)(y == source && bi == target));
  }
}

}  // namespace evalk
}  // namespace flr

using namespace flr;

extern "C" int flr_batchnorm_infer(const float* x, const float* gamma, const float* beta, const float* running_mean,
                                   const float* running_var, const float* residual, float* y, int64_t KC, int64_t HW,
                                   float eps, int relu, void* stream) {
  if (!x || !gamma || !beta || !running_mean || !running_var || !y || KC < 1 || KC > 65535 || HW < 1)
    return FLR_ERR_ARG;
  const dim3 grid((unsigned)std::min<int64_t>((HW + evalk::THREADS - 1) / evalk::THREADS, 64), (unsigned)KC);
  hipStream_t st = as_stream(stream);
#define FLR_BNI(R, S)                                                                                          \
  hipLaunchKernelGGL((evalk::bn_infer_kernel<R, S>), grid, dim3(evalk::THREADS), 0, st, x, gamma, beta,      \
                     running_mean, running_var, residual, y, HW, eps)
  if (relu && residual) FLR_BNI(true, true);
  else if (relu) FLR_BNI(true, false);
  else if (residual) FLR_BNI(false, true);
  else FLR_BNI(false, false);
#undef FLR_BNI
  return launch_status("batchnorm infer");
}

extern "C" int flr_classify_rows(const float* logits, const int64_t* labels, int64_t R, int64_t C, int64_t target,
                                 int64_t source, int32_t* pred, float* loss_rows, int64_t* counts, void* stream) {
  if (!logits || !pred || !counts || R < 0 || C < 1 || R >= ((int64_t)1 << 31) || (labels && !loss_rows))
    return FLR_ERR_ARG;
  if (R == 0) return FLR_OK;
  hipLaunchKernelGGL(evalk::classify_kernel, dim3((unsigned)((R + 3) / 4)), dim3(evalk::THREADS), 0,
                     as_stream(stream), logits, labels, (int)R, (int)C, target, source, pred, loss_rows,
                     reinterpret_cast<unsigned long long*>(counts));
  return launch_status("classify rows");
}
