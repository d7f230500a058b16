// a2 — per-client BatchNorm (training mode) with the ReLU and the residual add
// of the ResNet blocks fused in, forward and backward.
//
// Reference layers: nn.BatchNorm2d in train mode inside the conv blocks
// (src/models/cub200_cnn.py:71-77 template; ResNet-18 BasicBlock here) —
// batch statistics only; running stats are not parameters() and are never
// aggregated (run_experiments.py:238, 258).  torch's CPU kernels
// (batch_norm_cpu_update_stats / transform_input / backward) are restated:
//   mean = sum(x)/n   var = sum((x-mean)^2)/n   invstd = 1/sqrt(var + eps)
//   alpha = invstd*gamma   shift = beta - mean*alpha   y = x*alpha + shift
//   backward: s = sum(g), d = sum((x-mean) g), kk = d invstd^2 / n,
//   dx = (g - s/n - (x-mean) kk) invstd gamma,  dgamma = d invstd,  dbeta = s
// Fused: out = relu(y [+ residual]); backward takes g = dout * (out > 0) and
// also returns g as the residual branch's gradient.
//
// Layout: the grouped activation tensor x[b][kc][hw] (kc = client*C + channel,
// n = B*HW values per plane).  One wave owns 64/seg planes, seg = min(HW, 64)
// lanes per plane, so every load instruction reads 64 consecutive floats of
// one batch row; per-plane sums are xor-shuffle reductions inside the segment.
// Three passes over x (sum, centred sum of squares, write); passes 2-3 re-read
// the wave's few KB from cache.
#include "flr_common.h"

namespace flr {
namespace bn {

constexpr int THREADS = 256;

struct Plane {
  int64_t base;  // offset of (b = 0, kc, hw = hw0)
  int64_t bstride;
  int HW, seg, hw0;
  bool valid;
};

__device__ __forceinline__ Plane plane_of(int B, int KC, int HW, int seg_log2, int& kc) {
  const int wave = blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  Plane p;
  p.seg = 1 << seg_log2;
  p.HW = HW;
  p.hw0 = lane & (p.seg - 1);
  kc = wave * (64 >> seg_log2) + (lane >> seg_log2);
  p.valid = kc < KC;
  p.base = (int64_t)kc * HW + p.hw0;
  p.bstride = (int64_t)KC * HW;
  return p;
}

__device__ __forceinline__ float seg_sum(float v, int seg) {
  for (int o = seg >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <bool RELU, bool RES>
__global__ __launch_bounds__(THREADS) void fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float* __restrict__ res,
                                                      float* __restrict__ y, float* __restrict__ mean_out,
                                                      float* __restrict__ invstd_out, int B, int KC, int HW,
                                                      int seg_log2, float eps) {
  int kc;
  const Plane p = plane_of(B, KC, HW, seg_log2, kc);
  const float n = (float)B * (float)HW;
  float s = 0.f;
  if (p.valid)
    for (int b = 0; b < B; ++b)
      for (int hw = 0; hw + p.hw0 < HW; hw += p.seg) s += x[b * p.bstride + p.base + hw];
  const float mean = seg_sum(s, p.seg) / n;
  float q = 0.f;
  if (p.valid)
    for (int b = 0; b < B; ++b)
      for (int hw = 0; hw + p.hw0 < HW; hw += p.seg) {
        const float d = x[b * p.bstride + p.base + hw] - mean;
        q += d * d;
      }
  const float var = seg_sum(q, p.seg) / n;
  if (!p.valid) return;
  const float invstd = 1.0f / sqrtf(var + eps);
  const float alpha = invstd * gamma[kc];
  const float shift = beta[kc] - mean * alpha;
  for (int b = 0; b < B; ++b)
    for (int hw = 0; hw + p.hw0 < HW; hw += p.seg) {
      const int64_t i = b * p.bstride + p.base + hw;
      float v = x[i] * alpha + shift;
      if constexpr (RES) v = v + res[i];
      if constexpr (RELU) v = fmaxf(v, 0.f);
      y[i] = v;
    }
  if (p.hw0 == 0) {
    mean_out[kc] = mean;
    invstd_out[kc] = invstd;
  }
}

template <bool RELU, bool DRES>
__global__ __launch_bounds__(THREADS) void bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                      const float* __restrict__ y, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ invstd_in, float* __restrict__ dx,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                      float* __restrict__ dres, int B, int KC, int HW,
                                                      int seg_log2) {
  int kc;
  const Plane p = plane_of(B, KC, HW, seg_log2, kc);
  const float n = (float)B * (float)HW;
  const float mean = p.valid ? mean_in[kc] : 0.f;
  float s = 0.f, d = 0.f;
  if (p.valid)
    for (int b = 0; b < B; ++b)
      for (int hw = 0; hw + p.hw0 < HW; hw += p.seg) {
        const int64_t i = b * p.bstride + p.base + hw;
        float g = dy[i];
        if constexpr (RELU) g = y[i] > 0.f ? g : 0.f;
        s += g;
        d += (x[i] - mean) * g;
      }
  s = seg_sum(s, p.seg);
  d = seg_sum(d, p.seg);
  if (!p.valid) return;
  const float invstd = invstd_in[kc];
  const float kk = d * invstd * invstd / n;
  const float mdy = s / n;
  const float wscale = invstd * gamma[kc];
  for (int b = 0; b < B; ++b)
    for (int hw = 0; hw + p.hw0 < HW; hw += p.seg) {
      const int64_t i = b * p.bstride + p.base + hw;
      float g = dy[i];
      if constexpr (RELU) g = y[i] > 0.f ? g : 0.f;
      if constexpr (DRES) dres[i] = g;
      dx[i] = (g - mdy - (x[i] - mean) * kk) * wscale;
    }
  if (p.hw0 == 0) {
    dgamma[kc] = d * invstd;
    dbeta[kc] = s;
  }
}

inline int seg_log2_of(int HW) {
  int l = 0;
  while (l < 6 && (1 << (l + 1)) <= HW) ++l;
  return l;  // seg = largest power of two <= min(HW, 64)
}

inline dim3 grid_of(int KC, int seg_log2) {
  const int cpw = 64 >> seg_log2;
  const int waves = (KC + cpw - 1) / cpw;
  return dim3((unsigned)((waves + THREADS / 64 - 1) / (THREADS / 64)));
}

}  // namespace bn
}  // namespace flr

using namespace flr;

extern "C" int flr_batchnorm_fwd(const float* x, const float* gamma, const float* beta, const float* residual,
                                 float* y, float* mean, float* invstd, int64_t B, int64_t KC, int64_t HW, float eps,
                                 int relu, void* stream) {
  if (!x || !gamma || !beta || !y || !mean || !invstd || B < 1 || KC < 1 || HW < 1 ||
      B * KC * HW >= ((int64_t)1 << 31))
    return FLR_ERR_ARG;
  const int sl = bn::seg_log2_of((int)HW);
  const dim3 grid = bn::grid_of((int)KC, sl);
  hipStream_t st = as_stream(stream);
#define FLR_BN_FWD(R, S)                                                                                       \
  hipLaunchKernelGGL((bn::fwd_kernel<R, S>), grid, dim3(bn::THREADS), 0, st, x, gamma, beta, residual, y, mean, \
                     invstd, (int)B, (int)KC, (int)HW, sl, eps)
  if (relu && residual) FLR_BN_FWD(true, true);
  else if (relu) FLR_BN_FWD(true, false);
  else if (residual) FLR_BN_FWD(false, true);
  else FLR_BN_FWD(false, false);
#undef FLR_BN_FWD
  return launch_status("batchnorm fwd");
}

extern "C" int flr_batchnorm_bwd(const float* dy, const float* x, const float* y, const float* gamma,
                                 const float* mean, const float* invstd, float* dx, float* dgamma, float* dbeta,
                                 float* dresidual, int64_t B, int64_t KC, int64_t HW, int relu, void* stream) {
  if (!dy || !x || !gamma || !mean || !invstd || !dx || !dgamma || !dbeta || (relu && !y) || B < 1 || KC < 1 ||
      HW < 1 || B * KC * HW >= ((int64_t)1 << 31))
    return FLR_ERR_ARG;
  const int sl = bn::seg_log2_of((int)HW);
  const dim3 grid = bn::grid_of((int)KC, sl);
  hipStream_t st = as_stream(stream);
#define FLR_BN_BWD(R, D)                                                                                         \
  hipLaunchKernelGGL((bn::bwd_kernel<R, D>), grid, dim3(bn::THREADS), 0, st, dy, x, y, gamma, mean, invstd, dx, \
                     dgamma, dbeta, dresidual, (int)B, (int)KC, (int)HW, sl)
  if (relu && dresidual) FLR_BN_BWD(true, true);
  else if (relu) FLR_BN_BWD(true, false);
  else if (dresidual) FLR_BN_BWD(false, true);
  else FLR_BN_BWD(false, false);
#undef FLR_BN_BWD
  return launch_status("batchnorm bwd");
}
