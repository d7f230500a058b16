// a2 — 2-D max pooling of the image branch (the ResNet stem's 3x3/2 pad-1
// max-pool; the reference's conv blocks pool with nn.MaxPool2d,
// src/models/cub200_cnn.py:71-77 template), forward and backward, over the
// independent H x W planes of the engine's [K][C][B][H][W] activations.
//
// torch's CPU kernel (aten/src/ATen/native/cpu/MaxPoolKernel.cpp) is restated:
// the window is scanned row-major over its in-bounds elements and the first
// element with (v > max || isnan(v)) wins, starting from max = -inf; the
// backward adds each window's gradient to its argmax in output-raster order,
// so an input element shared by several windows sums their gradients in the
// same order (bit-identical, no atomics).
//
// Forward: one lane per output; the argmax is kept as a 1-byte window offset
// (kh*KW + kw).  Backward: one lane per INPUT element, gathering from the <=
// ceil(KH/S)*ceil(KW/S) windows that contain it, in raster order.  Planes are
// staged through LDS (H*W <= 4096).
#include "conv_common.h"

#include <algorithm>

namespace flr {
namespace pool {

constexpr int THREADS = 256;

struct PoolGeom {
  int H, W, Ho, Wo, KH, KW, S, P;
  conv::FastDiv d_hw, d_w, d_howo, d_wo;  // 32-bit index math (total < 2^31)
};

// A workgroup owns PPB consecutive planes (PPB * H * W <= LDS_FLOATS): the
// planes are staged in LDS with coalesced loads, every window / scatter is
// evaluated from LDS, and the results leave with coalesced stores.
constexpr int LDS_FLOATS = 4096;

// SC: the stride as a compile-time constant (1, 2: divisions become shifts) or 0
// (runtime g.S) — the backward's per-element window ranges are its VALU cost.
template <int SC>
__device__ __forceinline__ void window_range(int i, int P, int K, int Sr, int n_out, int& lo, int& hi) {
  const int S = SC ? SC : Sr;
  // outputs o with o*S - P <= i <= o*S - P + K - 1
  const int a = i + P - K + 1;  // o*S >= a
  lo = a <= 0 ? 0 : (a + S - 1) / S;
  hi = min(n_out - 1, (i + P) / S);
}

__global__ __launch_bounds__(THREADS) void fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                      uint8_t* __restrict__ arg, int64_t nplanes, int ppb,
                                                      PoolGeom g) {
  __shared__ float xs[LDS_FLOATS];
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int np = (int)min((int64_t)ppb, nplanes - p0);
  const int HW = g.H * g.W, HoWo = g.Ho * g.Wo;
  const float* xb = x + p0 * HW;
  for (int e = threadIdx.x; e < np * HW; e += THREADS) xs[e] = xb[e];
  __syncthreads();
  float* yb = y + p0 * HoWo;
  uint8_t* ab = arg + p0 * HoWo;
  for (int o = threadIdx.x; o < np * HoWo; o += THREADS) {
    const int pl = (int)conv::udiv(o, g.d_howo), q = o - pl * HoWo;
    const int oh = (int)conv::udiv(q, g.d_wo), ow = q - oh * g.Wo;
    const float* xp = xs + pl * HW;
    const int ih0 = oh * g.S - g.P, iw0 = ow * g.S - g.P;
    float best = -__builtin_huge_valf();
    int bi = -1;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = ih0 + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = iw0 + kw;
        if (iw < 0 || iw >= g.W) continue;
        const float v = xp[ih * g.W + iw];
        if (bi < 0) bi = kh * g.KW + kw;  // torch's initial maxindex: the first in-bounds element
        if (v > best || v != v) {
          best = v;
          bi = kh * g.KW + kw;
        }
      }
    }
    yb[o] = best;
    ab[o] = (uint8_t)bi;
  }
}

template <int SC>
__global__ __launch_bounds__(THREADS) void bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                      float* __restrict__ dx, int64_t nplanes, int ppb, PoolGeom g) {
  __shared__ __attribute__((aligned(16))) float ds[LDS_FLOATS];
  __shared__ __attribute__((aligned(16))) uint8_t as[LDS_FLOATS];
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int np = (int)min((int64_t)ppb, nplanes - p0);
  const int HW = g.H * g.W, HoWo = g.Ho * g.Wo;
  const int nin = np * HoWo;
  const float* dyb = dy + p0 * HoWo;
  const uint8_t* ab = arg + p0 * HoWo;
  if (((p0 * HoWo) & 3) == 0 && (nin & 3) == 0) {  // 16-B dy / 4-B argmax loads
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    for (int o = threadIdx.x; o < nin / 4; o += THREADS) {
      reinterpret_cast<f32x4*>(ds)[o] = reinterpret_cast<const f32x4*>(dyb)[o];
      reinterpret_cast<uint32_t*>(as)[o] = reinterpret_cast<const uint32_t*>(ab)[o];
    }
  } else {
    for (int o = threadIdx.x; o < nin; o += THREADS) {
      ds[o] = dyb[o];
      as[o] = ab[o];
    }
  }
  __syncthreads();
  float* xb = dx + p0 * HW;
  for (int e = threadIdx.x; e < np * HW; e += THREADS) {
    const int pl = (int)conv::udiv(e, g.d_hw), q = e - pl * HW;
    const int ih = (int)conv::udiv(q, g.d_w), iw = q - ih * g.W;
    int oh_lo, oh_hi, ow_lo, ow_hi;
    window_range<SC>(ih, g.P, g.KH, g.S, g.Ho, oh_lo, oh_hi);
    window_range<SC>(iw, g.P, g.KW, g.S, g.Wo, ow_lo, ow_hi);
    const float* dp = ds + pl * HoWo;
    const uint8_t* ap = as + pl * HoWo;
    float acc = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = ih - (oh * (SC ? SC : g.S) - g.P);
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = iw - (ow * (SC ? SC : g.S) - g.P);
        if (ap[oh * g.Wo + ow] == kh * g.KW + kw) acc = add_rn(acc, dp[oh * g.Wo + ow]);
      }
    }
    xb[e] = acc;
  }
}

// 3x3 / stride 2 / pad 1 (the ResNet stem pool): one thread per 2x2 input
// block (2m .. 2m+1, 2n .. 2n+1).  Window (oh, ow) covers rows 2oh-1 .. 2oh+1,
// so only windows (m .. m+1, n .. n+1) reach the block; their gradients are
// added to the block's four accumulators in window-raster order — the order of
// the generic gather, so the result is bit-identical.
__global__ __launch_bounds__(THREADS) void bwd_k3s2p1_kernel(const float* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg, float* __restrict__ dx,
                                                             int64_t nplanes, int ppb, PoolGeom g) {
  __shared__ __attribute__((aligned(16))) float ds[LDS_FLOATS];
  __shared__ __attribute__((aligned(16))) uint8_t as[LDS_FLOATS];
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int np = (int)min((int64_t)ppb, nplanes - p0);
  const int HW = g.H * g.W, HoWo = g.Ho * g.Wo;
  const int nin = np * HoWo;
  const float* dyb = dy + p0 * HoWo;
  const uint8_t* ab = arg + p0 * HoWo;
  if (((p0 * HoWo) & 3) == 0 && (nin & 3) == 0) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    for (int o = threadIdx.x; o < nin / 4; o += THREADS) {
      reinterpret_cast<f32x4*>(ds)[o] = reinterpret_cast<const f32x4*>(dyb)[o];
      reinterpret_cast<uint32_t*>(as)[o] = reinterpret_cast<const uint32_t*>(ab)[o];
    }
  } else {
    for (int o = threadIdx.x; o < nin; o += THREADS) {
      ds[o] = dyb[o];
      as[o] = ab[o];
    }
  }
  __syncthreads();
  const int Hb = (g.H + 1) >> 1, Wb = (g.W + 1) >> 1, nb = Hb * Wb;
  float* xb = dx + p0 * HW;
  for (int e = threadIdx.x; e < np * nb; e += THREADS) {
    const int pl = e / nb, q = e - pl * nb;
    const int m = q / Wb, n = q - m * Wb;
    const float* dp = ds + pl * HoWo;
    const uint8_t* ap = as + pl * HoWo;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};  // (2m, 2n), (2m, 2n+1), (2m+1, 2n), (2m+1, 2n+1)
#pragma unroll
    for (int w = 0; w < 4; ++w) {  // windows in raster order
      const int oh = m + (w >> 1), ow = n + (w & 1);
      if (oh >= g.Ho || ow >= g.Wo) continue;
      const int a = ap[oh * g.Wo + ow];
      const int kh = a / 3, kw = a - 3 * kh;
      const int dh = 2 * oh - 1 + kh - 2 * m, dw = 2 * ow - 1 + kw - 2 * n;  // argmax relative to the block
      if (dh < 0 || dh > 1 || dw < 0 || dw > 1) continue;
      acc[2 * dh + dw] = add_rn(acc[2 * dh + dw], dp[oh * g.Wo + ow]);
    }
    float* xp = xb + (int64_t)pl * HW;
    const int ih = 2 * m, iw = 2 * n;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      if (ih + dh >= g.H) continue;
      float* row = xp + (ih + dh) * g.W + iw;
      row[0] = acc[2 * dh];
      if (iw + 1 < g.W) row[1] = acc[2 * dh + 1];
    }
  }
}

inline bool geom(int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t S, int64_t P, PoolGeom& g) {
  if (H < 1 || W < 1 || KH < 1 || KW < 1 || S < 1 || P < 0 || 2 * P > KH || 2 * P > KW || KH * KW > 255)
    return false;
  g.H = (int)H; g.W = (int)W; g.KH = (int)KH; g.KW = (int)KW; g.S = (int)S; g.P = (int)P;
  g.Ho = (int)((H + 2 * P - KH) / S + 1);
  g.Wo = (int)((W + 2 * P - KW) / S + 1);
  if (g.Ho < 1 || g.Wo < 1) return false;
  g.d_hw = conv::make_fastdiv((uint32_t)(H * W));
  g.d_w = conv::make_fastdiv((uint32_t)W);
  g.d_howo = conv::make_fastdiv((uint32_t)(g.Ho * g.Wo));
  g.d_wo = conv::make_fastdiv((uint32_t)g.Wo);
  return true;
}

}  // namespace pool
}  // namespace flr

using namespace flr;

extern "C" int flr_maxpool2d_fwd(const float* x, float* y, uint8_t* argmax, int64_t nplanes, int64_t H, int64_t W,
                                 int64_t KH, int64_t KW, int64_t stride, int64_t pad, void* stream) {
  pool::PoolGeom g;
  if (!x || !y || !argmax || nplanes < 0 || !pool::geom(H, W, KH, KW, stride, pad, g)) return FLR_ERR_ARG;
  if (H * W > pool::LDS_FLOATS) return FLR_ERR_UNSUPPORTED;
  if (nplanes == 0) return FLR_OK;
  const int ppb = (int)std::max<int64_t>(1, std::min<int64_t>(pool::LDS_FLOATS / (H * W), 64));
  hipLaunchKernelGGL(pool::fwd_kernel, dim3((unsigned)((nplanes + ppb - 1) / ppb)), dim3(pool::THREADS), 0,
                     as_stream(stream), x, y, argmax, nplanes, ppb, g);
  return launch_status("maxpool fwd");
}

extern "C" int flr_maxpool2d_bwd(const float* dy, const uint8_t* argmax, float* dx, int64_t nplanes, int64_t H,
                                 int64_t W, int64_t KH, int64_t KW, int64_t stride, int64_t pad, void* stream) {
  pool::PoolGeom g;
  if (!dy || !dx || !argmax || nplanes < 0 || !pool::geom(H, W, KH, KW, stride, pad, g)) return FLR_ERR_ARG;
  if (H * W > pool::LDS_FLOATS) return FLR_ERR_UNSUPPORTED;
  if (nplanes == 0) return FLR_OK;
  const int ppb = (int)std::max<int64_t>(1, std::min<int64_t>(pool::LDS_FLOATS / (H * W), 64));
  auto kern = stride == 2 ? pool::bwd_kernel<2> : stride == 1 ? pool::bwd_kernel<1> : pool::bwd_kernel<0>;
  if (KH == 3 && KW == 3 && stride == 2 && pad == 1) kern = pool::bwd_k3s2p1_kernel;
  hipLaunchKernelGGL(kern, dim3((unsigned)((nplanes + ppb - 1) / ppb)), dim3(pool::THREADS), 0, as_stream(stream), dy,
                     argmax, dx, nplanes, ppb, g);
  return launch_status("maxpool bwd");
}
