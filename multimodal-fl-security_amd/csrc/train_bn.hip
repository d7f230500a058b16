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

// ---- register-resident fast path -------------------------------------------------
// The engine's layout hands every (client, channel) plane over as one contiguous
// run (B == 1).  When that run is n = 4 * L * V floats (L lanes per plane: a
// power of two <= 64, or 256 = the whole workgroup; V float4s per lane, <= 8),
// each value is read from HBM once as part of a 16-B load, kept in registers
// through the centred second pass and the normalisation, and written once
// (the general kernels above make three passes).  Per-plane sums: xor shuffles
// inside the L-lane segment, plus one LDS step across the 4 waves when L = 256.
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int L>
__device__ __forceinline__ float plane_sum(float v, float* red) {
  if constexpr (L <= 64) {
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();  // red is reused by the next call
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
  }
}

template <int L, int V>
struct FastPlane {
  static constexpr int PPB = L >= THREADS ? 1 : THREADS / L;  // planes per workgroup
  int kc, lane;
  bool valid;
  __device__ explicit FastPlane(int KC) {
    lane = (int)(threadIdx.x % L);
    kc = (int)blockIdx.x * PPB + (int)(threadIdx.x / L);
    valid = kc < KC;
  }
  __device__ int64_t at(int i) const { return (int64_t)kc * (L * V) + (int64_t)i * L + lane; }  // float4 index
};

template <int L, int V, bool RELU, bool RES>
__global__ __launch_bounds__(THREADS) void fwd_fast_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, const float* __restrict__ res,
                                                           float* __restrict__ y, float* __restrict__ mean_out,
                                                           float* __restrict__ invstd_out, int KC, float eps) {
  __shared__ float red[THREADS / 64];
  const FastPlane<L, V> pl(KC);
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  f32x4 v[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] = pl.valid ? x4[pl.at(i)] : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
  const float n = (float)(4 * L * V);
  const float mean = plane_sum<L>(s, red) / n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q += d * d;
    }
  const float var = plane_sum<L>(q, red) / n;
  if (!pl.valid) return;
  const float invstd = 1.0f / sqrtf(var + eps);
  const float alpha = invstd * gamma[pl.kc];
  const float shift = beta[pl.kc] - mean * alpha;
  f32x4* y4 = reinterpret_cast<f32x4*>(y);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    f32x4 r = {0.f, 0.f, 0.f, 0.f};
    if constexpr (RES) r = reinterpret_cast<const f32x4*>(res)[pl.at(i)];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = v[i][e] * alpha + shift;
      if constexpr (RES) t = t + r[e];
      if constexpr (RELU) t = fmaxf(t, 0.f);
      o[e] = t;
    }
    y4[pl.at(i)] = o;
  }
  if (pl.lane == 0) {
    mean_out[pl.kc] = mean;
    invstd_out[pl.kc] = invstd;
  }
}

template <int L, int V, bool RELU, bool DRES>
__global__ __launch_bounds__(THREADS) void bwd_fast_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ y, const float* __restrict__ gamma,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ invstd_in, float* __restrict__ dx,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float* __restrict__ dres, int KC) {
  __shared__ float red[THREADS / 64];
  const FastPlane<L, V> pl(KC);
  const float mean = pl.valid ? mean_in[pl.kc] : 0.f;
  f32x4 g[V], xc[V];
  float s = 0.f, d = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 gv = pl.valid ? reinterpret_cast<const f32x4*>(dy)[pl.at(i)] : z;
    f32x4 xv = pl.valid ? reinterpret_cast<const f32x4*>(x)[pl.at(i)] : z;
    if constexpr (RELU) {
      const f32x4 yv = pl.valid ? reinterpret_cast<const f32x4*>(y)[pl.at(i)] : z;
#pragma unroll
      for (int e = 0; e < 4; ++e) gv[e] = yv[e] > 0.f ? gv[e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xv[e] = xv[e] - mean;
      s += gv[e];
      d += xv[e] * gv[e];
    }
    g[i] = gv;
    xc[i] = xv;
  }
  s = plane_sum<L>(s, red);
  d = plane_sum<L>(d, red);
  if (!pl.valid) return;
  const float n = (float)(4 * L * V);
  const float invstd = invstd_in[pl.kc];
  const float kk = d * invstd * invstd / n;
  const float mdy = s / n;
  const float wscale = invstd * gamma[pl.kc];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (g[i][e] - mdy - xc[i][e] * kk) * wscale;
    if constexpr (DRES) reinterpret_cast<f32x4*>(dres)[pl.at(i)] = g[i];
    reinterpret_cast<f32x4*>(dx)[pl.at(i)] = o;
  }
  if (pl.lane == 0) {
    dgamma[pl.kc] = d * invstd;
    dbeta[pl.kc] = s;
  }
}

// (L, V) of the fast path for a plane of n floats, or false.
inline bool fast_shape(int64_t B, int64_t HW, int& L, int& V) {
  if (B != 1 || HW % 4 != 0) return false;
  const int64_t n4 = HW / 4;
  if ((n4 & (n4 - 1)) != 0 || n4 > 2048) return false;
  if (n4 <= 64) {
    L = (int)n4;
    V = 1;
  } else if (n4 <= 512) {
    L = 64;
    V = (int)(n4 / 64);
  } else {
    L = 256;
    V = (int)(n4 / 256);
  }
  return true;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

#define FLR_BN_FAST_SHAPES(X) \
  X(1, 1) X(2, 1) X(4, 1) X(8, 1) X(16, 1) X(32, 1) X(64, 1) X(64, 2) X(64, 4) X(64, 8) X(256, 4) X(256, 8)

template <bool RELU, bool RES>
bool fwd_fast(const float* x, const float* gamma, const float* beta, const float* res, float* y, float* mean,
              float* invstd, int64_t B, int64_t KC, int64_t HW, float eps, hipStream_t st) {
  int L, V;
  if (!fast_shape(B, HW, L, V) || !aligned16(x) || !aligned16(y) || (RES && !aligned16(res))) return false;
  const int ppb = L >= THREADS ? 1 : THREADS / L;
  const dim3 grid((unsigned)((KC + ppb - 1) / ppb));
#define FLR_BN_FWD_CASE(LL, VV)                                                                                  \
  if (L == LL && V == VV) {                                                                                      \
    hipLaunchKernelGGL((fwd_fast_kernel<LL, VV, RELU, RES>), grid, dim3(THREADS), 0, st, x, gamma, beta, res, y, \
                       mean, invstd, (int)KC, eps);                                                              \
    return true;                                                                                                 \
  }
  FLR_BN_FAST_SHAPES(FLR_BN_FWD_CASE)
#undef FLR_BN_FWD_CASE
  return false;
}

template <bool RELU, bool DRES>
bool bwd_fast(const float* dy, const float* x, const float* y, const float* gamma, const float* mean,
              const float* invstd, float* dx, float* dgamma, float* dbeta, float* dres, int64_t B, int64_t KC,
              int64_t HW, hipStream_t st) {
  int L, V;
  if (!fast_shape(B, HW, L, V) || !aligned16(dy) || !aligned16(x) || !aligned16(dx) || (RELU && !aligned16(y)) ||
      (DRES && !aligned16(dres)))
    return false;
  const int ppb = L >= THREADS ? 1 : THREADS / L;
  const dim3 grid((unsigned)((KC + ppb - 1) / ppb));
#define FLR_BN_BWD_CASE(LL, VV)                                                                                   \
  if (L == LL && V == VV) {                                                                                       \
    hipLaunchKernelGGL((bwd_fast_kernel<LL, VV, RELU, DRES>), grid, dim3(THREADS), 0, st, dy, x, y, gamma, mean, \
                       invstd, dx, dgamma, dbeta, dres, (int)KC);                                                 \
    return true;                                                                                                  \
  }
  FLR_BN_FAST_SHAPES(FLR_BN_BWD_CASE)
#undef FLR_BN_BWD_CASE
  return false;
}

// ---- the ResNet stem's BatchNorm + ReLU + 3x3/2/1 max-pool, fused -------------
// One workgroup per (client, channel) plane of NI images of 16 x 16 (NI = 16 or
// 32: the fast path's L = 256 lanes, V = NI / 4 float4s per lane; lane l's float4
// i is image 4i + l/64, row (l/4) % 16, columns 4 (l % 4) .. +3).  Forward: the
// fast kernel's BatchNorm + ReLU in registers, the activated plane staged in LDS,
// the pool evaluated from LDS exactly as pool::fwd_kernel (first in-bounds max,
// NaN wins, 1-byte argmax) — the BN output never goes to HBM.  Backward: the
// pooled gradient and argmax staged in LDS, each lane gathers its four pixels'
// gradients in window-raster order (pool::bwd_k3s2p1_kernel's order), the ReLU
// mask recomputed from x (t = x alpha + shift > 0, the forward's arithmetic),
// then bwd_fast_kernel's BatchNorm backward.  Bit-identical to the three-kernel
// composition (flr_batchnorm_fwd + flr_maxpool2d_fwd, flr_maxpool2d_bwd +
// flr_batchnorm_bwd) and two HBM round trips of the plane lighter each way.
constexpr int SP_H = 16, SP_W = 16, SP_HO = 8, SP_WO = 8;

template <int V>
__global__ __launch_bounds__(THREADS) void stem_bn_pool_fwd_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta,
                                                                   float* __restrict__ yp, uint8_t* __restrict__ arg,
                                                                   float* __restrict__ mean_out,
                                                                   float* __restrict__ invstd_out, int KC, float eps) {
  constexpr int L = 256, NI = 4 * V;
  __shared__ float red[THREADS / 64];
  __shared__ __attribute__((aligned(16))) float xs[NI * SP_H * SP_W];
  const FastPlane<L, V> pl(KC);
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  f32x4 v[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] = pl.valid ? x4[pl.at(i)] : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
  const float n = (float)(4 * L * V);
  const float mean = plane_sum<L>(s, red) / n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q += d * d;
    }
  const float var = plane_sum<L>(q, red) / n;
  if (!pl.valid) return;  // one plane per workgroup: uniform
  const float invstd = 1.0f / sqrtf(var + eps);
  const float alpha = invstd * gamma[pl.kc];
  const float shift = beta[pl.kc] - mean * alpha;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = fmaxf(v[i][e] * alpha + shift, 0.f);
    reinterpret_cast<f32x4*>(xs)[i * L + pl.lane] = o;
  }
  if (pl.lane == 0) {
    mean_out[pl.kc] = mean;
    invstd_out[pl.kc] = invstd;
  }
  __syncthreads();
  float* yb = yp + (int64_t)pl.kc * NI * SP_HO * SP_WO;
  uint8_t* ab = arg + (int64_t)pl.kc * NI * SP_HO * SP_WO;
  for (int o = threadIdx.x; o < NI * SP_HO * SP_WO; o += THREADS) {
    const int b = o / (SP_HO * SP_WO), qq = o % (SP_HO * SP_WO);
    const int oh = qq / SP_WO, ow = qq % SP_WO;
    const float* xp = xs + b * SP_H * SP_W;
    const int ih0 = 2 * oh - 1, iw0 = 2 * ow - 1;
    float best = -__builtin_huge_valf();
    int bi = -1;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = ih0 + kh;
      if (ih < 0 || ih >= SP_H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = iw0 + kw;
        if (iw < 0 || iw >= SP_W) continue;
        const float val = xp[ih * SP_W + iw];
        if (bi < 0) bi = kh * 3 + kw;  // torch's initial maxindex: the first in-bounds element
        if (val > best || val != val) {
          best = val;
          bi = kh * 3 + kw;
        }
      }
    }
    yb[o] = best;
    ab[o] = (uint8_t)bi;
  }
}

template <int V>
__global__ __launch_bounds__(THREADS) void stem_pool_bn_bwd_kernel(
    const float* __restrict__ dyp, const uint8_t* __restrict__ arg, const float* __restrict__ x,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ mean_in,
    const float* __restrict__ invstd_in, float* __restrict__ dx, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int KC) {
  constexpr int L = 256, NI = 4 * V, NO = NI * SP_HO * SP_WO;
  __shared__ float red[THREADS / 64];
  __shared__ __attribute__((aligned(16))) float ds[NO];
  __shared__ __attribute__((aligned(16))) uint8_t as[NO];
  const FastPlane<L, V> pl(KC);
  if (!pl.valid) return;  // one plane per workgroup: uniform
  const float* dyb = dyp + (int64_t)pl.kc * NO;
  const uint8_t* ab = arg + (int64_t)pl.kc * NO;
  for (int o = threadIdx.x; o < NO / 4; o += THREADS) {
    reinterpret_cast<f32x4*>(ds)[o] = reinterpret_cast<const f32x4*>(dyb)[o];
    reinterpret_cast<uint32_t*>(as)[o] = reinterpret_cast<const uint32_t*>(ab)[o];
  }
  __syncthreads();
  const float mean = mean_in[pl.kc];
  const float invstd = invstd_in[pl.kc];
  const float alpha = invstd * gamma[pl.kc];
  const float shift = beta[pl.kc] - mean * alpha;
  const int r = (pl.lane >> 2) & 15, c0 = 4 * (pl.lane & 3);
  const int m = r >> 1, dh = r & 1;
  f32x4 g[V], xc[V];
  float s = 0.f, d = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int b = 4 * i + (pl.lane >> 6);
    const float* dp = ds + b * SP_HO * SP_WO;
    const uint8_t* ap = as + b * SP_HO * SP_WO;
    // this lane's four pixels: 2x2 blocks n = c0/2 and c0/2 + 1, row dh of each
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int nn = (c0 >> 1) + nb;
#pragma unroll
      for (int w = 0; w < 4; ++w) {  // windows in raster order
        const int oh = m + (w >> 1), ow = nn + (w & 1);
        if (oh >= SP_HO || ow >= SP_WO) continue;
        const int a = ap[oh * SP_WO + ow];
        const int kh = a / 3, kw = a - 3 * kh;
        const int rh = 2 * oh - 1 + kh - 2 * m, rw = 2 * ow - 1 + kw - 2 * nn;  // argmax relative to the block
        if (rh != dh || rw < 0 || rw > 1) continue;
        acc[2 * nb + rw] = add_rn(acc[2 * nb + rw], dp[oh * SP_WO + ow]);
      }
    }
    f32x4 xv = reinterpret_cast<const f32x4*>(x)[pl.at(i)];
    f32x4 gv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float t = xv[e] * alpha + shift;  // the forward's pre-ReLU value
      gv[e] = fmaxf(t, 0.f) > 0.f ? acc[e] : 0.f;
      xv[e] = xv[e] - mean;
      s += gv[e];
      d += xv[e] * gv[e];
    }
    g[i] = gv;
    xc[i] = xv;
  }
  s = plane_sum<L>(s, red);
  d = plane_sum<L>(d, red);
  const float n = (float)(4 * L * V);
  const float kk = d * invstd * invstd / n;
  const float mdy = s / n;
  const float wscale = invstd * gamma[pl.kc];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (g[i][e] - mdy - xc[i][e] * kk) * wscale;
    reinterpret_cast<f32x4*>(dx)[pl.at(i)] = o;
  }
  if (pl.lane == 0) {
    dgamma[pl.kc] = d * invstd;
    dbeta[pl.kc] = s;
  }
}

inline bool stem_fused_ok(int64_t NI, int64_t H, int64_t W) { return H == SP_H && W == SP_W && (NI == 16 || NI == 32); }

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
  bool fast;
  if (relu && residual) fast = bn::fwd_fast<true, true>(x, gamma, beta, residual, y, mean, invstd, B, KC, HW, eps, st);
  else if (relu) fast = bn::fwd_fast<true, false>(x, gamma, beta, residual, y, mean, invstd, B, KC, HW, eps, st);
  else if (residual) fast = bn::fwd_fast<false, true>(x, gamma, beta, residual, y, mean, invstd, B, KC, HW, eps, st);
  else fast = bn::fwd_fast<false, false>(x, gamma, beta, residual, y, mean, invstd, B, KC, HW, eps, st);
  if (fast) return launch_status("batchnorm fwd (fast)");
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
  bool fast;
  if (relu && dresidual)
    fast = bn::bwd_fast<true, true>(dy, x, y, gamma, mean, invstd, dx, dgamma, dbeta, dresidual, B, KC, HW, st);
  else if (relu)
    fast = bn::bwd_fast<true, false>(dy, x, y, gamma, mean, invstd, dx, dgamma, dbeta, dresidual, B, KC, HW, st);
  else if (dresidual)
    fast = bn::bwd_fast<false, true>(dy, x, y, gamma, mean, invstd, dx, dgamma, dbeta, dresidual, B, KC, HW, st);
  else
    fast = bn::bwd_fast<false, false>(dy, x, y, gamma, mean, invstd, dx, dgamma, dbeta, dresidual, B, KC, HW, st);
  if (fast) return launch_status("batchnorm bwd (fast)");
#define FLR_BN_BWD(R, D)                                                                                       \
  hipLaunchKernelGGL((bn::bwd_kernel<R, D>), grid, dim3(bn::THREADS), 0, st, dy, x, y, gamma, mean, invstd, dx, \
                     dgamma, dbeta, dresidual, (int)B, (int)KC, (int)HW, sl)
  if (relu && dresidual) FLR_BN_BWD(true, true);
  else if (relu) FLR_BN_BWD(true, false);
  else if (dresidual) FLR_BN_BWD(false, true);
  else FLR_BN_BWD(false, false);
#undef FLR_BN_BWD
  return launch_status("batchnorm bwd");
}

extern "C" int flr_batchnorm_relu_maxpool_fwd(const float* x, const float* gamma, const float* beta, float* y_pool,
                                              uint8_t* argmax, float* mean, float* invstd, int64_t KC, int64_t NI,
                                              int64_t H, int64_t W, float eps, void* stream) {
  if (!x || !gamma || !beta || !y_pool || !argmax || !mean || !invstd || KC < 1 || NI < 1 ||
      KC * NI * H * W >= ((int64_t)1 << 31))
    return FLR_ERR_ARG;
  if (!bn::stem_fused_ok(NI, H, W) || !bn::aligned16(x) || !bn::aligned16(y_pool) ||
      (reinterpret_cast<uintptr_t>(argmax) & 3) != 0)
    return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  if (NI == 32)
    hipLaunchKernelGGL(bn::stem_bn_pool_fwd_kernel<8>, dim3((unsigned)KC), dim3(bn::THREADS), 0, st, x, gamma, beta,
                       y_pool, argmax, mean, invstd, (int)KC, eps);
  else
    hipLaunchKernelGGL(bn::stem_bn_pool_fwd_kernel<4>, dim3((unsigned)KC), dim3(bn::THREADS), 0, st, x, gamma, beta,
                       y_pool, argmax, mean, invstd, (int)KC, eps);
  return launch_status("batchnorm + relu + maxpool fwd");
}

extern "C" int flr_maxpool_relu_batchnorm_bwd(const float* dy_pool, const uint8_t* argmax, const float* x,
                                              const float* gamma, const float* beta, const float* mean,
                                              const float* invstd, float* dx, float* dgamma, float* dbeta, int64_t KC,
                                              int64_t NI, int64_t H, int64_t W, void* stream) {
  if (!dy_pool || !argmax || !x || !gamma || !beta || !mean || !invstd || !dx || !dgamma || !dbeta || KC < 1 ||
      NI < 1 || KC * NI * H * W >= ((int64_t)1 << 31))
    return FLR_ERR_ARG;
  if (!bn::stem_fused_ok(NI, H, W) || !bn::aligned16(x) || !bn::aligned16(dx) || !bn::aligned16(dy_pool) ||
      (reinterpret_cast<uintptr_t>(argmax) & 3) != 0)
    return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  if (NI == 32)
    hipLaunchKernelGGL(bn::stem_pool_bn_bwd_kernel<8>, dim3((unsigned)KC), dim3(bn::THREADS), 0, st, dy_pool, argmax,
                       x, gamma, beta, mean, invstd, dx, dgamma, dbeta, (int)KC);
  else
    hipLaunchKernelGGL(bn::stem_pool_bn_bwd_kernel<4>, dim3((unsigned)KC), dim3(bn::THREADS), 0, st, dy_pool, argmax,
                       x, gamma, beta, mean, invstd, dx, dgamma, dbeta, (int)KC);
  return launch_status("maxpool + relu + batchnorm bwd");
}
