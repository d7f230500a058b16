// a2 — the ResNet-18 stem convolution (7x7 / stride 2 / pad 3, Cin = 3 -> 64;
// BASELINE C2/C3 image branch, conv-block template src/models/cub200_cnn.py:
// 71-77, trained per client in run_experiments.py:216-235), forward and weight
// gradient, for all clients of a GPU.  The stem's input has no gradient.
//
// The reduction (Cin*KH*KW = 147) is too short for the tiled implicit GEMM to
// amortise its per-K-tile gathers, and an explicit im2col matrix is 620 MB per
// pass at C3.  Here a workgroup owns (client, NI images): the images are staged
// once, zero-padded, in LDS, and every MFMA operand of the image side is read
// from there.  The reduction index is reordered as (row = ci*KH + kh, kw
// padded to 8): one 16-deep MFMA k-step is two rows x 8 kw, lane half h taking
// row 2s + h, so a lane's eight B values are eight consecutive floats of one
// padded image row (four ds_read_b64).  Weight slots kw >= KW and rows >= Cin*KH
// are zero; the image values they meet are finite padding or image data.
//
// Products: fp32 operands split into three bf16 terms, six products per k-step
// on v_mfma_f32_32x32x16_bf16 (the engine's bf16x6 form, per-product error a
// few 2^-24 |a b|), fp32 accumulation in a fixed order (deterministic).
//
//   forward: y[k][co][b][oh][ow] = sum_(row, kw) w[k][co][row][kw] img(b; row, kw; oh, ow)
//     wave (co-tile c, pixel stream p): its 32 output channels' weight
//     fragments for every k-step are split once and held in registers.
//   weight gradient: dw[k][co][row][kw] = sum_pix dy[k][co][pix] img(pix; row, kw)
//     per (client, image group) partials over that group's pixels, reduced in
//     group order by reduce_kernel (which also drops the padded slots).
#include "conv_common.h"

#include <algorithm>
#include <cstdlib>

namespace flr {
namespace stem {

using conv::FastDiv;
using conv::udiv;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
using rsrc_t = __amdgpu_buffer_rsrc_t;

constexpr int NI = 4;        // images per workgroup
constexpr int THREADS = 256;
constexpr int NKS = 11;      // k-steps: ceil(Cin*KH / 2) = ceil(21 / 2) for the 3-channel 7x7 stem
constexpr int S = 2;         // stride
constexpr int NT = (2 * NKS * 8 + 31) / 32;  // weight-gradient n-tiles of 32 (row, kw) slots
constexpr int NTW = (NT + 1) / 2;            // per wave
constexpr int NSLOT = 32 * NT;
constexpr int MAX_LDS = 80 * 1024;

struct Args {
  int B, Cin, H, W, Cout, KH, KW, P, Ho, Wo, Hp, Wp, PL, IMG, CK;
  int64_t sxk, sxc, sxb, syk, syc;
  FastDiv d_hw, d_w, d_nhw, d_howo, d_wo;
};

__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a = (__bf16)v[j];
    const float r1 = v[j] - (float)a;
    const __bf16 b = (__bf16)r1;
    hi[j] = a;
    mid[j] = b;
    lo[j] = (__bf16)(r1 - (float)b);
  }
}

__device__ __forceinline__ f32x16 mfma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                        const bf16x8& bm, const bf16x8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int64_t nfloats) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane((int)(nfloats * 4));
  void* b = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, bytes, 0x00020000);
}

// img[bl][ci][Hp][Wp] <- the NI images b0 .. b0+NI-1 of client x, zero-padded
// (x is [Cin][B][H][W]: for a fixed channel the NI images are one contiguous
// run).  Every thread issues all of its (<= SV) 16-B loads before its first LDS
// store, so the staging costs one load latency, not one per element.
constexpr int SV = 16;  // float4 loads per thread: Cin * NI * H * W <= 4 * SV * THREADS
__device__ void stage(const Args& a, const float* __restrict__ xk, int b0, float* img) {
  const int tot = NI * a.IMG;
  const int HW = a.H * a.W, nhw = NI * HW, nv = a.Cin * nhw / 4;
  f32x4 v[SV];
#pragma unroll
  for (int i = 0; i < SV; ++i) {
    const int e = threadIdx.x + THREADS * i;
    if (e < nv) {
      const int f = 4 * e;
      const int ci = (int)udiv((uint32_t)f, a.d_nhw), r = f - ci * nhw;
      v[i] = *reinterpret_cast<const f32x4*>(xk + ci * a.sxc + (int64_t)b0 * a.sxb + r);
    }
  }
  for (int e = threadIdx.x; e < tot / 4; e += THREADS) reinterpret_cast<f32x4*>(img)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
#pragma unroll
  for (int i = 0; i < SV; ++i) {
    const int e = threadIdx.x + THREADS * i;
    if (e < nv) {
      const int f = 4 * e;  // W % 4 == 0: the four values share one image row
      const int ci = (int)udiv((uint32_t)f, a.d_nhw), r = f - ci * nhw;
      const int bl = (int)udiv((uint32_t)r, a.d_hw), q = r - bl * HW;
      const int ih = (int)udiv((uint32_t)q, a.d_w), iw = q - ih * a.W;
      float* d = img + bl * a.IMG + ci * a.PL + (ih + a.P) * a.Wp + iw + a.P;
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = v[i][j];
    }
  }
  __syncthreads();
}

// grid (B / NI, K, ceil(Cout / 64)); dynamic LDS NI * IMG floats
__global__ __launch_bounds__(THREADS, 2) void fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         float* __restrict__ y, const Args a) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  const int k = blockIdx.y, b0 = blockIdx.x * NI;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int c = wave & 1, ps = wave >> 1;
  const int co = 64 * blockIdx.z + 32 * c + l32;
  // this wave's weight fragments, every k-step, split once (issued before the staging)
  bf16x8 wh[NKS], wm[NKS], wl[NKS];
  {
    const int RW = a.CK * a.KW;  // torch order [Cout][Cin][KH][KW]
    const rsrc_t rw = make_rsrc(w + (int64_t)k * a.Cout * RW, (int64_t)a.Cout * RW);
    float v[NKS][8];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int row = 2 * s + h;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = co < a.Cout && row < a.CK && j < a.KW;
        const unsigned off = ok ? (unsigned)((co * RW + row * a.KW + j) * 4) : 0x80000000u;
        v[s][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, off, 0, 0));
      }
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) split3(v[s], wh[s], wm[s], wl[s]);
  }
  // LDS offset of (ci, kh) of this lane half's row, per k-step (rows past Cin*KH: any real row)
  int cb[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int row = min(2 * s + h, a.CK - 1);
    const int ci = row / a.KH, kh = row - ci * a.KH;
    cb[s] = ci * a.PL + kh * a.Wp;
  }
  stage(a, x + k * a.sxk, b0, img);
  const int HoWo = a.Ho * a.Wo, npix = NI * HoWo, ntiles = (npix + 31) / 32;
  const int64_t ybase = k * a.syk + (int64_t)b0 * HoWo;
  for (int t = ps; t < ntiles; t += 2) {
    const int n = 32 * t + l32;
    const bool nok = n < npix;
    const int bl = (int)udiv((uint32_t)n, a.d_howo), p = n - bl * HoWo;
    const int oh = (int)udiv((uint32_t)p, a.d_wo), ow = p - oh * a.Wo;
    const int pbase = nok ? bl * a.IMG + oh * S * a.Wp + ow * S : 0;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const float2* src = reinterpret_cast<const float2*>(img + pbase + cb[s]);  // 8-B aligned: even offsets
      float v[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 f = src[q];
        v[2 * q] = f.x;
        v[2 * q + 1] = f.y;
      }
      bf16x8 bh, bm, bl8;
      split3(v, bh, bm, bl8);
      acc = mfma6(wh[s], wm[s], wl[s], bh, bm, bl8, acc);
    }
    // C/D map: col = lane & 31 (pixel), row = (e & 3) + 8 (e >> 2) + 4 h (output channel)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int coe = 64 * blockIdx.z + 32 * c + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (nok && coe < a.Cout) y[ybase + coe * a.syc + n] = acc[e];
    }
  }
}

// grid (B / NI, K, ceil(Cout / 64)); part[k][group][64 * gridDim.z][NSLOT]
__global__ __launch_bounds__(THREADS, 2) void wgt_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                         float* __restrict__ part, const Args a) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  const int k = blockIdx.y, grp = blockIdx.x, b0 = grp * NI;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int c = wave & 1, tq = wave >> 1;
  const int co = 64 * blockIdx.z + 32 * c + l32;
  // this lane's (row, kw) slot of each of its n-tiles -> LDS offset (rows past Cin*KH: any real row)
  int lb[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int slot = 32 * (tq * NTW + t) + l32;
    const int row = min(slot >> 3, a.CK - 1), kw = slot & 7;
    const int ci = row / a.KH, kh = row - ci * a.KH;
    lb[t] = ci * a.PL + kh * a.Wp + kw;
  }
  const int HoWo = a.Ho * a.Wo;
  const rsrc_t rdy = make_rsrc(dy + k * a.syk, a.syk);
  const bool cok = co < a.Cout;
  const unsigned arow = (unsigned)((min(co, a.Cout - 1) * a.syc + (int64_t)b0 * HoWo) * 4);
  auto load_a = [&](int ks, float (&v)[8]) {
    const unsigned off = cok ? arow + (unsigned)((16 * ks + 8 * h) * 4) : 0x80000000u;
    const f32x4 p = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rdy, off, 0, 0));
    const f32x4 q = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rdy, off + 16u, 0, 0));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = p[e];
      v[4 + e] = q[e];
    }
  };
  float an[8];
  load_a(0, an);  // in flight during the staging
  stage(a, x + k * a.sxk, b0, img);
  f32x16 acc[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  const int nks = NI * HoWo / 16;  // HoWo % 16 == 0, Wo % 8 == 0: a lane half's 8 pixels share one output row
  for (int ks = 0; ks < nks; ++ks) {
    float av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) av[e] = an[e];
    if (ks + 1 < nks) load_a(ks + 1, an);
    const int p = 16 * ks + 8 * h;
    const int bl = (int)udiv((uint32_t)p, a.d_howo), q = p - bl * HoWo;
    const int oh = (int)udiv((uint32_t)q, a.d_wo), ow = q - oh * a.Wo;
    const int pb = bl * a.IMG + oh * S * a.Wp + ow * S;
    bf16x8 ah, am, al;
    split3(av, ah, am, al);
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      const float* src = img + pb + lb[t];
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[j * S];
      bf16x8 bh, bm, bl8;
      split3(v, bh, bm, bl8);
      acc[t] = mfma6(ah, am, al, bh, bm, bl8, acc[t]);
    }
  }
  const int cop = 64 * gridDim.z;
  float* pk = part + ((int64_t)k * gridDim.x + grp) * cop * NSLOT;
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int slot = 32 * (tq * NTW + t) + l32;
    if (tq * NTW + t >= NT) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int coe = 64 * blockIdx.z + 32 * c + (e & 3) + 8 * (e >> 2) + 4 * h;
      pk[(int64_t)coe * NSLOT + slot] = acc[t][e];
    }
  }
}

// dw[k][co][r] (torch order r = row*KW + kw) = sum over groups, in group order
__global__ void reduce_kernel(const float* __restrict__ part, int ngroups, int cop, const Args a,
                              float* __restrict__ dw) {
  const int k = blockIdx.y;
  const int R = a.CK * a.KW;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.Cout * R) return;
  const int co = e / R, r = e - co * R;
  const int row = r / a.KW, kw = r - row * a.KW;
  const float* p = part + ((int64_t)k * ngroups * cop + co) * NSLOT + row * 8 + kw;
  float v = p[0];
  for (int g = 1; g < ngroups; ++g) v += p[(int64_t)g * cop * NSLOT];
  dw[((int64_t)k * a.Cout) * R + e] = v;
}

inline bool make_args(const conv::Geom& g, Args& a) {
  a.B = g.B; a.Cin = g.Cin; a.H = g.H; a.W = g.W; a.Cout = g.Cout; a.KH = g.KH; a.KW = g.KW; a.P = g.pad;
  a.Ho = g.Ho; a.Wo = g.Wo;
  a.CK = g.Cin * g.KH;
  a.Hp = g.H + 2 * g.pad;
  a.Wp = std::max(g.W + 2 * g.pad, (g.Wo - 1) * S + 8);
  a.Wp += a.Wp & 1;  // even: 8-B aligned float2 reads
  a.PL = a.Hp * a.Wp;
  a.IMG = a.Cin * a.PL;
  a.IMG += (4 - a.IMG % 4) % 4;  // 16-B aligned image slots (zero fill by float4)
  a.sxk = g.sxk; a.sxc = g.sxc; a.sxb = g.sxb; a.syk = g.syk; a.syc = g.syc;
  a.d_hw = conv::make_fastdiv((uint32_t)(g.H * g.W));
  a.d_w = conv::make_fastdiv((uint32_t)g.W);
  a.d_nhw = conv::make_fastdiv((uint32_t)(NI * g.H * g.W));
  a.d_howo = conv::make_fastdiv((uint32_t)(g.Ho * g.Wo));
  a.d_wo = conv::make_fastdiv((uint32_t)g.Wo);
  return true;
}

}  // namespace stem

namespace convt {

// The direct stem kernels cover the ResNet stem class: stride 2, 5 <= KW <= 8,
// ceil(Cin*KH / 2) == 11 k-steps (Cin = 3, KH = 7), whole image groups, output
// rows of a multiple of 8 pixels, and NI padded images within MAX_LDS.
bool stem_eligible(const conv::Geom& g) {
  if (g.stride != stem::S || g.KW < 5 || g.KW > 8 || (g.Cin * g.KH + 1) / 2 != stem::NKS) return false;
  if (g.B % stem::NI != 0 || g.Wo % 8 != 0 || (g.Ho * g.Wo) % 16 != 0 || g.Cout > 64 * 16) return false;
  if (g.W % 4 != 0 || (int64_t)g.Cin * stem::NI * g.H * g.W > 4 * stem::SV * stem::THREADS) return false;
  stem::Args a;
  stem::make_args(g, a);
  return (int64_t)stem::NI * a.IMG * 4 <= stem::MAX_LDS && g.syk * 4 < (int64_t(1) << 31);
}

size_t stem_workspace(const conv::Geom& g) {
  const int cop = 64 * ((g.Cout + 63) / 64);
  return align_up((size_t)g.Kc * (g.B / stem::NI) * cop * stem::NSLOT * sizeof(float), 256);
}

int stem_fwd(const conv::Geom& g, const float* x, const float* w, float* y, hipStream_t st) {
  stem::Args a;
  stem::make_args(g, a);
  const dim3 grid((unsigned)(g.B / stem::NI), (unsigned)g.Kc, (unsigned)((g.Cout + 63) / 64));
  hipLaunchKernelGGL(stem::fwd_kernel, grid, dim3(stem::THREADS), (size_t)stem::NI * a.IMG * sizeof(float), st, x, w,
                     y, a);
  return launch_status("stem conv fwd");
}

int stem_wgrad(const conv::Geom& g, const float* x, const float* dy, float* dw, void* ws, size_t ws_bytes,
               hipStream_t st) {
  if (!ws || ws_bytes < stem_workspace(g)) return FLR_ERR_WORKSPACE;
  stem::Args a;
  stem::make_args(g, a);
  const int ng = g.B / stem::NI, cz = (g.Cout + 63) / 64;
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(stem::wgt_kernel, dim3((unsigned)ng, (unsigned)g.Kc, (unsigned)cz), dim3(stem::THREADS),
                     (size_t)stem::NI * a.IMG * sizeof(float), st, x, dy, part, a);
  int rc = launch_status("stem conv wgrad");
  if (rc != FLR_OK) return rc;
  const int n = g.Cout * a.CK * g.KW;
  hipLaunchKernelGGL(stem::reduce_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)g.Kc), dim3(256), 0, st, part,
                     ng, 64 * cz, a, dw);
  return launch_status("stem conv wgrad reduce");
}

}  // namespace convt
}  // namespace flr
