// Client-batched convolution: geometry shared by the conv kernels (gfx950).
#pragma once

#include "flr_common.h"

namespace flr {
namespace conv {

struct FastDiv {  // n / d for 0 <= n < 2^31 via mul-hi (Granlund-Montgomery)
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint32_t t = __umulhi(n, f.m);
  return (t + ((n - t) >> 1)) >> (f.s ? f.s - 1 : 0);
}
// d == 1 needs s = 0: (t + ((n - t) >> 1)) >> 0 with m = 1 gives n/2 ... handle explicitly
__device__ __forceinline__ uint32_t udiv(uint32_t n, const FastDiv& f) { return f.d == 1 ? n : fdiv(n, f); }

constexpr int MAXTAPS = 49;

// A tap list that is a (strided) rectangle: slot -> (kh0 + step*(slot / nkw),
// kw0 + step*(slot % nkw)).  Kernels decode a reduction slot with scalar
// arithmetic instead of indexing the by-value tap table, which the compiler
// can only read with a vector-memory load per K-tile (a full load latency on
// the critical path).  ok = false: the list is not a rectangle (use the table).
struct TapRect {
  int kh0, kw0, nkw, step;
  uint32_t nkw_m;  // ceil(2^16 / nkw): slot / nkw = (slot * nkw_m) >> 16 for slot < MAXTAPS
  bool ok;
};
inline TapRect make_rect(const int8_t* kh, const int8_t* kw, int n, int step) {
  TapRect r{0, 0, 1, step, 65536u, false};
  if (n == 0) { r.ok = true; return r; }
  r.kh0 = kh[0]; r.kw0 = kw[0];
  int nkw = 0;
  while (nkw < n && kh[nkw] == kh[0]) ++nkw;
  r.nkw = nkw;
  r.nkw_m = (65536u + (uint32_t)nkw - 1) / (uint32_t)nkw;
  if (n % nkw != 0) return r;
  for (int t = 0; t < n; ++t)
    if (kh[t] != r.kh0 + step * (t / nkw) || kw[t] != r.kw0 + step * (t % nkw)) return r;
  r.ok = true;
  return r;
}
__device__ __forceinline__ void rect_tap(const TapRect& r, int slot, int& kh, int& kw) {
  // exact for 0 <= slot < 2^16 / nkw (slot < MAXTAPS = 49, nkw <= 7); a multiply
  // and a shift on the scalar unit instead of a division sequence per K-tile
  const int i = (int)(((uint32_t)slot * r.nkw_m) >> 16);
  kh = r.kh0 + r.step * i;
  kw = r.kw0 + r.step * (slot - i * r.nkw);
}

struct Geom {
  int Kc, B, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo;
  // Activation layout x[K][Cin][B][H][W], y[K][Cout][B][Ho][Wo] ("client-
  // channel major"): for a fixed (client, channel) the GEMM's pixel dimension
  // n = b*H*W + h*W + w is one contiguous run of B*H*W floats.  Strides in
  // floats: client, channel, batch; extents = floats per client.
  int64_t sxk, sxc, sxb, syk, syc, syb, xext, yext;
  FastDiv d_howo, d_wo, d_hw, d_w, d_cin, d_cout;
  // Kernel taps that read at least one non-padding input pixel.  A tap that
  // only ever reads the zero padding contributes exact zeros to y, dx and dw,
  // so the reduction runs over (valid tap, channel) only: r = slot * C + c.
  int ntaps;
  int8_t tap_kh[MAXTAPS], tap_kw[MAXTAPS];
  TapRect rect;  // the live taps as a rectangle (step 1), when they are one
};

inline Geom make_geom(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH,
                      int64_t KW, int64_t stride, int64_t pad) {
  Geom g;
  g.Kc = (int)K; g.B = (int)B; g.Cin = (int)Cin; g.H = (int)H; g.W = (int)W; g.Cout = (int)Cout;
  g.KH = (int)KH; g.KW = (int)KW; g.stride = (int)stride; g.pad = (int)pad;
  g.Ho = (int)((H + 2 * pad - KH) / stride + 1);
  g.Wo = (int)((W + 2 * pad - KW) / stride + 1);
  g.sxb = H * W;
  g.sxc = B * H * W;
  g.sxk = Cin * B * H * W;
  g.syb = (int64_t)g.Ho * g.Wo;
  g.syc = B * g.syb;
  g.syk = Cout * g.syc;
  g.xext = g.sxk;
  g.yext = g.syk;
  g.d_howo = make_fastdiv((uint32_t)(g.Ho * g.Wo));
  g.d_wo = make_fastdiv((uint32_t)g.Wo);
  g.d_hw = make_fastdiv((uint32_t)(H * W));
  g.d_w = make_fastdiv((uint32_t)W);
  g.d_cin = make_fastdiv((uint32_t)Cin);
  g.d_cout = make_fastdiv((uint32_t)Cout);
  g.ntaps = 0;
  for (int kh = 0; kh < KH; ++kh) {
    bool hv = false;
    for (int oh = 0; oh < g.Ho && !hv; ++oh) { const int ih = oh * (int)stride - (int)pad + kh; hv = ih >= 0 && ih < H; }
    for (int kw = 0; kw < KW; ++kw) {
      bool wv = false;
      for (int ow = 0; ow < g.Wo && !wv; ++ow) { const int iw = ow * (int)stride - (int)pad + kw; wv = iw >= 0 && iw < W; }
      if (hv && wv) { g.tap_kh[g.ntaps] = (int8_t)kh; g.tap_kw[g.ntaps] = (int8_t)kw; ++g.ntaps; }
    }
  }
  g.rect = make_rect(g.tap_kh, g.tap_kw, g.ntaps, 1);
  return g;
}

inline bool geom_ok(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                    int64_t stride, int64_t pad) {
  if (K < 1 || B < 1 || Cin < 1 || H < 1 || W < 1 || Cout < 1 || KH < 1 || KW < 1 || stride < 1 || pad < 0)
    return false;
  if (H + 2 * pad < KH || W + 2 * pad < KW || KH * KW > MAXTAPS) return false;
  // 32-bit index space per client for the GEMM dims and offsets
  return K * Cin * H * W * B < (int64_t(1) << 31) && K * Cout * H * W * B < (int64_t(1) << 31) &&
         K <= 65535;
}

}  // namespace conv

// Explicit-im2col path for convs with a short reduction (the 7x7 stem:
// Cin*KH*KW = 147), implemented in train_conv_t.hip and used by the
// generic-layout entry points of train_conv.hip.
namespace convt {
bool im2col_eligible(const conv::Geom& g);
size_t im2col_workspace(const conv::Geom& g);
int fwd_im2col(const conv::Geom& g, const float* x, const float* w, float* y, void* ws, size_t ws_bytes,
               hipStream_t st);
int wgrad_im2col(const conv::Geom& g, const float* x, const float* dy, float* dw, void* ws, size_t ws_bytes,
                 hipStream_t st, bool have_col);
// The direct ResNet-stem kernels (train_stem.hip): images staged in LDS, no im2col.
bool stem_eligible(const conv::Geom& g);
size_t stem_workspace(const conv::Geom& g);
int stem_fwd(const conv::Geom& g, const float* x, const float* w, float* y, hipStream_t st);
int stem_wgrad(const conv::Geom& g, const float* x, const float* dy, float* dw, void* ws, size_t ws_bytes,
               hipStream_t st);
}  // namespace convt
}  // namespace flr
