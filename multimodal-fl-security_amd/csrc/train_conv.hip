// a2 — client-batched convolution (forward, backward-data, backward-weight)
// for the image encoder, on exact-fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Reference layer: nn.Conv2d(bias=False) inside the conv blocks
// (src/models/cub200_cnn.py:71-77 template; ResNet-18 BasicBlock here),
// trained per client in run_experiments.py:216-235.  The engine runs every
// client of a GPU in one launch: grid.z = client, each client with its own
// weights [Cout][Cin][KH][KW] (a block of the parameter-major training state)
// and activations in the grouped layout x[b][k*Cin + c][h][w] (client k's
// channels are contiguous; torch's grouped-conv layout, so BatchNorm/ReLU/
// pooling kernels see per-(client, channel) planes).
//
// All three products are one implicit-GEMM template: C_k[M][N] = sum_r
// A_k(m, r) B_k(n, r).  Operand elements are gathered straight from the
// activation / weight tensors (im2col is never materialised); tiles of
// 64(M) x 64(N) x 32(R) are staged through LDS as [r][m] / [r][n] images
// (row stride 65 floats: conflict-free for both the transposing stores and
// the MFMA operand reads), register-staged one tile ahead.  Each of the 4
// waves owns a 32x32 output block: 16 MFMAs per tile, lane half h feeding
// reduction index 16h + q to MFMA q.  fp32 in, fp32 accumulate, one
// rounding per product (a k-ordered fmaf chain) — fp32 numerics, as the
// reference's CPU conv.
#include "conv_common.h"

#include <algorithm>
#include <cstdlib>

namespace flr {
namespace conv {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 32, THREADS = 256;
constexpr int LDS_STRIDE = 65;

// ---- problem accessors -----------------------------------------------------
// A(m, r) and B(n, r); FAST_*: the dimension consecutive threads walk when
// loading a tile (true = m / n, false = r), chosen for contiguous addresses.
// Tile slot mapping (the kernel's LDS stash uses the same): element e = tid +
// 256 i of a 64 x 32 tile sits at (e % 64, e / 64) when FAST along m / n and at
// (e / 32, e % 32) when FAST along r.
__device__ __forceinline__ void slot_of(bool fast_mn, int tid, int i, int& mn, int& kk) {
  const int e = tid + THREADS * i;
  if (fast_mn) { mn = e % BM; kk = e / BM; } else { kk = e % BK; mn = e / BK; }
}

// Generic accessors (any channel count; the stem's Cin = 3): every element's
// index is decomposed on its own.

struct FwdG {  // y = conv(x, w): M = Cout, N = B*Ho*Wo, R = Cin*KH*KW
  Geom g;
  const float* x;
  const float* w;
  float* y;
  static constexpr bool FAST_A_M = false, FAST_B_N = true;
  __host__ __device__ int M() const { return g.Cout; }
  __host__ __device__ int N() const { return g.B * g.Ho * g.Wo; }
  __host__ __device__ int R() const { return g.ntaps * g.Cin; }
  __device__ float a(int k, int m, int r) const {
    const uint32_t slot = udiv(r, g.d_cin), ci = r - slot * g.Cin;
    return w[(((int64_t)k * g.Cout + m) * g.Cin + ci) * (g.KH * g.KW) + g.tap_kh[slot] * g.KW + g.tap_kw[slot]];
  }
  __device__ float b(int k, int n, int r) const {
    const uint32_t slot = udiv(r, g.d_cin), ci = r - slot * g.Cin;
    const int kh = g.tap_kh[slot], kw = g.tap_kw[slot];
    const uint32_t bb = udiv(n, g.d_howo), p = n - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    const int ih = (int)(oh * g.stride + kh) - g.pad, iw = (int)(ow * g.stride + kw) - g.pad;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return 0.f;
    return x[k * g.sxk + ci * g.sxc + bb * g.sxb + ih * g.W + iw];
  }
  __device__ void store(int k, int m, int n, float v) const {
    const uint32_t bb = udiv(n, g.d_howo), p = n - bb * g.Ho * g.Wo;
    y[k * g.syk + m * g.syc + bb * g.syb + p] = v;
  }
};

struct WgtG {  // dw = sum_q dy(co, q) im(r, q): M = Cout, N = R, reduction over q = B*Ho*Wo
  Geom g;
  const float* x;
  const float* dy;
  float* dw;
  static constexpr bool FAST_A_M = false, FAST_B_N = false;
  __host__ __device__ int M() const { return g.Cout; }
  __host__ __device__ int N() const { return g.ntaps * g.Cin; }
  __host__ __device__ int R() const { return g.B * g.Ho * g.Wo; }
  __device__ float a(int k, int m, int q) const {
    const uint32_t bb = udiv(q, g.d_howo), p = q - bb * g.Ho * g.Wo;
    return dy[k * g.syk + m * g.syc + bb * g.syb + p];
  }
  __device__ float b(int k, int r, int q) const {
    const uint32_t slot = udiv(r, g.d_cin), ci = r - slot * g.Cin;
    const int kh = g.tap_kh[slot], kw = g.tap_kw[slot];
    const uint32_t bb = udiv(q, g.d_howo), p = q - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    const int ih = (int)(oh * g.stride + kh) - g.pad, iw = (int)(ow * g.stride + kw) - g.pad;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return 0.f;
    return x[k * g.sxk + ci * g.sxc + bb * g.sxb + ih * g.W + iw];
  }
  __device__ void store(int k, int m, int n, float v) const {
    const uint32_t slot = udiv(n, g.d_cin), ci = n - slot * g.Cin;
    dw[(((int64_t)k * g.Cout + m) * g.Cin + ci) * (g.KH * g.KW) + g.tap_kh[slot] * g.KW + g.tap_kw[slot]] = v;
  }
};

struct DgradG {  // dx = conv^T(dy, w): M = Cin, N = B*H*W, R = Cout*KH*KW
  Geom g;
  const float* dy;
  const float* w;
  float* dx;
  static constexpr bool FAST_A_M = false, FAST_B_N = true;
  __host__ __device__ int M() const { return g.Cin; }
  __host__ __device__ int N() const { return g.B * g.H * g.W; }
  __host__ __device__ int R() const { return g.ntaps * g.Cout; }
  __device__ float a(int k, int m, int r) const {
    const uint32_t slot = udiv(r, g.d_cout), co = r - slot * g.Cout;
    return w[(((int64_t)k * g.Cout + co) * g.Cin + m) * (g.KH * g.KW) + g.tap_kh[slot] * g.KW + g.tap_kw[slot]];
  }
  __device__ float b(int k, int n, int r) const {
    const uint32_t slot = udiv(r, g.d_cout), co = r - slot * g.Cout;
    const int kh = g.tap_kh[slot], kw = g.tap_kw[slot];
    const uint32_t bb = udiv(n, g.d_hw), p = n - bb * g.H * g.W;
    const uint32_t ih = udiv(p, g.d_w), iw = p - ih * g.W;
    const int nh = (int)ih + g.pad - kh, nw = (int)iw + g.pad - kw;
    if (nh < 0 || nw < 0) return 0.f;
    const int oh = nh / g.stride, ow = nw / g.stride;
    if (oh * g.stride != nh || ow * g.stride != nw || oh >= g.Ho || ow >= g.Wo) return 0.f;
    return dy[k * g.syk + co * g.syc + bb * g.syb + oh * g.Wo + ow];
  }
  __device__ void store(int k, int m, int n, float v) const {
    const uint32_t bb = udiv(n, g.d_hw), p = n - bb * g.H * g.W;
    dx[k * g.sxk + m * g.sxc + bb * g.sxb + p] = v;
  }
};


template <class G>
struct GenericLoad : G {
  struct State { int k, m0, n0, tid; };
  __device__ State init(int k, int m0, int n0, int tid) const { return State{k, m0, n0, tid}; }
  __device__ void load(const State& s, int r0, int re, float (&ra)[8], float (&rb)[8]) const {
    const int M = this->M(), N = this->N();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int mm, ak, nn, bk;
      slot_of(G::FAST_A_M, s.tid, i, mm, ak);
      slot_of(G::FAST_B_N, s.tid, i, nn, bk);
      const int m = s.m0 + mm, r = r0 + ak, n = s.n0 + nn, rr = r0 + bk;
      ra[i] = (m < M && r < re) ? this->a(s.k, m, r) : 0.f;
      rb[i] = (n < N && rr < re) ? this->b(s.k, n, rr) : 0.f;
    }
  }
};
using Fwd = GenericLoad<FwdG>;
using Wgt = GenericLoad<WgtG>;
using Dgrad = GenericLoad<DgradG>;

// ---- fast accessors (channel counts multiple of 32; Wgt: Cin multiple of 64) --
// r = slot * C + c with C % 32 == 0, so a 32-deep K-tile never straddles two
// kernel taps: the tap and channel base are tile-uniform (scalar), each
// thread's spatial coordinates are decomposed once per kernel, and an element
// costs one add + one load.

struct FwdF : FwdG {  // A fast along r (ci), B fast along n (pixels)
  struct State {
    const float* wk; const float* xk;
    int abase[8]; bool mok[8];
    int ih0, iw0, xoff, rl;  // B: this thread's pixel
    bool nok;
  };
  __device__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.wk = w + (int64_t)k * g.Cout * g.Cin * g.KH * g.KW;
    s.xk = x + k * g.sxk;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + tid / BK + 8 * i;
      s.mok[i] = m < g.Cout;
      s.abase[i] = m * g.Cin * g.KH * g.KW + (tid % BK) * g.KH * g.KW;
    }
    const int n = n0 + tid % BN;
    s.nok = n < g.B * g.Ho * g.Wo;
    const uint32_t bb = udiv(n, g.d_howo), p = n - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    s.ih0 = (int)oh * g.stride - g.pad;
    s.iw0 = (int)ow * g.stride - g.pad;
    s.xoff = (int)(bb * g.sxb + (tid / BN) * g.sxc);
    s.rl = tid / BN;
    return s;
  }
  __device__ void load(const State& s, int r0, int re, float (&ra)[8], float (&rb)[8]) const {
    const int slot = __builtin_amdgcn_readfirstlane(r0 / g.Cin);
    const int ci0 = r0 - slot * g.Cin;
    int kh, kw;
    if (g.rect.ok) rect_tap(g.rect, slot, kh, kw); else { kh = g.tap_kh[slot]; kw = g.tap_kw[slot]; }
    const int KK = g.KH * g.KW, HW = (int)g.sxc;  // channel stride
    const int aoff = ci0 * KK + kh * g.KW + kw;
#pragma unroll
    for (int i = 0; i < 8; ++i) ra[i] = s.mok[i] ? s.wk[s.abase[i] + aoff] : 0.f;
    const int ih = s.ih0 + kh, iw = s.iw0 + kw;
    const bool ok = s.nok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
    const int boff = s.xoff + ci0 * HW + ih * g.W + iw;
#pragma unroll
    for (int i = 0; i < 8; ++i) rb[i] = ok ? s.xk[boff + 4 * i * HW] : 0.f;
  }
};

struct DgradF : DgradG {  // A fast along m (ci), B fast along n (input pixels)
  static constexpr bool FAST_A_M = true, FAST_B_N = true;
  struct State {
    const float* wk; const float* dyk;
    int abase; bool mok;
    int ih, iw, yoff;
    bool nok;
  };
  __device__ State init(int k, int m0, int n0, int tid) const {
    State s;
    const int KK = g.KH * g.KW;
    s.wk = w + (int64_t)k * g.Cout * g.Cin * KK;
    s.dyk = dy + k * g.syk;
    const int m = m0 + tid % BM;
    s.mok = m < g.Cin;
    s.abase = m * KK + (tid / BM) * g.Cin * KK;
    const int n = n0 + tid % BN;
    s.nok = n < g.B * g.H * g.W;
    const uint32_t bb = udiv(n, g.d_hw), p = n - bb * g.H * g.W;
    const uint32_t ih = udiv(p, g.d_w), iw = p - ih * g.W;
    s.ih = (int)ih + g.pad;
    s.iw = (int)iw + g.pad;
    s.yoff = (int)(bb * g.syb + (tid / BN) * g.syc);
    return s;
  }
  __device__ void load(const State& s, int r0, int re, float (&ra)[8], float (&rb)[8]) const {
    const int slot = __builtin_amdgcn_readfirstlane(r0 / g.Cout);
    const int co0 = r0 - slot * g.Cout;
    int kh, kw;
    if (g.rect.ok) rect_tap(g.rect, slot, kh, kw); else { kh = g.tap_kh[slot]; kw = g.tap_kw[slot]; }
    const int KK = g.KH * g.KW, HoWo = (int)g.syc;  // channel stride
    const int aoff = co0 * g.Cin * KK + kh * g.KW + kw;
#pragma unroll
    for (int i = 0; i < 8; ++i) ra[i] = s.mok ? s.wk[s.abase + aoff + 4 * i * g.Cin * KK] : 0.f;
    const int nh = s.ih - kh, nw = s.iw - kw;
    int oh, ow;
    bool ok = s.nok && nh >= 0 && nw >= 0;
    if (g.stride == 1) {
      oh = nh; ow = nw;
    } else {
      oh = nh / g.stride; ow = nw / g.stride;
      ok = ok && oh * g.stride == nh && ow * g.stride == nw;
    }
    ok = ok && oh < g.Ho && ow < g.Wo;
    const int boff = s.yoff + co0 * HoWo + oh * g.Wo + ow;
#pragma unroll
    for (int i = 0; i < 8; ++i) rb[i] = ok ? s.dyk[boff + 4 * i * HoWo] : 0.f;
  }
};

struct WgtF : WgtG {  // n-tile inside one tap (Cin % 64 == 0); A and B fast along r (q)
  struct State {
    const float* dyk; const float* xk;
    int abase[8]; bool mok[8];
    int bbase[8];
    int kh, kw, ci0, ql;
  };
  __device__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.dyk = dy + k * g.syk;
    s.xk = x + k * g.sxk;
    const int slot = n0 / g.Cin;
    s.ci0 = n0 - slot * g.Cin;
    s.kh = g.tap_kh[slot];
    s.kw = g.tap_kw[slot];
    s.ql = tid % BK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + tid / BK + 8 * i;
      s.mok[i] = m < g.Cout;
      s.abase[i] = (int)(m * g.syc);
      s.bbase[i] = (int)((s.ci0 + tid / BK + 8 * i) * g.sxc);
    }
    return s;
  }
  __device__ void load(const State& s, int r0, int re, float (&ra)[8], float (&rb)[8]) const {
    const int q = r0 + s.ql;
    const bool qok = q < re;
    const uint32_t bb = udiv(q, g.d_howo), p = q - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    const int aoff = (int)(bb * g.syb + p);
#pragma unroll
    for (int i = 0; i < 8; ++i) ra[i] = (qok && s.mok[i]) ? s.dyk[s.abase[i] + aoff] : 0.f;
    const int ih = (int)oh * g.stride - g.pad + s.kh, iw = (int)ow * g.stride - g.pad + s.kw;
    const bool ok = qok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
    const int boff = (int)(bb * g.sxb) + ih * g.W + iw;
#pragma unroll
    for (int i = 0; i < 8; ++i) rb[i] = ok ? s.xk[s.bbase[i] + boff] : 0.f;
  }
};

// ---- the implicit-GEMM kernel ---------------------------------------------
// Split-K: blockIdx.z = client * S + split; split s reduces the BK-aligned
// range [rb, re) and, when S > 1, writes its tile to part[(s*K + k)][M][N];
// cgemm_reduce then adds the S partials in split order (deterministic).
template <class Prob>
__global__ __launch_bounds__(THREADS, 2) void cgemm_kernel(const Prob pb, int S, float* __restrict__ part) {
  __shared__ float As[2][BK * LDS_STRIDE];
  __shared__ float Bs[2][BK * LDS_STRIDE];
  const int k = blockIdx.z / S, split = blockIdx.z % S;
  const int M = pb.M(), N = pb.N(), R = pb.R();
  const int ktiles = cdiv(R, BK);
  const int rb = (int)((int64_t)ktiles * split / S) * BK, re = min(R, (int)((int64_t)ktiles * (split + 1) / S) * BK);
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;

  float ra[8], rb_[8];
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int am, ak, bn, bk;
      slot_of(Prob::FAST_A_M, tid, i, am, ak);
      slot_of(Prob::FAST_B_N, tid, i, bn, bk);
      As[buf][ak * LDS_STRIDE + am] = ra[i];
      Bs[buf][bk * LDS_STRIDE + bn] = rb_[i];
    }
  };
  const auto st = pb.init(k, m0, n0, tid);

  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  auto loadr = [&](int r0) { pb.load(st, r0, re, ra, rb_); };
  loadr(rb);
  stash(0);
  __syncthreads();
  int cur = 0;
  for (int r0 = rb; r0 < re; r0 += BK) {
    const bool more = r0 + BK < re;
    if (more) loadr(r0 + BK);  // in flight during the MFMAs below
    const float* Ab = As[cur] + 32 * wm + l32;
    const float* Bb = Bs[cur] + 32 * wn + l32;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int kk = 16 * h + q;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ab[kk * LDS_STRIDE], Bb[kk * LDS_STRIDE], acc, 0, 0, 0);
    }
    if (more) stash(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  // C/D map of 32x32 MFMA: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int n = n0 + 32 * wn + l32;
    if (m < M && n < N) {
      if (S == 1) pb.store(k, m, n, acc[e]);
      else part[(((int64_t)split * pb.g.Kc + k) * M + m) * N + n] = acc[e];
    }
  }
}

// dw[e] = 0 for every element of a dead kernel tap (e % KK in the dead mask).
// A kernel rather than hipMemsetAsync: a memset captured inside the training
// phase's HIP graph was observed not to take effect on replays.
__global__ void zero_dead_taps_kernel(float* __restrict__ dw, int64_t n, int KK, uint64_t dead) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    if ((dead >> (int)(e % KK)) & 1ull) dw[e] = 0.f;
}

template <class Prob>
__global__ void cgemm_reduce(const Prob pb, int S, const float* __restrict__ part) {
  const int M = pb.M(), N = pb.N(), K = pb.g.Kc;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = (int64_t)M * N;
  if (idx >= MN * K) return;
  const int k = (int)(idx / MN);
  const int m = (int)((idx % MN) / N), n = (int)(idx % N);
  float v = part[idx];
  for (int s = 1; s < S; ++s) v += part[(int64_t)s * MN * K + idx];
  pb.store(k, m, n, v);
}

// Splits so that a launch has >= ~2048 workgroups while each split keeps >= 8 K-tiles.
// Split-K count from the PER-CLIENT problem only (never the client count K):
// a client's reduction order — and so its trained weights — must not depend
// on how many clients share its GPU (bit-identical results at 1/2/4/8 GPUs).
// 16 tiles per client = the 2048-workgroup target at the nominal 128 clients.
inline int choose_splits(int M, int N, int R, int /*K*/) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int ktiles = cdiv(R, BK);
  int S = 1;
  while (S < 16 && tiles * S < 16 && ktiles / (2 * S) >= 8) S *= 2;
  return S;
}

template <class Prob>
size_t splits_workspace(const Prob& pb) {
  const int S = choose_splits(pb.M(), pb.N(), pb.R(), pb.g.Kc);
  return S > 1 ? (size_t)S * pb.g.Kc * pb.M() * pb.N() * sizeof(float) : 0;
}

template <class Prob>
int launch(const Prob& pb, void* ws, size_t ws_bytes, hipStream_t st, const char* name) {
  const int M = pb.M(), N = pb.N(), R = pb.R(), K = pb.g.Kc;
  if (R == 0) return FLR_OK;
  int S = choose_splits(M, N, R, K);
  if (S > 1 && (!ws || ws_bytes < splits_workspace(pb))) S = 1;  // no workspace: single split
  dim3 grid((unsigned)cdiv(N, BN), (unsigned)cdiv(M, BM), (unsigned)(K * S));
  hipLaunchKernelGGL(cgemm_kernel<Prob>, grid, dim3(THREADS), 0, st, pb, S, static_cast<float*>(ws));
  int rc = launch_status(name);
  if (rc != FLR_OK || S == 1) return rc;
  const int64_t total = (int64_t)M * N * K;
  hipLaunchKernelGGL(cgemm_reduce<Prob>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, pb, S,
                     static_cast<const float*>(ws));
  return launch_status(name);
}

}  // namespace conv
}  // namespace flr

using namespace flr;
using namespace flr::conv;

// FLR_CONV_GENERIC=1 forces the generic gathers (A/B timing and cross-checks).
static int generic_conv_forced() {
  static const int v = [] {
    const char* e = flr::knob("FLR_CONV_GENERIC");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v;
}

extern "C" size_t flr_conv2d_workspace(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                                       int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  if (!geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad)) return 0;
  const Geom g = make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  Fwd f; f.g = g; Dgrad d; d.g = g; Wgt w; w.g = g;
  size_t m = splits_workspace(f);
  m = std::max(m, splits_workspace(d));
  m = std::max(m, splits_workspace(w));
  if (convt::im2col_eligible(g)) m = std::max(m, convt::im2col_workspace(g));
  return m;
}

extern "C" int flr_conv2d_fwd(const float* x, const float* w, float* y, int64_t K, int64_t B, int64_t Cin, int64_t H,
                              int64_t W, int64_t Cout, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                              void* ws, size_t ws_bytes, void* stream) {
  if (!x || !w || !y || !geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad)) return FLR_ERR_ARG;
  const Geom g = make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  if (generic_conv_forced() == 0 && convt::im2col_eligible(g) && ws && ws_bytes >= convt::im2col_workspace(g))
    return convt::fwd_im2col(g, x, w, y, ws, ws_bytes, as_stream(stream));
  if (Cin % BK == 0 && generic_conv_forced() == 0) {
    FwdF pb;
    pb.g = g; pb.x = x; pb.w = w; pb.y = y;
    return launch(pb, ws, ws_bytes, as_stream(stream), "conv fwd");
  }
  Fwd pb;
  pb.g = g; pb.x = x; pb.w = w; pb.y = y;
  return launch(pb, ws, ws_bytes, as_stream(stream), "conv fwd");
}

extern "C" int flr_conv2d_bwd_data(const float* dy, const float* w, float* dx, int64_t K, int64_t B, int64_t Cin,
                                   int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                   int64_t pad, void* ws, size_t ws_bytes, void* stream) {
  if (!dy || !w || !dx || !geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad)) return FLR_ERR_ARG;
  const Geom g = make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  if (Cout % BK == 0 && generic_conv_forced() == 0) {
    DgradF pb;
    pb.g = g; pb.dy = dy; pb.w = w; pb.dx = dx;
    return launch(pb, ws, ws_bytes, as_stream(stream), "conv bwd data");
  }
  Dgrad pb;
  pb.g = g; pb.dy = dy; pb.w = w; pb.dx = dx;
  return launch(pb, ws, ws_bytes, as_stream(stream), "conv bwd data");
}

static int bwd_weight(const float* x, const float* dy, float* dw, int64_t K, int64_t B, int64_t Cin, int64_t H,
                      int64_t W, int64_t Cout, int64_t KH, int64_t KW, int64_t stride, int64_t pad, void* ws,
                      size_t ws_bytes, void* stream, bool have_col) {
  if (!x || !dy || !dw || !geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad)) return FLR_ERR_ARG;
  const Geom g = make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  hipStream_t st = as_stream(stream);
  if (g.ntaps < KH * KW) {  // dead taps get exact-zero gradients
    if (KH * KW > 64) return FLR_ERR_UNSUPPORTED;
    uint64_t dead = (KH * KW == 64) ? ~0ull : ((1ull << (KH * KW)) - 1);
    for (int t = 0; t < g.ntaps; ++t) dead &= ~(1ull << (g.tap_kh[t] * KW + g.tap_kw[t]));
    const int64_t n = K * Cout * Cin * KH * KW;
    hipLaunchKernelGGL(zero_dead_taps_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                       st, dw, n, (int)(KH * KW), dead);
    const int rc = launch_status("conv bwd weight: zero dead taps");
    if (rc != FLR_OK) return rc;
  }
  if (generic_conv_forced() == 0 && convt::im2col_eligible(g) && ws && ws_bytes >= convt::im2col_workspace(g))
    return convt::wgrad_im2col(g, x, dy, dw, ws, ws_bytes, st, have_col);
  if (Cin % BN == 0 && generic_conv_forced() == 0) {
    WgtF pb;
    pb.g = g; pb.x = x; pb.dy = dy; pb.dw = dw;
    return launch(pb, ws, ws_bytes, st, "conv bwd weight");
  }
  Wgt pb;
  pb.g = g; pb.x = x; pb.dy = dy; pb.dw = dw;
  return launch(pb, ws, ws_bytes, st, "conv bwd weight");
}

extern "C" int flr_conv2d_bwd_weight(const float* x, const float* dy, float* dw, int64_t K, int64_t B, int64_t Cin,
                                     int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                     int64_t pad, void* ws, size_t ws_bytes, void* stream) {
  return bwd_weight(x, dy, dw, K, B, Cin, H, W, Cout, KH, KW, stride, pad, ws, ws_bytes, stream, false);
}

extern "C" int flr_conv2d_bwd_weight_reuse(const float* x, const float* dy, float* dw, int64_t K, int64_t B,
                                           int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                                           int64_t stride, int64_t pad, void* ws, size_t ws_bytes, void* stream) {
  return bwd_weight(x, dy, dw, K, B, Cin, H, W, Cout, KH, KW, stride, pad, ws, ws_bytes, stream, true);
}
