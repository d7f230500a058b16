// a2 — client-batched convolution with TAP-MAJOR weights, the training
// engine's layout for every conv whose channel counts are multiples of 64
// (all of ResNet-18 but the stem).  Same products as train_conv.hip
// (nn.Conv2d(bias=False) of the conv blocks, src/models/cub200_cnn.py:71-77
// template; trained per client in run_experiments.py:216-235), with the
// weights of client k stored as W_t[k][kh][kw][Cin][Cout] instead of torch's
// [Cout][Cin][kh][kw].  The trainer converts at the round boundaries
// (load_global / export); inside the round nothing else sees the layout.
//
// Why: at a fixed kernel tap the weight slab is a plain [Cin][Cout] matrix, so
//   fwd   A(m = co, k = ci) is contiguous along m -> 16-B loads, [k][m] LDS image
//   dgrad A(m = ci, k = co) is contiguous along k -> 16-B loads, [m][k] LDS image
//   wgrad writes C(m = ci, n = co) with coalesced rows.
// The activation operand is an im2col gather; it uses raw buffer loads whose
// per-element stride sits in soffset (an SGPR) and whose padding taps carry an
// out-of-range voffset (the hardware returns 0), so a gathered element costs
// no VALU work — f32 MFMA shares the VALU's issue rate on gfx950, so address
// arithmetic comes straight out of matrix throughput.
//
// Tiles: 64 x 64 outputs per workgroup, 32-deep K-tiles (one kernel tap each:
// C % 64 == 0), 4 waves of 32 x 32, v_mfma_f32_32x32x2_f32; MFMA (j, t) of a
// K-tile feeds reduction index 8j + 4h + t from lane half h, so an operand
// held as [row][k] is read with one ds_read_b128 per four MFMAs and one held
// as [k][row] with ds_read_b32.  Register-staged one K-tile ahead, double-
// buffered LDS, deterministic split-K for long reductions (partials reduced
// in split order).
#include "conv_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

// The file compiles as one translation unit, or (Makefile) as five parts that
// build in parallel, -DFLR_CT_PART=0..4: 0 the im2col / stem path and the
// workspace query, 1 the forward, 2 the data gradient, 3 the weight gradient,
// 4 the batched GEMM and row sums.  Device templates are shared; each part
// instantiates only the kernels its entry points launch.
#ifdef FLR_CT_PART
#define FLR_CT_P0 (FLR_CT_PART == 0)
#define FLR_CT_P1 (FLR_CT_PART == 1)
#define FLR_CT_P2 (FLR_CT_PART == 2)
#define FLR_CT_P3 (FLR_CT_PART == 3)
#define FLR_CT_P4 (FLR_CT_PART == 4)
#else
#define FLR_CT_P0 1
#define FLR_CT_P1 1
#define FLR_CT_P2 1
#define FLR_CT_P3 1
#define FLR_CT_P4 1
#endif

namespace flr {
namespace convt {

using conv::Geom;
using conv::udiv;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 64, BN = 64, BK = 32, THREADS = 256;
constexpr int SKR = 68;  // [k][row] image row stride (floats)
constexpr int SRK = 36;  // [row][k] image row stride
constexpr int TILE = 64 * SRK;
constexpr unsigned SENT = 0x80000000u;  // out-of-range voffset: the load returns 0

enum Lay { KR_VEC = 0, KR_GATHER = 1, RK_VEC = 2, RK_GATHER = 3 };

using rsrc_t = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int64_t nfloats) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane((int)(nfloats * 4));
  void* b = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float ld1(rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ f32x4 ld4(rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// ---- LDS images -------------------------------------------------------------
template <int LAY>
__device__ __forceinline__ void stash(float* buf, const float (&v)[8], int tid) {
  if constexpr (LAY == KR_VEC) {  // thread: 4 rows (tid % 16), k = tid / 16 + 16 i
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *reinterpret_cast<f32x4*>(buf + (tid / 16 + 16 * i) * SKR + 4 * (tid % 16)) =
          f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
  } else if constexpr (LAY == KR_GATHER) {  // row tid % 64, k = tid / 64 + 4 i
#pragma unroll
    for (int i = 0; i < 8; ++i) buf[(tid / 64 + 4 * i) * SKR + tid % 64] = v[i];
  } else if constexpr (LAY == RK_VEC) {  // row tid / 8 + 32 i, k = 4 (tid % 8) .. +3
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *reinterpret_cast<f32x4*>(buf + (tid / 8 + 32 * i) * SRK + 4 * (tid % 8)) =
          f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
  } else {  // RK_GATHER: row tid / 32 + 8 i, k = tid % 32
#pragma unroll
    for (int i = 0; i < 8; ++i) buf[(tid / 32 + 8 * i) * SRK + tid % 32] = v[i];
  }
}

// Operand values of MFMAs (j, 0..3) for this lane: k = 8j + 4h + t, row = rb.
template <int LAY>
__device__ __forceinline__ f32x4 frag(const float* buf, int rb, int j, int h) {
  if constexpr (LAY == RK_VEC || LAY == RK_GATHER) {
    return *reinterpret_cast<const f32x4*>(buf + rb * SRK + 8 * j + 4 * h);
  } else {
    const float* p = buf + (8 * j + 4 * h) * SKR + rb;
    return f32x4{p[0], p[SKR], p[2 * SKR], p[3 * SKR]};
  }
}

// ---- the bf16x6 MFMA form ----------------------------------------------------
// f32 MFMA runs at 1/16 of the bf16 rate on gfx950.  Each f32 operand is split
// into three round-to-nearest bf16 terms, x = hi + mid + lo (the residual is
// below 2^-24 |x|: 24 significand bits in three 8-bit pieces), and the six
// products whose order is above 2^-24 (hi*hi, hi*mid, mid*hi, mid*mid, hi*lo,
// lo*hi; every bf16 x bf16 product is exact in the fp32 accumulator) run on
// v_mfma_f32_32x32x16_bf16: 6 x 32 cycles per 16-deep k-step against 8 x 64 for
// v_mfma_f32_32x32x2_f32, at a per-product error of a few 2^-24 |a b| — the
// rounding of an fp32 product.  The LDS images stay fp32; each wave splits
// the eight values of its fragment: lane (l32, h) supplies row l32 and
// reduction indices k0 .. k0+7, k0 = 16 s + 8 h.
template <int LAY>
__device__ __forceinline__ void frag8(const float* buf, int rb, int k0, float (&v)[8]) {
  if constexpr (LAY == RK_VEC || LAY == RK_GATHER) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(buf + rb * SRK + k0);
    const f32x4 b = *reinterpret_cast<const f32x4*>(buf + rb * SRK + k0 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = a[e];
      v[4 + e] = b[e];
    }
  } else {
    const float* p = buf + k0 * SKR + rb;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p[e * SKR];
  }
}

// The residuals r = v - (float)bf16(v) come from v_dot2_f32_bf16 against
// (-1, 0) / (0, -1): one instruction per value instead of a bf16 -> fp32
// expansion plus a subtraction.  r is exact either way (|r| <= half a bf16
// ulp of v, representable in fp32), so the split is bit-identical to the
// plain form (tools/hip/split_check.hip checks 2^24 random patterns).
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#ifdef FLR_AB_SPLIT_PLAIN  // A/B build (tools/ab_build.sh): expansion + subtraction
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a = (__bf16)v[j];
    const float r1 = v[j] - (float)a;
    const __bf16 b = (__bf16)r1;
    hi[j] = a;
    mid[j] = b;
    lo[j] = (__bf16)(r1 - (float)b);
  }
  return;
#endif
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  // (-1, 0) and (0, -1) as opaque SGPRs: hipcc encodes a (-1, 0) constant as the
  // inline constant -1.0, which the hardware reads as the fp32 bits, i.e. (0, -1)
  unsigned klo, khi;  // non-volatile: the compiler may hoist / share them
  asm("s_mov_b32 %0, 0xbf80" : "=s"(klo));
  asm("s_mov_b32 %0, 0xbf800000" : "=s"(khi));
  const bf16x2 nl = __builtin_bit_cast(bf16x2, klo), nh = __builtin_bit_cast(bf16x2, khi);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float v0 = v[2 * p], v1 = v[2 * p + 1];
    const bf16x2 a = {(__bf16)v0, (__bf16)v1};
    const float r0 = __builtin_amdgcn_fdot2_f32_bf16(a, nl, v0, false);
    const float r1 = __builtin_amdgcn_fdot2_f32_bf16(a, nh, v1, false);
    const bf16x2 b = {(__bf16)r0, (__bf16)r1};
    const float s0 = __builtin_amdgcn_fdot2_f32_bf16(b, nl, r0, false);
    const float s1 = __builtin_amdgcn_fdot2_f32_bf16(b, nh, r1, false);
    hi[2 * p] = a[0];
    hi[2 * p + 1] = a[1];
    mid[2 * p] = b[0];
    mid[2 * p + 1] = b[1];
    lo[2 * p] = (__bf16)s0;
    lo[2 * p + 1] = (__bf16)s1;
  }
}

// FLR_GEMM=f32 selects the exact-f32 MFMA (A/B timing, cross-checks); read per
// launch so one process can compare both forms.
// FLR_XCD=0 turns the XCD-aware tile order off (A/B timing).
// bit 0: the XCD-aware tile order; A/B (split-at-stash kernels): bits 8-15
// FLR_GEMM_STAGGER = n, workgroups of odd XCD slot start n x 512 cycles late;
// bit 16 FLR_GEMM_SPRIO=1, those workgroups at s_setprio 1 for the whole loop
inline int xcd_remap() {
  const char* e = flr::knob("FLR_XCD");
  int r = (e && e[0] == '0') ? 0 : 1;
  const char* st = flr::knob("FLR_GEMM_STAGGER");
  if (st) r |= (std::min(255, std::max(0, atoi(st))) << 8);
  const char* sp = flr::knob("FLR_GEMM_SPRIO");
  if (sp && sp[0] == '1') r |= 1 << 16;
  return r;
}
// the A/B controls above, at the start of a split-at-stash kernel
__device__ __forceinline__ void odd_slot_controls(int remap) {
  const int lid = (int)blockIdx.x + (int)gridDim.x * ((int)blockIdx.y + (int)gridDim.y * (int)blockIdx.z);
  if (((lid >> 3) & 1) == 0) return;
  if ((remap >> 16) & 1) __builtin_amdgcn_s_setprio(1);
  for (int i = (remap >> 8) & 255; i > 0; --i) __builtin_amdgcn_s_sleep(8);
}

// Wave priority raised around each MFMA cluster (FLR_PRIO=0: off, for A/B).
inline int mfma_prio() {  // measured +0-5 % on the encoder GEMMs and the 3x3 convs (FLR_PRIO=0 turns it off)
  const char* e = flr::knob("FLR_PRIO");
  return (e && e[0] == '0') ? 0 : 1;
}

// 0: exact f32 MFMA; 2: bf16x6, product-major, software-pipelined; 5 (default):
// split at stash time where the plan supports it (fwd / dgrad / batched GEMM),
// else 2.  FLR_GEMM=f32 | pipe | stash.  The tools build (make ABLATION=1) adds
// the measured-slower forms 1 (accumulator-chain order, FLR_GEMM=chain) and 4
// (the unpipelined loop, =old), and the wrong-result timing ablation 3 (=A).
inline int gemm_form() {
  const char* e = flr::knob("FLR_GEMM");
  if (e && e[0] == 'f') return 0;
#ifdef FLR_ABLATION
  if (e && e[0] == 'c') return 1;
  if (e && e[0] == 'A') return 3;  // ablation (timing only, wrong results): one bf16 term, no split; tools build only
  if (e && e[0] == 'o') return 4;  // the unpipelined product-major loop (A/B timing)
#endif
  if (e && e[0] == 'p') return 2;  // the pipelined loop for every plan
  return 5;  // split at stash (bf16 LDS images) where the plan has k8 loads, else pipelined
}

// ---- load plans ---------------------------------------------------------------
// Tap of a reduction slot: W_t offset of (tap, 0, 0) = tap_index * Cin * Cout.
// (kh, kw) of a tile-uniform reduction slot, by rectangle arithmetic (the host
// accepts only geometries whose live taps form a rectangle: args_ok)
__device__ __forceinline__ void slot_tap(const Geom& g, int slot, int& kh, int& kw) {
  conv::rect_tap(g.rect, slot, kh, kw);
}
__device__ __forceinline__ int tap_index(const Geom& g, int slot) {
  int kh, kw;
  slot_tap(g, slot, kh, kw);
  return kh * g.KW + kw;
}
// Tile-uniform values the compiler cannot prove uniform (the tap table is
// indexed by a computed slot): broadcast so they live in SGPRs and the buffer
// loads that take them as soffset need no waterfall loop.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Split-at-stash forms (sgemm_body): the thread that loads 8 consecutive k of
// one operand row stashes them as bf16x8.  Row-contiguous operands put the 64
// lanes of a wave on 64 consecutive rows (coalesced along the row); a
// k-contiguous operand instead puts 4 lanes on each row (QUAD: row tid / 4,
// k 8 (tid % 4)), so a wave's load covers 16 rows x 128 B instead of 64 rows x
// 32 B (64 cache lines per instruction).  FLR_QUAD=0 at build time: the plain
// mapping everywhere (A/B).
#ifndef FLR_QUAD
#define FLR_QUAD 1
#endif
template <bool QUAD> __device__ __forceinline__ int stash_row(int tid) { return QUAD ? tid >> 2 : tid & 63; }
template <bool QUAD> __device__ __forceinline__ int stash_k(int tid) { return QUAD ? 8 * (tid & 3) : 8 * (tid >> 6); }

struct FwdT {  // y = conv(x, W_t): M = Cout, N = B*Ho*Wo, R = ntaps*Cin
  static constexpr bool QUAD_A = false, QUAD_B = false;
  Geom g;
  const float* x;
  const float* w;
  float* y;
  int64_t wsk;  // weight floats between clients (KK*Cin*Cout; 0: every client reads one shared copy)
  static constexpr int LA = KR_VEC, LB = KR_GATHER;
  __host__ __device__ __forceinline__ int M() const { return g.Cout; }
  __host__ __device__ __forceinline__ int N() const { return g.B * g.Ho * g.Wo; }
  __host__ __device__ __forceinline__ int R() const { return g.ntaps * g.Cin; }
  struct State {
    rsrc_t ra, rb;
    unsigned a0;            // byte offset of (k-row tid/16, m 4*(tid%16)) at tap 0, ci 0
    int ih0, iw0, xoff;     // this thread's output pixel (B operand)
    bool nok;
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    const int KK = g.KH * g.KW;
    s.ra = make_rsrc(w + (int64_t)k * wsk, (int64_t)KK * g.Cin * g.Cout);
    s.rb = make_rsrc(x + k * g.sxk, g.xext);
    s.a0 = (unsigned)(((tid / 16) * g.Cout + m0 + 4 * (tid % 16)) * 4);
    const int n = n0 + tid % 64;
    s.nok = n < N();
    const uint32_t bb = udiv(n, g.d_howo), p = n - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    s.ih0 = (int)oh * g.stride - g.pad;
    s.iw0 = (int)ow * g.stride - g.pad;
    s.xoff = (int)(bb * g.sxb + (tid / 64) * g.sxc);
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const int slot = uni(r0 / g.Cin), ci0 = r0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    kh = uni(kh);
    kw = uni(kw);
    const int arow = ((kh * g.KW + kw) * g.Cin + ci0) * g.Cout * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 q = ld4(s.ra, s.a0, arow + i * 16 * g.Cout * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[4 * i + e] = q[e];
    }
  }
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const int slot = uni(r0 / g.Cin), ci0 = r0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    kh = uni(kh);
    kw = uni(kw);
    const int HW = (int)g.sxc;  // channel stride
    const int ih = s.ih0 + kh, iw = s.iw0 + kw;
    // bitwise & (no short-circuit): the gather stays branch-free, one basic block with the MFMAs
    const bool ok = s.nok & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
    const unsigned addr = (unsigned)((s.xoff + ih * g.W + iw) * 4);
    const unsigned vb = ok ? addr : SENT;
    const int cb = ci0 * HW * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = ld1(s.rb, vb, cb + i * 4 * HW * 4);
  }
  // y[k][m][n]: n = b*Ho*Wo + p is linear in the [K][C][B][Ho][Wo] layout
  __device__ __forceinline__ void store(int k, int m, int n, float v) const { y[k * g.syk + m * g.syc + n] = v; }
  __device__ __forceinline__ bool linear() const { return true; }
  __device__ __forceinline__ float* out() const { return y; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return k * g.syk + m0 * g.syc + n0; }
  __device__ __forceinline__ int64_t ldm() const { return g.syc; }
  // ---- k-contiguous loads for the split-at-stash kernel: thread (row = tid & 63,
  // k = 8 (tid >> 6) .. +7) of a 64 x 32 sub-tile
  struct State8 {
    rsrc_t ra, rb;
    unsigned a0;
    int ih0, iw0, xoff;
    bool nok;
  };
  __device__ __forceinline__ State8 init8(int k, int m0, int n0, int tid) const {
    State8 s;
    const int KK = g.KH * g.KW;
    const int row = tid & 63, k0 = 8 * (tid >> 6);
    s.ra = make_rsrc(w + (int64_t)k * wsk, (int64_t)KK * g.Cin * g.Cout);
    s.rb = make_rsrc(x + k * g.sxk, g.xext);
    s.a0 = (unsigned)((k0 * g.Cout + m0 + row) * 4);
    const int n = n0 + row;
    s.nok = n < N();
    const uint32_t bb = udiv(n, g.d_howo), p = n - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    s.ih0 = (int)oh * g.stride - g.pad;
    s.iw0 = (int)ow * g.stride - g.pad;
    s.xoff = (int)(bb * g.sxb + k0 * g.sxc);
    return s;
  }
  __device__ __forceinline__ void load_a8(const State8& s, int r0, float (&a)[8]) const {  // A(co, ci): lanes along co
    const int slot = uni((int)udiv((uint32_t)r0, g.d_cin)), ci0 = r0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    const int arow = uni(((kh * g.KW + kw) * g.Cin + ci0) * g.Cout * 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = ld1(s.ra, s.a0, arow + e * g.Cout * 4);
  }
  __device__ __forceinline__ void load_b8(const State8& s, int r0, float (&b)[8]) const {  // B(pixel, ci): 8 channels
    const int slot = uni((int)udiv((uint32_t)r0, g.d_cin)), ci0 = r0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    kh = uni(kh);
    kw = uni(kw);
    const int HW = (int)g.sxc;
    const int ih = s.ih0 + kh, iw = s.iw0 + kw;
    const bool ok = s.nok & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
    const unsigned addr = (unsigned)((s.xoff + ih * g.W + iw) * 4);
    const unsigned vb = ok ? addr : SENT;
    const int cb = ci0 * HW * 4;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = ld1(s.rb, vb, cb + e * HW * 4);
  }
};

// dx = conv^T(dy, W_t) over ONE stride-parity class of input pixels:
// ih = ca + stride*ihc, iw = cb + stride*iwc.  Only the taps kh = (ih + pad)
// mod stride (same for kw) reach such a pixel, so a class is a dense GEMM
// M = Cin, N = B*Hc*Wc, R = ntc*Cout with no zero-padded taps — a stride-2
// dgrad runs the four classes and does the fwd's MFMA work, not four times
// it.  Stride 1 is the single class (0, 0) with every live tap.
struct DgradT {
  static constexpr bool QUAD_A = FLR_QUAD != 0, QUAD_B = false;
  Geom g;
  const float* dy;
  const float* w;
  float* dx;
  const float* add;  // optional addend in dx's layout: dx = dgrad + add (one rounding)
  int64_t wsk;       // weight floats between clients (KK*Cin*Cout; 0: one shared copy)
  int ca, cb, Hc, Wc, ntc;
  conv::FastDiv d_hcwc, d_wc;
  int8_t ckh[conv::MAXTAPS], ckw[conv::MAXTAPS];
  conv::TapRect crect;  // the class taps: a rectangle of step = stride
  static constexpr int LA = RK_VEC, LB = KR_GATHER;
  __host__ __device__ __forceinline__ int M() const { return g.Cin; }
  __host__ __device__ __forceinline__ int N() const { return g.B * Hc * Wc; }
  __host__ __device__ __forceinline__ int R() const { return ntc * g.Cout; }
  struct State {
    rsrc_t ra, rb;
    unsigned a0;
    int ih, iw, yoff;  // ih, iw: this lane's input pixel + pad
    bool nok;
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    const int KK = g.KH * g.KW;
    s.ra = make_rsrc(w + (int64_t)k * wsk, (int64_t)KK * g.Cin * g.Cout);
    s.rb = make_rsrc(dy + k * g.syk, g.yext);
    s.a0 = (unsigned)(((m0 + tid / 8) * g.Cout + 4 * (tid % 8)) * 4);
    const int n = n0 + tid % 64;
    s.nok = n < N();
    const uint32_t bb = udiv(n, d_hcwc), p = n - bb * Hc * Wc;
    const uint32_t ihc = udiv(p, d_wc), iwc = p - ihc * Wc;
    s.ih = ca + (int)ihc * g.stride + g.pad;
    s.iw = cb + (int)iwc * g.stride + g.pad;
    s.yoff = (int)(bb * g.syb + (tid / 64) * g.syc);
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const int slot = uni(r0 / g.Cout), co0 = r0 - slot * g.Cout;
    int kh, kw;
    conv::rect_tap(crect, slot, kh, kw);
    kh = uni(kh);
    kw = uni(kw);
    const int abase = ((kh * g.KW + kw) * g.Cin * g.Cout + co0) * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 q = ld4(s.ra, s.a0, abase + i * 32 * g.Cout * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[4 * i + e] = q[e];
    }
  }
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const int slot = uni(r0 / g.Cout), co0 = r0 - slot * g.Cout;
    int kh, kw;
    conv::rect_tap(crect, slot, kh, kw);
    kh = uni(kh);
    kw = uni(kw);
    // the class guarantees (ih + pad - kh) % stride == 0
    const int nh = s.ih - kh, nw = s.iw - kw;
    const int oh = g.stride == 1 ? nh : nh / g.stride, ow = g.stride == 1 ? nw : nw / g.stride;
    const bool ok = s.nok & (nh >= 0) & (nw >= 0) & (oh < g.Ho) & (ow < g.Wo);
    const unsigned addr = (unsigned)((s.yoff + oh * g.Wo + ow) * 4);
    const unsigned vb = ok ? addr : SENT;
    const int cs = (int)g.syc;  // channel stride
    const int cb0 = co0 * cs * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = ld1(s.rb, vb, cb0 + i * 4 * cs * 4);
  }
  __device__ __forceinline__ void store(int k, int m, int n, float v) const {
    const uint32_t bb = udiv(n, d_hcwc), p = n - bb * Hc * Wc;
    const uint32_t ihc = udiv(p, d_wc), iwc = p - ihc * Wc;
    const int ih = ca + (int)ihc * g.stride, iw = cb + (int)iwc * g.stride;
    const int64_t i = k * g.sxk + m * g.sxc + bb * g.sxb + ih * g.W + iw;
    dx[i] = add ? __fadd_rn(v, add[i]) : v;
  }
  __device__ __forceinline__ int64_t index(int k, int m, int n) const {  // dx offset of output (m, n) of client k
    const uint32_t bb = udiv(n, d_hcwc), p = n - bb * Hc * Wc;
    const uint32_t ihc = udiv(p, d_wc), iwc = p - ihc * Wc;
    const int ih = ca + (int)ihc * g.stride, iw = cb + (int)iwc * g.stride;
    return k * g.sxk + m * g.sxc + bb * g.sxb + ih * g.W + iw;
  }
  // stride 1 (the one class is every pixel): dx[k][m][n] is linear in n
  __device__ __forceinline__ bool linear() const { return g.stride == 1; }
  __device__ __forceinline__ float* out() const { return dx; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return k * g.sxk + m0 * g.sxc + n0; }
  __device__ __forceinline__ int64_t ldm() const { return g.sxc; }
  struct State8 {
    rsrc_t ra, rb;
    unsigned a0;
    int ih, iw, yoff;
    bool nok;
  };
  __device__ __forceinline__ State8 init8(int k, int m0, int n0, int tid) const {
    State8 s;
    const int KK = g.KH * g.KW;
    const int row = tid & 63, k0 = 8 * (tid >> 6);
    s.ra = make_rsrc(w + (int64_t)k * wsk, (int64_t)KK * g.Cin * g.Cout);
    s.rb = make_rsrc(dy + k * g.syk, g.yext);
    // A = W(ci, co) is k-contiguous: quad lanes (stash_row / stash_k, QUAD_A)
    s.a0 = (unsigned)(((m0 + stash_row<QUAD_A>(tid)) * g.Cout + stash_k<QUAD_A>(tid)) * 4);
    const int n = n0 + row;
    s.nok = n < N();
    const uint32_t bb = udiv(n, d_hcwc), p = n - bb * Hc * Wc;
    const uint32_t ihc = udiv(p, d_wc), iwc = p - ihc * Wc;
    s.ih = ca + (int)ihc * g.stride + g.pad;
    s.iw = cb + (int)iwc * g.stride + g.pad;
    s.yoff = (int)(bb * g.syb + k0 * g.syc);
    return s;
  }
  __device__ __forceinline__ void load_a8(const State8& s, int r0, float (&a)[8]) const {  // A(ci, co): 8 consecutive co
    const int slot = uni((int)udiv((uint32_t)r0, g.d_cout)), co0 = r0 - slot * g.Cout;
    int kh, kw;
    conv::rect_tap(crect, slot, kh, kw);
    const int abase = uni(((kh * g.KW + kw) * g.Cin * g.Cout + co0) * 4);
    const f32x4 q0 = ld4(s.ra, s.a0, abase), q1 = ld4(s.ra, s.a0, abase + 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = q0[e];
      a[4 + e] = q1[e];
    }
  }
  __device__ __forceinline__ void load_b8(const State8& s, int r0, float (&b)[8]) const {  // B(input pixel, co): 8 channels
    const int slot = uni((int)udiv((uint32_t)r0, g.d_cout)), co0 = r0 - slot * g.Cout;
    int kh, kw;
    conv::rect_tap(crect, slot, kh, kw);
    kh = uni(kh);
    kw = uni(kw);
    const int nh = s.ih - kh, nw = s.iw - kw;
    const int oh = g.stride == 1 ? nh : nh / g.stride, ow = g.stride == 1 ? nw : nw / g.stride;
    const bool ok = s.nok & (nh >= 0) & (nw >= 0) & (oh < g.Ho) & (ow < g.Wo);
    const unsigned addr = (unsigned)((s.yoff + oh * g.Wo + ow) * 4);
    const unsigned vb = ok ? addr : SENT;
    const int cs = (int)g.syc;
    const int cb0 = co0 * cs * 4;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = ld1(s.rb, vb, cb0 + e * cs * 4);
  }
};

// The parity classes of a dgrad (stride^2 of them, fewer when H or W < stride).
inline int dgrad_classes(const Geom& g, DgradT* out) {
  int n = 0;
  for (int ca = 0; ca < std::min(g.stride, g.H); ++ca)
    for (int cb = 0; cb < std::min(g.stride, g.W); ++cb) {
      DgradT& c = out[n++];
      c.g = g;
      c.ca = ca;
      c.cb = cb;
      c.Hc = (g.H - ca + g.stride - 1) / g.stride;
      c.Wc = (g.W - cb + g.stride - 1) / g.stride;
      c.d_hcwc = conv::make_fastdiv((uint32_t)(c.Hc * c.Wc));
      c.d_wc = conv::make_fastdiv((uint32_t)c.Wc);
      c.ntc = 0;
      for (int t = 0; t < g.ntaps; ++t) {
        const int kh = g.tap_kh[t], kw = g.tap_kw[t];
        if (((ca + g.pad - kh) % g.stride + g.stride) % g.stride != 0) continue;
        if (((cb + g.pad - kw) % g.stride + g.stride) % g.stride != 0) continue;
        c.ckh[c.ntc] = (int8_t)kh;
        c.ckw[c.ntc] = (int8_t)kw;
        ++c.ntc;
      }
      c.crect = conv::make_rect(c.ckh, c.ckw, c.ntc, g.stride);
    }
  return n;
}
constexpr int MAX_CLASSES = 16;

// dW_t[tap][ci][co] = sum_q x(q; tap, ci) dy(q; co): M = ntaps*Cin (slot, ci),
// N = Cout, R = B*Ho*Wo.  A 64-row m-tile lies inside one tap (Cin % 64 == 0).
template <bool BVEC>
struct WgtT {
  static constexpr bool QUAD_A = false, QUAD_B = false;
  Geom g;
  const float* x;
  const float* dy;
  float* dw;
  // optional clip-norm partials (flr_conv2d_bwd_weight_t_sq): one fp64 sum of
  // squares per output tile (split-K 1) or per 256-value treduce block, at
  // sq[k * sq_ld + slot] — the optimizer's clip norm then never re-reads dw
  double* sq = nullptr;
  int sq_ld = 0;
  static constexpr int LA = RK_GATHER, LB = BVEC ? RK_VEC : RK_GATHER;
  __host__ __device__ __forceinline__ int M() const { return g.ntaps * g.Cin; }
  __host__ __device__ __forceinline__ int N() const { return g.Cout; }
  __host__ __device__ __forceinline__ int R() const { return g.B * g.Ho * g.Wo; }
  struct State {
    rsrc_t ra, rb;
    int kh, kw, aoff, boff;
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.ra = make_rsrc(x + k * g.sxk, g.xext);
    s.rb = make_rsrc(dy + k * g.syk, g.yext);
    const int slot = uni(m0 / g.Cin), ci0 = m0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    s.kh = uni(kh);
    s.kw = uni(kw);
    s.aoff = (int)((ci0 + tid / 32) * g.sxc);
    s.boff = (int)((BVEC ? (n0 + tid / 8) : (n0 + tid / 32)) * g.syc);
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const int tid = threadIdx.x;
    const int HoWo = g.Ho * g.Wo, R = this->R();
    {  // A: x gathered at q = r0 + tid % 32
      const int q = r0 + tid % 32;
      const uint32_t bb = udiv(q, g.d_howo), p = q - bb * HoWo;
      const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
      const int ih = (int)oh * g.stride - g.pad + s.kh, iw = (int)ow * g.stride - g.pad + s.kw;
      const bool ok = (q < R) & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
      const unsigned addr = (unsigned)(((int)(bb * g.sxb) + s.aoff + ih * g.W + iw) * 4);
      const unsigned va = ok ? addr : SENT;
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = ld1(s.ra, va, i * 8 * (int)g.sxc * 4);
    }
  }
  // B: dy[co][q] with q = b*Ho*Wo + p contiguous per channel ([K][C][B][Ho][Wo])
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const int tid = threadIdx.x, R = this->R();
    if constexpr (BVEC) {  // q = r0 + 4 (tid % 8) .. +3
      const int q = r0 + 4 * (tid % 8);
      const unsigned vb = q < R ? (unsigned)((s.boff + q) * 4) : SENT;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = ld4(s.rb, vb, i * 32 * (int)g.syc * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) b[4 * i + e] = v[e];
      }
    } else {  // q = r0 + tid % 32
      const int q = r0 + tid % 32;
      const unsigned vb = q < R ? (unsigned)((s.boff + q) * 4) : SENT;
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = ld1(s.rb, vb, i * 8 * (int)g.syc * 4);
    }
  }
  __device__ __forceinline__ void store(int k, int m, int n, float v) const {
    const int slot = (int)udiv(m, g.d_cin), ci = m - slot * g.Cin;
    dw[(((int64_t)k * g.KH * g.KW + tap_index(g, slot)) * g.Cin + ci) * g.Cout + n] = v;
  }
  __device__ __forceinline__ bool linear() const { return true; }
  __device__ __forceinline__ float* out() const { return dw; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const {
    const int slot = m0 / g.Cin, ci0 = m0 - slot * g.Cin;
    return (((int64_t)k * g.KH * g.KW + tap_index(g, slot)) * g.Cin + ci0) * g.Cout + n0;
  }
  __device__ __forceinline__ int64_t ldm() const { return g.Cout; }
  struct State8 {
    rsrc_t ra, rb;
    int kh, kw, k0;
    unsigned aoff, boff;
  };
  __device__ __forceinline__ State8 init8(int k, int m0, int n0, int tid) const {
    State8 s;
    s.ra = make_rsrc(x + k * g.sxk, g.xext);
    s.rb = make_rsrc(dy + k * g.syk, g.yext);
    const int slot = uni(m0 / g.Cin), ci0 = m0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    s.kh = uni(kh);
    s.kw = uni(kw);
    const int row = tid & 63;
    s.k0 = uni(8 * (tid >> 6));  // the wave's k-group: its 8 pixels are wave-uniform
    s.aoff = (unsigned)((ci0 + row) * g.sxc * 4);
    s.boff = (unsigned)((n0 + row) * g.syc * 4);
    return s;
  }
  // A(ci, pixel q): the 8 pixels of the wave's k-group are wave-uniform, so their
  // decomposition and padding test run on the scalar unit (soffset per pixel)
  __device__ __forceinline__ void load_a8(const State8& s, int r0, float (&a)[8]) const {
    const int R = this->R(), HoWo = g.Ho * g.Wo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = uni(r0 + s.k0 + e);
      const int bb = uni((int)udiv((uint32_t)q, g.d_howo)), p = q - bb * HoWo;
      const int oh = uni((int)udiv((uint32_t)p, g.d_wo)), ow = p - oh * g.Wo;
      const int ih = oh * g.stride - g.pad + s.kh, iw = ow * g.stride - g.pad + s.kw;
      const bool ok = (q < R) & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
      const int soff = uni(ok ? (bb * (int)g.sxb + ih * g.W + iw) * 4 : 0);
      a[e] = ld1(s.ra, ok ? s.aoff : SENT, soff);
    }
  }
  // B(co, q): dy[co][q], q contiguous per channel
  __device__ __forceinline__ void load_b8(const State8& s, int r0, float (&b)[8]) const {
    const int R = this->R();
    const int q0 = r0 + s.k0;
    if constexpr (BVEC) {  // syc % 4 == 0, R % 4 == 0
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = q0 + 4 * i < R;
        const f32x4 v = ld4(s.rb, ok ? s.boff + (unsigned)((q0 + 4 * i) * 4) : SENT, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) b[4 * i + e] = v[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = ld1(s.rb, (q0 + e < R) ? s.boff + (unsigned)((q0 + e) * 4) : SENT, 0);
    }
  }
  // ---- transposed-image loads (wsgemm_kernel): thread t holds rows 8 (t >> 5) .. +7 of
  // the 64-row sub-tile at reduction index k = t & 31 — the 32 lanes of a half-wave
  // read 32 consecutive pixels of one row (128 B), and the thread's 8 values are
  // the 8 consecutive rows of one k, one 16-B chunk of a [k][row] LDS image
  struct StateT {
    rsrc_t ra, rb;
    int kh, kw;
    unsigned arow, brow;
  };
  __device__ __forceinline__ StateT initT(int k, int m0, int n0, int tid) const {
    StateT s;
    s.ra = make_rsrc(x + k * g.sxk, g.xext);
    s.rb = make_rsrc(dy + k * g.syk, g.yext);
    const int slot = uni(m0 / g.Cin), ci0 = m0 - slot * g.Cin;
    int kh, kw;
    slot_tap(g, slot, kh, kw);
    s.kh = uni(kh);
    s.kw = uni(kw);
    const int rg = tid >> 5;
    s.arow = (unsigned)((ci0 + 8 * rg) * g.sxc * 4);
    s.brow = (unsigned)((n0 + 8 * rg) * g.syc * 4);
    return s;
  }
  __device__ __forceinline__ void load_at8(const StateT& s, int r0, float (&a)[8]) const {  // x(ci, pixel q of tap (kh, kw))
    const int q = r0 + (int)(threadIdx.x & 31), HoWo = g.Ho * g.Wo;
    const uint32_t bb = udiv(q, g.d_howo), p = q - bb * HoWo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    const int ih = (int)oh * g.stride - g.pad + s.kh, iw = (int)ow * g.stride - g.pad + s.kw;
    const bool ok = (q < R()) & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
    const unsigned va = ok ? s.arow + (unsigned)(((int)(bb * g.sxb) + ih * g.W + iw) * 4) : SENT;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = ld1(s.ra, va, i * (int)g.sxc * 4);
  }
  __device__ __forceinline__ void load_bt8(const StateT& s, int r0, float (&b)[8]) const {  // dy(co, q), q contiguous
    const int q = r0 + (int)(threadIdx.x & 31);
    const unsigned vb = q < R() ? s.brow + (unsigned)(q * 4) : SENT;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = ld1(s.rb, vb, i * (int)g.syc * 4);
  }
};

// ---- explicit im2col (short reductions: the stem) -----------------------------
// col[k][pix][RP], pix = b*Ho*Wo + oh*Wo + ow, r = (ci*KH + kh)*KW + kw (torch
// weight order), zero for padding taps and for r >= R (RP = R rounded up to 4).
// The weights are used as wp[k][co][RP] (a zero-padded copy), so both GEMM
// operands are k-contiguous rows and load as 16-B vectors.
struct DenseFwd {  // y[co][pix] = sum_r wp[co][r] col[pix][r]: M = Cout, N = B*Ho*Wo, R = RP
  Geom g;
  int RP;
  const float* col;
  const float* wp;
  float* y;
  static constexpr int LA = RK_VEC, LB = RK_VEC;
  __host__ __device__ __forceinline__ int M() const { return g.Cout; }
  __host__ __device__ __forceinline__ int N() const { return g.B * g.Ho * g.Wo; }
  __host__ __device__ __forceinline__ int R() const { return RP; }
  struct State {
    rsrc_t ra, rb;
    unsigned a0, b0;
    bool aok[2], bok[2];
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.ra = make_rsrc(wp + (int64_t)k * g.Cout * RP, (int64_t)g.Cout * RP);
    s.rb = make_rsrc(col + (int64_t)k * N() * RP, (int64_t)N() * RP);
    s.a0 = (unsigned)(((m0 + tid / 8) * RP + 4 * (tid % 8)) * 4);
    s.b0 = (unsigned)(((n0 + tid / 8) * RP + 4 * (tid % 8)) * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      s.aok[i] = m0 + tid / 8 + 32 * i < M();
      s.bok[i] = n0 + tid / 8 + 32 * i < N();
    }
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const bool kok = r0 + 4 * (int)(threadIdx.x % 8) < RP;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 qa = ld4(s.ra, (kok && s.aok[i]) ? s.a0 + (unsigned)((r0 + 32 * i * RP) * 4) : SENT, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[4 * i + e] = qa[e];
    }
  }
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const bool kok = r0 + 4 * (int)(threadIdx.x % 8) < RP;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 qb = ld4(s.rb, (kok && s.bok[i]) ? s.b0 + (unsigned)((r0 + 32 * i * RP) * 4) : SENT, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) b[4 * i + e] = qb[e];
    }
  }
  // y[k][m][n]: n = b*Ho*Wo + p is linear in the [K][C][B][Ho][Wo] layout
  __device__ __forceinline__ void store(int k, int m, int n, float v) const { y[k * g.syk + m * g.syc + n] = v; }
  __device__ __forceinline__ bool linear() const { return true; }
  __device__ __forceinline__ float* out() const { return y; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return k * g.syk + m0 * g.syc + n0; }
  __device__ __forceinline__ int64_t ldm() const { return g.syc; }
};

struct DenseWgt {  // dwp[co][r] = sum_pix dy[co][pix] col[pix][r]: M = Cout, N = RP, R = B*Ho*Wo (HoWo % 4 == 0)
  Geom g;
  int RP;
  const float* col;
  const float* dy;
  float* dwp;
  static constexpr int LA = RK_VEC, LB = KR_VEC;
  __host__ __device__ __forceinline__ int M() const { return g.Cout; }
  __host__ __device__ __forceinline__ int N() const { return RP; }
  __host__ __device__ __forceinline__ int R() const { return g.B * g.Ho * g.Wo; }
  struct State {
    rsrc_t ra, rb;
    int arow;
    bool aok[2], nok;
    unsigned b0;
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.ra = make_rsrc(dy + k * g.syk, g.yext);
    s.rb = make_rsrc(col + (int64_t)k * R() * RP, (int64_t)R() * RP);
    s.arow = (int)((m0 + tid / 8) * g.syc);
#pragma unroll
    for (int i = 0; i < 2; ++i) s.aok[i] = m0 + tid / 8 + 32 * i < M();
    const int n = n0 + 4 * (tid % 16);
    s.nok = n < RP;
    s.b0 = (unsigned)(((tid / 16) * RP + n) * 4);
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const int tid = threadIdx.x, R = this->R();
    const int q = r0 + 4 * (tid % 8);  // dy[co][q]: q = b*Ho*Wo + p contiguous per channel
    const unsigned va = (unsigned)((s.arow + q) * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 qa = ld4(s.ra, (q < R && s.aok[i]) ? va + (unsigned)(i * 32 * (int)g.syc * 4) : SENT, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[4 * i + e] = qa[e];
    }
  }
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const int tid = threadIdx.x, R = this->R();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pix = r0 + tid / 16 + 16 * i;
      const f32x4 qb = ld4(s.rb, (pix < R && s.nok) ? s.b0 + (unsigned)((r0 + 16 * i) * RP * 4) : SENT, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) b[4 * i + e] = qb[e];
    }
  }
  __device__ __forceinline__ void store(int k, int m, int n, float v) const { dwp[((int64_t)k * g.Cout + m) * RP + n] = v; }
  __device__ __forceinline__ bool linear() const { return true; }
  __device__ __forceinline__ float* out() const { return dwp; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return ((int64_t)k * g.Cout + m0) * RP + n0; }
  __device__ __forceinline__ int64_t ldm() const { return RP; }
};

// The same two GEMMs with the im2col operand gathered on the fly from x
// ([K][C][B][H][W]; one client's image batch, 393 KB at the C3 stem, stays in
// L2 across its 49 taps): no column matrix is written or read.  Reduction
// index r = (ci*KH + kh)*KW + kw (torch weight order), zero past R = Cin*KH*KW.
struct StemFwd {  // y[co][pix] = sum_r wp[co][r] x(pix; r): M = Cout, N = B*Ho*Wo, R = RP
  Geom g;
  int RP, RR;  // RR = Cin*KH*KW
  conv::FastDiv d_kk, d_kw;
  const float* x;
  const float* wp;
  float* y;
  static constexpr int LA = RK_VEC, LB = KR_GATHER;
  __host__ __device__ __forceinline__ int M() const { return g.Cout; }
  __host__ __device__ __forceinline__ int N() const { return g.B * g.Ho * g.Wo; }
  __host__ __device__ __forceinline__ int R() const { return RP; }
  struct State {
    rsrc_t ra, rb;
    unsigned a0;
    bool aok[2], nok;
    int ih0, iw0, xoff;
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.ra = make_rsrc(wp + (int64_t)k * g.Cout * RP, (int64_t)g.Cout * RP);
    s.a0 = (unsigned)(((m0 + tid / 8) * RP + 4 * (tid % 8)) * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) s.aok[i] = m0 + tid / 8 + 32 * i < M();
    s.rb = make_rsrc(x + k * g.sxk, g.xext);
    const int n = n0 + tid % 64;
    s.nok = n < N();
    const uint32_t bb = udiv(n, g.d_howo), p = n - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    s.ih0 = (int)oh * g.stride - g.pad;
    s.iw0 = (int)ow * g.stride - g.pad;
    s.xoff = (int)(bb * g.sxb);
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const bool kok = r0 + 4 * (int)(threadIdx.x % 8) < RP;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 qa = ld4(s.ra, (kok && s.aok[i]) ? s.a0 + (unsigned)((r0 + 32 * i * RP) * 4) : SENT, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[4 * i + e] = qa[e];
    }
  }
  // k-row tid/64 + 4i is the wave's: (ci, kh, kw) are wave-uniform (SGPRs)
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const int KK = g.KH * g.KW;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = uni(r0 + (int)(threadIdx.x / 64) + 4 * i);
      const int ci = uni((int)udiv((uint32_t)r, d_kk)), rem = r - ci * KK;
      const int kh = uni((int)udiv((uint32_t)rem, d_kw)), kw = rem - kh * g.KW;
      const int ih = s.ih0 + kh, iw = s.iw0 + kw;
      const bool ok = s.nok & (r < RR) & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
      const unsigned addr = (unsigned)((s.xoff + ih * g.W + iw) * 4);
      const unsigned vb = ok ? addr : SENT;
      b[i] = ld1(s.rb, vb, uni(ci * (int)g.sxc * 4));
    }
  }
  __device__ __forceinline__ void store(int k, int m, int n, float v) const { y[k * g.syk + m * g.syc + n] = v; }
  __device__ __forceinline__ bool linear() const { return true; }
  __device__ __forceinline__ float* out() const { return y; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return k * g.syk + m0 * g.syc + n0; }
  __device__ __forceinline__ int64_t ldm() const { return g.syc; }
};

struct StemWgt {  // dwp[co][r] = sum_pix dy[co][pix] x(pix; r): M = Cout, N = RP, R = B*Ho*Wo (HoWo % 4 == 0)
  Geom g;
  int RP, RR;
  conv::FastDiv d_kk, d_kw;
  const float* x;
  const float* dy;
  float* dwp;
  static constexpr int LA = RK_VEC, LB = KR_VEC;
  __host__ __device__ __forceinline__ int M() const { return g.Cout; }
  __host__ __device__ __forceinline__ int N() const { return RP; }
  __host__ __device__ __forceinline__ int R() const { return g.B * g.Ho * g.Wo; }
  struct State {
    rsrc_t ra, rb;
    int arow;
    bool aok[2];
    int roff[4];          // this thread's 4 reduction columns r: ci*sxc + kh*W + kw
    int8_t kh[4], kw[4];  // (kh = -128: r past R)
  };
  __device__ __forceinline__ State init(int k, int m0, int n0, int tid) const {
    State s;
    s.ra = make_rsrc(dy + k * g.syk, g.yext);
    s.arow = (int)((m0 + tid / 8) * g.syc);
#pragma unroll
    for (int i = 0; i < 2; ++i) s.aok[i] = m0 + tid / 8 + 32 * i < M();
    s.rb = make_rsrc(x + k * g.sxk, g.xext);
    const int KK = g.KH * g.KW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = n0 + 4 * (tid % 16) + e;
      const int ci = (int)udiv((uint32_t)r, d_kk), rem = r - ci * KK;
      const int kh = (int)udiv((uint32_t)rem, d_kw), kw = rem - kh * g.KW;
      const bool ok = r < RR;
      s.kh[e] = ok ? (int8_t)kh : (int8_t)-128;
      s.kw[e] = (int8_t)kw;
      s.roff[e] = ok ? ci * (int)g.sxc + kh * g.W + kw : 0;
    }
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&a)[8]) const {
    const int tid = threadIdx.x, R = this->R();
    const int q = r0 + 4 * (tid % 8);  // dy[co][q]: q = b*Ho*Wo + p contiguous per channel
    const unsigned va = (unsigned)((s.arow + q) * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 qa = ld4(s.ra, (q < R && s.aok[i]) ? va + (unsigned)(i * 32 * (int)g.syc * 4) : SENT, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[4 * i + e] = qa[e];
    }
  }
  // KR_VEC image: pixel k-rows tid/16 + 16i, columns r = n0 + 4 (tid % 16) + e
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&b)[8]) const {
    const int tid = threadIdx.x, R = this->R(), HoWo = g.Ho * g.Wo;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = r0 + tid / 16 + 16 * i;
      const uint32_t bb = udiv((uint32_t)q, g.d_howo), p = (uint32_t)q - bb * HoWo;
      const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
      const int ih0 = (int)oh * g.stride - g.pad, iw0 = (int)ow * g.stride - g.pad;
      const int base = (int)(bb * g.sxb) + ih0 * g.W + iw0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ih = ih0 + s.kh[e], iw = iw0 + s.kw[e];
        const bool ok = (q < R) & (s.kh[e] >= 0) & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
        const unsigned addr = (unsigned)((base + s.roff[e]) * 4);
        b[4 * i + e] = ld1(s.rb, ok ? addr : SENT, 0);
      }
    }
  }
  __device__ __forceinline__ void store(int k, int m, int n, float v) const { dwp[((int64_t)k * g.Cout + m) * RP + n] = v; }
  __device__ __forceinline__ bool linear() const { return true; }
  __device__ __forceinline__ float* out() const { return dwp; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return ((int64_t)k * g.Cout + m0) * RP + n0; }
  __device__ __forceinline__ int64_t ldm() const { return RP; }
};

// col[k][pix][RP] (grid: pixel blocks x K).  A workgroup builds IM_PB whole
// rows in LDS — one thread per (pix, ci, kh) fills the KW-long run
// r = (ci*KH + kh)*KW + 0..KW-1 — then streams the IM_PB*RP contiguous floats
// out as 16-B stores (RP % 4 == 0).
// ---- batched dense GEMM (the text branch and the late-fusion MLP) -------------
// C_k[m][n] = (bias_k[n] | add_k[m][n]) + sum_r A_k(m, r) B_k(n, r) for every
// client k, with arbitrary strides: A(m, r) at a + k a_k + m a_m + r a_r, etc.
// Operand modes: RK (r contiguous: 16-B loads along r), KR (m / n contiguous:
// 16-B loads along the row index), G (anything else: scalar gathers).  Same
// tiled exact-fp32 MFMA kernel and split-K rule as the convolutions, so a
// client's result never depends on how many clients share the launch.
struct BatchDim {
  int Kc;
};
enum BMode { BM_RK = 0, BM_KR = 1, BM_G = 2 };

struct BGemmArgs {
  BatchDim g;
  int m, n, r;
  const float* a;
  int64_t a_k, a_m, a_r, a_ext;
  const float* b;
  int64_t b_k, b_n, b_r, b_ext;
  float* c;
  int64_t c_k, c_m, c_n;
  const float* bias;  // bias[k * bias_k + n]
  int64_t bias_k;
  const float* add;   // add[k*c_k + m*c_m + n*c_n] (may alias c)
  // epilogue (flr_bgemm_ex): pre <- v; v <- act(v [, aux]); v <- v * mul
  int act;            // FLR_ACT_*
  const float* mul;   // indexed like c (may be NULL)
  const float* aux;   // indexed like c: the saved activation input/output of the D* modes
  float* pre;         // indexed like c: the pre-activation value (may be NULL)
};

// exact-erf GELU as torch's CPU kernel: x * 0.5 * (1 + erf(x * M_SQRT1_2))
__device__ __forceinline__ float gelu_erf(float x) {
  return __fmul_rn(__fmul_rn(x, 0.5f), __fadd_rn(1.f, erff(__fmul_rn(x, 0.70710678118654752440f))));
}
// d/dx GELU: 0.5 (1 + erf(x / sqrt 2)) + x exp(-x^2 / 2) / sqrt(2 pi)
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752440f));
  const float pdf = expf(-0.5f * x * x) * 0.39894228040143267794f;
  return cdf + x * pdf;
}

// the activation given the aux value (the D* modes' saved input / output)
__device__ __forceinline__ float apply_act_v(int act, float v, float ax) {
  switch (act) {
    case FLR_ACT_RELU: return v > 0.f ? v : 0.f;
    case FLR_ACT_GELU: return gelu_erf(v);
    case FLR_ACT_TANH: return tanhf(v);
    case FLR_ACT_DRELU: return ax > 0.f ? v : 0.f;
    case FLR_ACT_DGELU: return v * gelu_erf_grad(ax);
    case FLR_ACT_DTANH: return v * (1.f - ax * ax);
    default: return v;
  }
}

__device__ __forceinline__ float apply_act(int act, float v, const float* aux, int64_t i) {
  switch (act) {
    case FLR_ACT_RELU: return v > 0.f ? v : 0.f;
    case FLR_ACT_GELU: return gelu_erf(v);
    case FLR_ACT_TANH: return tanhf(v);
    case FLR_ACT_DRELU: return aux[i] > 0.f ? v : 0.f;
    case FLR_ACT_DGELU: return v * gelu_erf_grad(aux[i]);
    case FLR_ACT_DTANH: { const float y = aux[i]; return v * (1.f - y * y); }
    default: return v;
  }
}

template <int AM, int BMD>
struct BGemm : BGemmArgs {
  static constexpr int AMODE = AM, BMODE = BMD;
  static constexpr bool QUAD_A = FLR_QUAD != 0 && AM == BM_RK, QUAD_B = FLR_QUAD != 0 && BMD == BM_RK;
  static constexpr int LA = AM == BM_RK ? RK_VEC : (AM == BM_KR ? KR_VEC : RK_GATHER);
  static constexpr int LB = BMD == BM_RK ? RK_VEC : (BMD == BM_KR ? KR_VEC : RK_GATHER);
  __host__ __device__ __forceinline__ int M() const { return m; }
  __host__ __device__ __forceinline__ int N() const { return n; }
  __host__ __device__ __forceinline__ int R() const { return r; }
  struct State {
    rsrc_t ra, rb;
    int arow, brow;
  };
  // one operand (rows = m or n) of a 64 x 32 tile, in the layout its mode stashes
  template <int MODE>
  __device__ __forceinline__ static void load_op(rsrc_t rs, int base_row, int rows, int r0, int R, int64_t s_row, int64_t s_r,
                                 float (&v)[8]) {
    const int tid = threadIdx.x;
    if constexpr (MODE == BM_RK) {  // rows tid/8 + 32 i, k = r0 + 4 (tid % 8) .. +3
      const int kk = r0 + 4 * (tid % 8);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = base_row + tid / 8 + 32 * i;
        const bool ok = (row < rows) & (kk < R);
        const unsigned addr = (unsigned)((row * s_row + kk) * 4);
        const f32x4 q = ld4(rs, ok ? addr : SENT, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * i + e] = q[e];
      }
    } else if constexpr (MODE == BM_KR) {  // rows 4 (tid % 16) .. +3, k = r0 + tid/16 + 16 i
      const int row = base_row + 4 * (tid % 16);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kk = r0 + tid / 16 + 16 * i;
        const bool ok = (row < rows) & (kk < R);
        const unsigned addr = (unsigned)((kk * s_r + row) * 4);
        const f32x4 q = ld4(rs, ok ? addr : SENT, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * i + e] = q[e];
      }
    } else {  // rows tid/32 + 8 i, k = r0 + tid % 32
      const int kk = r0 + tid % 32;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = base_row + tid / 32 + 8 * i;
        const bool ok = (row < rows) & (kk < R);
        const unsigned addr = (unsigned)((row * s_row + kk * s_r) * 4);
        v[i] = ld1(rs, ok ? addr : SENT, 0);
      }
    }
  }
  __device__ __forceinline__ State init(int k, int m0, int n0, int) const {
    State s;
    s.ra = make_rsrc(a + k * a_k, a_ext);
    s.rb = make_rsrc(b + k * b_k, b_ext);
    s.arow = m0;
    s.brow = n0;
    return s;
  }
  __device__ __forceinline__ void load_a(const State& s, int r0, float (&v)[8]) const {
    load_op<AM>(s.ra, s.arow, m, r0, r, a_m, a_r, v);
  }
  __device__ __forceinline__ void load_b(const State& s, int r0, float (&v)[8]) const {
    load_op<BMD>(s.rb, s.brow, n, r0, r, b_n, b_r, v);
  }
  __device__ __forceinline__ void store(int k, int mm, int nn, float v) const {
    const int64_t i = k * c_k + mm * c_m + nn * c_n;
    if (bias) v = bias[k * bias_k + nn] + v;
    if (add) v = add[i] + v;
    if (pre) pre[i] = v;
    if (act) v = apply_act(act, v, aux, i);
    if (mul) v = v * mul[i];
    c[i] = v;
  }
  // The S == 1 epilogue of one 32 x 32 accumulator tile (lane column n, rows
  // m[e]): every epilogue operand of the lane's 16 values is loaded before the
  // first store.  Per value, store()'s load -> store chain serialised on memory
  // latency (the stores may alias the operands): the bias epilogue cost 141 us
  // of 252 on the GRU input projection.  Same operations in the same order.
  __device__ __forceinline__ void store_tile(int k, int tm0, int tn0, int ml0, int nl, const f32x16& acc, int M,
                                             int N) const {
    // the plain epilogue's addressing: one uniform tile base, per value the
    // offset ml c_m + nl c_n (ml = ml0 + r, r = (e & 3) + 8 (e >> 2)), bounds as
    // predicates (no early exit)
    const int64_t tb = k * c_k + (int64_t)tm0 * c_m + (int64_t)tn0 * c_n;
    const bool nok = tn0 + nl < N;
    const float bv = (bias && nok) ? bias[k * bias_k + tn0 + nl] : 0.f;
    const bool use_aux = act >= FLR_ACT_DRELU && aux;
    float av[16], xv[16], mv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ml = ml0 + (e & 3) + 8 * (e >> 2);
      const bool ok = nok && tm0 + ml < M;
      const int64_t o = tb + ml * c_m + nl * c_n;
      av[e] = (add && ok) ? add[o] : 0.f;
      xv[e] = (use_aux && ok) ? aux[o] : 0.f;
      mv[e] = (mul && ok) ? mul[o] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ml = ml0 + (e & 3) + 8 * (e >> 2);
      if (nok && tm0 + ml < M) {
        const int64_t o = tb + ml * c_m + nl * c_n;
        float v = acc[e];
        if (bias) v = bv + v;
        if (add) v = av[e] + v;
        if (pre) pre[o] = v;
        if (act) v = apply_act_v(act, v, xv[e]);
        if (mul) v = v * mv[e];
        c[o] = v;
      }
    }
  }
  // the plain epilogue (row-major output, at most a bias: added there as bias + v)
  __device__ __forceinline__ bool linear() const { return c_n == 1 && !add && !act && !mul && !pre; }
  __device__ __forceinline__ float* out() const { return c; }
  __device__ __forceinline__ int64_t tile_base(int k, int m0, int n0) const { return k * c_k + m0 * c_m + n0; }
  __device__ __forceinline__ int64_t ldm() const { return c_m; }
  using State8 = State;
  template <int MODE>
  __device__ __forceinline__ static void load_op8(rsrc_t rs, int base_row, int rows, int r0, int R, int64_t s_row, int64_t s_r,
                                  float (&v)[8]) {
    const int tid = threadIdx.x;
    constexpr bool Q = FLR_QUAD != 0 && MODE == BM_RK;
    const int row = base_row + stash_row<Q>(tid), kk0 = r0 + stash_k<Q>(tid);
    const bool rok = row < rows;
    if constexpr (MODE == BM_RK) {  // r contiguous, R % 4 == 0
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = rok & (kk0 + 4 * i < R);
        const unsigned addr = (unsigned)((row * s_row + kk0 + 4 * i) * 4);
        const f32x4 q = ld4(rs, ok ? addr : SENT, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * i + e] = q[e];
      }
    } else {  // KR (rows contiguous: lanes coalesce) and G
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = rok & (kk0 + e < R);
        const unsigned addr = (unsigned)((row * s_row + (kk0 + e) * s_r) * 4);
        v[e] = ld1(rs, ok ? addr : SENT, 0);
      }
    }
  }
  __device__ __forceinline__ State8 init8(int k, int m0, int n0, int tid) const { return init(k, m0, n0, tid); }
  __device__ __forceinline__ void load_a8(const State8& s, int r0, float (&v)[8]) const {
    load_op8<AM>(s.ra, s.arow, m, r0, r, a_m, a_r, v);
  }
  __device__ __forceinline__ void load_b8(const State8& s, int r0, float (&v)[8]) const {
    load_op8<BMD>(s.rb, s.brow, n, r0, r, b_n, b_r, v);
  }
  // transposed-image loads of a k-contiguous (RK) operand (wsgemm_kernel): thread t
  // reads k = r0 + (t & 31) of rows 8 (t >> 5) .. +7 — a half-wave covers 128 B of a row
  using StateT = State;
  __device__ __forceinline__ StateT initT(int k, int m0, int n0, int tid) const { return init(k, m0, n0, tid); }
  __device__ __forceinline__ static void load_opT(rsrc_t rs, int base_row, int rows, int r0, int R, int64_t s_row, float (&v)[8]) {
    const int kk = r0 + (int)(threadIdx.x & 31);
    const int row0 = base_row + 8 * (int)(threadIdx.x >> 5);
    const unsigned base = (unsigned)((row0 * s_row + kk) * 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool ok = (row0 + i < rows) & (kk < R);
      v[i] = ld1(rs, ok ? base + (unsigned)(i * s_row * 4) : SENT, 0);
    }
  }
  __device__ __forceinline__ void load_at8(const StateT& s, int r0, float (&v)[8]) const {
    load_opT(s.ra, s.arow, m, r0, r, a_m, v);
  }
  __device__ __forceinline__ void load_bt8(const StateT& s, int r0, float (&v)[8]) const {
    load_opT(s.rb, s.brow, n, r0, r, b_n, v);
  }
  // LDS-DMA fill of one 128-row x 32-k operand image (dsgemm_kernel): 16 pieces of
  // 1 KB, one buffer_load_dwordx4 ... lds each, pieces 4 wave .. 4 wave + 3 issued by
  // this wave.  The destination is lane-linear, so the images' swizzles are applied
  // to the SOURCE address (lane -> the logical chunk its physical slot holds):
  //   RK [128 rows][32 k]: physical 16-B chunk of (row, q) = q ^ ((row >> 1) & 7)
  //      (a ds_read_b128 group of 16 rows hits 16 distinct bank groups);
  //   KR [32 k][128 rows]: physical 4-row chunk of (k, c) = c ^ (8 ((k >> 3) & 1))
  //      (the two half-waves' ds_read_b32, k and k + 8, on disjoint bank halves).
  // Out-of-range rows / reductions read 0 (raw buffer bounds), as the register loads.
  template <int MODE>
  __device__ __forceinline__ static void dma_op(rsrc_t rs, float* img, int base_row, int rows, int r0, int R, int64_t s_row,
                                int64_t s_r, int wave, int lane) {
    static_assert(MODE == BM_RK || MODE == BM_KR, "LDS-DMA images hold RK or KR operands");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = 4 * wave + i;  // wave-uniform: the LDS base goes to M0
      unsigned voff;
      if constexpr (MODE == BM_RK) {  // 8 rows x 128 B per piece
        const int rl = 8 * piece + (lane >> 3);
        const int q = (lane & 7) ^ ((rl >> 1) & 7);
        const int row = base_row + rl, kk = r0 + 4 * q;
        voff = ((row < rows) & (kk < R)) ? (unsigned)((row * s_row + kk) * 4) : SENT;
      } else {  // 2 k-rows x 512 B per piece
        const int kl = 2 * piece + (lane >> 5);
        const int q = (lane & 31) ^ (((kl >> 3) & 1) << 3);
        const int row = base_row + 4 * q, kk = r0 + kl;
        voff = ((row < rows) & (kk < R)) ? (unsigned)((kk * s_r + row) * 4) : SENT;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + piece * 256), 16,
                                               voff, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void dma_a(const State& s, float* img, int r0, int wave, int lane) const {
    dma_op<AM>(s.ra, img, s.arow, m, r0, r, a_m, a_r, wave, lane);
  }
  __device__ __forceinline__ void dma_b(const State& s, float* img, int r0, int wave, int lane) const {
    dma_op<BMD>(s.rb, img, s.brow, n, r0, r, b_n, b_r, wave, lane);
  }
};

#if FLR_CT_P4
// out[k][n] = sum_m X[k][m][n] (bias gradients of the batched GEMMs).  Eight
// interleaved accumulators (rows m = 8i + j go to accumulator j), combined in a
// fixed tree: deterministic, and eight independent load/add chains per lane
// instead of one M-long dependent chain.
__global__ void sum_rows_kernel(const float* __restrict__ x, int64_t x_k, int64_t x_m, int M, int N,
                                float* __restrict__ out, int64_t out_k) {
  const int k = blockIdx.y;
  const int nn = blockIdx.x * blockDim.x + threadIdx.x;
  if (nn >= N) return;
  const float* p = x + k * x_k + nn;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int mm = 0;
  for (; mm + 8 <= M; mm += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += p[(int64_t)(mm + j) * x_m];
  }
  for (int j = 0; mm < M; ++mm, ++j) a[j] += p[(int64_t)mm * x_m];
  out[k * out_k + nn] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}
#endif

[[maybe_unused]] constexpr int IM_PB = 32, IM_MAXRP = 512;
#if FLR_CT_P0
__global__ __launch_bounds__(THREADS) void im2col_kernel(const Geom g, const float* __restrict__ x, int RP,
                                                         float* __restrict__ col) {
  extern __shared__ __attribute__((aligned(16))) float rows[];  // [IM_PB][RP]
  const int k = blockIdx.y;
  const int N = g.B * g.Ho * g.Wo, CK = g.Cin * g.KH, R = CK * g.KW;
  const int pix0 = blockIdx.x * IM_PB;
  const int np = min(IM_PB, N - pix0);
  const float* xk = x + k * g.sxk;
  for (int e = threadIdx.x; e < np * CK; e += THREADS) {
    const int pl = e / CK, j = e - pl * CK;
    const int ci = j / g.KH, kh = j - ci * g.KH;
    const int pix = pix0 + pl;
    const uint32_t bb = udiv(pix, g.d_howo), p = pix - bb * g.Ho * g.Wo;
    const uint32_t oh = udiv(p, g.d_wo), ow = p - oh * g.Wo;
    const int ih = (int)oh * g.stride - g.pad + kh, iw0 = (int)ow * g.stride - g.pad;
    const bool hok = ih >= 0 && ih < g.H;
    const float* src = xk + bb * g.sxb + ci * g.sxc + (int64_t)ih * g.W;
    float* dst = rows + pl * RP + j * g.KW;
    for (int kw = 0; kw < g.KW; ++kw) {
      const int iw = iw0 + kw;
      dst[kw] = (hok && iw >= 0 && iw < g.W) ? src[iw] : 0.f;
    }
  }
  for (int e = threadIdx.x; e < np * (RP - R); e += THREADS) rows[(e / (RP - R)) * RP + R + e % (RP - R)] = 0.f;
  __syncthreads();
  f32x4* out = reinterpret_cast<f32x4*>(col + ((int64_t)k * N + pix0) * RP);
  const f32x4* in = reinterpret_cast<const f32x4*>(rows);
  for (int e = threadIdx.x; e < np * RP / 4; e += THREADS) out[e] = in[e];
}
#endif

#if FLR_CT_P0
// dst[k][co][RP] <- src[k][co][R] (zero pad) or the reverse (unpad) (grid: chunks x K)
__global__ __launch_bounds__(THREADS) void repad_kernel(const float* __restrict__ src, int sld, float* __restrict__ dst,
                                                        int dld, int rows, int R) {
  const int k = blockIdx.y;
  const int64_t total = (int64_t)rows * dld;
  for (int64_t e = (int64_t)blockIdx.x * THREADS + threadIdx.x; e < total; e += (int64_t)gridDim.x * THREADS) {
    const int row = (int)(e / dld), r = (int)(e - (int64_t)row * dld);
    dst[(int64_t)k * total + e] = r < R ? src[((int64_t)k * rows + row) * sld + r] : 0.f;
  }
}
#endif

// ---- the kernel ---------------------------------------------------------------
// Workgroup tile (64*MS) x (64*NS): MS A sub-tiles and NS B sub-tiles of 64
// rows each are staged per K-tile; wave (wm, wn) owns rows 32 wm .. +31 and
// columns 32 wn .. +31 of every (i, j) sub-tile pair, so a fragment read from
// LDS feeds NS (A) or MS (B) MFMAs and the MS*NS accumulator chains are
// independent.  MS or NS = 2 halves the loads, LDS traffic and barriers per
// MFMA of the 64 x 64 tile.
// XCD-aware tile order.  The hardware deals workgroups round-robin over the 8
// XCDs (linear id i -> XCD i % 8), each with its own 4 MB L2.  The remap gives
// XCD x one contiguous range of logical tiles (bijective for any grid size), so
// the tiles of one client — which re-read the same activations once per kernel
// tap and the same weight slabs once per pixel tile — run on one XCD and share
// its L2 instead of streaming every client through all eight.
__device__ __forceinline__ void xcd_tile(int& bx, int& by, int& bz) {
  const int gx = (int)gridDim.x, gy = (int)gridDim.y;
  const int n = gx * gy * (int)gridDim.z;
  const int lid = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
  const int xcd = lid & 7, slot = lid >> 3;
  const int q = n >> 3, r = n & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  bx = t % gx;
  by = (t / gx) % gy;
  bz = t / (gx * gy);
}

template <class P> struct has_sq : std::false_type {};
template <bool V> struct has_sq<WgtT<V>> : std::true_type {};

// Sum over the workgroup in a fixed order (fp64): each thread's own value, a
// butterfly over the wave, the waves in index order; the result is thread 0's.
// Every thread of the workgroup must call it (one barrier).
__device__ __forceinline__ double block_sumsq(double s, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;
}

// the epilogue's optional addend (DgradT: the other gradient path of a residual
// block, summed where autograd would add the two paths)
template <class P> __device__ inline const float* plan_add(const P&) { return nullptr; }
__device__ inline const float* plan_add(const DgradT& p) { return p.add; }
template <class Plan, int MS, int NS, int X6>
__global__ __launch_bounds__(THREADS, 2) void tgemm_kernel(const Plan pl, int S, float* __restrict__ part, int remap,
                                                           int prio) {
  __shared__ __attribute__((aligned(16))) float As[2][MS][TILE];
  __shared__ __attribute__((aligned(16))) float Bs[2][NS][TILE];
  int bx = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
  if (remap & 1) xcd_tile(bx, by, bz);
  const int k = bz / S, split = bz % S;
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const int ktiles = cdiv(R, BK);
  const int rbeg = (int)((int64_t)ktiles * split / S) * BK;
  const int rend = std::min(R, (int)((int64_t)ktiles * (split + 1) / S) * BK);
  const int m0 = by * BM * MS, n0 = bx * BN * NS;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;

  typename Plan::State sa[MS], sb[NS];
#pragma unroll
  for (int i = 0; i < MS; ++i) sa[i] = pl.init(k, m0 + BM * i, n0, tid);
#pragma unroll
  for (int j = 0; j < NS; ++j) sb[j] = pl.init(k, m0, n0 + BN * j, tid);
  float ra[MS][8], rb[NS][8];
  f32x16 acc[MS][NS];
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  auto load = [&](int r) {
#pragma unroll
    for (int i = 0; i < MS; ++i) pl.load_a(sa[i], r, ra[i]);
#pragma unroll
    for (int j = 0; j < NS; ++j) pl.load_b(sb[j], r, rb[j]);
  };
  auto stash_all = [&](int buf) {
#pragma unroll
    for (int i = 0; i < MS; ++i) stash<Plan::LA>(As[buf][i], ra[i], tid);
#pragma unroll
    for (int j = 0; j < NS; ++j) stash<Plan::LB>(Bs[buf][j], rb[j], tid);
  };
  if constexpr (X6 == 2) {
    // Software-pipelined bf16x6 loop (the default form).  A wave issues in
    // order, so its fragment reads, bf16 splits, LDS stash and global loads
    // only overlap its own MFMAs when they sit between them in one basic
    // block.  Per K-tile t (two 16-deep k-steps, fragments F of step 0 ready):
    //   phase 0: MFMAs of step 0 || read + split step 1 -> F1, stash tile t+1
    //   barrier (publishes tile t+1; every read of the buffer it reuses is done)
    //   phase 1: MFMAs of step 1 || global loads of tile t+2, read + split
    //            step 0 of tile t+1 -> F0
    // Tiles past the last are clamped to it (duplicate loads / stashes / splits
    // that nothing consumes), so both phases are branch-free.
    static_assert(BK == 32, "two k-steps per K-tile");
    const int ntile = rend > rbeg ? (rend - rbeg + BK - 1) / BK : 0;
    if (ntile > 0) {
      const int rlast = rbeg + (ntile - 1) * BK;
      bf16x8 ah0[MS], am0[MS], al0[MS], bh0[NS], bm0[NS], bl0[NS];
      bf16x8 ah1[MS], am1[MS], al1[MS], bh1[NS], bm1[NS], bl1[NS];
      float va[MS][8], vb[NS][8];
      auto read_frags = [&](int buf, int s) {
#pragma unroll
        for (int i = 0; i < MS; ++i) frag8<Plan::LA>(As[buf][i], 32 * wm + l32, 16 * s + 8 * h, va[i]);
#pragma unroll
        for (int j = 0; j < NS; ++j) frag8<Plan::LB>(Bs[buf][j], 32 * wn + l32, 16 * s + 8 * h, vb[j]);
      };
#define FLR_SPLIT_ALL(AH, AM, AL, BH, BM, BL)                                       \
  _Pragma("unroll") for (int i = 0; i < MS; ++i) split3(va[i], AH[i], AM[i], AL[i]); \
  _Pragma("unroll") for (int j = 0; j < NS; ++j) split3(vb[j], BH[j], BM[j], BL[j]);
#define FLR_X6P(AV, BV)                                                                           \
  _Pragma("unroll") for (int i = 0; i < MS; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(AV[i], BV[j], acc[i][j], 0, 0, 0);
#define FLR_X6P_ALL(AH, AM, AL, BH, BM, BL) \
  FLR_X6P(AM, BM) FLR_X6P(AH, BL) FLR_X6P(AL, BH) FLR_X6P(AH, BM) FLR_X6P(AM, BH) FLR_X6P(AH, BH)
      load(rbeg);
      stash_all(0);
      __syncthreads();
      load(std::min(rbeg + BK, rlast));
      read_frags(0, 0);
      FLR_SPLIT_ALL(ah0, am0, al0, bh0, bm0, bl0)
      int cur = 0;
      for (int t = 0; t < ntile; ++t) {
        const int r0 = rbeg + t * BK;
        // phase 0
        read_frags(cur, 1);
        FLR_X6P_ALL(ah0, am0, al0, bh0, bm0, bl0)
        FLR_SPLIT_ALL(ah1, am1, al1, bh1, bm1, bl1)
        stash_all(cur ^ 1);
        __syncthreads();
        // phase 1
        load(std::min(r0 + 2 * BK, rlast));
        read_frags(cur ^ 1, 0);
        FLR_X6P_ALL(ah1, am1, al1, bh1, bm1, bl1)
        FLR_SPLIT_ALL(ah0, am0, al0, bh0, bm0, bl0)
        cur ^= 1;
      }
#undef FLR_SPLIT_ALL
#undef FLR_X6P
#undef FLR_X6P_ALL
    }
  } else {
  if (rbeg < rend) {
    load(rbeg);
    stash_all(0);
  }
  __syncthreads();
  int cur = 0;
  for (int r0 = rbeg; r0 < rend; r0 += BK) {
    const bool more = r0 + BK < rend;
    if (more) load(r0 + BK);  // in flight during the MFMAs below
    if constexpr (X6 != 0) {
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 ah[MS], am[MS], al[MS], bh[NS], bm[NS], bl[NS];
#pragma unroll
        for (int i = 0; i < MS; ++i) {
          float v[8];
          frag8<Plan::LA>(As[cur][i], 32 * wm + l32, 16 * s + 8 * h, v);
          if constexpr (X6 == 3) {
#pragma unroll
            for (int q = 0; q < 8; ++q) ah[i][q] = am[i][q] = al[i][q] = (__bf16)v[q];
          } else {
            split3(v, ah[i], am[i], al[i]);
          }
        }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          float v[8];
          frag8<Plan::LB>(Bs[cur][j], 32 * wn + l32, 16 * s + 8 * h, v);
          if constexpr (X6 == 3) {
#pragma unroll
            for (int q = 0; q < 8; ++q) bh[j][q] = bm[j][q] = bl[j][q] = (__bf16)v[q];
          } else {
            split3(v, bh[j], bm[j], bl[j]);
          }
        }
        if (prio) __builtin_amdgcn_s_setprio(1);
        if constexpr (X6 >= 3) {
          // product-major: the MS*NS accumulator chains interleave, so a chain's
          // next MFMA never waits on its own previous one (small terms first)
#define FLR_X6_STEP(AV, BV)                                                              \
  _Pragma("unroll") for (int i = 0; i < MS; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(AV[i], BV[j], acc[i][j], 0, 0, 0);
          FLR_X6_STEP(am, bm)
          FLR_X6_STEP(ah, bl)
          FLR_X6_STEP(al, bh)
          FLR_X6_STEP(ah, bm)
          FLR_X6_STEP(am, bh)
          FLR_X6_STEP(ah, bh)
#undef FLR_X6_STEP
        } else {
#pragma unroll
          for (int i = 0; i < MS; ++i)
#pragma unroll
            for (int j = 0; j < NS; ++j) {  // small terms first
              f32x16 c = acc[i][j];
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], c, 0, 0, 0);
              acc[i][j] = c;
            }
        }
        if (prio) __builtin_amdgcn_s_setprio(0);
      }
    } else {
      f32x4 fa[MS][4], fb[NS][4];  // all of the tile's fragments first: the reads overlap the MFMA chain
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
#pragma unroll
        for (int i = 0; i < MS; ++i) fa[i][jj] = frag<Plan::LA>(As[cur][i], 32 * wm + l32, jj, h);
#pragma unroll
        for (int j = 0; j < NS; ++j) fb[j][jj] = frag<Plan::LB>(Bs[cur][j], 32 * wn + l32, jj, h);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the chain (the scheduler would interleave them)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < MS; ++i)
#pragma unroll
            for (int j = 0; j < NS; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][jj][t], fb[j][jj][t], acc[i][j], 0, 0, 0);
    }
    if (more) stash_all(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  }  // old loop (FLR_GEMM=f32 | chain | old | A)
  // C/D map of the 32x32 MFMA: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int tm0 = m0 + BM * i, tn0 = n0 + BN * j;
      if (S == 1 && pl.linear()) {  // one tile base, then row * ldm + col per element
        float* base = pl.out() + pl.tile_base(k, tm0, tn0);
        const int64_t ldm = pl.ldm();
        const int nl = 32 * wn + l32;
        if constexpr (std::is_base_of<BGemmArgs, Plan>::value) {
          if (pl.bias) {  // the batched GEMM's bias: one value per lane column, bias + v
            const float bv = tn0 + nl < N ? pl.bias[k * pl.bias_k + tn0 + nl] : 0.f;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = bv + acc[i][j][e];
          }
        }
        if (const float* abase = plan_add(pl)) {  // all 16 addends in flight before the first store
          abase += pl.tile_base(k, tm0, tn0);
          float av[16];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int ml = 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            av[e] = (tm0 + ml < M && tn0 + nl < N) ? abase[ml * ldm + nl] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = __fadd_rn(acc[i][j][e], av[e]);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int ml = 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (tm0 + ml < M && tn0 + nl < N) base[ml * ldm + nl] = acc[i][j][e];
        }
        continue;
      }
      if constexpr (std::is_same<Plan, DgradT>::value) {
        if (S == 1 && pl.add) {  // parity-class stores: the addends loaded before any store
          int64_t ix[16];
          float av[16];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = tm0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            const int n = tn0 + 32 * wn + l32;
            ix[e] = (m < M && n < N) ? pl.index(k, m, n) : -1;
            av[e] = ix[e] >= 0 ? pl.add[ix[e]] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (ix[e] >= 0) pl.dx[ix[e]] = __fadd_rn(acc[i][j][e], av[e]);
          continue;
        }
      }
      if constexpr (std::is_base_of<BGemmArgs, Plan>::value) {
        if (S == 1) {
          pl.store_tile(k, tm0, tn0, 32 * wm + 4 * h, 32 * wn + l32, acc[i][j], M, N);
          continue;
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = tm0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int n = tn0 + 32 * wn + l32;
        if (m < M && n < N) {
          if (S == 1) pl.store(k, m, n, acc[i][j][e]);
          else part[(((int64_t)split * pl.g.Kc + k) * M + m) * N + n] = acc[i][j][e];
        }
      }
    }
  if constexpr (has_sq<Plan>::value) {
    if (S == 1 && pl.sq) {  // this tile's clip-norm partial (split-K: the treduce pass writes them)
      double sq = 0.0;
#pragma unroll
      for (int i = 0; i < MS; ++i)
#pragma unroll
        for (int j = 0; j < NS; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = m0 + BM * i + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            const int n = n0 + BN * j + 32 * wn + l32;
            const double v = (m < M && n < N) ? (double)acc[i][j][e] : 0.0;
            sq += v * v;
          }
      __shared__ double red[THREADS / 64];
      const double t = block_sumsq(sq, red);
      if (tid == 0) pl.sq[(int64_t)k * pl.sq_ld + by * (int)gridDim.x + bx] = t;
    }
  }
}

// ---- the split-at-stash form (FLR_GEMM=stash) ------------------------------
// Each value is split into bf16 hi/mid/lo ONCE, by the thread that loaded it,
// instead of once per wave that reads its fragment: the LDS holds three bf16
// images per sub-tile, [64 rows][32 k] with the four 16-B k-chunks of a row
// XOR-swizzled by zswz(row) (no padding: conflict-free ds_read_b128 fragment
// reads and ds_write_b128 stashes under both stash mappings, checked
// exhaustively over the lane groups), and an MFMA fragment is one
// ds_read_b128 per term.  48 KB per 128 x 128 tile, so three workgroups fit a
// CU's LDS (the padded 80-B rows took 61 KB: two).  The loads are k-contiguous (thread: row tid & 63,
// k 8 (tid >> 6) .. +7, the plans' init8 / load_a8 / load_b8), so a thread's
// stash is three 16-B writes per sub-tile.  Single LDS buffer, two barriers
// per K-tile; the split of tile t+1 sits between tile t's MFMAs.  Every
// accumulator sees the same bf16 products in the same order as the other
// bf16x6 forms: the results are bit-identical to them.
#ifndef FLR_LDS_SWZ
#define FLR_LDS_SWZ 1
#endif
#if FLR_LDS_SWZ
constexpr int SB = 32;            // bf16 per image row (chunks swizzled, no pad)
#else
constexpr int SB = 40;            // bf16 per image row (32 + 8 pad; A/B build)
#endif
constexpr int TERM_B = 64 * SB;   // bf16 per term image
// bf16 offset of (row, k-chunk c = k / 8) in a row-major term image
__device__ __forceinline__ int zimg(int row, int c) {
#if FLR_LDS_SWZ
  const int f = ((row >> 2) & 1) | ((((row >> 1) ^ (row >> 3)) & 1) << 1);
  return row * SB + 8 * (c ^ f);
#else
  return row * SB + 8 * c;
#endif
}
// waves per SIMD the split-at-stash kernels are compiled for (FLR_SG_OCC=3: at
// most 168 VGPRs, three 128 x 128 workgroups per CU)
#ifndef FLR_SG_OCC
#define FLR_SG_OCC 2
#endif
#ifndef FLR_FRAG_AHEAD
#define FLR_FRAG_AHEAD 1
#endif
template <class P> struct has_k8 : std::false_type {};
template <> struct has_k8<FwdT> : std::true_type {};
template <> struct has_k8<DgradT> : std::true_type {};
// WgtT has k8 loads but stays on the pipelined form: its x operand is k-contiguous
// only along pixels, so the k8 mapping puts the lanes on channels (sxc apart, a
// cache line per lane): l1 wgrad 202 -> 366 us measured.
template <int A, int B> struct has_k8<BGemm<A, B>> : std::true_type {};

// The epilogue of the split-at-stash and LDS-DMA forms: this wave's MSW x NS
// accumulator tiles (32 x 32 each, at (m0 + m_off(i), n0 + n_off(j))) to the
// plan's output (S == 1: epilogue operands loaded before the stores) or to the
// split-K partials.
template <int MSW, int NS>
struct TileOffs {
  int m[MSW], n[NS];  // the wave's 32 x 32 blocks' row / column offsets from (m0, n0)
};
template <class Plan, int MSW, int NS>
__device__ __forceinline__ void sg_store(const Plan& pl, int S, float* __restrict__ part, int k, int split, int m0,
                                         int n0, int h, int l32, int M, int N, f32x16 (&acc)[MSW][NS],
                                         const TileOffs<MSW, NS> off) {
  // C/D map of the 32x32 MFMA: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < MSW; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      // (tm0, tn0): this wave's 32 x 32 block; offsets inside it below
      const int tm0 = m0 + off.m[i], tn0 = n0 + off.n[j];
      if (S == 1 && pl.linear()) {
        float* base = pl.out() + pl.tile_base(k, tm0, tn0);
        const int64_t ldm = pl.ldm();
        const int nl = l32;
        if constexpr (std::is_base_of<BGemmArgs, Plan>::value) {
          if (pl.bias) {  // the batched GEMM's bias: one value per lane column, bias + v
            const float bv = tn0 + nl < N ? pl.bias[k * pl.bias_k + tn0 + nl] : 0.f;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = bv + acc[i][j][e];
          }
        }
        if (const float* abase = plan_add(pl)) {  // all 16 addends in flight before the first store
          abase += pl.tile_base(k, tm0, tn0);
          float av[16];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int ml = (e & 3) + 8 * (e >> 2) + 4 * h;
            av[e] = (tm0 + ml < M && tn0 + nl < N) ? abase[ml * ldm + nl] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = __fadd_rn(acc[i][j][e], av[e]);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int ml = (e & 3) + 8 * (e >> 2) + 4 * h;
          if (tm0 + ml < M && tn0 + nl < N) base[ml * ldm + nl] = acc[i][j][e];
        }
        continue;
      }
      if constexpr (std::is_same<Plan, DgradT>::value) {
        if (S == 1 && pl.add) {  // parity-class stores: the addends loaded before any store
          int64_t ix[16];
          float av[16];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = tm0 + (e & 3) + 8 * (e >> 2) + 4 * h;
            const int n = tn0 + l32;
            ix[e] = (m < M && n < N) ? pl.index(k, m, n) : -1;
            av[e] = ix[e] >= 0 ? pl.add[ix[e]] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (ix[e] >= 0) pl.dx[ix[e]] = __fadd_rn(acc[i][j][e], av[e]);
          continue;
        }
      }
      if constexpr (std::is_base_of<BGemmArgs, Plan>::value) {
        if (S == 1) {
          pl.store_tile(k, tm0, tn0, 4 * h, l32, acc[i][j], M, N);
          continue;
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = tm0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int n = tn0 + l32;
        if (m < M && n < N) {
          if (S == 1) pl.store(k, m, n, acc[i][j][e]);
          else part[(((int64_t)split * pl.g.Kc + k) * M + m) * N + n] = acc[i][j][e];
        }
      }
    }
}

// Two LDS stages (one barrier per K-tile, tile t+1 stashed into the other stage
// during tile t's MFMAs, one workgroup per CU by LDS) were measured 20-35 %
// slower than this one-stage form at two workgroups per CU (C3 conv and C4
// GEMM shapes, profiles/r3_sgemm_db.txt).
//
// Producer / consumer waves (8 consumer waves over a 128 x 256 tile + 4 waves that
// only stash into the other of two LDS stages, one barrier per K-tile; or 4 + 4 over
// 128 x 128) were measured, bit-identical, 7-40 % slower than this loop on the C4
// GEMM and C3 conv shapes (profiles/r3_gemm_loop/pc8_*): the consumer waves, which
// wait for their fragment reads after every barrier, set the pace.
//
// A half-phase schedule (one barrier per 16-deep k-step; waves 0-1 stash k-step 0's
// half of the next tile beside k-step 1's MFMAs, waves 2-3 k-step 1's half beside
// the next k-step 0; lane pairs instead of quads on k-contiguous rows) was
// bit-identical and 0-25 % slower per conv layer, 8-27 % on the C4 GEMMs, C3 round
// 60.0 -> 61.5 ms (profiles/r3_gemm_loop/half_phase.txt): twice the barriers per MFMA.
// Issuing tile t+2's global loads before the first barrier instead of after the
// stash: neutral on the GEMMs, C3 round 58.7 -> 59.6 ms (same file).
// NAR (narrow N, the l4 convolutions' N = B * 1 * 1 = 32 pixels): NS = 1 and the four
// waves stacked along M over MS 64-row A sub-tiles, each wave MS / 2 MFMA blocks of
// 32 x 32 on the first 32 columns of the B image — a 64-wide N tile would leave half
// its MFMAs on empty columns.  Same products per output: bit-identical.
template <class Plan, int MS, int NS, int D, int ABL = 0, bool NAR = false>
__device__ __forceinline__ void sgemm_body(const Plan& pl, int S, float* __restrict__ part, int remap) {
  static_assert(!NAR || (NS == 1 && (MS == 2 || MS == 4)), "narrow tiles: 128 or 256 x 32");
  constexpr int MSW = NAR ? MS / 2 : MS;  // MFMA blocks per wave along M (NAR), or A sub-tiles
  constexpr int NST = 1;
  __shared__ __attribute__((aligned(16))) __bf16 Ls[NST][MS + NS][3][TERM_B];
  int bx = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
  if (remap & 1) xcd_tile(bx, by, bz);
  if (remap >> 8) odd_slot_controls(remap);
  const int k = bz / S, split = bz % S;
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const int ktiles = cdiv(R, BK);
  const int rbeg = (int)((int64_t)ktiles * split / S) * BK;
  const int rend = std::min(R, (int)((int64_t)ktiles * (split + 1) / S) * BK);
  const int m0 = by * BM * MS, n0 = bx * BN * NS;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;
  // this thread's stash row and k offset per operand (Plan::QUAD_A / QUAD_B)
  const int srowA = stash_row<Plan::QUAD_A>(tid), skA = stash_k<Plan::QUAD_A>(tid);
  const int srowB = stash_row<Plan::QUAD_B>(tid), skB = stash_k<Plan::QUAD_B>(tid);

  typename Plan::State8 sa[MS], sb[NS];
#pragma unroll
  for (int i = 0; i < MS; ++i) sa[i] = pl.init8(k, m0 + BM * i, n0, tid);
#pragma unroll
  for (int j = 0; j < NS; ++j) sb[j] = pl.init8(k, m0, n0 + BN * j, tid);
  // register sets; D == 3 keeps two tiles of global loads in flight (measured: no gain over D == 2 at the
  // C3 conv and C4 GEMM shapes — the loop is not load-latency-bound; D == 2 is the one instantiated)
  float ra[2][MS][8], rb[2][NS][8];
  bf16x8 pa[MS][3], pb[NS][3];
  f32x16 acc[MSW][NS];
#pragma unroll
  for (int i = 0; i < MSW; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // this wave's MFMA block i: A sub-tile and row band (NAR: wave-stacked), and its
  // row / column offset from (m0, n0)
  auto a_sub = [&](int i) { return NAR ? (wave * MSW + i) >> 1 : i; };
  auto a_row = [&](int i) { return NAR ? 32 * ((wave * MSW + i) & 1) + l32 : 32 * wm + l32; };
  auto b_row = [&]() { return NAR ? l32 : 32 * wn + l32; };
  auto m_off = [&](int i) { return NAR ? 32 * (wave * MSW + i) : BM * i + 32 * wm; };
  auto n_off = [&](int j) { return NAR ? 0 : BN * j + 32 * wn; };
  auto load = [&](int r, auto qc) {
    constexpr int Q = decltype(qc)::value;
#pragma unroll
    for (int i = 0; i < MS; ++i) pl.load_a8(sa[i], r, ra[Q][i]);
#pragma unroll
    for (int j = 0; j < NS; ++j) pl.load_b8(sb[j], r, rb[Q][j]);
  };
  auto split_all = [&](auto qc) {
    constexpr int Q = decltype(qc)::value;
#pragma unroll
    for (int i = 0; i < MS; ++i) split3(ra[Q][i], pa[i][0], pa[i][1], pa[i][2]);
#pragma unroll
    for (int j = 0; j < NS; ++j) split3(rb[Q][j], pb[j][0], pb[j][1], pb[j][2]);
  };
  auto write_all = [&](auto stc) {
    constexpr int ST = decltype(stc)::value;
#pragma unroll
    for (int i = 0; i < MS; ++i)
#pragma unroll
      for (int t = 0; t < 3; ++t) *reinterpret_cast<bf16x8*>(&Ls[ST][i][t][zimg(srowA, skA >> 3)]) = pa[i][t];
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int t = 0; t < 3; ++t) *reinterpret_cast<bf16x8*>(&Ls[ST][MS + j][t][zimg(srowB, skB >> 3)]) = pb[j][t];
  };
  // FLR_FRAG_AHEAD (default): both k-steps' fragments are read before the
  // first MFMA, so the second k-step's LDS latency runs under the first's MFMAs
  // and the reads are complete by the barrier that follows (the compiler keeps
  // the reads ahead of that barrier and moves the second k-step's MFMAs after
  // it); 0: read per k-step (A/B build).  Same operands, same MFMA order.
  auto compute_tile = [&](auto stc) {
      constexpr int ST = decltype(stc)::value;
      constexpr int NKS = BK / 16;
#if FLR_FRAG_AHEAD
      bf16x8 fa[NKS][MSW][3], fb[NKS][NS][3];
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const int ko = 16 * s + 8 * h;
#pragma unroll
        for (int i = 0; i < MSW; ++i)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            fa[s][i][q] = *reinterpret_cast<const bf16x8*>(&Ls[ST][a_sub(i)][q][zimg(a_row(i), ko >> 3)]);
#pragma unroll
        for (int j = 0; j < NS; ++j)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            fb[s][j][q] = *reinterpret_cast<const bf16x8*>(&Ls[ST][MS + j][q][zimg(b_row(), ko >> 3)]);
      }
      __builtin_amdgcn_sched_barrier(0);  // the scheduler would sink the second k-step's reads again
#define FLR_SX(TA, TB)                                                                              \
  _Pragma("unroll") for (int i = 0; i < MSW; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][TA], fb[s][j][TB], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        // product-major, small terms first (term 0 = hi, 1 = mid, 2 = lo)
        FLR_SX(1, 1) FLR_SX(0, 2) FLR_SX(2, 0) FLR_SX(0, 1) FLR_SX(1, 0) FLR_SX(0, 0)
      }
#undef FLR_SX
#else
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        bf16x8 fa[MSW][3], fb[NS][3];
        const int ko = 16 * s + 8 * h;
#pragma unroll
        for (int i = 0; i < MSW; ++i)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            fa[i][q] = *reinterpret_cast<const bf16x8*>(&Ls[ST][a_sub(i)][q][zimg(a_row(i), ko >> 3)]);
#pragma unroll
        for (int j = 0; j < NS; ++j)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            fb[j][q] = *reinterpret_cast<const bf16x8*>(&Ls[ST][MS + j][q][zimg(b_row(), ko >> 3)]);
#define FLR_SX(TA, TB)                                                                              \
  _Pragma("unroll") for (int i = 0; i < MSW; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][TA], fb[j][TB], acc[i][j], 0, 0, 0);
        // product-major, small terms first (term 0 = hi, 1 = mid, 2 = lo)
        FLR_SX(1, 1) FLR_SX(0, 2) FLR_SX(2, 0) FLR_SX(0, 1) FLR_SX(1, 0) FLR_SX(0, 0)
#undef FLR_SX
      }
#endif
  };
  const int ntile = rend > rbeg ? (rend - rbeg + BK - 1) / BK : 0;
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  if (ntile > 0) {
    const int rlast = rbeg + (ntile - 1) * BK;
    load(rbeg, Q0{});
    split_all(Q0{});
    write_all(Q0{});
    load(std::min(rbeg + BK, rlast), Q0{});
    if constexpr (D == 3) load(std::min(rbeg + 2 * BK, rlast), Q1{});
    __syncthreads();
    {
      // one K-tile: the MFMAs of tile t from the LDS images, the split of tile t+1
      // (register set Q) between them, its stash, then the global loads of tile
      // t+D-1 into the set just freed (clamped past the last tile: duplicates)
      auto tile_body = [&](int t, auto qc) {
        const int r0 = rbeg + t * BK;
        // ABL (tools build only, timing ablations with wrong results): 1 no global loads,
        // 2 no stash writes, 4 no first barrier, 8 no split, 16 no MFMAs / fragment reads
        // (profiles/r3_gemm_loop/: without the stash writes the loop is 36 % shorter; with
        // only the fragment reads and MFMAs it runs at ~0.55 of the bf16x6 ceiling)
        if constexpr (!(ABL & 16)) compute_tile(Q0{});
        if constexpr (!(ABL & 8)) split_all(qc);
        if constexpr (!(ABL & 4)) __syncthreads();  // every wave's fragment reads of tile t are done
        if constexpr (!(ABL & 2)) write_all(Q0{});
        if constexpr (!(ABL & 1)) load(std::min(r0 + D * BK, rlast), qc);
        __syncthreads();
      };
      if constexpr (D == 3) {
        for (int t = 0; t < ntile; t += 2) {
          tile_body(t, Q0{});
          if (t + 1 < ntile) tile_body(t + 1, Q1{});
        }
      } else {
        for (int t = 0; t < ntile; ++t) tile_body(t, Q0{});
      }
    }
  }
  TileOffs<MSW, NS> off;
#pragma unroll
  for (int i = 0; i < MSW; ++i) off.m[i] = m_off(i);
#pragma unroll
  for (int j = 0; j < NS; ++j) off.n[j] = n_off(j);
  sg_store<Plan, MSW, NS>(pl, S, part, k, split, m0, n0, h, l32, M, N, acc, off);
}

template <class Plan, int MS, int NS, int D, int ABL = 0, bool NAR = false>
__global__ __launch_bounds__(THREADS, FLR_SG_OCC) void sgemm_kernel(const Plan pl, int S, float* __restrict__ part,
                                                                     int remap) {
  sgemm_body<Plan, MS, NS, D, ABL, NAR>(pl, S, part, remap);
}

// ---- the LDS-DMA form (FLR_BGEMM_DMA=1, batched GEMMs with RK / KR operands) ---
// 128 x 128 tiles, four waves of 64 x 64.  The fp32 operand tiles go global ->
// LDS by buffer_load_dwordx4 ... lds (BGemm::dma_op): no VGPR staging and no
// ds_write pass (the split-at-stash form spends 36 % of its loop in the stash
// writes, profiles/r3_gemm_loop/).  Two LDS stages of 32 KB, one barrier per
// K-tile: tile t+1's DMA runs under tile t's MFMAs.  Each wave splits its own
// fragments into bf16 hi / mid / lo at read time (twice the split work of the
// stash form, on the VALU beside the MFMAs).  Every accumulator sees the same
// bf16 products in the same order as sgemm_body: bit-identical.
constexpr int DG_IMG = 128 * BK;  // floats per operand image
template <class Plan>
__global__ __launch_bounds__(THREADS, 2) void dsgemm_kernel(const Plan pl, int S, float* __restrict__ part,
                                                            int remap) {
  constexpr int MSW = 2, NS = 2;
  __shared__ __attribute__((aligned(16))) float Lf[2][2][DG_IMG];  // [stage][A, B]
  int bx = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
  if (remap & 1) xcd_tile(bx, by, bz);
  const int k = bz / S, split = bz % S;
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const int ktiles = cdiv(R, BK);
  const int rbeg = (int)((int64_t)ktiles * split / S) * BK;
  const int rend = std::min(R, (int)((int64_t)ktiles * (split + 1) / S) * BK);
  const int m0 = by * 128, n0 = bx * 128;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;
  const typename Plan::State8 st = pl.init8(k, m0, n0, tid);
  f32x16 acc[MSW][NS];
#pragma unroll
  for (int i = 0; i < MSW; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  auto dma = [&](int r0, int sg) {
    pl.dma_a(st, &Lf[sg][0][0], r0, wave, lane);
    pl.dma_b(st, &Lf[sg][1][0], r0, wave, lane);
  };
  // lane (l32, h): row `row` of the image, k = 16 s + 8 h .. +7
  auto frag = [&](const float* img, auto modec, int row, int s, float (&v)[8]) {
    constexpr int MODE = decltype(modec)::value;
    if constexpr (MODE == BM_RK) {
      const int f = (row >> 1) & 7, q0 = 4 * s + 2 * h;
      const f32x4 a = *reinterpret_cast<const f32x4*>(img + row * BK + 4 * (q0 ^ f));
      const f32x4 b = *reinterpret_cast<const f32x4*>(img + row * BK + 4 * ((q0 + 1) ^ f));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = a[e];
        v[4 + e] = b[e];
      }
    } else {
      const float* p = img + (16 * s + 8 * h) * 128 + 4 * ((row >> 2) ^ (h << 3)) + (row & 3);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = p[e * 128];
    }
  };
  using MA = std::integral_constant<int, Plan::AMODE>;
  using MB = std::integral_constant<int, Plan::BMODE>;
  auto compute = [&](int sg) {
    const float* ia = &Lf[sg][0][0];
    const float* ib = &Lf[sg][1][0];
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 fa[MSW][3], fb[NS][3];
#pragma unroll
      for (int i = 0; i < MSW; ++i) {
        float v[8];
        frag(ia, MA{}, 64 * i + 32 * wm + l32, s, v);
        split3(v, fa[i][0], fa[i][1], fa[i][2]);
      }
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        float v[8];
        frag(ib, MB{}, 64 * j + 32 * wn + l32, s, v);
        split3(v, fb[j][0], fb[j][1], fb[j][2]);
      }
#define FLR_DX(TA, TB)                                                                              \
  _Pragma("unroll") for (int i = 0; i < MSW; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][TA], fb[j][TB], acc[i][j], 0, 0, 0);
      // product-major, small terms first: sgemm_body's order
      FLR_DX(1, 1) FLR_DX(0, 2) FLR_DX(2, 0) FLR_DX(0, 1) FLR_DX(1, 0) FLR_DX(0, 0)
#undef FLR_DX
    }
  };
  const int ntile = rend > rbeg ? (rend - rbeg + BK - 1) / BK : 0;
  if (ntile > 0) {
    dma(rbeg, 0);
    for (int t = 0; t < ntile; ++t) {
      // this wave's DMA of tile t landed; after the barrier every wave's has, and
      // every wave's fragment reads of tile t-1 (the stage refilled next) are done
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < ntile) dma(rbeg + (t + 1) * BK, (t + 1) & 1);
      compute(t & 1);
    }
  }
  auto m_off = [&](int i) { return 64 * i + 32 * wm; };
  auto n_off = [&](int j) { return 64 * j + 32 * wn; };
  TileOffs<MSW, NS> off;
#pragma unroll
  for (int i = 0; i < MSW; ++i) off.m[i] = m_off(i);
#pragma unroll
  for (int j = 0; j < NS; ++j) off.n[j] = n_off(j);
  sg_store<Plan, MSW, NS>(pl, S, part, k, split, m0, n0, h, l32, M, N, acc, off);
}

// FLR_BGEMM_DMA=1 selects the LDS-DMA form (read per launch).  Off by default:
// bit-identical, but 0-18 % SLOWER than split-at-stash at every C4 encoder shape
// (vit.qkv 461 vs 391 us, vit.fc1 519 vs 489, vit.fc2 480 vs 455 at 32 clients;
// profiles/r4_bgemm_dma_ab.txt): the per-wave split doubles the VALU split work
// of the stash form, which costs more than the ds_write pass it removes.
inline bool bgemm_dma() {
  const char* e = flr::knob("FLR_BGEMM_DMA");
  return e && e[0] == '1';
}
// ---- the pre-split form (batched GEMMs with 128 x 128 tiles, FLR_BGEMM_PRESPLIT=1; measured slower) --
// Each operand is split into bf16 hi / mid / lo ONCE per GEMM by presplit_kernel
// (the same split3 as every other form) into k-contiguous planes in the
// workspace, [3][K][rows_pad][R_pad] with rows padded to 128 and R to 32 by
// zeros.  The GEMM (psgemm_kernel) is then a plain six-product bf16 loop: each
// 16-deep k-step's three A and three B planes go global -> LDS by
// buffer_load_dwordx4 ... lds into a ring of three 24-KB stages (two k-steps in
// flight, counted vmcnt, raw barrier), fragments are one ds_read_b128 per term,
// no VGPR staging, no ds_write, no split in the loop.  Same bf16 terms, same
// products in the same order per accumulator: bit-identical to sgemm_body.
constexpr int PS_ROWS = 128;                 // tile rows per operand
constexpr int PS_PLANE = PS_ROWS * 16;       // bf16 per plane per stage (16 k per row)
constexpr int PS_STAGE = 6 * PS_PLANE;       // A hi/mid/lo, B hi/mid/lo
constexpr int PS_NST = 3;                    // ring stages
constexpr int PS_PIECES = 6 * PS_PLANE * 2 / 1024;  // 1-KB DMA pieces per stage (24)
static_assert(PS_PIECES % 4 == 0, "pieces split over four waves");

inline int64_t ps_pad(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
inline size_t ps_plane_bytes(int64_t K, int64_t rows, int64_t R) {
  return (size_t)3 * K * ps_pad(rows, PS_ROWS) * ps_pad(R, BK) * 2;
}

// planes[t][k][row][c] = term t of src(k, row, c) (0 outside rows x R)
template <int MODE>
__global__ __launch_bounds__(THREADS) void presplit_kernel(const float* __restrict__ src, int64_t s_k, int64_t s_row,
                                                           int64_t s_r, int K, int rows, int R, int rows_pad,
                                                           int R_pad, __bf16* __restrict__ planes) {
  const int ngrp = R_pad / 8;  // 8-wide k groups per row
  const int64_t per_k = (int64_t)rows_pad * ngrp;
  const int64_t total = (int64_t)K * per_k;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * THREADS) {
    const int k = (int)(i / per_k);
    const int64_t rem = i - (int64_t)k * per_k;
    int row, grp;
    if constexpr (MODE == BM_RK) {  // lanes along k: each reads 32 contiguous bytes
      row = (int)(rem / ngrp);
      grp = (int)(rem - (int64_t)row * ngrp);
    } else {  // lanes along rows: each load instruction reads consecutive rows
      grp = (int)(rem / rows_pad);
      row = (int)(rem - (int64_t)grp * rows_pad);
    }
    float v[8];
    const float* base = src + k * s_k + (int64_t)row * s_row;
    if constexpr (MODE == BM_RK) {  // s_r == 1, R % 4 == 0, 16-B aligned rows: two float4 loads
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = 8 * grp + 4 * q;
        const f32x4 x = (row < rows && c < R) ? *reinterpret_cast<const f32x4*>(base + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = x[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 8 * grp + e;
        v[e] = (row < rows && c < R) ? base[(int64_t)c * s_r] : 0.f;
      }
    }
    bf16x8 t0, t1, t2;
    split3(v, t0, t1, t2);
    const int64_t plane = (int64_t)K * rows_pad * R_pad;
    const int64_t o = ((int64_t)k * rows_pad + row) * R_pad + 8 * grp;
    *reinterpret_cast<bf16x8*>(planes + o) = t0;
    *reinterpret_cast<bf16x8*>(planes + plane + o) = t1;
    *reinterpret_cast<bf16x8*>(planes + 2 * plane + o) = t2;
  }
}

template <class Plan>
__global__ __launch_bounds__(THREADS, 2) void psgemm_kernel(const Plan pl, int S, float* __restrict__ part, int remap,
                                                            const __bf16* __restrict__ pa, const __bf16* __restrict__ pb,
                                                            int Mp, int Np, int Rp) {
  constexpr int MSW = 2, NS = 2;
  __shared__ __attribute__((aligned(16))) __bf16 L[PS_NST * PS_STAGE];  // one array: no compiler vmcnt(0)
  int bx = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
  if (remap & 1) xcd_tile(bx, by, bz);
  const int k = bz / S, split = bz % S;
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const int ktiles = cdiv(R, BK);
  const int rbeg = (int)((int64_t)ktiles * split / S) * BK;
  const int rend = std::min(R, (int)((int64_t)ktiles * (split + 1) / S) * BK);
  const int m0 = by * 128, n0 = bx * 128;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;
  // plane (operand o, term t) of client k: rows from m0 / n0, all of R_pad
  const int64_t pla = (int64_t)pl.g.Kc * Mp * Rp, plb = (int64_t)pl.g.Kc * Np * Rp;
  const rsrc_t ra = make_rsrc(reinterpret_cast<const float*>(pa), 3 * pla / 2);
  const rsrc_t rb = make_rsrc(reinterpret_cast<const float*>(pb), 3 * plb / 2);
  f32x16 acc[MSW][NS];
#pragma unroll
  for (int i = 0; i < MSW; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // one 16-deep k-step into ring stage sg: piece p = (operand, term, 32-row block);
  // lane: row (lane >> 1) of the block, its 16-B half (lane & 1) holds the k half
  // (lane & 1) ^ ((row >> 3) & 1) (source-side swizzle)
  auto dma = [&](int k0, int sg) {
#pragma unroll
    for (int q = 0; q < PS_PIECES / 4; ++q) {
      const int piece = (PS_PIECES / 4) * wave + q;
      const int op = piece / 12, t = (piece % 12) / 4, blk = piece % 4;
      const int row = 32 * blk + (lane >> 1);
      const int half = (lane & 1) ^ ((row >> 3) & 1);
      const int64_t rows_pad = op ? Np : Mp;
      const int64_t e = (int64_t)t * (op ? plb : pla) + ((int64_t)k * rows_pad + (op ? n0 : m0) + row) * Rp + k0 +
                        8 * half;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(op ? rb : ra,
                                               (__attribute__((address_space(3))) void*)(L + sg * PS_STAGE +
                                                                                        piece * 512),
                                               16, (unsigned)(e * 2), 0, 0, 0);
    }
  };
  auto frag = [&](int sg, int op, int t, int row) {
    const int off = sg * PS_STAGE + (op * 3 + t) * PS_PLANE + row * 16 + 8 * (h ^ ((row >> 3) & 1));
    return *reinterpret_cast<const bf16x8*>(L + off);
  };
  const int nstep = rend > rbeg ? 2 * ((rend - rbeg + BK - 1) / BK) : 0;
  if (nstep > 0) {
    dma(rbeg, 0);
    if (nstep > 1) dma(rbeg + 16, 1);
    for (int s = 0; s < nstep; ++s) {
      // this wave's DMA of step s landed (step s+1's may still fly); after the
      // barrier every wave's has, and every wave's reads of step s-1 are done
      if (s + 1 < nstep) {
        static_assert(PS_PIECES / 4 == 6, "vmcnt immediate below");
        asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < nstep) dma(rbeg + 16 * (s + 2), (s + 2) % PS_NST);
      const int sg = s % PS_NST;
      bf16x8 fa[MSW][3], fb[NS][3];
#pragma unroll
      for (int i = 0; i < MSW; ++i)
#pragma unroll
        for (int t = 0; t < 3; ++t) fa[i][t] = frag(sg, 0, t, 64 * i + 32 * wm + l32);
#pragma unroll
      for (int j = 0; j < NS; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t) fb[j][t] = frag(sg, 1, t, 64 * j + 32 * wn + l32);
#define FLR_PX(TA, TB)                                                                              \
  _Pragma("unroll") for (int i = 0; i < MSW; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][TA], fb[j][TB], acc[i][j], 0, 0, 0);
      FLR_PX(1, 1) FLR_PX(0, 2) FLR_PX(2, 0) FLR_PX(0, 1) FLR_PX(1, 0) FLR_PX(0, 0)
#undef FLR_PX
    }
  }
  TileOffs<MSW, NS> off;
#pragma unroll
  for (int i = 0; i < MSW; ++i) off.m[i] = 64 * i + 32 * wm;
#pragma unroll
  for (int j = 0; j < NS; ++j) off.n[j] = 64 * j + 32 * wn;
  sg_store<Plan, MSW, NS>(pl, S, part, k, split, m0, n0, h, l32, M, N, acc, off);
}

// FLR_BGEMM_PRESPLIT=1 selects the pre-split form (read per launch and per
// workspace query).  Off by default: bit-identical, but 1.6-3x SLOWER than
// split-at-stash at the C4 encoder shapes (vit.qkv 624 vs 392 us, vit.fc1.dw 1484
// vs 499 us at 32 clients; profiles/r4_bgemm_presplit_ab.txt).  Three bf16 planes
// are 6 B per operand value against the stash form's 4 B of fp32: the 128 x 128
// tiles re-read their operands from L2 once per opposite tile, so the loop moves
// 1.5x the bytes (2.8 GB per vit.qkv GEMM at 32 clients), and the split pass
// itself transposes the row-contiguous (KR) operands of the weight gradients.
inline bool bgemm_presplit() {
  const char* e = flr::knob("FLR_BGEMM_PRESPLIT");
  return e && e[0] == '1';
}

template <class P> struct dma_ok : std::false_type {};
template <int A, int B> struct dma_ok<BGemm<A, B>> : std::integral_constant<bool, A != BM_G && B != BM_G> {};

// ---- the weight gradient on split-at-stash images, transposed ----------------
// Both operands of dW are contiguous along the reduction (pixels), so the loads
// put a half-wave on 32 consecutive pixels of one channel (coalesced) and each
// thread holds 8 consecutive channels at one pixel (StateT).  The split images
// are [k = 32][row = 64] bf16 per term (128-B k-rows, 16-B chunks of 8 rows
// XOR-swizzled by tswz(k): conflict-free ds_write_b128 stashes and transposed
// reads), and an MFMA fragment (8 consecutive k of one row) is two
// ds_read_b64_tr_b16: each 16-lane group reads a 4 k x 16 row block and gets it
// column-major.  Products and their order per accumulator are the other bf16x6
// forms': bit-identical dw and clip-norm partials.
typedef short s16x4 __attribute__((ext_vector_type(4)));
__host__ __device__ constexpr int tswz(int k) { return (k & 3) | ((((k >> 1) ^ (k >> 2)) & 1) << 2); }
constexpr int TIMG = 32 * 64;  // bf16 per transposed term image

template <class Plan, int MS, int NS, int D, bool TA, bool TB>
__global__ __launch_bounds__(THREADS, FLR_SG_OCC) void wsgemm_kernel(const Plan pl, int S, float* __restrict__ part,
                                                            int remap) {
  // a term image: transposed [32 k][64 rows] (TIMG) or row-major [64 rows][SB] (TERM_B)
  constexpr int IMG = (TA || TB) && !(TA && TB) ? TERM_B : (TA ? TIMG : TERM_B);
  __shared__ __attribute__((aligned(16))) __bf16 Lt[MS + NS][3][IMG];
  int bx = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
  if (remap & 1) xcd_tile(bx, by, bz);
  if (remap >> 8) odd_slot_controls(remap);
  const int k = bz / S, split = bz % S;
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const int ktiles = cdiv(R, BK);
  const int rbeg = (int)((int64_t)ktiles * split / S) * BK;
  const int rend = std::min(R, (int)((int64_t)ktiles * (split + 1) / S) * BK);
  const int m0 = by * BM * MS, n0 = bx * BN * NS;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;
  // stash slot: k = tid & 31, chunk (tid >> 5) ^ tswz(k)
  const int skq = tid & 31;
  const int sidx = skq * 64 + 8 * ((tid >> 5) ^ tswz(skq));
  // transposed-read lane addresses (bf16 index in a term image) for the two 4-k halves
  // of this lane's 8-k fragment; k-step s adds 16 * 64
  const int gq = (lane & 15) >> 2, gp = lane & 3, g1 = (lane >> 4) & 1;
  int ra_off[2], rb_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kk = 8 * h + 4 * j + gq;
    const int ca = 4 * wm + 2 * g1 + (gp >> 1), cb = 4 * wn + 2 * g1 + (gp >> 1);
    ra_off[j] = kk * 64 + 8 * (ca ^ tswz(kk)) + 4 * (gp & 1);
    rb_off[j] = kk * 64 + 8 * (cb ^ tswz(kk)) + 4 * (gp & 1);
  }

  // row-major images: the split-at-stash kernel's stash slot and fragment rows
  const int srowA = stash_row<Plan::QUAD_A>(tid), skA = stash_k<Plan::QUAD_A>(tid);
  const int srowB = stash_row<Plan::QUAD_B>(tid), skB = stash_k<Plan::QUAD_B>(tid);
  using SA = std::conditional_t<TA, typename Plan::StateT, typename Plan::State8>;
  using SBt = std::conditional_t<TB, typename Plan::StateT, typename Plan::State8>;
  SA sa[MS];
  SBt sb[NS];
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if constexpr (TA) sa[i] = pl.initT(k, m0 + BM * i, n0, tid);
    else sa[i] = pl.init8(k, m0 + BM * i, n0, tid);
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    if constexpr (TB) sb[j] = pl.initT(k, m0, n0 + BN * j, tid);
    else sb[j] = pl.init8(k, m0, n0 + BN * j, tid);
  }
  // register sets; D == 3 keeps two tiles of global loads in flight (measured: no gain over D == 2 at the
  // C3 conv and C4 GEMM shapes — the loop is not load-latency-bound; D == 2 is the one instantiated)
  float ra[2][MS][8], rb[2][NS][8];
  bf16x8 pa[MS][3], pb[NS][3];
  f32x16 acc[MS][NS];
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  auto load = [&](int r, auto qc) {
    constexpr int Q = decltype(qc)::value;
#pragma unroll
    for (int i = 0; i < MS; ++i) {
      if constexpr (TA) pl.load_at8(sa[i], r, ra[Q][i]);
      else pl.load_a8(sa[i], r, ra[Q][i]);
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      if constexpr (TB) pl.load_bt8(sb[j], r, rb[Q][j]);
      else pl.load_b8(sb[j], r, rb[Q][j]);
    }
  };
  auto split_all = [&](auto qc) {
    constexpr int Q = decltype(qc)::value;
#pragma unroll
    for (int i = 0; i < MS; ++i) split3(ra[Q][i], pa[i][0], pa[i][1], pa[i][2]);
#pragma unroll
    for (int j = 0; j < NS; ++j) split3(rb[Q][j], pb[j][0], pb[j][1], pb[j][2]);
  };
  auto write_all = [&]() {
#pragma unroll
    for (int i = 0; i < MS; ++i)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        *reinterpret_cast<bf16x8*>(&Lt[i][t][TA ? sidx : zimg(srowA, skA >> 3)]) = pa[i][t];
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        *reinterpret_cast<bf16x8*>(&Lt[MS + j][t][TB ? sidx : zimg(srowB, skB >> 3)]) = pb[j][t];
  };
  auto tread = [&](const __bf16* img, const int (&off)[2], int s) -> bf16x8 {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off[0] + 1024 * s));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off[1] + 1024 * s));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  auto compute_tile = [&]() {
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 fa[MS][3], fb[NS][3];
#pragma unroll
        for (int i = 0; i < MS; ++i)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            if constexpr (TA) fa[i][q] = tread(Lt[i][q], ra_off, s);
            else fa[i][q] = *reinterpret_cast<const bf16x8*>(&Lt[i][q][zimg(32 * wm + l32, 2 * s + h)]);
          }
#pragma unroll
        for (int j = 0; j < NS; ++j)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            if constexpr (TB) fb[j][q] = tread(Lt[MS + j][q], rb_off, s);
            else fb[j][q] = *reinterpret_cast<const bf16x8*>(&Lt[MS + j][q][zimg(32 * wn + l32, 2 * s + h)]);
          }
#define FLR_SX(TA, TB)                                                                              \
  _Pragma("unroll") for (int i = 0; i < MS; ++i) _Pragma("unroll") for (int j = 0; j < NS; ++j) \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][TA], fb[j][TB], acc[i][j], 0, 0, 0);
        // product-major, small terms first (term 0 = hi, 1 = mid, 2 = lo)
        FLR_SX(1, 1) FLR_SX(0, 2) FLR_SX(2, 0) FLR_SX(0, 1) FLR_SX(1, 0) FLR_SX(0, 0)
#undef FLR_SX
      }
  };
  const int ntile = rend > rbeg ? (rend - rbeg + BK - 1) / BK : 0;
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  if (ntile > 0) {
    const int rlast = rbeg + (ntile - 1) * BK;
    load(rbeg, Q0{});
    split_all(Q0{});
    write_all();
    load(std::min(rbeg + BK, rlast), Q0{});
    if constexpr (D == 3) load(std::min(rbeg + 2 * BK, rlast), Q1{});
    __syncthreads();
    // one K-tile: the MFMAs of tile t from the LDS images, the split of tile t+1
    // (register set Q) between them, its stash, then the global loads of tile
    // t+D-1 into the set just freed (clamped past the last tile: duplicates)
    auto tile_body = [&](int t, auto qc) {
      const int r0 = rbeg + t * BK;
      compute_tile();
      split_all(qc);
      __syncthreads();  // every wave's fragment reads of tile t are done
      write_all();
      load(std::min(r0 + D * BK, rlast), qc);
      __syncthreads();
    };
    if constexpr (D == 3) {
      for (int t = 0; t < ntile; t += 2) {
        tile_body(t, Q0{});
        if (t + 1 < ntile) tile_body(t + 1, Q1{});
      }
    } else {
      for (int t = 0; t < ntile; ++t) tile_body(t, Q0{});
    }
  }
  // C/D map of the 32x32 MFMA: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int tm0 = m0 + BM * i, tn0 = n0 + BN * j;
      if (S == 1 && pl.linear()) {  // one tile base, then row * ldm + col per element
        float* base = pl.out() + pl.tile_base(k, tm0, tn0);
        const int64_t ldm = pl.ldm();
        const int nl = 32 * wn + l32;
        if constexpr (std::is_base_of<BGemmArgs, Plan>::value) {
          if (pl.bias) {  // the batched GEMM's bias: one value per lane column, bias + v
            const float bv = tn0 + nl < N ? pl.bias[k * pl.bias_k + tn0 + nl] : 0.f;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = bv + acc[i][j][e];
          }
        }
        if (const float* abase = plan_add(pl)) {  // all 16 addends in flight before the first store
          abase += pl.tile_base(k, tm0, tn0);
          float av[16];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int ml = 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            av[e] = (tm0 + ml < M && tn0 + nl < N) ? abase[ml * ldm + nl] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = __fadd_rn(acc[i][j][e], av[e]);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int ml = 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (tm0 + ml < M && tn0 + nl < N) base[ml * ldm + nl] = acc[i][j][e];
        }
        continue;
      }
      if constexpr (std::is_same<Plan, DgradT>::value) {
        if (S == 1 && pl.add) {  // parity-class stores: the addends loaded before any store
          int64_t ix[16];
          float av[16];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = tm0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            const int n = tn0 + 32 * wn + l32;
            ix[e] = (m < M && n < N) ? pl.index(k, m, n) : -1;
            av[e] = ix[e] >= 0 ? pl.add[ix[e]] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (ix[e] >= 0) pl.dx[ix[e]] = __fadd_rn(acc[i][j][e], av[e]);
          continue;
        }
      }
      if constexpr (std::is_base_of<BGemmArgs, Plan>::value) {
        if (S == 1) {
          pl.store_tile(k, tm0, tn0, 32 * wm + 4 * h, 32 * wn + l32, acc[i][j], M, N);
          continue;
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = tm0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int n = tn0 + 32 * wn + l32;
        if (m < M && n < N) {
          if (S == 1) pl.store(k, m, n, acc[i][j][e]);
          else part[(((int64_t)split * pl.g.Kc + k) * M + m) * N + n] = acc[i][j][e];
        }
      }
    }
  if constexpr (has_sq<Plan>::value) {
    if (S == 1 && pl.sq) {  // this tile's clip-norm partial (split-K: the treduce pass writes them)
      double sq = 0.0;
#pragma unroll
      for (int i = 0; i < MS; ++i)
#pragma unroll
        for (int j = 0; j < NS; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = m0 + BM * i + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            const int n = n0 + BN * j + 32 * wn + l32;
            const double v = (m < M && n < N) ? (double)acc[i][j][e] : 0.0;
            sq += v * v;
          }
      __shared__ double red[THREADS / 64];
      const double t = block_sumsq(sq, red);
      if (tid == 0) pl.sq[(int64_t)k * pl.sq_ld + by * (int)gridDim.x + bx] = t;
    }
  }
}

template <class Plan>
__global__ void treduce_kernel(const Plan pl, int S, const float* __restrict__ part) {
  // grid (cdiv(M*N, 256), K): one client per grid row, 32-bit index math
  const int M = pl.M(), N = pl.N(), K = pl.g.Kc;
  const int k = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = (int64_t)M * N;
  float v = 0.f;
  if (e < MN) {
    const int m = e / N, n = e - m * N;
    const int64_t idx = k * MN + e;
    v = part[idx];
    for (int s = 1; s < S; ++s) v += part[(int64_t)s * MN * K + idx];
    pl.store(k, m, n, v);
  }
  if constexpr (has_sq<Plan>::value) {
    if (pl.sq) {  // this block's clip-norm partial (slot = blockIdx.x)
      __shared__ double red[4];
      const double t = block_sumsq((double)v * (double)v, red);
      if (threadIdx.x == 0) pl.sq[(int64_t)k * pl.sq_ld + blockIdx.x] = t;
    }
  }
}

#if FLR_CT_P3
// dw_t slabs [k][t] of the taps set in `dead` = 0 (grid: 64 x K).
__global__ void zero_taps_kernel(float* __restrict__ dw, int KK, int64_t slab, uint64_t dead) {
  const int k = blockIdx.y;
  for (int t = 0; t < KK; ++t) {
    if (!((dead >> t) & 1)) continue;
    f32x4* p = reinterpret_cast<f32x4*>(dw + ((int64_t)k * KK + t) * slab);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slab / 4; i += (int64_t)gridDim.x * blockDim.x)
      p[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}
#endif

// Split-K count from the PER-CLIENT problem only (never the client count K):
// a client's reduction order — and so its trained weights — must not depend
// on how many clients share its GPU (bit-identical results at 1/2/4/8 GPUs).
// 16 tiles per client = the 2048-workgroup target at the nominal 128 clients.
// min_kt: fewest K-tiles a split may keep (8 for the convolutions; the batched
// GEMMs read FLR_BGEMM_MINKT, default 32: 8 cost 1.7 ms per C3 round in split-K partials and reduce passes).
inline int choose_splits(int M, int N, int R, int /*K*/, int sub = 1, int min_kt = 8) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN) / sub;
  const int ktiles = cdiv(R, BK);
  int S = 1;
  while (S < 16 && tiles * S < 16 && ktiles / (2 * S) >= min_kt) S *= 2;
  return S;
}

inline int bgemm_min_kt() {
  static const int v = [] {
    const char* e = flr::knob("FLR_BGEMM_MINKT");
    const int x = e ? atoi(e) : 0;
    return x >= 1 && x <= 64 ? x : 32;
  }();
  return v;
}

// Fewest K-tiles per conv split-K part.  32 (measured per layer against 8 and 16,
// tools/conv_bench.py): a workgroup's unhidden prologue (first load, split,
// barrier) amortises over more K-tiles; the l3b / l4 forward and dgrad gain the
// most.  FLR_CONV_MINKT overrides (A/B timing).
inline int conv_min_kt() {
  static const int v = [] {
    const char* e = flr::knob("FLR_CONV_MINKT");
    const int x = e ? atoi(e) : 0;
    return x >= 1 && x <= 256 ? x : 32;
  }();
  return v;
}

// Stride-1 dgrad (one class: the forward's GEMM shape, transposed) takes the
// forward's split rule unless FLR_DGRAD_MINKT1 overrides it (A/B timing).
inline int dgrad_min_kt1() {
  static const int v = [] {
    const char* e = flr::knob("FLR_DGRAD_MINKT1");
    const int x = e ? atoi(e) : 0;
    return x >= 1 && x <= 256 ? x : 0;
  }();
  return v ? v : conv_min_kt();
}

// Strided dgrad classes (FLR_DGRAD_MINKT2 overrides 8 for A/B timing).
inline int dgrad_min_kt2() {
  static const int v = [] {
    const char* e = flr::knob("FLR_DGRAD_MINKT2");
    const int x = e ? atoi(e) : 0;
    return x >= 1 && x <= 256 ? x : 8;
  }();
  return v;
}

template <class Plan>
inline int plan_min_kt(const Plan& pl) {
  if (std::is_base_of<BGemmArgs, Plan>::value) return bgemm_min_kt();
  // a strided dgrad's parity class has few tiles per client (l3a: one 128 x 128
  // tile): it keeps the deeper split-K, or the launch runs ~128 workgroups on 256 CUs
  if constexpr (std::is_same<Plan, DgradT>::value) return pl.g.stride == 1 ? dgrad_min_kt1() : dgrad_min_kt2();
  return conv_min_kt();
}

template <class Plan>
size_t splits_bytes(const Plan& pl) {  // enough for any sub-tile count (1, 2, 3, 4)
  int S = 1;
  for (int sub : {1, 2, 3, 4}) S = std::max(S, choose_splits(pl.M(), pl.N(), pl.R(), pl.g.Kc, sub, plan_min_kt(pl)));
  return S > 1 ? (size_t)S * pl.g.Kc * pl.M() * pl.N() * sizeof(float) : 0;
}

// Workgroup tile: 64 x 64 (MS = NS = 1: 4 waves of 32 x 32, 4 workgroups/CU)
// or 128 x 128 (MS = NS = 2: each wave 64 x 64, its A and B fragments — and
// their bf16 splits — reused twice; 2 workgroups/CU).  Measured per ResNet-18
// layer on MI355X (tools/conv_bench.py): 128 x 128 wins where both dimensions
// allow it and the tile still has work — a reduction of >= 512 or more than
// 128 x 512 outputs per client; 64 x 64 everywhere else.
// FLR_CONV_TILE=11|21|12|22 forces a shape (read per launch, for A/B runs).
inline int tile_choice(int M, int N, int R) {
  const char* e = flr::knob("FLR_CONV_TILE");
  const int forced = e ? atoi(e) : 0;
  if (forced == 11) return 11;
  if (forced == 21 && M % 128 == 0) return 21;
  if (forced == 12 && N % 128 == 0) return 12;
  const bool big = M % 128 == 0 && N % 128 == 0;
  if (forced == 22 && big) return 22;
  if (forced == 0 && big && (R >= 512 || (int64_t)M * N > 128 * 512)) return 22;
  return 11;
}

template <class P> struct is_bgemm_t : std::false_type {
  static constexpr bool ta = false, tb = false;
};
template <int A, int B> struct is_bgemm_t<BGemm<A, B>> : std::true_type {
  static constexpr bool ta = A == BM_RK, tb = B == BM_RK;
};
// FLR_BGEMM_TIMG=1: k-contiguous batched-GEMM operands on transposed images
// (A/B; off by default: the eight 4-B loads per thread cost more than the
// quad-lane stash's 2-way bank conflicts save — vit.qkv 493 vs 426 us at K=32,
// profiles/r3_bgemm_timg.txt)
inline bool bgemm_timg() {
  const char* e = flr::knob("FLR_BGEMM_TIMG");
  return e && e[0] == '1';
}

template <class Plan, int MS, int NS>
int launch_tiles(const Plan& pl, void* ws, size_t ws_bytes, hipStream_t st, const char* name, int split_sub = 0) {
  const int M = pl.M(), N = pl.N(), R = pl.R(), K = pl.g.Kc;
  // split_sub: the sub-tile count the split-K choice is made for (0: this tile's);
  // a launch on smaller tiles with the default tile's split count computes the
  // same sums in the same order (fill_tile below)
  int S = choose_splits(M, N, R, K, split_sub > 0 ? split_sub : MS * NS, plan_min_kt(pl));
  if (S > 1 && (!ws || ws_bytes < (size_t)S * K * M * N * sizeof(float))) {
    // a clip-norm launch must write the slots sq_slots() promised: no silent fallback
    if constexpr (has_sq<Plan>::value) {
      if (pl.sq) return FLR_ERR_WORKSPACE;
    }
    S = 1;
  }
  const dim3 grid((unsigned)cdiv(N, BN * NS), (unsigned)cdiv(M, BM * MS), (unsigned)(K * S));
  int form = gemm_form();
  if constexpr (is_bgemm_t<Plan>::ta || is_bgemm_t<Plan>::tb) {
    // batched GEMMs with a k-contiguous operand: that operand on a transposed
    // image (coalesced 128-B row reads, conflict-free stashes; the row-major
    // image of a quad-lane load stashes 2-way bank-conflicted)
#ifdef FLR_ABLATION
    if (form == 5 && bgemm_timg()) {
      hipLaunchKernelGGL((wsgemm_kernel<Plan, MS, NS, 2, is_bgemm_t<Plan>::ta, is_bgemm_t<Plan>::tb>), grid,
                         dim3(THREADS), 0, st, pl, S, static_cast<float*>(ws), xcd_remap());
      form = -1;
    }
#endif
  }
  float* partp = static_cast<float*>(ws);  // split-K partials (after the planes in the pre-split form)
#ifdef FLR_ABLATION  // the measured-slower batched-GEMM forms: tools build only
  if constexpr (std::is_base_of<BGemmArgs, Plan>::value && MS == 2 && NS == 2) {
    if (form == 5 && bgemm_presplit()) {
      const size_t pa_b = (ps_plane_bytes(K, M, R) + 255) / 256 * 256;
      const size_t pb_b = (ps_plane_bytes(K, N, R) + 255) / 256 * 256;
      const size_t need = pa_b + pb_b + (S > 1 ? (size_t)S * K * M * N * sizeof(float) : 0);
      // the planes' byte offsets must fit the 31-bit buffer voffset
      if (ws && ws_bytes >= need && pa_b < (size_t(1) << 31) && pb_b < (size_t(1) << 31)) {
        __bf16* pa = static_cast<__bf16*>(ws);
        __bf16* pb = reinterpret_cast<__bf16*>(static_cast<char*>(ws) + pa_b);
        partp = reinterpret_cast<float*>(static_cast<char*>(ws) + pa_b + pb_b);
        const int Mp = (int)ps_pad(M, PS_ROWS), Np = (int)ps_pad(N, PS_ROWS), Rp = (int)ps_pad(R, BK);
        auto pgrid = [](int64_t n) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384))); };
        hipLaunchKernelGGL((presplit_kernel<Plan::AMODE>), pgrid((int64_t)K * Mp * Rp / 8), dim3(THREADS), 0, st, pl.a,
                           pl.a_k, pl.a_m, pl.a_r, K, M, R, Mp, Rp, pa);
        hipLaunchKernelGGL((presplit_kernel<Plan::BMODE>), pgrid((int64_t)K * Np * Rp / 8), dim3(THREADS), 0, st, pl.b,
                           pl.b_k, pl.b_n, pl.b_r, K, N, R, Np, Rp, pb);
        hipLaunchKernelGGL((psgemm_kernel<Plan>), grid, dim3(THREADS), 0, st, pl, S, partp, xcd_remap(), pa, pb, Mp,
                           Np, Rp);
        form = -1;
      }
    }
  }
  if constexpr (dma_ok<Plan>::value && MS == 2 && NS == 2) {
    if (form == 5 && bgemm_dma()) {
      hipLaunchKernelGGL((dsgemm_kernel<Plan>), grid, dim3(THREADS), 0, st, pl, S, static_cast<float*>(ws),
                         xcd_remap());
      form = -1;
    }
  }
#endif
  if constexpr (has_k8<Plan>::value) {
#ifdef FLR_ABLATION
    if constexpr (MS == 2 && NS == 2) {
      const char* ae = flr::knob("FLR_SG_ABL");  // timing ablations of the main loop (tools build only)
      const int abl = ae ? atoi(ae) : 0;
#define FLR_SG_ABL_CASE(A)                                                                                  \
  if (form == 5 && abl == A) {                                                                               \
    hipLaunchKernelGGL((sgemm_kernel<Plan, MS, NS, 2, A>), grid, dim3(THREADS), 0, st, pl, S,               \
                       static_cast<float*>(ws), xcd_remap());                                                \
    form = -1;                                                                                               \
  }
      FLR_SG_ABL_CASE(1) FLR_SG_ABL_CASE(2) FLR_SG_ABL_CASE(3) FLR_SG_ABL_CASE(4) FLR_SG_ABL_CASE(8)
      FLR_SG_ABL_CASE(10) FLR_SG_ABL_CASE(16) FLR_SG_ABL_CASE(11) FLR_SG_ABL_CASE(15) FLR_SG_ABL_CASE(23)
#undef FLR_SG_ABL_CASE
    }
#endif
    if (form == 5) {
      hipLaunchKernelGGL((sgemm_kernel<Plan, MS, NS, 2>), grid, dim3(THREADS), 0, st, pl, S, static_cast<float*>(ws),
                         xcd_remap());
      form = -1;
    }
  }
  if constexpr (std::is_same<Plan, WgtT<true>>::value || std::is_same<Plan, WgtT<false>>::value) {
    if (form == 5) {
      hipLaunchKernelGGL((wsgemm_kernel<Plan, MS, NS, 2, true, true>), grid, dim3(THREADS), 0, st, pl, S,
                         static_cast<float*>(ws), xcd_remap());
      form = -1;
    }
  }
  if (form == 5) form = 2;  // plans without k8 loads
  switch (form) {  // every form keeps each accumulator's product order: results do not depend on it
    case -1:
      break;
    case 0:
      hipLaunchKernelGGL((tgemm_kernel<Plan, MS, NS, 0>), grid, dim3(THREADS), 0, st, pl, S,
                         static_cast<float*>(ws), xcd_remap(), mfma_prio());
      break;
#ifdef FLR_ABLATION
    case 1:
      hipLaunchKernelGGL((tgemm_kernel<Plan, MS, NS, 1>), grid, dim3(THREADS), 0, st, pl, S,
                         static_cast<float*>(ws), xcd_remap(), mfma_prio());
      break;
    case 3:
      hipLaunchKernelGGL((tgemm_kernel<Plan, MS, NS, 3>), grid, dim3(THREADS), 0, st, pl, S,
                         static_cast<float*>(ws), xcd_remap(), mfma_prio());
      break;
    case 4:
      hipLaunchKernelGGL((tgemm_kernel<Plan, MS, NS, 4>), grid, dim3(THREADS), 0, st, pl, S,
                         static_cast<float*>(ws), xcd_remap(), mfma_prio());
      break;
#endif
    default:
      hipLaunchKernelGGL((tgemm_kernel<Plan, MS, NS, 2>), grid, dim3(THREADS), 0, st, pl, S,
                         static_cast<float*>(ws), xcd_remap(), mfma_prio());
  }
  int rc = launch_status(name);
  if (rc != FLR_OK || S == 1) return rc;
  const int64_t mn = (int64_t)M * N;
  hipLaunchKernelGGL(treduce_kernel<Plan>, dim3((unsigned)((mn + 255) / 256), (unsigned)K), dim3(256), 0, st, pl, S,
                     static_cast<const float*>(partp));
  return launch_status(name);
}

// Tile code 10 * MS + NS.  Besides the square shapes above, the tap-major
// convolutions take 64 x 192 / 192 x 64 (13 / 31) and 64 x 256 / 256 x 64
// (14 / 41): a 64-row operand (layer1's 64 channels) then feeds three or four
// MFMA sub-tiles per fragment read instead of one or two (LDS: five sub-tiles
// of bf16 images, still two workgroups per CU).
template <class Plan>
constexpr bool wide_tiles() {
  return std::is_same<Plan, FwdT>::value || std::is_same<Plan, DgradT>::value ||
         std::is_same<Plan, WgtT<true>>::value || std::is_same<Plan, WgtT<false>>::value;
}

template <class Plan>
inline int plan_tile(const Plan& pl) {
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const char* e = flr::knob("FLR_CONV_TILE");
  const int forced = e ? atoi(e) : 0;
  if (forced) {  // A/B timing: any shape that leaves no sub-tile empty
    const int ms = forced / 10, ns = forced % 10;
    const bool ok = ms >= 1 && ns >= 1 && ms * ns <= 4 && (wide_tiles<Plan>() || (ms <= 2 && ns <= 2)) &&
                    M > 64 * (ms - 1) && N > 64 * (ns - 1);
    if (ok) return forced;
  }
  int tile = tile_choice(M, N, R);
  // dgrad with 64 input channels (layer1): 64 x 128 tiles, the A fragment feeding
  // two B sub-tiles (measured 178 -> 147 us at l1)
  if (std::is_same<Plan, DgradT>::value && tile == 11 && M == 64 && N % 128 == 0) tile = 12;
  return tile;
}

// Clip-norm partial slots per client a WgtT launch writes (the tile count at
// split-K 1, else one per 256-value treduce block), under the launch's own
// tile and split choice — given a workspace of splits_bytes(pl).
template <class Plan>
int sq_slots(const Plan& pl) {
  const int M = pl.M(), N = pl.N(), R = pl.R();
  const int tile = plan_tile(pl);
  const int ms = tile / 10, ns = tile % 10;
  const int S = choose_splits(M, N, R, pl.g.Kc, ms * ns, plan_min_kt(pl));
  if (S == 1) return cdiv(N, BN * ns) * cdiv(M, BM * ms);
  return (int)(((int64_t)M * N + 255) / 256);
}

// Narrow-N tiles (sgemm_body NAR) for the conv forward / data gradient whose GEMM has
// at most 32 columns (the l4 layers at 32 x 32 inputs: B * 1 * 1); FLR_CONV_NARROW=0:
// the 64-wide tiles (A/B, read per launch).
inline bool conv_narrow() {
  const char* e = flr::knob("FLR_CONV_NARROW");
  return !(e && e[0] == '0');
}
template <class Plan>
int launch_narrow(const Plan& pl, void* ws, size_t ws_bytes, hipStream_t st, const char* name) {
  const int M = pl.M(), N = pl.N(), R = pl.R(), K = pl.g.Kc;
  int S = choose_splits(M, N, R, K, 2, plan_min_kt(pl));
  if (S > 1 && (!ws || ws_bytes < (size_t)S * K * M * N * sizeof(float))) S = 1;
  const dim3 grid((unsigned)cdiv(N, BN), (unsigned)cdiv(M, 2 * BM), (unsigned)(K * S));
  hipLaunchKernelGGL((sgemm_kernel<Plan, 2, 1, 2, 0, true>), grid, dim3(THREADS), 0, st, pl, S,
                     static_cast<float*>(ws), xcd_remap());
  int rc = launch_status(name);
  if (rc != FLR_OK || S == 1) return rc;
  const int64_t mn = (int64_t)M * N;
  hipLaunchKernelGGL(treduce_kernel<Plan>, dim3((unsigned)((mn + 255) / 256), (unsigned)K), dim3(256), 0, st, pl, S,
                     static_cast<const float*>(ws));
  return launch_status(name);
}

// Small client counts (K/G clients per GPU at G = 8: 16 at C3) leave the
// default tiles' grids below one wave of the chip: layer2 / layer3 of ResNet-18
// launch 4 workgroups of 128 x 128 per client.  Forward and data-gradient
// launches whose grid would hold fewer than FILL_WG workgroups then run on
// 64 x 64 tiles with the DEFAULT tile's split-K count: every output element is
// the same K-tile / k-step / product sequence, so the result is bit-identical
// to the default tiles (and the model to the one at G = 1).  The weight
// gradients keep their tiles: their clip-norm partial slots follow the tile.
// FLR_CONV_FILL=0: off (A/B, read per launch).
constexpr int FILL_WG = 512;  // two 128 x 128 workgroups per CU on 256 CUs
inline bool conv_fill() {
  const char* e = flr::knob("FLR_CONV_FILL");
  return !(e && e[0] == '0');
}
template <class Plan>
bool fill_tile(const Plan& pl, int tile) {
  if constexpr (!(std::is_same<Plan, FwdT>::value || std::is_same<Plan, DgradT>::value)) {
    return false;
  } else {
    const int ms = tile / 10, ns = tile % 10;
    if (ms * ns == 1 || !conv_fill()) return false;
    const int M = pl.M(), N = pl.N(), R = pl.R();
    const int S = choose_splits(M, N, R, pl.g.Kc, ms * ns, plan_min_kt(pl));
    const int64_t wg = (int64_t)pl.g.Kc * cdiv(M, BM * ms) * cdiv(N, BN * ns) * S;
    return wg < FILL_WG;
  }
}

template <class Plan>
int launch(const Plan& pl, void* ws, size_t ws_bytes, hipStream_t st, const char* name) {
  if (pl.R() == 0 && !std::is_same<Plan, DgradT>::value) return FLR_OK;  // a dgrad class with no tap stores zeros
  if constexpr (std::is_same<Plan, FwdT>::value || std::is_same<Plan, DgradT>::value) {
    if (pl.N() <= 32 && pl.M() % (2 * BM) == 0 && pl.R() > 0 && gemm_form() == 5 && conv_narrow()) {
      // a narrow launch under one wave of the chip (few clients per GPU): the 64 x 64
      // tiles with the narrow tiles' split count — twice the workgroups, the same bits
      const int S = choose_splits(pl.M(), pl.N(), pl.R(), pl.g.Kc, 2, plan_min_kt(pl));
      if (conv_fill() && (int64_t)pl.g.Kc * cdiv(pl.M(), 2 * BM) * S < FILL_WG / 2)
        return launch_tiles<Plan, 1, 1>(pl, ws, ws_bytes, st, name, 2);
      return launch_narrow(pl, ws, ws_bytes, st, name);
    }
  }
  const int tile = plan_tile(pl);
  if (fill_tile(pl, tile)) return launch_tiles<Plan, 1, 1>(pl, ws, ws_bytes, st, name, (tile / 10) * (tile % 10));
  if constexpr (wide_tiles<Plan>()) {
    switch (tile) {
      case 13: return launch_tiles<Plan, 1, 3>(pl, ws, ws_bytes, st, name);
      case 31: return launch_tiles<Plan, 3, 1>(pl, ws, ws_bytes, st, name);
      case 14: return launch_tiles<Plan, 1, 4>(pl, ws, ws_bytes, st, name);
      case 41: return launch_tiles<Plan, 4, 1>(pl, ws, ws_bytes, st, name);
      default: break;
    }
  }
  switch (tile) {
    case 21: return launch_tiles<Plan, 2, 1>(pl, ws, ws_bytes, st, name);
    case 12: return launch_tiles<Plan, 1, 2>(pl, ws, ws_bytes, st, name);
    case 22: return launch_tiles<Plan, 2, 2>(pl, ws, ws_bytes, st, name);
    default: return launch_tiles<Plan, 1, 1>(pl, ws, ws_bytes, st, name);
  }
}

inline bool shape_ok(int64_t Cin, int64_t Cout) { return Cin % 64 == 0 && Cout % 64 == 0; }

// ---- im2col path (declared in conv_common.h) ----------------------------------
inline int padded_r(const Geom& g) { return (g.Cin * g.KH * g.KW + 3) / 4 * 4; }

#if FLR_CT_P0
bool im2col_eligible(const Geom& g) {
  const int64_t N = (int64_t)g.B * g.Ho * g.Wo;
  return padded_r(g) <= IM_MAXRP && !shape_ok(g.Cin, g.Cout) && (g.Ho * g.Wo) % 4 == 0 &&
         N * padded_r(g) * 4 < (int64_t(1) << 31) && (int64_t)g.Cout * padded_r(g) * 4 < (int64_t(1) << 31);
}
#endif

#if FLR_CT_P0
size_t im2col_workspace(const Geom& g) {
  const size_t col = align_up((size_t)g.Kc * g.B * g.Ho * g.Wo * padded_r(g) * sizeof(float), 256);
  const size_t wp = align_up((size_t)g.Kc * g.Cout * padded_r(g) * sizeof(float), 256);
  DenseFwd f; f.g = g; f.RP = padded_r(g);
  DenseWgt w; w.g = g; w.RP = padded_r(g);
  StemFwd sf; sf.g = g; sf.RP = padded_r(g);
  StemWgt sw; sw.g = g; sw.RP = padded_r(g);
  const size_t gemm = col + wp + std::max(std::max(splits_bytes(f), splits_bytes(w)), std::max(splits_bytes(sf), splits_bytes(sw)));
  return std::max(gemm, stem_eligible(g) ? stem_workspace(g) : 0);
}
#endif

#if FLR_CT_P0
static int run_im2col(const Geom& g, const float* x, float* col, hipStream_t st) {
  const int N = g.B * g.Ho * g.Wo, RP = padded_r(g);
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)cdiv(N, IM_PB), (unsigned)g.Kc), dim3(THREADS),
                     (size_t)IM_PB * RP * sizeof(float), st, g, x, RP, col);
  return launch_status("conv im2col");
}
#endif

#if FLR_CT_P0
// FLR_STEM=col: the explicit im2col column matrix; =gather: the tiled GEMM with the
// im2col operand gathered on the fly (A/B timing); default: the direct stem
// kernels (train_stem.hip) where eligible, else the gathered GEMM.
inline bool stem_col() {
  const char* e = flr::knob("FLR_STEM");
  return e && e[0] == 'c';
}
#endif
#if FLR_CT_P0
inline bool stem_direct(const Geom& g) {
  const char* e = flr::knob("FLR_STEM");
  return !(e && (e[0] == 'c' || e[0] == 'g')) && stem_eligible(g);
}
#endif

#if FLR_CT_P0
template <class Plan>
inline void stem_divs(Plan& pl, const Geom& g) {
  pl.RR = g.Cin * g.KH * g.KW;
  pl.d_kk = conv::make_fastdiv((uint32_t)(g.KH * g.KW));
  pl.d_kw = conv::make_fastdiv((uint32_t)g.KW);
}
#endif

#if FLR_CT_P0
int fwd_im2col(const Geom& g, const float* x, const float* w, float* y, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!ws || ws_bytes < im2col_workspace(g)) return FLR_ERR_WORKSPACE;
  if (stem_direct(g)) return stem_fwd(g, x, w, y, st);
  const int RP = padded_r(g), R = g.Cin * g.KH * g.KW;
  char* base = static_cast<char*>(ws);
  float* col = reinterpret_cast<float*>(base);
  const size_t colb = align_up((size_t)g.Kc * g.B * g.Ho * g.Wo * RP * sizeof(float), 256);
  float* wp = reinterpret_cast<float*>(base + colb);
  const size_t wpb = align_up((size_t)g.Kc * g.Cout * RP * sizeof(float), 256);
  const int64_t wtot = (int64_t)g.Cout * RP;
  hipLaunchKernelGGL(repad_kernel, dim3((unsigned)std::min<int64_t>((wtot + THREADS - 1) / THREADS, 256), (unsigned)g.Kc),
                     dim3(THREADS), 0, st, w, R, wp, RP, g.Cout, R);
  int rc = launch_status("conv pad weights");
  if (rc != FLR_OK) return rc;
  if (!stem_col()) {
    StemFwd pl;
    pl.g = g; pl.RP = RP; pl.x = x; pl.wp = wp; pl.y = y;
    stem_divs(pl, g);
    return launch(pl, base + colb + wpb, ws_bytes - colb - wpb, st, "conv fwd (gathered im2col)");
  }
  if ((rc = run_im2col(g, x, col, st)) != FLR_OK) return rc;
  DenseFwd pl;
  pl.g = g; pl.RP = RP; pl.col = col; pl.wp = wp; pl.y = y;
  return launch(pl, base + colb + wpb, ws_bytes - colb - wpb, st, "conv fwd (im2col)");
}
#endif

#if FLR_CT_P0
int wgrad_im2col(const Geom& g, const float* x, const float* dy, float* dw, void* ws, size_t ws_bytes,
                 hipStream_t st, bool have_col) {
  if (!ws || ws_bytes < im2col_workspace(g)) return FLR_ERR_WORKSPACE;
  if (stem_direct(g)) return stem_wgrad(g, x, dy, dw, ws, ws_bytes, st);
  const int RP = padded_r(g), R = g.Cin * g.KH * g.KW;
  char* base = static_cast<char*>(ws);
  float* col = reinterpret_cast<float*>(base);
  const size_t colb = align_up((size_t)g.Kc * g.B * g.Ho * g.Wo * RP * sizeof(float), 256);
  float* dwp = reinterpret_cast<float*>(base + colb);
  const size_t wpb = align_up((size_t)g.Kc * g.Cout * RP * sizeof(float), 256);
  int rc = FLR_OK;
  if (!stem_col()) {
    StemWgt pl;
    pl.g = g; pl.RP = RP; pl.x = x; pl.dy = dy; pl.dwp = dwp;
    stem_divs(pl, g);
    rc = launch(pl, base + colb + wpb, ws_bytes - colb - wpb, st, "conv bwd weight (gathered im2col)");
  } else {
    if (!have_col) rc = run_im2col(g, x, col, st);  // have_col: the forward's column matrix
    if (rc != FLR_OK) return rc;
    DenseWgt pl;
    pl.g = g; pl.RP = RP; pl.col = col; pl.dy = dy; pl.dwp = dwp;
    rc = launch(pl, base + colb + wpb, ws_bytes - colb - wpb, st, "conv bwd weight (im2col)");
  }
  if (rc != FLR_OK) return rc;
  const int64_t wtot = (int64_t)g.Cout * R;
  hipLaunchKernelGGL(repad_kernel, dim3((unsigned)std::min<int64_t>((wtot + THREADS - 1) / THREADS, 256), (unsigned)g.Kc),
                     dim3(THREADS), 0, st, dwp, RP, dw, R, g.Cout, R);
  return launch_status("conv unpad dw");
}
#endif

inline bool args_ok(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                    int64_t stride, int64_t pad) {
  if (!conv::geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad) || !shape_ok(Cin, Cout)) return false;
  // byte offsets inside one client's buffer view must fit the 31-bit voffset
  if (!(B * K * Cin * H * W * 4 < (int64_t(1) << 31) && B * K * Cout * H * W * 4 < (int64_t(1) << 31) &&
        KH * KW * Cin * Cout * 4 < (int64_t(1) << 31)))
    return false;
  // the kernels decode taps by rectangle arithmetic (true for any stride <= 4
  // conv whose live rows / columns are contiguous: every ResNet shape)
  if (stride > 4) return false;
  const conv::Geom g = conv::make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  if (!g.rect.ok) return false;
  DgradT cls[MAX_CLASSES];
  const int nc = dgrad_classes(g, cls);
  for (int c = 0; c < nc; ++c)
    if (!cls[c].crect.ok) return false;
  return true;
}

}  // namespace convt
}  // namespace flr

using namespace flr;

#if FLR_CT_P0
extern "C" int flr_conv2d_tap_major_ok(int64_t Cin, int64_t Cout) { return convt::shape_ok(Cin, Cout) ? 1 : 0; }
#endif

#if FLR_CT_P0
extern "C" size_t flr_conv2d_t_workspace(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                                         int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  if (!convt::args_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad)) return 0;
  const conv::Geom g = conv::make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  convt::FwdT f; f.g = g;
  convt::WgtT<false> w; w.g = g;
  size_t m = std::max(convt::splits_bytes(f), convt::splits_bytes(w));
  if (stride <= 4) {
    convt::DgradT cls[convt::MAX_CLASSES];
    const int nc = convt::dgrad_classes(g, cls);
    for (int c = 0; c < nc; ++c) m = std::max(m, convt::splits_bytes(cls[c]));
  }
  return m;
}
#endif

#if FLR_CT_P1
extern "C" int flr_conv2d_fwd_t(const float* x, const float* w_t, float* y, int64_t K, int64_t B, int64_t Cin,
                                int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                int64_t pad, void* ws, size_t ws_bytes, void* stream) {
  return flr_conv2d_fwd_t_ex(x, w_t, KH * KW * Cin * Cout, y, K, B, Cin, H, W, Cout, KH, KW, stride, pad, ws,
                             ws_bytes, stream);
}
#endif

#if FLR_CT_P1
extern "C" int flr_conv2d_fwd_t_ex(const float* x, const float* w_t, int64_t w_stride, float* y, int64_t K, int64_t B,
                                   int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                                   int64_t stride, int64_t pad, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !w_t || !y || w_stride < 0) return FLR_ERR_ARG;
  if (!convt::args_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad))
    return conv::geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad) ? FLR_ERR_UNSUPPORTED : FLR_ERR_ARG;
  convt::FwdT pl;
  pl.g = conv::make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  pl.x = x; pl.w = w_t; pl.y = y; pl.wsk = w_stride;
  return convt::launch(pl, ws, ws_bytes, as_stream(stream), "conv fwd (tap-major)");
}
#endif

#if FLR_CT_P2
extern "C" int flr_conv2d_bwd_data_t(const float* dy, const float* w_t, float* dx, int64_t K, int64_t B, int64_t Cin,
                                     int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                     int64_t pad, void* ws, size_t ws_bytes, void* stream) {
  return flr_conv2d_bwd_data_t_add(dy, w_t, nullptr, dx, K, B, Cin, H, W, Cout, KH, KW, stride, pad, ws, ws_bytes,
                                   stream);
}
#endif

#if FLR_CT_P2
extern "C" int flr_conv2d_bwd_data_t_add(const float* dy, const float* w_t, const float* add, float* dx, int64_t K,
                                         int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH,
                                         int64_t KW, int64_t stride, int64_t pad, void* ws, size_t ws_bytes,
                                         void* stream) {
  return flr_conv2d_bwd_data_t_ex(dy, w_t, KH * KW * Cin * Cout, add, dx, K, B, Cin, H, W, Cout, KH, KW, stride, pad,
                                  ws, ws_bytes, stream);
}
#endif

#if FLR_CT_P2
extern "C" int flr_conv2d_bwd_data_t_ex(const float* dy, const float* w_t, int64_t w_stride, const float* add,
                                        float* dx, int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W,
                                        int64_t Cout, int64_t KH, int64_t KW, int64_t stride, int64_t pad, void* ws,
                                        size_t ws_bytes, void* stream) {
  if (!dy || !w_t || !dx || w_stride < 0) return FLR_ERR_ARG;
  if (!convt::args_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad))
    return conv::geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad) ? FLR_ERR_UNSUPPORTED : FLR_ERR_ARG;
  if (stride > 4) return FLR_ERR_UNSUPPORTED;  // <= MAX_CLASSES parity classes
  const conv::Geom g = conv::make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  convt::DgradT cls[convt::MAX_CLASSES];
  const int nc = convt::dgrad_classes(g, cls);
  for (int c = 0; c < nc; ++c) {
    // in-place accumulation (add == dx): a class no tap reaches adds nothing
    if (add == dx && cls[c].R() == 0) continue;
    cls[c].dy = dy; cls[c].w = w_t; cls[c].dx = dx; cls[c].add = add; cls[c].wsk = w_stride;
    const int rc = convt::launch(cls[c], ws, ws_bytes, as_stream(stream), "conv bwd data (tap-major)");
    if (rc != FLR_OK) return rc;
  }
  return FLR_OK;
}
#endif

#if FLR_CT_P3
extern "C" int flr_conv2d_bwd_weight_t(const float* x, const float* dy, float* dw_t, int64_t K, int64_t B,
                                       int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                                       int64_t stride, int64_t pad, int zero_dead_taps, void* ws, size_t ws_bytes,
                                       void* stream) {
  return flr_conv2d_bwd_weight_t_sq(x, dy, dw_t, K, B, Cin, H, W, Cout, KH, KW, stride, pad, zero_dead_taps, nullptr,
                                    0, ws, ws_bytes, stream);
}
#endif

#if FLR_CT_P3
extern "C" int64_t flr_conv2d_bwd_weight_t_sq_slots(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W,
                                                    int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                                    int64_t pad) {
  if (!convt::args_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad)) return -1;
  convt::WgtT<true> pl;  // the slot count does not depend on the B-operand load form
  pl.g = conv::make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  return pl.R() == 0 ? 0 : convt::sq_slots(pl);
}
#endif

#if FLR_CT_P3
extern "C" int flr_conv2d_bwd_weight_t_sq(const float* x, const float* dy, float* dw_t, int64_t K, int64_t B,
                                          int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                                          int64_t stride, int64_t pad, int zero_dead_taps, double* sq,
                                          int64_t sq_ld, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !dy || !dw_t) return FLR_ERR_ARG;
  if (!convt::args_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad))
    return conv::geom_ok(K, B, Cin, H, W, Cout, KH, KW, stride, pad) ? FLR_ERR_UNSUPPORTED : FLR_ERR_ARG;
  const conv::Geom g = conv::make_geom(K, B, Cin, H, W, Cout, KH, KW, stride, pad);
  hipStream_t st = as_stream(stream);
  if (zero_dead_taps && g.ntaps < KH * KW) {  // dead taps: exact-zero gradients, one slab each
    uint64_t dead = (KH * KW >= 64) ? ~0ull : ((1ull << (KH * KW)) - 1);
    for (int t = 0; t < g.ntaps; ++t) dead &= ~(1ull << (g.tap_kh[t] * KW + g.tap_kw[t]));
    hipLaunchKernelGGL(convt::zero_taps_kernel, dim3(64, (unsigned)K), dim3(256), 0, st, dw_t, (int)(KH * KW),
                       (int64_t)Cin * Cout, dead);
    const int rc = launch_status("conv bwd weight: zero dead taps");
    if (rc != FLR_OK) return rc;
  }
  if (sq) {  // the partial slots follow the launch's split choice, which needs the full workspace
    convt::WgtT<true> probe;
    probe.g = g;
    if (sq_ld < convt::sq_slots(probe) || ws_bytes < convt::splits_bytes(probe) ||
        (convt::splits_bytes(probe) > 0 && !ws))
      return FLR_ERR_WORKSPACE;
  }
  if ((g.Ho * g.Wo) % 4 == 0) {
    convt::WgtT<true> pl;
    pl.g = g; pl.x = x; pl.dy = dy; pl.dw = dw_t; pl.sq = sq; pl.sq_ld = (int)sq_ld;
    return convt::launch(pl, ws, ws_bytes, st, "conv bwd weight (tap-major)");
  }
  convt::WgtT<false> pl;
  pl.g = g; pl.x = x; pl.dy = dy; pl.dw = dw_t; pl.sq = sq; pl.sq_ld = (int)sq_ld;
  return convt::launch(pl, ws, ws_bytes, st, "conv bwd weight (tap-major)");
}
#endif

#if FLR_CT_P4
namespace {
// operand mode from strides: RK (r contiguous) / KR (rows contiguous) / G
int bgemm_mode(const float* p, int64_t s_k, int64_t s_row, int64_t s_r, int64_t rows, int64_t R) {
  const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0 && s_k % 4 == 0;
  if (s_r == 1 && al && s_row % 4 == 0 && R % 4 == 0) return convt::BM_RK;
  if (s_row == 1 && al && s_r % 4 == 0 && rows % 4 == 0) return convt::BM_KR;
  return convt::BM_G;
}
// Workgroup tile of the batched GEMM: 128 x 128 (each wave 64 x 64, its
// fragments and bf16 splits reused twice) for the encoder-sized products
// (M, N >= 128 and a long reduction or many outputs), 64 x 64 for the small
// ones (the GRU recurrence and the head, M = batch = 32).  Partial edge tiles
// are bounds-checked in the loads and stores.  FLR_BGEMM_TILE=11|22 forces it.
inline int bgemm_tile(int M, int N, int R) {
  const char* e = flr::knob("FLR_BGEMM_TILE");
  const int forced = e ? atoi(e) : 0;
  if (forced == 11 || forced == 22) return forced;
  return (M >= 128 && N >= 128 && (R >= 256 || (int64_t)M * N >= 128 * 512)) ? 22 : 11;
}
template <int AM, int BMD>
int bgemm_run(const convt::BGemmArgs& args, void* ws, size_t ws_bytes, hipStream_t st) {
  convt::BGemm<AM, BMD> pl;
  static_cast<convt::BGemmArgs&>(pl) = args;
  if (bgemm_tile(args.m, args.n, args.r) == 22)
    return convt::launch_tiles<convt::BGemm<AM, BMD>, 2, 2>(pl, ws, ws_bytes, st, "batched gemm");
  return convt::launch_tiles<convt::BGemm<AM, BMD>, 1, 1>(pl, ws, ws_bytes, st, "batched gemm");
}
template <int AM>
int bgemm_b(int bm, const convt::BGemmArgs& args, void* ws, size_t wsb, hipStream_t st) {
  switch (bm) {
    case convt::BM_RK: return bgemm_run<AM, convt::BM_RK>(args, ws, wsb, st);
    case convt::BM_KR: return bgemm_run<AM, convt::BM_KR>(args, ws, wsb, st);
    default: return bgemm_run<AM, convt::BM_G>(args, ws, wsb, st);
  }
}
}  // namespace

extern "C" size_t flr_bgemm_workspace(int64_t batch, int64_t M, int64_t N, int64_t R) {
  if (batch < 1 || M < 1 || N < 1 || R < 0 || M > INT32_MAX || N > INT32_MAX || R > INT32_MAX) return 0;
  // the larger of the two tile shapes' split counts (sub-tile count 1 or 4)
  const int S = std::max(convt::choose_splits((int)M, (int)N, (int)R, (int)batch, 1, convt::bgemm_min_kt()),
                         convt::choose_splits((int)M, (int)N, (int)R, (int)batch, 4, convt::bgemm_min_kt()));
  size_t n = S > 1 ? (size_t)S * batch * M * N * sizeof(float) : 0;
#ifdef FLR_ABLATION
  // the pre-split form's bf16 planes of both operands (128 x 128 tiles), before the partials
  if (convt::bgemm_presplit() && bgemm_tile((int)M, (int)N, (int)R) == 22)
    n += (convt::ps_plane_bytes(batch, M, R) + 255) / 256 * 256 + (convt::ps_plane_bytes(batch, N, R) + 255) / 256 * 256;
#endif
  return n;
}

extern "C" int flr_bgemm(const float* A, int64_t a_k, int64_t a_m, int64_t a_r, const float* B, int64_t b_k,
                         int64_t b_n, int64_t b_r, float* C, int64_t c_k, int64_t c_m, int64_t c_n, const float* bias,
                         int64_t bias_k, const float* add, int64_t batch, int64_t M, int64_t N, int64_t R, void* ws,
                         size_t ws_bytes, void* stream) {
  return flr_bgemm_ex(A, a_k, a_m, a_r, B, b_k, b_n, b_r, C, c_k, c_m, c_n, bias, bias_k, add, FLR_ACT_NONE, nullptr,
                      nullptr, nullptr, batch, M, N, R, ws, ws_bytes, stream);
}

extern "C" int flr_bgemm_ex(const float* A, int64_t a_k, int64_t a_m, int64_t a_r, const float* B, int64_t b_k,
                            int64_t b_n, int64_t b_r, float* C, int64_t c_k, int64_t c_m, int64_t c_n,
                            const float* bias, int64_t bias_k, const float* add, int act, const float* mul,
                            const float* aux, float* pre, int64_t batch, int64_t M, int64_t N, int64_t R, void* ws,
                            size_t ws_bytes, void* stream) {
  if (!A || !B || !C || batch < 1 || batch > 65535 || M < 1 || N < 1 || R < 1) return FLR_ERR_ARG;
  if (act < FLR_ACT_NONE || act > FLR_ACT_DTANH) return FLR_ERR_ARG;
  if (act >= FLR_ACT_DRELU && !aux) return FLR_ERR_ARG;
  if (a_k < 0 || a_m < 0 || a_r < 0 || b_k < 0 || b_n < 0 || b_r < 0 || c_k < 0 || c_m < 0 || c_n < 0)
    return FLR_ERR_ARG;
  const int64_t a_ext = (M - 1) * a_m + (R - 1) * a_r + 1;
  const int64_t b_ext = (N - 1) * b_n + (R - 1) * b_r + 1;
  if (a_ext * 4 >= (int64_t(1) << 31) || b_ext * 4 >= (int64_t(1) << 31) || M * N >= (int64_t(1) << 31) ||
      R >= (int64_t(1) << 30))
    return FLR_ERR_UNSUPPORTED;
  convt::BGemmArgs p;
  p.g.Kc = (int)batch;
  p.m = (int)M; p.n = (int)N; p.r = (int)R;
  p.a = A; p.a_k = a_k; p.a_m = a_m; p.a_r = a_r; p.a_ext = a_ext;
  p.b = B; p.b_k = b_k; p.b_n = b_n; p.b_r = b_r; p.b_ext = b_ext;
  p.c = C; p.c_k = c_k; p.c_m = c_m; p.c_n = c_n;
  p.bias = bias; p.bias_k = bias_k; p.add = add;
  p.act = act; p.mul = mul; p.aux = aux; p.pre = pre;
  hipStream_t st = as_stream(stream);
  const int am = bgemm_mode(A, a_k, a_m, a_r, M, R), bm = bgemm_mode(B, b_k, b_n, b_r, N, R);
  switch (am) {
    case convt::BM_RK: return bgemm_b<convt::BM_RK>(bm, p, ws, ws_bytes, st);
    case convt::BM_KR: return bgemm_b<convt::BM_KR>(bm, p, ws, ws_bytes, st);
    default: return bgemm_b<convt::BM_G>(bm, p, ws, ws_bytes, st);
  }
}

namespace flr {
namespace convt {
// Long reductions (the encoders' bias gradients sum M = 2080 rows) are cut
// into fixed 256-row chunks: stage 1 sums each chunk with the 8-accumulator
// kernel into a partial row, stage 2 adds the partials in chunk order.  The
// chunking depends on M alone, so a client's sum never depends on the launch.
constexpr int SR_CHUNK = 256;
constexpr int SR_MAXCHUNK = 64;

__global__ void sum_rows_chunks_kernel(const float* __restrict__ x, int64_t x_k, int64_t x_m, int M, int N,
                                       float* __restrict__ part, int nch) {
  const int k = blockIdx.z, c = blockIdx.y;
  const int nn = blockIdx.x * blockDim.x + threadIdx.x;
  if (nn >= N) return;
  const int m0 = c * SR_CHUNK, m1 = min(M, m0 + SR_CHUNK);
  const float* p = x + k * x_k + (int64_t)m0 * x_m + nn;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int mm = 0;
  const int R = m1 - m0;
  for (; mm + 8 <= R; mm += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += p[(int64_t)(mm + j) * x_m];
  }
  for (int j = 0; mm < R; ++mm, ++j) a[j] += p[(int64_t)mm * x_m];
  part[((int64_t)k * nch + c) * N + nn] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

__global__ void sum_rows_finish_kernel(const float* __restrict__ part, int nch, int N, float* __restrict__ out,
                                       int64_t out_k) {
  const int k = blockIdx.y;
  const int nn = blockIdx.x * blockDim.x + threadIdx.x;
  if (nn >= N) return;
  const float* p = part + (int64_t)k * nch * N + nn;
  float s = p[0];
  for (int c = 1; c < nch; ++c) s += p[(int64_t)c * N];
  out[k * out_k + nn] = s;
}
}  // namespace convt
}  // namespace flr

extern "C" size_t flr_sum_rows_workspace(int64_t batch, int64_t M, int64_t N) {
  if (batch < 1 || M <= convt::SR_CHUNK || N < 1) return 0;
  const int64_t nch = std::min<int64_t>((M + convt::SR_CHUNK - 1) / convt::SR_CHUNK, convt::SR_MAXCHUNK);
  return align_up((size_t)batch * nch * N * sizeof(float), 256);
}

extern "C" int flr_sum_rows(const float* X, int64_t x_k, int64_t x_m, int64_t batch, int64_t M, int64_t N, float* out,
                            int64_t out_k, void* stream) {
  return flr_sum_rows_ex(X, x_k, x_m, batch, M, N, out, out_k, nullptr, 0, stream);
}

extern "C" int flr_sum_rows_ex(const float* X, int64_t x_k, int64_t x_m, int64_t batch, int64_t M, int64_t N,
                               float* out, int64_t out_k, void* workspace, size_t workspace_bytes, void* stream) {
  if (!X || !out || batch < 1 || batch > 65535 || M < 0 || N < 1) return FLR_ERR_ARG;
  const size_t need = flr_sum_rows_workspace(batch, M, N);
  if (need == 0 || !workspace || workspace_bytes < need ||
      (M + convt::SR_CHUNK - 1) / convt::SR_CHUNK > convt::SR_MAXCHUNK) {
    hipLaunchKernelGGL(convt::sum_rows_kernel, dim3((unsigned)((N + 255) / 256), (unsigned)batch), dim3(256), 0,
                       as_stream(stream), X, x_k, x_m, (int)M, (int)N, out, out_k);
    return launch_status("sum_rows");
  }
  const int nch = (int)((M + convt::SR_CHUNK - 1) / convt::SR_CHUNK);
  float* part = static_cast<float*>(workspace);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(convt::sum_rows_chunks_kernel, dim3((unsigned)((N + 255) / 256), (unsigned)nch, (unsigned)batch),
                     dim3(256), 0, st, X, x_k, x_m, (int)M, (int)N, part, nch);
  int rc = launch_status("sum_rows_chunks");
  if (rc != FLR_OK) return rc;
  hipLaunchKernelGGL(convt::sum_rows_finish_kernel, dim3((unsigned)((N + 255) / 256), (unsigned)batch), dim3(256), 0,
                     st, part, nch, (int)N, out, out_k);
  return launch_status("sum_rows_finish");
}

#endif