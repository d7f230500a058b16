// a9, reference-exact mode — Krum distances bit-identical to the reference's
// fp32 `torch.norm(flat_i - flat_j).item()` (src/defenses/krum.py:89-97).
//
// The reference's norm on an fp32 CPU tensor accumulates (SURVEY.md App. C,
// probed on this image's torch; oracle/norm_ref.c restates it and
// tests/test_oracle.py pins it against torch.norm):
//   d = fl(x_i - x_j) elementwise;
//   8 fp32 lanes ("chains"), chain c = fma(d[8r+c], d[8r+c], chain c)
//   sequentially over the steps r = 0 .. R-1, R = P / 8;
//   s = chain 0 + chain 1 + ... + chain 7 (in that order);
//   the tail t >= 8R: while 4 or more remain, the next 4 as
//   s = s + fl(d[t] * d[t]) (separate multiply and add), then the last
//   0..3 as s = fma(d[t], d[t], s);
//   sqrt_f32(s) (correctly rounded), widened to fp64 by .item().
// Every fp32 operation here is that operation, in that order, so D is the
// reference's D bit for bit — no tolerance, no margin argument.
//
// Design.  The parallelism is fixed by the reference: K(K-1)/2 pairs x 8
// chains, each chain a sequential fma over R steps (65,024 chains of 1.475 M
// steps at C3): about one chain per lane of one wave per SIMD, so every step of
// a wave must be cheap and no wave may wait for another.
//  * Chain-major operands: a segment of X is first rewritten chain-major
//    (chain_transpose_kernel, Xc[k][c][s] = X[k][8(r0+s)+c], one read and one
//    write of the segment at HBM rate) so each chain's steps are contiguous.
//  * One wave per workgroup, one chain per lane: a wave holds 4 I rows (its
//    16-lane DPP rows) x 16 J rows (the lanes of a row) — 64 pairs — and
//    stages only the J rows it reads, so no wave waits at a barrier for
//    another (a shared 64-row J block behind a workgroup barrier cost 2.1 of
//    10.3 ms at C3: tools/gpu_r5_l.sh, profiles/r5_ref/).
//  * x_j per lane from LDS: per chunk of CS = 64 steps the wave stages its 16
//    (diagonal tiles: 20) J rows' 256-B chain pieces by LDS-DMA (one
//    global_load_lds_dwordx4 per 4 rows, XOR-swizzled 16-B slots so the
//    ds_read_b128 lane groups hit distinct banks) into a ring of NSTAGE stages
//    (DMA NSTAGE - 1 chunks ahead); each lane reads its row's 16 pieces with
//    ds_read_b128 one chunk ahead (two register buffers).
//  * x_i by DPP: lane L of each 16-lane row holds 4 steps of the chunk (one
//    16-B load per lane per chunk); step S reaches every lane of the row by a
//    row_newbcast of lane S / 4 folded into the subtraction (v_sub_f32_dpp).
//  * chain c = the XCD (blockIdx % 8): an XCD's L2 holds only its own chain's
//    streams.  40 KB of LDS per workgroup: four per CU, one wave per SIMD.
// Chains longer than the segment carry their partial sums in A between segments.
#include <cstdint>
#include <type_traits>
#include <utility>
#include <vector>

#include "flr_common.h"

namespace flr {
namespace pwref {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int IW = 4;              // I rows per wave: its 16-lane DPP rows
constexpr int JW = 16;             // J rows per wave: the lanes of a DPP row
constexpr int SB = 32;             // rows per super-block (tiles below)
constexpr int OFF_W = (SB / IW) * (SB / JW);  // waves of an off-diagonal super-block pair (16)
constexpr int DIAG_W = SB / IW;               // waves of a diagonal super-block (8)
constexpr int CS = 64;             // chain steps per staged chunk (256 B of one chain stream)
constexpr int NQ = CS / 4;         // 16-B pieces per chunk row
constexpr int RPD = 256 / CS;      // chunk rows per 1-KB DMA instruction (4)
constexpr int SROWS = 20;          // staged rows per stage (diagonal tiles read 19)
#ifndef FLR_REF_NSTAGE
#define FLR_REF_NSTAGE 8
#endif
constexpr int NSTAGE = FLR_REF_NSTAGE;    // LDS ring = the loop's unroll (DMA NSTAGE - 1 chunks ahead)
constexpr int STAGE = SROWS * CS;         // floats per stage (5 KB)
constexpr int64_t XC_CAP = int64_t(8) << 30;  // bytes of one chain-major segment
constexpr int64_t XC_SLACK = 4096;            // bytes past the last stream the chunk prefetch may read
// A segment's streams are zero-filled from its last step up to a multiple of
// XC_GROUP steps (one loop trip of the chain kernel): fma(0, 0, s) = s for the
// non-negative sums, so the loop runs whole groups without a per-chunk check
// and the last, partial chunk needs no separate path.
constexpr int64_t XC_GROUP = (int64_t)NSTAGE * CS;
static_assert(CS == 64 && NQ == 16, "x_i layout: 16 lanes x 4 steps per chunk");
static_assert(NSTAGE % 2 == 0 && NSTAGE >= 4, "two register buffers");
static_assert((NSTAGE - 1) * CS * 4 <= XC_SLACK, "the prefetch past a stream stays inside the slack");
static_assert((NSTAGE - 1) * STAGE * 4 < 65536, "ds_read_b128's 16-bit offset reaches every stage");
static_assert(NSTAGE * STAGE * 4 > 163840 / 5, "LDS caps the CU at four workgroups: one wave per SIMD");
template <bool DIAG>
struct Staging {
  static constexpr int DPW = (DIAG ? SROWS : JW) / RPD;  // DMA instructions per chunk (5 | 4)
  static constexpr int OPB = DPW + 1;                   // vector-memory ops per body: the DMAs, then x_i
  static_assert((NSTAGE - 2) * OPB + 1 < 64, "vmcnt counts to 63");
};

// the XOR swizzle of a staged row's 16-B slots: the rows one ds_read_b128 lane
// group ({0-3,12-15,20-27}, {4-11,16-19,28-31} and +32) reads are distinct
// modulo 16, or the same row (a broadcast), on both tile kinds
__host__ __device__ constexpr int slot_swz(int row) { return row & 15; }

// Tiles (per chain): one wave each.  The K rows form super-blocks of 32;
// super-block pair (X, Y), X <= Y:
//  * X < Y: 32 x 32 pairs in OFF_W waves (g, h): I rows 32X + 4g + r (DPP row
//    r), J rows 32Y + 16h + lane % 16;
//  * X == Y: the super-block's 32 * 31 / 2 pairs as a circulant: I row a takes
//    J rows a + 1 .. a + 16 (mod 32), the antipodal pair (a, a + 16) once
//    (from a < 16); wave g holds a = 4g + r, so its J rows are 4g + 1 ..
//    4g + 19 (mod 32): 20 staged rows, lane (r, o - 1) reading row r + o - 1.
//    496 of 512 lanes hold a pair.
// Tiles are numbered Y-major: Y's tiles start at 8 Y^2; within Y the
// off-diagonal pairs X = 0 .. Y-1 (16 waves each, w = 2g + h), then the diagonal.
__host__ __device__ inline int tiles_before(int Y) { return DIAG_W * Y * Y; }
__host__ __device__ inline int ntiles_of(int K) { return tiles_before((K + SB - 1) / SB); }
struct Tile {
  int X, Y, g, h;
  bool diag;
};
__host__ __device__ inline Tile tile_of(int t) {
  int Y = 0;
  while (tiles_before(Y + 1) <= t) ++Y;  // at most ~K / 32 steps
  const int local = t - tiles_before(Y);
  Tile r;
  r.Y = Y;
  if (local < Y * OFF_W) {
    r.X = local / OFF_W;
    r.g = (local % OFF_W) >> 1;
    r.h = local & 1;
    r.diag = false;
  } else {
    r.X = Y;
    r.g = local - Y * OFF_W;
    r.h = 0;
    r.diag = true;
  }
  return r;
}
// the tile that computes pair (i, j), i < j
__host__ __device__ inline int tile_of_pair(int i, int j) {
  const int X = i / SB, Y = j / SB;
  if (X < Y) return tiles_before(Y) + X * OFF_W + 2 * ((i % SB) / IW) + (j % SB) / JW;
  const int a = i % SB, b = j % SB, o = b - a;  // 1 .. 31
  const int ii = o <= SB / 2 ? a : b;           // the row whose circulant half holds the pair
  return tiles_before(Y) + Y * OFF_W + ii / IW;
}

// Xc[k][c][s] = X[k][8 (r0 + s) + c] for s < steps; stream stride ldc (x 8 per row).
// Each wave moves 256 steps (8 KB) on its own: 8 lane-contiguous 16-B loads
// (1 KB per instruction), the floats scattered into a chain-major LDS image
// (rows of 256 + 4 floats: the b32 writes of a 32-lane group hit 32 banks),
// then per chain one 16-B read of 4 steps per lane and a lane-contiguous 1-KB
// store.  (Per-lane 128-B rows read at 3 TB/s: 64 cache lines per load.)
constexpr int TW = 256;        // steps per wave
constexpr int TROW = TW + 4;   // LDS floats per chain row
// The waves to run, as runs of consecutive wave indices (wave w: steps
// w TW .. w TW + TW - 1): the host leaves out every wave whose 2048
// coordinates lie inside one tap-major block (tap_chain_kernel writes those),
// so no workgroup is launched only to find it has nothing to do.
struct WaveRuns {
  static constexpr int MAX = 48;
  int n;
  int64_t w0[MAX], pre[MAX + 1];  // run r: waves w0[r] .., launch ordinals pre[r] .. pre[r + 1] - 1
};
__global__ __launch_bounds__(256) void chain_transpose_kernel(const float* __restrict__ X, int64_t ldx, int64_t r0,
                                                              int64_t steps, int64_t ldc, float* __restrict__ Xc,
                                                              const WaveRuns runs) {
  __shared__ __attribute__((aligned(16))) float t[4 * 8 * TROW];
  const int k = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + wave;
  if (q >= runs.pre[runs.n]) return;  // the whole wave (no workgroup barrier below)
  int r = 0;
  while (q >= runs.pre[r + 1]) ++r;
  const int64_t s0 = (runs.w0[r] + q - runs.pre[r]) * TW;
  const int nv = (int)(steps - s0 < TW ? steps - s0 : TW);
  const float* src = X + (int64_t)k * ldx + 8 * (r0 + s0);
  float* tw = t + wave * 8 * TROW;
  const int h = lane & 1, sl = lane >> 1;
  f32x4 v[8];
  if (nv == TW) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src) + 64 * q + lane);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      v[q] = 32 * q + sl < nv ? reinterpret_cast<const f32x4*>(src)[64 * q + lane] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) tw[(4 * h + e) * TROW + 32 * q + sl] = v[q][e];
  // same wave: its LDS ops complete in order; the clobber keeps the compiler
  // from moving the reads above the writes
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float* dst = Xc + (int64_t)k * 8 * ldc + s0 + 4 * lane;
  if (nv == TW) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
      *reinterpret_cast<f32x4*>(dst + (int64_t)c * ldc) = *reinterpret_cast<const f32x4*>(tw + c * TROW + 4 * lane);
  } else {
    for (int c = 0; c < 8; ++c)
      for (int e = 0; e < 4 && 4 * lane + e < nv; ++e) dst[(int64_t)c * ldc + e] = tw[c * TROW + 4 * lane + e];
  }
}

// The tap-major blocks of a training-order client matrix (a convolution
// weight stored [KK][Cin][Cout], KK = kh * kw, whose reference order is
// torch's [Cout][Cin][KK]): chain_transpose_kernel skips them, this kernel
// writes their coordinates chain-major.  A workgroup takes a tile of 32 output
// channels x CI input channels x every tap of one row: coalesced 128-B reads of
// the training layout (32 channels of one (tap, input channel)) into LDS, then,
// per output channel, its run of CI * KK consecutive torch coordinates written
// chain-major (chain c = u % 8, step u / 8 - r0: CI * KK / 8 consecutive floats
// per chain).  The next CI of the same channels continues those runs: tiles
// are numbered channel-group-major and dealt to the XCDs in contiguous ranges
// (blockIdx % 8 is the XCD), so the workgroups that fill one stretch of a chain
// stream share an L2 and run together.  Grid (tiles, K).
constexpr int TAP_CO = 32;
constexpr int TAP_ROWS = 288;  // LDS tile rows (tap, input channel): CI = TAP_ROWS / KK
// the dense write enumeration divides item indices < TAP_CO * TAP_ROWS through
// a float reciprocal: exact while they stay far below 2^24 / (the divisor)
static_assert(TAP_CO * TAP_ROWS < (1 << 14), "dense write items exact in fp32");
template <int KKT, bool VEC>  // KKT: 9, 1, or 0 = KK at run time; VEC: 16-B aligned tile rows
__global__ __launch_bounds__(256) void tap_chain_kernel(const float* __restrict__ X, int64_t ldx, int64_t off,
                                                        int Cout, int Cin, int KKr, int64_t r0, int64_t steps,
                                                        int64_t ldc, float* __restrict__ Xc,
                                                        const float* __restrict__ gdead, uint64_t dead, int nneg) {
  constexpr int TCO = TAP_CO, TROWS = TAP_ROWS;
  __shared__ float tile[TROWS][TCO + 1];
  const int KK = KKT > 0 ? KKT : KKr;
  const int CI = TROWS / KK;
  const int nci_t = (Cin + CI - 1) / CI, ntiles = (int)gridDim.x;
  // XCD-contiguous tile numbering: XCD x = blockIdx % 8 takes tiles
  // [x * ntiles / 8, (x + 1) * ntiles / 8)
  const int x = (int)(blockIdx.x & 7), j = (int)(blockIdx.x >> 3);
  const int tl = x * (ntiles / 8) + min(x, ntiles % 8) + j;
  const int co0 = (tl / nci_t) * TCO, ci0 = (tl % nci_t) * CI;
  const int nci = min(CI, Cin - ci0), nco_v = min(TCO, Cout - co0);
  const int k = blockIdx.y;
  const float* row = X + (int64_t)k * ldx + off;
  // dead taps (flr_pairwise_l2_reference_tap_dead): read from the global
  // vector at the same offset, negated on the sign-flipped rows
  const float* grow = gdead ? gdead + off : row;
  const float gs = k < nneg ? -1.f : 1.f;
  auto is_dead = [&](int t) { return t < 64 && ((dead >> t) & 1); };
  auto src = [&](int t) { return is_dead(t) ? grow : row; };
  auto sgn = [&](int t) { return is_dead(t) ? gs : 1.f; };  // (x * 1 == x, -x exact)
  const int nrows = KK * CI;
  // load: tile row r = t * CI + ci, column = output channel; every load of a
  // thread issued before its LDS stores
  if constexpr (VEC) {  // nco_v == TCO: a row is TCO / 4 pieces of 16 B
    constexpr int LPR = TCO / 4, RPP = 256 / LPR;  // lanes per row, rows per pass
    const int sub = threadIdx.x % LPR, rr = threadIdx.x / LPR;
    constexpr int IT = (TROWS + RPP - 1) / RPP;
    f32x4 v[IT];
#pragma unroll
    for (int q = 0; q < IT; ++q) {
      const int r = rr + RPP * q, t = r / CI, ci = r - t * CI;
      const int64_t e = ((int64_t)t * Cin + ci0 + ci) * Cout + co0 + 4 * sub;
      if (!(r < nrows && ci < nci))
        v[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      else if (is_dead(t))  // the global vector, re-read by every client: cached loads
        v[q] = *reinterpret_cast<const f32x4*>(grow + e) * gs;
      else
        v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + e));
    }
#pragma unroll
    for (int q = 0; q < IT; ++q) {
      const int r = rr + RPP * q;
      if (r < nrows)
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[r][4 * sub + e] = v[q][e];
    }
  } else {
    for (int e = threadIdx.x; e < nrows * TCO; e += 256) {
      const int co = e % TCO, r = e / TCO, t = r / CI, ci = r % CI;
      if (ci < nci && co < nco_v) tile[r][co] = src(t)[((int64_t)t * Cin + ci0 + ci) * Cout + co0 + co] * sgn(t);
    }
  }
  __syncthreads();
  // write: output channel co's run [u0, u0 + nci * KK) (at most 288
  // coordinates: 38 steps per chain), clipped to the segment
  // [8 r0, 8 (r0 + steps)), chain-major: a wave writes consecutive steps of
  // a chain stream
  const int64_t L = (int64_t)nci * KK;
  const int64_t ulo = 8 * r0, uhi = 8 * (r0 + steps);
  float* out = Xc + (int64_t)k * 8 * ldc;
  {
    // every co's run whole inside the segment, and the same chain split for
    // every co (Cin KK and L multiples of 8: m steps per chain): the items
    // enumerated densely, (co, chain, step) with step fastest — every lane
    // busy, against 36 or 37 of 64 in the general loop below (-13 % time)
    const int64_t CL = (int64_t)Cin * KK;
    const int64_t ufirst = off + ((int64_t)co0 * Cin + ci0) * KK;
    if (CL % 8 == 0 && L % 8 == 0 && ufirst >= ulo && ufirst + (nco_v - 1) * CL + L <= uhi) {
      const int Li = (int)L, m = Li / 8, a0 = (int)(ufirst & 7);
      const int64_t sb0 = (ufirst >> 3) - r0, CLs = CL / 8;
      const float inv_L = 1.f / (float)Li, inv_m = 1.f / (float)m;
      const int n = nco_v * Li;
#pragma unroll 4
      for (int i = threadIdx.x; i < n; i += 256) {
        const int co = (int)(((float)i + 0.5f) * inv_L);  // exact: i < 2^14
        const int q = i - co * Li;
        const int c = (int)(((float)q + 0.5f) * inv_m);
        const int jj = q - c * m;
        const int dc = (c - a0) & 7;  // chain c's first coordinate in the run: u0 + dc
        const int rel = dc + 8 * jj, ci = rel / KK, t = rel - ci * KK;
        out[(int64_t)c * ldc + sb0 + co * CLs + ((a0 + dc) >> 3) + jj] = tile[t * CI + ci][co];
      }
      return;
    }
  }
  // the general tile (ragged, or crossing a segment end): item i -> (co =
  // i / 512, chain = i / 64 % 8, step slot i % 64)
  static_assert(TROWS / 8 + 1 <= 64, "a run's steps fit its slots");
#pragma unroll 4
  for (int i = threadIdx.x; i < nco_v * 512; i += 256) {
    const int ns = i & 63, c = (i >> 6) & 7, co = i >> 9;
    const int64_t u0 = off + ((int64_t)(co0 + co) * Cin + ci0) * KK;
    const int64_t u = 8 * ((u0 >> 3) + ns) + c;
    if (u >= u0 && u < u0 + L && u >= ulo && u < uhi) {
      const int rel = (int)(u - u0), ci = rel / KK, t = rel - ci * KK;
      out[(int64_t)c * ldc + ((u >> 3) - r0)] = tile[t * CI + ci][co];
    }
  }
}

// One chunk (CS = 64 steps) of a lane's chain: step S subtracts its x_j from
// x_i's step S, which lane S / 4 of each 16-lane row holds (component S % 4) and
// a DPP row_newbcast hands to every lane, folded into the subtraction
// (v_sub_f32_dpp), then acc = fma(d, d, acc).  Inline asm fixes the order
// (the subtraction of step S + 2 in the gap before the dependent fma of step
// S; blocks of 16 steps, three rotating temporaries).  The s_nop before the
// first block covers the DPP read-after-VALU-write hazard on x_i (the compiler
// cannot see a DPP inside asm; the later blocks follow asm that writes only the
// temporaries and acc).
// FLR_REF_ABL (tools build, timing only, wrong results): 1 plain v_sub instead
// of the DPP broadcast, 2 no LDS reads, 3 no DMA / x_i loads, 4 no barrier,
// 5 no chain arithmetic
#ifndef FLR_REF_ABL
#define FLR_REF_ABL 0
#endif
#if FLR_REF_ABL == 1
#define FLR_CHAIN16(A, B, C, D, NOP) \
  NOP \
  "v_sub_f32 %[t0], %[x0], %[j0]\n\t" \
  "v_sub_f32 %[t1], %[x1], %[j1]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32 %[t2], %[x2], %[j2]\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32 %[t0], %[x3], %[j3]\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32 %[t1], %[x0], %[j4]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32 %[t2], %[x1], %[j5]\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32 %[t0], %[x2], %[j6]\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32 %[t1], %[x3], %[j7]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32 %[t2], %[x0], %[j8]\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32 %[t0], %[x1], %[j9]\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32 %[t1], %[x2], %[j10]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32 %[t2], %[x3], %[j11]\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32 %[t0], %[x0], %[j12]\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32 %[t1], %[x1], %[j13]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32 %[t2], %[x2], %[j14]\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32 %[t0], %[x3], %[j15]\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t"
#else
#define FLR_CHAIN16(A, B, C, D, NOP) \
  NOP \
  "v_sub_f32_dpp %[t0], %[x0], %[j0] row_newbcast:" #A " row_mask:0xf bank_mask:0xf\n\t" \
  "v_sub_f32_dpp %[t1], %[x1], %[j1] row_newbcast:" #A " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32_dpp %[t2], %[x2], %[j2] row_newbcast:" #A " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32_dpp %[t0], %[x3], %[j3] row_newbcast:" #A " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32_dpp %[t1], %[x0], %[j4] row_newbcast:" #B " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32_dpp %[t2], %[x1], %[j5] row_newbcast:" #B " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32_dpp %[t0], %[x2], %[j6] row_newbcast:" #B " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32_dpp %[t1], %[x3], %[j7] row_newbcast:" #B " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32_dpp %[t2], %[x0], %[j8] row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32_dpp %[t0], %[x1], %[j9] row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32_dpp %[t1], %[x2], %[j10] row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32_dpp %[t2], %[x3], %[j11] row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32_dpp %[t0], %[x0], %[j12] row_newbcast:" #D " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_sub_f32_dpp %[t1], %[x1], %[j13] row_newbcast:" #D " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t" \
  "v_sub_f32_dpp %[t2], %[x2], %[j14] row_newbcast:" #D " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t1], %[t1]\n\t" \
  "v_sub_f32_dpp %[t0], %[x3], %[j15] row_newbcast:" #D " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[t2], %[t2]\n\t" \
  "v_fmac_f32 %[acc], %[t0], %[t0]\n\t"
#endif
#define FLR_CHAIN_BLOCK(b, A, B, C, D, NOP)                                                                 \
  asm volatile(FLR_CHAIN16(A, B, C, D, NOP)                                                                \
               : [acc] "+v"(acc), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)                        \
               : [x0] "v"(xv[0]), [x1] "v"(xv[1]), [x2] "v"(xv[2]), [x3] "v"(xv[3]), [j0] "v"(v[4 * (b) + 0][0]), [j1] "v"(v[4 * (b) + 0][1]), [j2] "v"(v[4 * (b) + 0][2]), [j3] "v"(v[4 * (b) + 0][3]), [j4] "v"(v[4 * (b) + 1][0]), [j5] "v"(v[4 * (b) + 1][1]), [j6] "v"(v[4 * (b) + 1][2]), [j7] "v"(v[4 * (b) + 1][3]), [j8] "v"(v[4 * (b) + 2][0]), [j9] "v"(v[4 * (b) + 2][1]), [j10] "v"(v[4 * (b) + 2][2]), [j11] "v"(v[4 * (b) + 2][3]), [j12] "v"(v[4 * (b) + 3][0]), [j13] "v"(v[4 * (b) + 3][1]), [j14] "v"(v[4 * (b) + 3][2]), [j15] "v"(v[4 * (b) + 3][3]))
__device__ __forceinline__ float chain_chunk(f32x4 xv, const f32x4 (&v)[NQ], float acc) {
  static_assert(NQ == 16, "four blocks of 16 steps");
  float t0, t1, t2;
  FLR_CHAIN_BLOCK(0, 0, 1, 2, 3, "s_nop 1\n\t");
  FLR_CHAIN_BLOCK(1, 4, 5, 6, 7, "");
  FLR_CHAIN_BLOCK(2, 8, 9, 10, 11, "");
  FLR_CHAIN_BLOCK(3, 12, 13, 14, 15, "");
  return acc;
}
#undef FLR_CHAIN_BLOCK
#undef FLR_CHAIN16

// Two chains per lane (K >= 256, off-diagonal tiles, ref_chain2_kernel): the
// lane's pairs (i, j) and (i + 4, j) share the staged x_j; per step two
// v_sub_f32_dpp (x_i and x_i2 broadcast by row_newbcast, as above) and two
// v_fmac, the previous step's squares one slot behind its subtraction.
#define FLR_STEP2(XA, XB, J, L, TA, TB, PA, PB) \
  "v_sub_f32_dpp %[" #TA "], %[" #XA "], %[" #J "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t" \
  "v_sub_f32_dpp %[" #TB "], %[" #XB "], %[" #J "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f32 %[acc], %[" #PA "], %[" #PA "]\n\t" \
  "v_fmac_f32 %[acc2], %[" #PB "], %[" #PB "]\n\t"
#define FLR_STEP2_FIRST(XA, XB, J, L, TA, TB) \
  "v_sub_f32_dpp %[" #TA "], %[" #XA "], %[" #J "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t" \
  "v_sub_f32_dpp %[" #TB "], %[" #XB "], %[" #J "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define FLR_CHAIN16_2(A, B, C, D, NOP) \
  NOP \
  FLR_STEP2_FIRST(x0, y0, j0, A, a0, b0) \
  FLR_STEP2(x1, y1, j1, A, a1, b1, a0, b0) FLR_STEP2(x2, y2, j2, A, a0, b0, a1, b1) \
  FLR_STEP2(x3, y3, j3, A, a1, b1, a0, b0) FLR_STEP2(x0, y0, j4, B, a0, b0, a1, b1) \
  FLR_STEP2(x1, y1, j5, B, a1, b1, a0, b0) FLR_STEP2(x2, y2, j6, B, a0, b0, a1, b1) \
  FLR_STEP2(x3, y3, j7, B, a1, b1, a0, b0) FLR_STEP2(x0, y0, j8, C, a0, b0, a1, b1) \
  FLR_STEP2(x1, y1, j9, C, a1, b1, a0, b0) FLR_STEP2(x2, y2, j10, C, a0, b0, a1, b1) \
  FLR_STEP2(x3, y3, j11, C, a1, b1, a0, b0) FLR_STEP2(x0, y0, j12, D, a0, b0, a1, b1) \
  FLR_STEP2(x1, y1, j13, D, a1, b1, a0, b0) FLR_STEP2(x2, y2, j14, D, a0, b0, a1, b1) \
  FLR_STEP2(x3, y3, j15, D, a1, b1, a0, b0) \
  "v_fmac_f32 %[acc], %[a1], %[a1]\n\t" \
  "v_fmac_f32 %[acc2], %[b1], %[b1]\n\t"
#define FLR_CHAIN_BLOCK2(b, A, B, C, D, NOP)                                                                   \
  asm volatile(FLR_CHAIN16_2(A, B, C, D, NOP)                                                                 \
               : [acc] "+v"(acc), [acc2] "+v"(acc2), [a0] "=&v"(a0), [b0] "=&v"(b0), [a1] "=&v"(a1),          \
                 [b1] "=&v"(b1)                                                                              \
               : [x0] "v"(xv[0]), [x1] "v"(xv[1]), [x2] "v"(xv[2]), [x3] "v"(xv[3]), [y0] "v"(yv[0]),           \
                 [y1] "v"(yv[1]), [y2] "v"(yv[2]), [y3] "v"(yv[3]), [j0] "v"(v[4 * (b) + 0][0]),              \
                 [j1] "v"(v[4 * (b) + 0][1]), [j2] "v"(v[4 * (b) + 0][2]), [j3] "v"(v[4 * (b) + 0][3]),        \
                 [j4] "v"(v[4 * (b) + 1][0]), [j5] "v"(v[4 * (b) + 1][1]), [j6] "v"(v[4 * (b) + 1][2]),        \
                 [j7] "v"(v[4 * (b) + 1][3]), [j8] "v"(v[4 * (b) + 2][0]), [j9] "v"(v[4 * (b) + 2][1]),        \
                 [j10] "v"(v[4 * (b) + 2][2]), [j11] "v"(v[4 * (b) + 2][3]), [j12] "v"(v[4 * (b) + 3][0]),     \
                 [j13] "v"(v[4 * (b) + 3][1]), [j14] "v"(v[4 * (b) + 3][2]), [j15] "v"(v[4 * (b) + 3][3]))
__device__ __forceinline__ void chain_chunk2(f32x4 xv, f32x4 yv, const f32x4 (&v)[NQ], float& acc, float& acc2) {
  float a0, b0, a1, b1;
  FLR_CHAIN_BLOCK2(0, 0, 1, 2, 3, "s_nop 1\n\t");
  FLR_CHAIN_BLOCK2(1, 4, 5, 6, 7, "");
  FLR_CHAIN_BLOCK2(2, 8, 9, 10, 11, "");
  FLR_CHAIN_BLOCK2(3, 12, 13, 14, 15, "");
}
#undef FLR_CHAIN_BLOCK2
#undef FLR_CHAIN16_2
#undef FLR_STEP2_FIRST
#undef FLR_STEP2

template <class F, int... U>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, U...>) {
  (f(std::integral_constant<int, U>{}), ...);
}

// One segment of steps of one tile (one wave): chain c of each lane's pair; the
// running chain sums in A[c][min(i,j)][max(i,j)] (first: start from 0).
//
// Body ch (stage u = ch % NSTAGE, static in the unrolled loop):
//   wait  DMA(ch + 1) and x_i(ch) landed (counted vmcnt: the DMA's LDS writes
//         are then visible to this wave), the ds_reads of chunk ch landed
//         (lgkmcnt(0): stage (ch - 1) % NSTAGE is free)
//   issue DMA(ch + NSTAGE - 1) into that stage and x_i(ch + NSTAGE - 1);
//         ds_read_b128 x 16 of chunk ch + 1 into the other register buffer
//   chain chunk ch (registers read in body ch - 1)
// Every body issues the same vector-memory ops (past the last group they read
// the next stream or the workspace slack: nothing consumes them), so the counts
// are static; the loop runs whole groups of NSTAGE chunks over the zero-filled
// streams (XC_GROUP), without a per-chunk check; the LDS reads and the register loads are inline asm
// with explicit waits (the compiler's waitcnt pass, merging across the
// rotated registers, drained vmcnt(0) every chunk).  No workgroup barrier:
// the wave is the workgroup and reads only what it staged.
// NST: the ring's stages (the loop's unroll); TWO: two chains per lane, pairs
// (i, j) and (i + 4, j) of an off-diagonal tile (ref_chain2_kernel).
template <bool DIAG, int NST = NSTAGE, bool TWO = false>
__device__ __forceinline__ void ref_chain_tile(float* lds, const Tile T, const int c, const float* __restrict__ Xc,
                                               int64_t ldc, int K, int64_t steps, int first,
                                               float* __restrict__ A) {
  using S = Staging<DIAG>;
  static_assert(!(TWO && DIAG), "two chains per lane on off-diagonal tiles only");
  static_assert(NST % 2 == 0 && NST >= 4, "two register buffers");
  constexpr int NXI = TWO ? 2 : 1;               // x_i loads per body
  constexpr int OPB = S::DPW + NXI;              // vector-memory ops per body
  static_assert((NST - 2) * OPB + NXI < 64, "vmcnt counts to 63");
  const int lane = threadIdx.x & 63, r = lane >> 4, jl = lane & 15;
  // this lane's pair (i, j) and the staged row it reads
  int i, j, srow;
  bool keep = true;
  if (DIAG) {
    const int a = IW * T.g + r, o = jl + 1;
    i = SB * T.X + a;
    j = SB * T.X + ((a + o) & (SB - 1));
    srow = r + jl;
    keep = o < SB / 2 || a < SB / 2;  // the antipodal pair once
  } else {
    i = SB * T.X + (TWO ? 2 * IW : IW) * T.g + r;  // TWO: I rows 8g + r and 8g + 4 + r
    j = SB * T.Y + JW * T.h + jl;
    srow = jl;
  }
  const int i2 = i + IW;  // TWO: the lane's second pair (i2, j), i2 < j
  const bool valid2 = TWO && i2 < K && j < K;
  const bool valid = keep && i < K && j < K;
  const int lo = i < j ? i : j, hi = i < j ? j : i;  // A holds the pair at [lo][hi]
  const int64_t rs = 8 * ldc;

  // the running sum of the previous segments: an asm load and a full wait
  // before any DMA, so no compiler-tracked load reaches into the loop
  float acc = 0.f, acc2 = 0.f;
  if (!first) {
    const float* ap = A + ((int64_t)c * K + (lo < K ? lo : K - 1)) * K + (hi < K ? hi : K - 1);
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(acc) : "v"(ap) : "memory");
    acc = valid ? acc : 0.f;
    if constexpr (TWO) {
      const float* ap2 = A + ((int64_t)c * K + (i2 < K ? i2 : K - 1)) * K + (j < K ? j : K - 1);
      asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(acc2) : "v"(ap2) : "memory");
      acc2 = valid2 ? acc2 : 0.f;
    }
  }

  // staging: DMA instruction u moves staged rows RPD u .. RPD u + 3, lane ->
  // row RPD u + lane / NQ, LDS slot lane % NQ holding the piece slot ^ slot_swz(row).
  // Global addresses as a uniform base (SGPRs, advanced per chunk) + a 32-bit
  // per-lane offset (the saddr form: no 64-bit address arithmetic per DMA);
  // the DMAs of a chunk share one M0 (the stage + 2 KB) and differ in the
  // instruction offset (u - 2) KB, which applies to the global and the LDS
  // address alike (13-bit signed: -2 .. +2 KB), so the lane offsets carry
  // 2 KB - (u - 2) KB of slack and the base sits 2 KB low.
  const int jrow0 = DIAG ? SB * T.X : min(SB * T.Y + JW * T.h, K - 1);  // lowest staged row (clamped)
  const char* sbj = reinterpret_cast<const char*>(Xc + (int64_t)jrow0 * rs + (int64_t)c * ldc) - 2048;
  uint32_t voj[S::DPW];
#pragma unroll
  for (int u = 0; u < S::DPW; ++u) {
    const int s = RPD * u + lane / NQ;
    int gj = DIAG ? SB * T.X + ((IW * T.g + 1 + s) & (SB - 1)) : SB * T.Y + JW * T.h + s;
    gj = gj < K ? gj : K - 1;
    voj[u] = (uint32_t)((int64_t)(gj - jrow0) * rs * 4 + 16 * ((lane % NQ) ^ slot_swz(s)) - 1024 * (u - 2) + 2048);
  }
  // x_i: lane jl of DPP row r loads steps 4 jl .. 4 jl + 3 of the row's I row
  const int irow0 = min(DIAG ? SB * T.X + IW * T.g : i - r, K - 1);
  const char* sbi = reinterpret_cast<const char*>(Xc + (int64_t)irow0 * rs + (int64_t)c * ldc);
  const uint32_t voi = (uint32_t)((int64_t)((i < K ? i : K - 1) - irow0) * rs * 4 + 16 * jl);
  const uint32_t voi2 = (uint32_t)((int64_t)((i2 < K ? i2 : K - 1) - irow0) * rs * 4 + 16 * jl);
  // whole loop trips of NST chunks inside the zero-filled streams (padded to
  // XC_GROUP steps, a multiple of NST * CS)
  static_assert(XC_GROUP % (NST * CS) == 0, "trips inside the zero fill");
  const int ngroup = (int)((steps + NST * CS - 1) / (NST * CS));
  // DMA(ch) into stage `slot`, then x_i(ch) into register set x (inline asm:
  // hipcc built 64-bit addresses per DMA instead of the saddr form)
  auto issue = [&](int ch, int slot, f32x4& x, f32x4& x2) {
    // the chunk's byte offset in a stream: the prefetch runs up to NSTAGE - 1
    // chunks past the last one (reads nothing consumes; the workspace carries
    // XC_SLACK bytes past the last stream)
    const int64_t co = (int64_t)ch * CS * 4;
    if (FLR_REF_ABL == 3) return;
    const char* sb = sbj + co;
    const uint32_t m = (uint32_t)(uintptr_t)lds + 4 * slot * STAGE + 2048;
    // M0 written in the statement that reads it; no other instruction of this
    // kernel reads M0 (the compiler emits none: checked in the ISA), so it is
    // not restored
#define FLR_DMA(n, off) "global_load_lds_dwordx4 %[v" #n "], %[sb] offset:" #off "\n\t"
    if constexpr (S::DPW == 5)
      asm volatile("s_mov_b32 m0, %[m]\n\ts_nop 0\n\t" FLR_DMA(0, -2048) FLR_DMA(1, -1024) FLR_DMA(2, 0)
                       FLR_DMA(3, 1024) FLR_DMA(4, 2048)
                   :
                   : [m] "s"(m), [sb] "s"(sb), [v0] "v"(voj[0]), [v1] "v"(voj[1]), [v2] "v"(voj[2]), [v3] "v"(voj[3]),
                     [v4] "v"(voj[S::DPW - 1])
                   : "memory");
    else
      asm volatile("s_mov_b32 m0, %[m]\n\ts_nop 0\n\t" FLR_DMA(0, -2048) FLR_DMA(1, -1024) FLR_DMA(2, 0)
                       FLR_DMA(3, 1024)
                   :
                   : [m] "s"(m), [sb] "s"(sb), [v0] "v"(voj[0]), [v1] "v"(voj[1]), [v2] "v"(voj[2]), [v3] "v"(voj[3])
                   : "memory");
#undef FLR_DMA
    static_assert(S::DPW == 4 || S::DPW == 5, "the DMA statements above");
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(x) : "v"(voi), "s"(sbi + co) : "memory");
    if constexpr (TWO) asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(x2) : "v"(voi2), "s"(sbi + co) : "memory");
  };
  // per-lane LDS byte addresses of staged row srow's 16 swizzled pieces in stage 0
  const int rsw = slot_swz(srow);
  uint32_t ra[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) ra[q] = (uint32_t)(uintptr_t)(lds + srow * CS + 4 * (q ^ rsw));
  auto rows = [](auto st, f32x4(&v)[NQ], const uint32_t(&a)[NQ]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (FLR_REF_ABL != 2)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[q]) : "v"(a[q]), "n"(decltype(st)::value * STAGE * 4)
                     : "memory");
  };

  f32x4 va[NQ], vb[NQ];
  f32x4 xs[NST], xs2[NST];
  auto body = [&](auto U, int ch, f32x4(&vc)[NQ], f32x4(&vn)[NQ]) {
    constexpr int u = decltype(U)::value;
    // DMA(ch + 1) was issued in body ch + 2 - NSTAGE; younger than it: its
    // x_i load and the NSTAGE - 3 bodies since (x_i(ch) is older: covered)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 3) * OPB + NXI) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // chunk ch's x_j
    // chunk ch's operands arrived at the waits above: tie them to here
    asm volatile("" : "+v"(vc[0]), "+v"(vc[1]), "+v"(vc[2]), "+v"(vc[3]), "+v"(vc[4]), "+v"(vc[5]), "+v"(vc[6]),
                 "+v"(vc[7]), "+v"(vc[8]), "+v"(vc[9]), "+v"(vc[10]), "+v"(vc[11]), "+v"(vc[12]), "+v"(vc[13]),
                 "+v"(vc[14]), "+v"(vc[15]), "+v"(xs[u]));
    if constexpr (TWO) asm volatile("" : "+v"(xs2[u]));
    issue(ch + NST - 1, (u + NST - 1) % NST, xs[(u + NST - 1) % NST], xs2[(u + NST - 1) % NST]);
    rows(std::integral_constant<int, (u + 1) % NST>{}, vn, ra);
    if constexpr (TWO)
      chain_chunk2(xs[u], xs2[u], vc, acc, acc2);
    else if (FLR_REF_ABL != 5)
      acc = chain_chunk(xs[u], vc, acc);
  };
  // prologue = the issues of bodies -(NSTAGE-1) .. -1, then chunk 0's rows
#pragma unroll
  for (int u = 0; u < NST - 1; ++u) issue(u, u, xs[u], xs2[u]);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * OPB + NXI) : "memory");  // DMA(0)
  rows(std::integral_constant<int, 0>{}, va, ra);
  for (int ch = 0; ch < ngroup * NST; ch += NST)
    static_for(
        [&](auto U) {
          constexpr int u = decltype(U)::value;
          if constexpr (u % 2 == 0)
            body(U, ch + u, va, vb);
          else
            body(U, ch + u, vb, va);
        },
        std::make_integer_sequence<int, NST>{});
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (valid) A[((int64_t)c * K + lo) * K + hi] = acc;
  if (valid2) A[((int64_t)c * K + i2) * K + j] = acc2;
}

// grid 8 x (t1 - t0) one-wave workgroups: chain c = blockIdx % 8 (the XCD),
// tile t0 + blockIdx / 8
__global__ __launch_bounds__(64) void ref_chain_kernel(const float* __restrict__ Xc, int64_t ldc, int K,
                                                       int64_t steps, int t0, int first, float* __restrict__ A) {
  // ONE __shared__ array (a second __shared__ object makes hipcc wait vmcnt(0)
  // before the LDS reads, draining the DMA ring)
  __shared__ __attribute__((aligned(16))) float lds[NSTAGE * STAGE];
  const int c = (int)(blockIdx.x & 7);
  const Tile T = tile_of(t0 + (int)(blockIdx.x >> 3));
  if (T.diag)
    ref_chain_tile<true>(lds, T, c, Xc, ldc, K, steps, first, A);
  else
    ref_chain_tile<false>(lds, T, c, Xc, ldc, K, steps, first, A);
}

// K >= 256 (more tiles than SIMDs: the chains are throughput-bound, not
// latency-bound): off-diagonal super-block pairs as 8 waves of 8 I rows x 16 J
// rows, two chains per lane sharing the staged x_j (half the LDS reads per chain
// step), diagonal super-blocks as the 1-I circulant tiles above; a 4-stage ring
// (20 KB) and at most 256 VGPRs, so two waves per SIMD.  Tiles per Y: the
// off-diagonal pairs X = 0 .. Y-1 (8 waves each: w = 2g + h), then the diagonal.
constexpr int NST2 = 4;
__host__ __device__ inline int tiles2_before(int Y) { return 4 * Y * (Y + 1); }
__host__ __device__ inline int ntiles2_of(int K) { return tiles2_before((K + SB - 1) / SB); }
__host__ __device__ inline Tile tile2_of(int t) {
  int Y = 0;
  while (tiles2_before(Y + 1) <= t) ++Y;
  const int local = t - tiles2_before(Y);
  Tile r;
  r.Y = Y;
  if (local < 8 * Y) {
    r.X = local / 8;
    r.g = (local % 8) >> 1;
    r.h = local & 1;
    r.diag = false;
  } else {
    r.X = Y;
    r.g = local - 8 * Y;
    r.h = 0;
    r.diag = true;
  }
  return r;
}
__global__ __launch_bounds__(64, 2) void ref_chain2_kernel(const float* __restrict__ Xc, int64_t ldc, int K,
                                                           int64_t steps, int first, float* __restrict__ A) {
  __shared__ __attribute__((aligned(16))) float lds[NST2 * STAGE];
  const int c = (int)(blockIdx.x & 7);
  const Tile T = tile2_of((int)(blockIdx.x >> 3));
  if (T.diag)
    ref_chain_tile<true, NST2, false>(lds, T, c, Xc, ldc, K, steps, first, A);
  else
    ref_chain_tile<false, NST2, true>(lds, T, c, Xc, ldc, K, steps, first, A);
}

// the two-chain form, opt-in (FLR_REF_2I=1, from two super-blocks, K > 32):
// measured -6 % at K=512 P=2M but +10 % at K=256 P=4M and +6 % on the C5
// distances (profiles/r6_ref/two_chain_ab.json), so off by default
inline bool use_two_chains(int64_t K) {
  const char* e = flr::knob("FLR_REF_2I");
  return e && e[0] == '1' && K > SB;
}

// K >= 480 (every pair, no tap-major blocks): the throughput form.  Measured
// on gfx950 (tools/hip/pk_rate.hip, profiles/r6_ref/pk_rate.json): at two waves
// per SIMD a plain v_fmac_f32 costs the SIMD 2.3 cycles, a v_sub_f32_dpp about
// 6.6, and packed f32 ops no fewer cycles per element than plain ones; so once
// there are two waves per SIMD to run, the cheapest chain step is a plain
// v_sub_f32 with x_i as an SGPR operand and a plain v_fmac_f32 — 2 SIMD issue
// slots of 2.3 cycles.  A wave holds 8 I rows (wave-uniform, scalar loads) x 64
// J rows (one per lane): 8 chains per lane, each x_j element serves 8 chain
// steps, so the chip's L2 traffic stays at 0.56 B per chain step.
// Operand layout (per segment, quad_transpose_kernel): Xq[c][b][k][e] =
// X[k][8 (r0 + 4 b + e) + c] — per chain c and 4-step block b, the Kp rows'
// 16-B pieces contiguous: lane j's x_j is one coalesced 1-KB load per wave,
// the 8 I rows' block 128 contiguous bytes (two s_load_dwordx16).
constexpr int QJ = 64;   // J rows per wave (lanes)
constexpr int QTB = 16;  // transpose tile: rows x 4-step blocks
constexpr int QD = 8;    // x_j blocks in flight per lane
static_assert(XC_GROUP % (4 * QTB) == 0 && XC_GROUP % (4 * QD) == 0, "padded segments hold whole tiles / trips");
__host__ __device__ inline int64_t quad_rows(int64_t K) { return (K + QJ - 1) / QJ * QJ; }
// tiles of J block q (rows 64 q .. 64 q + 63): I blocks of ni rows a = 0 ..
// min(64 / ni (q + 1), ceil(K / ni)) - 1
__host__ __device__ inline int quad_ni(int q, int K, int ni) {
  const int a = QJ / ni * (q + 1), b = (K + ni - 1) / ni;
  return a < b ? a : b;
}
// bytes past a segment's last block the x_j / x_i prefetches may read
inline int64_t quad_slack(int64_t K) { return (QD + 4) * quad_rows(K) * 16; }
inline int quad_ntiles(int K, int ni) {
  int n = 0;
  for (int q = 0; q * QJ < K; ++q) n += quad_ni(q, K, ni);
  return n;
}

// Xq tile: rows k0 .. k0 + 15 x blocks b0 .. b0 + 15 (64 steps = 512 coordinates
// = 2 KB of each row): coalesced 1-KB row reads into LDS, then thread (k, block)
// takes its row's 32 coordinates of the block and stores 8 chain pieces (16 B:
// 4 steps each), 256-B runs of consecutive rows.  Steps past `steps` are 0.
__global__ __launch_bounds__(256) void quad_transpose_kernel(const float* __restrict__ X, int64_t ldx, int K,
                                                             int64_t r0, int64_t steps, int64_t NB, int64_t Kp,
                                                             float* __restrict__ Xq) {
  __shared__ f32x4 t[QTB][QTB * 8 + 1];
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * QTB;
  const int k0 = blockIdx.y * QTB;
  const int64_t u0 = 8 * (r0 + 4 * b0), uend = 8 * (r0 + steps);  // this tile's first coordinate, the segment's end
  f32x4 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int idx = q * 256 + tid, row = idx >> 7, p = idx & 127;
    const int64_t u = u0 + 4 * p;
    v[q] = (k0 + row < K && u < uend)
               ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(X + (int64_t)(k0 + row) * ldx + u))
               : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int idx = q * 256 + tid;
    t[idx >> 7][idx & 127] = v[q];
  }
  __syncthreads();
  const int k = tid & 15, bl = tid >> 4;
  if (k0 + k >= K) return;  // rows past K: never a valid pair's operand
  f32x4 w[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) w[q] = t[k][8 * bl + q];
  // coordinate 32 bl + 4 q + m = 8 (4 bl + e) + c: step e = q / 2, chain c = 4 (q % 2) + m
  float* out = Xq + ((b0 + bl) * Kp + k0 + k) * 4;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int h = c >> 2, m = c & 3;
    *reinterpret_cast<f32x4*>(out + (int64_t)c * NB * Kp * 4) = f32x4{w[h][m], w[2 + h][m], w[4 + h][m], w[6 + h][m]};
  }
}

// One wave: chain c = blockIdx % 8 (the XCD) of tile blockIdx / 8 — J block q,
// I block a: lane l's pairs (NI a + r, 64 q + l), r < NI, valid where i < j < K.
// x_j: one 16-B load per lane and 4-step block, QD blocks in flight (vmcnt, in
// order).  x_i: NI rows x 4 steps x BT blocks per scalar round trip (NI BT / 4
// s_load_dwordx16 into one of two SGPR buffers).  Scalar loads return out of
// order, so a wait for one buffer waits for every scalar load issued: the next
// buffer's loads go out right AFTER the wait for the current one, and the
// latency they can hide is one buffer's compute, 2 NI 4 BT VALU — the reason for
// BT > 1 at NI = 4 (measured: NI = 8, BT = 1 stalled ~650 cycles per buffer,
// profiles/r6_ref/).  Per step the NI chains d = fl(x_i - x_j),
// acc = fma(d, d, acc): the reference's operations in its order.
// one step of the NI chains: plain v_sub_f32 (x_i an SGPR operand) and
// v_fmac_f32, each square one slot behind its difference (inline asm: the
// compiler otherwise SLP-packs the rows into v_pk_* ops whose SGPR pairs cost an
// s_mov per operand).  g0: rows 0-3 of the block (row r's step e at 4 r + e), g1:
// rows 4-7
template <int E>
__device__ __forceinline__ void sgpr_step(float (&acc)[4], const i32x16& g0, const i32x16&, float xjv) {
  float t0, t1;
  asm volatile(
      "v_sub_f32 %[t0], %[s0], %[x]\n\t"
      "v_sub_f32 %[t1], %[s1], %[x]\n\t"
      "v_fmac_f32 %[a0], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s2], %[x]\n\t"
      "v_fmac_f32 %[a1], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s3], %[x]\n\t"
      "v_fmac_f32 %[a2], %[t0], %[t0]\n\t"
      "v_fmac_f32 %[a3], %[t1], %[t1]\n\t"
      : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [t0] "=&v"(t0), [t1] "=&v"(t1)
      : [s0] "s"(g0[E]), [s1] "s"(g0[4 + E]), [s2] "s"(g0[8 + E]), [s3] "s"(g0[12 + E]), [x] "v"(xjv));
}
template <int E>
__device__ __forceinline__ void sgpr_step(float (&acc)[8], const i32x16& g0, const i32x16& g1, float xjv) {
  float t0, t1;
  asm volatile(
      "v_sub_f32 %[t0], %[s0], %[x]\n\t"
      "v_sub_f32 %[t1], %[s1], %[x]\n\t"
      "v_fmac_f32 %[a0], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s2], %[x]\n\t"
      "v_fmac_f32 %[a1], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s3], %[x]\n\t"
      "v_fmac_f32 %[a2], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s4], %[x]\n\t"
      "v_fmac_f32 %[a3], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s5], %[x]\n\t"
      "v_fmac_f32 %[a4], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s6], %[x]\n\t"
      "v_fmac_f32 %[a5], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s7], %[x]\n\t"
      "v_fmac_f32 %[a6], %[t0], %[t0]\n\t"
      "v_fmac_f32 %[a7], %[t1], %[t1]\n\t"
      : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]),
        [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7]), [t0] "=&v"(t0), [t1] "=&v"(t1)
      : [s0] "s"(g0[E]), [s1] "s"(g0[4 + E]), [s2] "s"(g0[8 + E]), [s3] "s"(g0[12 + E]), [s4] "s"(g1[E]),
        [s5] "s"(g1[4 + E]), [s6] "s"(g1[8 + E]), [s7] "s"(g1[12 + E]), [x] "v"(xjv));
}

// FLR_REF_S_ABL (tools build, timing only, wrong results): 1 no x_j loads in the
// loop, 2 no x_i loads, 3 no chain arithmetic, 4 x_i loaded but never waited for
#ifndef FLR_REF_S_ABL
#define FLR_REF_S_ABL 0
#endif
template <int NI, int BT>
__global__ __launch_bounds__(64) void ref_chain_s_kernel(const float* __restrict__ Xq, int64_t NB, int64_t Kp, int K,
                                                         int first, float* __restrict__ A) {
  static_assert(NI == 4 || NI == 8, "the step forms above");
  constexpr int NL = NI * BT / 4;  // s_load_dwordx16 per buffer
  static_assert(QD % (2 * BT) == 0, "whole ping-pong pairs of buffers per trip");
  const int c = (int)(blockIdx.x & 7), lane = threadIdx.x;
  int t = (int)(blockIdx.x >> 3), q = 0;
  for (int n = quad_ni(0, K, NI); t >= n; n = quad_ni(q, K, NI)) {
    t -= n;
    ++q;
  }
  const int i0 = NI * t, j = QJ * q + lane;
  const float* __restrict__ base = Xq + (int64_t)c * NB * Kp * 4;
  float acc[NI];
  if (first) {
#pragma unroll
    for (int r = 0; r < NI; ++r) acc[r] = 0.f;
  } else {  // asm loads and a full wait: no compiler-tracked load reaches into the loop
#pragma unroll
    for (int r = 0; r < NI; ++r) {
      const float* ap = A + ((int64_t)c * K + i0 + r) * K + (j < K ? j : K - 1);
      asm volatile("global_load_dword %0, %1, off" : "=v"(acc[r]) : "v"(ap) : "memory");
    }
    // the wait ties the loaded values: nothing reads them above it
    if constexpr (NI == 4)
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]) : : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)"
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                     "+v"(acc[6]), "+v"(acc[7])
                   :
                   : "memory");
#pragma unroll
    for (int r = 0; r < NI; ++r) acc[r] = (i0 + r < j && j < K) ? acc[r] : 0.f;
  }
  // uniform block pointers advanced per block (the prefetches run up to QD
  // blocks past the segment's last: the workspace's quad slack) and the lane's
  // 32-bit byte offset (the saddr load form)
  const int64_t bb = Kp * 16;  // bytes per block
  const uint32_t voff = (uint32_t)j * 16;
  const char* pjn = reinterpret_cast<const char*>(base);                      // the next x_j block to load
  const char* pin = reinterpret_cast<const char*>(base) + (int64_t)i0 * 16;  // the next x_i buffer
  auto ldj = [&](f32x4& x) {
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(x) : "v"(voff), "s"(pjn) : "memory");
    pjn += bb;
    asm volatile("" : "+s"(pjn));  // one running pointer, not QD precomputed ones
  };
  // buffer: block u's 4-row groups at buf[u NI / 4 ..]
  auto ldi = [&](i32x16(&buf)[NL]) {
    const char* pu = pin;
#pragma unroll
    for (int u = 0; u < BT; ++u) {
#pragma unroll
      for (int h = 0; h < NI / 4; ++h)
        asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(buf[u * (NI / 4) + h]) : "s"(pu), "n"(64 * h) : "memory");
      pu += bb;
      asm volatile("" : "+s"(pu));
    }
    pin = pu;
  };
  f32x4 xj[QD];
  i32x16 xa[NL], xb[NL];
#pragma unroll
  for (int u = 0; u < QD; ++u) ldj(xj[u]);
  ldi(xa);
  // a buffer's BT blocks: x_i(buffer) landed, then the next buffer issued;
  // per block x_j(b) landed, its 4 steps, x_j(b + QD) issued into the freed registers
  auto trip = [&](auto U0, const i32x16(&cur)[NL], i32x16(&nxt)[NL]) {
    constexpr int u0 = decltype(U0)::value;
    if (FLR_REF_S_ABL != 2 && FLR_REF_S_ABL != 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (FLR_REF_S_ABL != 2) ldi(nxt);
#pragma unroll
    for (int v = 0; v < BT; ++v) {
      f32x4& x = xj[u0 + v];
      if (FLR_REF_S_ABL != 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QD - 1) : "memory");
      asm volatile("" : "+v"(x));  // x arrived at the wait above
      const i32x16& g0 = cur[v * (NI / 4)];
      const i32x16& g1 = cur[v * (NI / 4) + (NI / 4) - 1];
      if (FLR_REF_S_ABL != 3) {
        sgpr_step<0>(acc, g0, g1, x[0]);
        sgpr_step<1>(acc, g0, g1, x[1]);
        sgpr_step<2>(acc, g0, g1, x[2]);
        sgpr_step<3>(acc, g0, g1, x[3]);
      }
      if (FLR_REF_S_ABL != 1) ldj(x);
    }
  };
  for (int64_t b0 = 0; b0 < NB; b0 += QD)
    static_for(
        [&](auto P) {
          constexpr int p = decltype(P)::value;
          trip(std::integral_constant<int, 2 * BT * p>{}, xa, xb);
          trip(std::integral_constant<int, 2 * BT * p + BT>{}, xb, xa);
        },
        std::make_integer_sequence<int, QD / (2 * BT)>{});
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int r = 0; r < NI; ++r) {
    const int i = i0 + r;
    if (i < j && j < K) A[((int64_t)c * K + i) * K + j] = acc[r];
  }
}

// The workgroup form (default for the throughput path): 4 waves = 4 I blocks
// (32 rows) of one J block share its x_j through LDS.  Measured, the one-wave
// form above is bound by its x_j stream, not its arithmetic (without any chain
// arithmetic it ran 21.5 of 22.1 ms at K = 512, P = 2M, profiles/r6_sgpr/): its
// waves drift apart, the L2 no longer serves one J block to the many waves that
// read it, and the chip streams ~7.7 TB/s.  Here a 4-wave workgroup stages each
// chunk of WCB blocks of its J rows (WCB KB) once by LDS-DMA into a ring of WNS
// stages — one barrier per chunk keeps its waves together — and each lane reads
// its row's 16-B piece per block with ds_read_b128 (1 KB per wave: ~4 LDS cycles
// per 64 VALU).  x_i as above (SGPR operands, one block ahead).
constexpr int WCB = 8;  // 4-step blocks per staged chunk (WCB KB: one 1-KB DMA per block)
constexpr int WNS = 4;  // ring stages
static_assert(WCB % 8 == 0 && (XC_GROUP / 4) % WCB == 0, "two DMAs per wave per chunk; whole chunks per segment");
__host__ __device__ inline int wg_groups(int q, int K) { return (quad_ni(q, K, 8) + 3) / 4; }
inline int wg_ntiles(int K) {
  int n = 0;
  for (int q = 0; q * QJ < K; ++q) n += wg_groups(q, K);
  return n;
}
// the step with x_i in VGPRs (XL: every lane holds the same value, read from LDS)
template <int E>
__device__ __forceinline__ void vgpr_step(float (&acc)[8], const f32x4 (&xi)[8], float xjv) {
  float t0, t1;
  asm volatile(
      "v_sub_f32 %[t0], %[s0], %[x]\n\t"
      "v_sub_f32 %[t1], %[s1], %[x]\n\t"
      "v_fmac_f32 %[a0], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s2], %[x]\n\t"
      "v_fmac_f32 %[a1], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s3], %[x]\n\t"
      "v_fmac_f32 %[a2], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s4], %[x]\n\t"
      "v_fmac_f32 %[a3], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s5], %[x]\n\t"
      "v_fmac_f32 %[a4], %[t0], %[t0]\n\t"
      "v_sub_f32 %[t0], %[s6], %[x]\n\t"
      "v_fmac_f32 %[a5], %[t1], %[t1]\n\t"
      "v_sub_f32 %[t1], %[s7], %[x]\n\t"
      "v_fmac_f32 %[a6], %[t0], %[t0]\n\t"
      "v_fmac_f32 %[a7], %[t1], %[t1]\n\t"
      : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]),
        [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7]), [t0] "=&v"(t0), [t1] "=&v"(t1)
      : [s0] "v"(xi[0][E]), [s1] "v"(xi[1][E]), [s2] "v"(xi[2][E]), [s3] "v"(xi[3][E]), [s4] "v"(xi[4][E]),
        [s5] "v"(xi[5][E]), [s6] "v"(xi[6][E]), [s7] "v"(xi[7][E]), [x] "v"(xjv));
}

// XL: x_i staged through LDS too (the group's 32 I rows, 512 B per block) and
// read as broadcast ds_read_b128 into VGPR operands — no scalar loads (their
// round trip, ~600 cycles under load, bounded the SGPR form: one block's
// compute is all a scalar prefetch can hide, as they complete out of order)
template <bool XL>
__global__ __launch_bounds__(256, 3) void ref_chain_w_kernel(const float* __restrict__ Xq, int64_t NB, int64_t Kp,
                                                             int K, int first, float* __restrict__ A) {
  constexpr int SJ = WCB * QJ * 16;              // x_j bytes per stage
  constexpr int SI = XL ? WCB * 32 * 16 : 0;     // x_i bytes per stage
  constexpr int NDMA = XL ? 3 : 2;               // DMA instructions per wave per chunk
  __shared__ __attribute__((aligned(16))) float xs[WNS * (SJ + SI) / 4];  // [stage]{[block][row][4] x_j, x_i}
  const int c = (int)(blockIdx.x & 7), lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform (SGPR operands)
  int t = (int)(blockIdx.x >> 3), q = 0;
  for (int n = wg_groups(0, K); t >= n; n = wg_groups(q, K)) {
    t -= n;
    ++q;
  }
  // this wave's I block; past the J block's last one (a ragged group) the wave
  // still stages and meets every barrier, and stores nothing
  const int a = 4 * t + wave, na = quad_ni(q, K, 8);
  const bool live = a < na;
  const int i0 = 8 * (live ? a : na - 1), j = QJ * q + lane;
  const float* __restrict__ base = Xq + (int64_t)c * NB * Kp * 4;
  float acc[8];
  if (first || !live) {
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = 0.f;
  } else {  // asm loads and a full wait: no compiler-tracked load reaches into the loop
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float* ap = A + ((int64_t)c * K + i0 + r) * K + (j < K ? j : K - 1);
      asm volatile("global_load_dword %0, %1, off" : "=v"(acc[r]) : "v"(ap) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
                   "+v"(acc[7])
                 :
                 : "memory");
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = (i0 + r < j && j < K) ? acc[r] : 0.f;
  }
  const int64_t bb = Kp * 16;   // bytes per block
  const int64_t nch = NB / WCB;  // chunks in the segment
  // staging: wave w moves x_j blocks 2w, 2w + 1 of a chunk (the J block's 64
  // rows, 1 KB contiguous each) and (XL) the x_i of the same two blocks (the
  // group's 32 rows, 512 B each: lanes 0-31 block 2w, 32-63 block 2w + 1)
  const char* jsrc = reinterpret_cast<const char*>(base) + (int64_t)(QJ * q) * 16;
  const char* isrc = reinterpret_cast<const char*>(base) + (int64_t)(32 * t) * 16;
  const uint32_t vj = (uint32_t)lane * 16;
  const uint32_t vi = (uint32_t)(((lane >> 5) * Kp + (lane & 31)) * 16);
  const uint32_t lds0 = (uint32_t)(uintptr_t)xs;
  auto dma = [&](int64_t ch) {
    const int64_t cc = ch < nch ? ch : nch - 1;  // past the last chunk: the last again (nothing reads it)
    const uint32_t sb = lds0 + (uint32_t)((int)(ch % WNS) * (SJ + SI));
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int blk = 2 * wave + v;
      const char* src = jsrc + (cc * WCB + blk) * bb;
      const uint32_t m = sb + (uint32_t)(blk * QJ * 16);
      // M0 written in the statement that reads it; nothing else in the kernel reads M0
      asm volatile("s_mov_b32 m0, %[m]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[v], %[s] offset:0"
                   :
                   : [m] "s"(m), [v] "v"(vj), [s] "s"(src)
                   : "memory");
    }
    if constexpr (XL) {
      const char* src = isrc + (cc * WCB + 2 * wave) * bb;
      const uint32_t m = sb + SJ + (uint32_t)(2 * wave * 32 * 16);
      asm volatile("s_mov_b32 m0, %[m]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[v], %[s] offset:0"
                   :
                   : [m] "s"(m), [v] "v"(vi), [s] "s"(src)
                   : "memory");
    }
  };
  const char* pin = reinterpret_cast<const char*>(base) + (int64_t)i0 * 16;  // the next x_i block (SGPR form)
  auto ldi = [&](i32x16& lo, i32x16& hi) {
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40" : "=s"(lo), "=s"(hi) : "s"(pin) : "memory");
    pin += bb;
    asm volatile("" : "+s"(pin));
  };
  auto rdj = [&](f32x4& x, uint32_t addr, auto U) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x) : "v"(addr), "n"(decltype(U)::value * QJ * 16) : "memory");
  };
  // XL: row r of this wave's 8 at byte 16 (32 u + 8 wave + r) of the stage's x_i
  // (the same address in every lane: a broadcast)
  auto rdi = [&](f32x4(&x)[8], uint32_t addr, auto U) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(x[r])
                   : "v"(addr), "n"(SJ + decltype(U)::value * 32 * 16 + 16 * r)
                   : "memory");
  };
  i32x16 al, ah, bl, bh;
  f32x4 j0, j1, ia[8], ib[8];
#pragma unroll
  for (int p = 0; p < WNS - 1; ++p) dma(p);
  if constexpr (!XL) ldi(al, ah);
  // block u of chunk ch: x_i(b) and x_j(b) landed; x_i(b + 1) issued (the SGPR
  // form: always; XL: inside the chunk, like x_j(b + 1)); the block's 4 steps
  auto body = [&](auto U, uint32_t sbase, uint32_t ibase, f32x4& xc, f32x4& xn, const i32x16& cl,
                  const i32x16& ch_, i32x16& nl, i32x16& nh, f32x4(&ic)[8], f32x4(&in)[8]) {
    constexpr int u = decltype(U)::value;
    if constexpr (XL) {
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(xc), "+v"(ic[0]), "+v"(ic[1]), "+v"(ic[2]), "+v"(ic[3]), "+v"(ic[4]), "+v"(ic[5]),
                     "+v"(ic[6]), "+v"(ic[7])
                   :
                   : "memory");
      if constexpr (u + 1 < WCB) {
        rdj(xn, sbase, std::integral_constant<int, u + 1>{});
        rdi(in, ibase, std::integral_constant<int, u + 1>{});
      }
      vgpr_step<0>(acc, ic, xc[0]);
      vgpr_step<1>(acc, ic, xc[1]);
      vgpr_step<2>(acc, ic, xc[2]);
      vgpr_step<3>(acc, ic, xc[3]);
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xc) : : "memory");
      ldi(nl, nh);
      if constexpr (u + 1 < WCB) rdj(xn, sbase, std::integral_constant<int, u + 1>{});
      sgpr_step<0>(acc, cl, ch_, xc[0]);
      sgpr_step<1>(acc, cl, ch_, xc[1]);
      sgpr_step<2>(acc, cl, ch_, xc[2]);
      sgpr_step<3>(acc, cl, ch_, xc[3]);
    }
  };
  static_assert(WCB % 2 == 0, "x_i / x_j ping-pong");
  for (int64_t ch = 0; ch < nch; ++ch) {
    // this wave's DMAs of chunk ch landed (the younger ones: chunks ch + 1 ..
    // ch + WNS - 2), then every wave's (the barrier), which also marks every
    // wave done with chunk ch - 1, whose stage the next DMA refills
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NDMA * (WNS - 2)) : "memory");
    dma(ch + WNS - 1);
    const uint32_t st = lds0 + (uint32_t)((int)(ch % WNS) * (SJ + SI));
    const uint32_t sbase = st + vj;
    const uint32_t ibase = st + (uint32_t)(wave * 8 * 16);  // uniform: a broadcast address
    rdj(j0, sbase, std::integral_constant<int, 0>{});
    if constexpr (XL) rdi(ia, ibase, std::integral_constant<int, 0>{});
    static_for(
        [&](auto P) {
          constexpr int p = decltype(P)::value;
          body(std::integral_constant<int, 2 * p>{}, sbase, ibase, j0, j1, al, ah, bl, bh, ia, ib);
          body(std::integral_constant<int, 2 * p + 1>{}, sbase, ibase, j1, j0, bl, bh, al, ah, ib, ia);
        },
        std::make_integer_sequence<int, WCB / 2>{});
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (live) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int i = i0 + r;
      if (i < j && j < K) A[((int64_t)c * K + i) * K + j] = acc[r];
    }
  }
}

// the throughput form: every pair in one call, no tap-major blocks, K >= 480
// (at least two waves per SIMD); FLR_REF_SGPR=0 off, =1 from K > 64
inline bool use_quad(int64_t K, int64_t ntaps, bool all_tiles) {
  if (!all_tiles || ntaps > 0 || K <= QJ) return false;
  const char* e = flr::knob("FLR_REF_SGPR");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return K >= 480;
}

// D[i][j] = D[j][i] for the pairs of tiles [t0, t1): chains summed 0..7 in
// order, the tail, correctly rounded sqrt; the other pairs 0 (the ranks' parts
// are then summed: exactly one rank holds each pair), the diagonal 0.
// the columns of the tail coordinates 8R .. P-1 (at most 7)
struct TailCols {
  int64_t c[8];
};
__global__ void ref_finish_kernel(const float* __restrict__ A, int chains, const float* __restrict__ X,
                                  const TailCols tc, int K, int64_t P, int64_t ldx, int64_t R, int t0, int t1,
                                  double* __restrict__ D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)K * K) return;
  const int i = (int)(idx / K), j = (int)(idx % K);
  if (i == j) {
    D[idx] = 0.0;
    return;
  }
  if (i > j) return;
  const int tile = tile_of_pair(i, j);
  double v = 0.0;
  if (tile >= t0 && tile < t1) {
    float s = 0.f;
    if (chains) {
      const int64_t kk = (int64_t)K * K, p = (int64_t)i * K + j;
      s = A[p];
#pragma unroll
      for (int c = 1; c < 8; ++c) s = add_rn(s, A[c * kk + p]);
    }
    const float* xi = X + (int64_t)i * ldx;
    const float* xj = X + (int64_t)j * ldx;
    int64_t t = R * 8;
    auto col = [&](int64_t c) { return tc.c[c - R * 8]; };
    if (t + 4 <= P)
      for (const int64_t e = t + 4; t < e; ++t) {
        const float d = xi[col(t)] - xj[col(t)];
        s = add_rn(s, mul_rn(d, d));
      }
    for (; t < P; ++t) {
      const float d = xi[col(t)] - xj[col(t)];
      s = __builtin_fmaf(d, d, s);
    }
    v = (double)sqrt_rn(s);
  }
  D[(int64_t)i * K + j] = v;
  D[(int64_t)j * K + i] = v;
}

// workspace layout: A [8][K][K] fp32 (256-B aligned), then the chain-major segment
inline size_t a_bytes(int64_t K) { return align_up((size_t)(8 * K * K) * 4, 256); }

}  // namespace pwref
}  // namespace flr

using namespace flr;
using namespace flr::pwref;

extern "C" size_t flr_pairwise_l2_reference_workspace(int64_t K, int64_t P) {
  if (K < 1 || P < 0) return 0;
  const int64_t R = P / 8;
  size_t n = a_bytes(K);
  if (K < 2 || R == 0) return n;
  const int64_t Rc = (R + XC_GROUP - 1) / XC_GROUP * XC_GROUP;
  // the throughput form's segments hold K rounded up to 64 rows (use_quad)
  const int64_t per_step = (K > QJ ? quad_rows(K) : K) * 8 * 4;
  const int64_t nseg = (per_step * Rc + XC_CAP - 1) / XC_CAP;
  const int64_t Rs = ((R + nseg - 1) / nseg + XC_GROUP - 1) / XC_GROUP * XC_GROUP;
  return n + (size_t)(per_step * Rs + XC_SLACK + (K > QJ ? quad_slack(K) : 0));
}

extern "C" int flr_pairwise_l2_reference_tiles(int64_t K) {
  if (K < 2 || K > (1 << 15)) return 0;
  return ntiles_of((int)K);
}

// The transpose's waves for segment [r0, r0 + steps): every wave not inside
// one tap block (the blocks ascending and disjoint, checked by the caller).
// Past WaveRuns::MAX runs the shortest gaps are bridged (those waves then
// also run; the tap kernel, launched after, rewrites their coordinates).
static WaveRuns wave_runs(const int64_t* taps, int64_t ntaps, int64_t r0, int64_t steps) {
  const int64_t nw = (steps + TW - 1) / TW;
  std::vector<std::pair<int64_t, int64_t>> v;  // [first, last + 1) wave runs
  int64_t b = 0;
  for (int64_t w = 0; w < nw; ++w) {
    const int64_t u0 = 8 * (r0 + w * TW), u1 = u0 + 8 * TW;
    while (b < ntaps && taps[4 * b] + taps[4 * b + 1] * taps[4 * b + 2] * taps[4 * b + 3] <= u0) ++b;
    const bool inside = b < ntaps && u0 >= taps[4 * b] &&
                        u1 <= taps[4 * b] + taps[4 * b + 1] * taps[4 * b + 2] * taps[4 * b + 3];
    if (inside) continue;
    if (!v.empty() && v.back().second == w)
      v.back().second = w + 1;
    else
      v.push_back({w, w + 1});
  }
  while ((int)v.size() > WaveRuns::MAX) {  // bridge the shortest gap
    size_t best = 1;
    for (size_t i = 2; i < v.size(); ++i)
      if (v[i].first - v[i - 1].second < v[best].first - v[best - 1].second) best = i;
    v[best - 1].second = v[best].second;
    v.erase(v.begin() + (int64_t)best);
  }
  WaveRuns wr;
  wr.n = (int)v.size();
  wr.pre[0] = 0;
  for (int i = 0; i < wr.n; ++i) {
    wr.w0[i] = v[i].first;
    wr.pre[i + 1] = wr.pre[i] + (v[i].second - v[i].first);
  }
  return wr;
}

// The chains of tiles [t0, t1) over `steps` chain steps of X (coordinates
// 0 .. 8 steps - 1 of each row), continuing the sums in A (first: from 0):
// per segment the chain-major transpose (skipping the tap-major blocks), the
// tap blocks' rewrite, the chain kernel.
static int run_chains(const float* X, int64_t K, int64_t steps_total, int64_t ldx, const int64_t* taps, int64_t ntaps,
                      const uint64_t* dead, const float* gdead, int64_t nneg, int first, float* A, void* ws,
                      size_t ws_bytes, int t0, int t1, hipStream_t st, hipEvent_t after_rewrite = nullptr) {
  const size_t na = a_bytes(K);
  if (ws_bytes < na) return FLR_ERR_WORKSPACE;
  const int64_t R = steps_total;
  if (ws_bytes < na + (size_t)XC_SLACK) return FLR_ERR_WORKSPACE;
  if (use_quad(K, ntaps, t0 == 0 && t1 == ntiles_of((int)K))) {  // the throughput form (Xq segments)
    const int64_t Kp = quad_rows(K), qstep = Kp * 8 * 4;
    const char* rows_knob = flr::knob("FLR_REF_SGPR_ROWS");  // 4 (default) or 8 I rows per wave
    const bool eight = rows_knob && rows_knob[0] == '8';
    const char* form_knob = flr::knob("FLR_REF_SGPR_FORM");  // "wave": the one-wave forms (A/B)
    const bool wg = !(form_knob && form_knob[0] == 'w' && form_knob[1] == 'a');
    const bool xl = !(form_knob && form_knob[0] == 's');  // "sgpr": the workgroup form with scalar x_i
    if (ws_bytes < na + (size_t)(XC_SLACK + quad_slack(K))) return FLR_ERR_WORKSPACE;
    const int64_t cap =
        (int64_t)((ws_bytes - na - XC_SLACK - quad_slack(K)) / (size_t)qstep) / XC_GROUP * XC_GROUP;
    if (cap < XC_GROUP) return FLR_ERR_WORKSPACE;
    const int64_t nseg = (R + cap - 1) / cap;
    const int64_t Rs = ((R + nseg - 1) / nseg + XC_GROUP - 1) / XC_GROUP * XC_GROUP;  // <= cap
    float* Xq = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + na);
    for (int64_t seg = 0; seg < nseg; ++seg) {
      const int64_t r0 = seg * Rs, steps = (R - r0 < Rs) ? R - r0 : Rs;
      if (steps <= 0) break;
      const int64_t NB = (steps + XC_GROUP - 1) / XC_GROUP * XC_GROUP / 4;
      hipLaunchKernelGGL(quad_transpose_kernel, dim3((unsigned)(NB / QTB), (unsigned)((K + QTB - 1) / QTB)), dim3(256),
                         0, st, X, ldx, (int)K, r0, steps, NB, Kp, Xq);
      int rc = launch_status("quad_transpose_kernel");
      if (rc != FLR_OK) return rc;
      if (after_rewrite && seg == nseg - 1 && hipEventRecord(after_rewrite, st) != hipSuccess) return FLR_ERR_HIP;
      const int fst = (first && seg == 0) ? 1 : 0;
      if (wg && xl)
        hipLaunchKernelGGL(ref_chain_w_kernel<true>, dim3((unsigned)(8 * wg_ntiles((int)K))), dim3(256), 0, st, Xq, NB,
                           Kp, (int)K, fst, A);
      else if (wg)
        hipLaunchKernelGGL(ref_chain_w_kernel<false>, dim3((unsigned)(8 * wg_ntiles((int)K))), dim3(256), 0, st, Xq,
                           NB, Kp, (int)K, fst, A);
      else if (eight)
        hipLaunchKernelGGL((ref_chain_s_kernel<8, 1>), dim3((unsigned)(8 * quad_ntiles((int)K, 8))), dim3(64), 0, st,
                           Xq, NB, Kp, (int)K, fst, A);
      else
        hipLaunchKernelGGL((ref_chain_s_kernel<4, 2>), dim3((unsigned)(8 * quad_ntiles((int)K, 4))), dim3(64), 0, st,
                           Xq, NB, Kp, (int)K, fst, A);
      if ((rc = launch_status("ref_chain_s_kernel")) != FLR_OK) return rc;
    }
    return FLR_OK;
  }
  const int64_t per_step = K * 8 * 4;
  const int64_t ldc = (int64_t)((ws_bytes - na - XC_SLACK) / (size_t)per_step) / XC_GROUP * XC_GROUP;
  if (ldc < XC_GROUP) return FLR_ERR_WORKSPACE;
  const int64_t nseg = (R + ldc - 1) / ldc;
  const int64_t Rs = ((R + nseg - 1) / nseg + XC_GROUP - 1) / XC_GROUP * XC_GROUP;  // <= ldc
  float* Xc = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + na);
  for (int64_t seg = 0; seg < nseg; ++seg) {
    const int64_t r0 = seg * Rs, steps = (R - r0 < Rs) ? R - r0 : Rs;
    if (steps <= 0) break;
    const WaveRuns runs = wave_runs(taps, ntaps, r0, steps);
    int rc = FLR_OK;
    if (runs.pre[runs.n] > 0) {
      hipLaunchKernelGGL(chain_transpose_kernel, dim3((unsigned)((runs.pre[runs.n] + 3) / 4), (unsigned)K), dim3(256),
                         0, st, X, ldx, r0, steps, ldc, Xc, runs);
      if ((rc = launch_status("chain_transpose_kernel")) != FLR_OK) return rc;
    }
    for (int64_t b = 0; b < ntaps; ++b) {  // the tap-major blocks of this segment, rewritten
      const int64_t off = taps[4 * b], co = taps[4 * b + 1], ci = taps[4 * b + 2], kk = taps[4 * b + 3];
      if (off + co * ci * kk <= 8 * r0 || off >= 8 * (r0 + steps)) continue;
      const int64_t tiles = (co + TAP_CO - 1) / TAP_CO * ((ci + TAP_ROWS / kk - 1) / (TAP_ROWS / kk));
      const bool vec = off % 4 == 0 && co % TAP_CO == 0;  // 16-B aligned rows, full 32-channel tiles
      auto kern = kk == 9 ? (vec ? tap_chain_kernel<9, true> : tap_chain_kernel<9, false>)
                : kk == 1 ? (vec ? tap_chain_kernel<1, true> : tap_chain_kernel<1, false>)
                          : (vec ? tap_chain_kernel<0, true> : tap_chain_kernel<0, false>);
      const uint64_t dm = dead ? dead[b] : 0;
      hipLaunchKernelGGL(kern, dim3((unsigned)tiles, (unsigned)K), dim3(256), 0, st, X, ldx, off, (int)co, (int)ci,
                         (int)kk, r0, steps, ldc, Xc, dm ? gdead : nullptr, dm, (int)std::min<int64_t>(nneg, K));
      if ((rc = launch_status("tap_chain_kernel")) != FLR_OK) return rc;
    }
    const int64_t padded = (steps + XC_GROUP - 1) / XC_GROUP * XC_GROUP;  // <= Rs <= ldc
    if (padded > steps &&
        hipMemset2DAsync(Xc + steps, (size_t)ldc * 4, 0, (size_t)(padded - steps) * 4, (size_t)(K * 8), st) != hipSuccess)
      return FLR_ERR_HIP;
    // every read of X done (the last segment's rewrite): the caller may now
    // write X's dead-tap slabs beside the chains (flr_pairwise_l2_reference_tap_dead)
    if (after_rewrite && seg == nseg - 1 && hipEventRecord(after_rewrite, st) != hipSuccess) return FLR_ERR_HIP;
    if (t0 == 0 && t1 == ntiles_of((int)K) && use_two_chains(K)) {  // every pair: the two-chain tiles
      hipLaunchKernelGGL(ref_chain2_kernel, dim3(8 * ntiles2_of((int)K)), dim3(64), 0, st, Xc, ldc, (int)K, steps,
                         (first && seg == 0) ? 1 : 0, A);
      rc = launch_status("ref_chain2_kernel");
    } else {
      hipLaunchKernelGGL(ref_chain_kernel, dim3(8 * (t1 - t0)), dim3(64), 0, st, Xc, ldc, (int)K, steps, t0,
                         (first && seg == 0) ? 1 : 0, A);
      rc = launch_status("ref_chain_kernel");
    }
    if (rc != FLR_OK) return rc;
  }
  return FLR_OK;
}

static int check_rows(const float* X, int64_t K, int64_t n, int64_t ldx) {
  // 16-B loads of the rows
  if (K > 1 && n >= 8 && (((reinterpret_cast<uintptr_t>(X) & 15) != 0) || (ldx % 4) != 0)) return FLR_ERR_ARG;
  return FLR_OK;
}

extern "C" int flr_pairwise_l2_reference_tap_dead(const float* X, int64_t K, int64_t P, int64_t ldx,
                                                  const int64_t* taps, int64_t ntaps, const uint64_t* dead,
                                                  const float* gdead, int64_t nneg, double* D, void* ws,
                                                  size_t ws_bytes, int64_t part, int64_t nparts, void* after_rewrite,
                                                  void* stream) {
  if (K < 1 || P < 0 || ldx < P || !D || (K > 1 && P > 0 && !X) || nparts < 1 || part < 0 || part >= nparts)
    return FLR_ERR_ARG;
  if (K > (1 << 15)) return FLR_ERR_UNSUPPORTED;
  if (ntaps < 0 || (ntaps > 0 && !taps) || nneg < 0) return FLR_ERR_ARG;
  bool any_dead = false;
  for (int64_t b = 0; dead && b < ntaps; ++b) {  // bit t names tap t < min(KK, 64)
    if (taps[4 * b + 3] < 64 && (dead[b] >> taps[4 * b + 3]) != 0) return FLR_ERR_ARG;
    any_dead |= dead[b] != 0;
  }
  if (any_dead && !gdead) return FLR_ERR_ARG;
  // tap-major blocks: {off, Cout, Cin, KK}, inside [0, P), ascending, disjoint
  for (int64_t b = 0, end = 0; b < ntaps; ++b) {
    const int64_t off = taps[4 * b], co = taps[4 * b + 1], ci = taps[4 * b + 2], kk = taps[4 * b + 3];
    if (off < end || co < 1 || ci < 1 || kk < 1 || kk > TAP_ROWS || co > INT32_MAX || ci > INT32_MAX ||
        off + co * ci * kk > P)
      return FLR_ERR_ARG;
    end = off + co * ci * kk;
  }
  int rc = check_rows(X, K, P, ldx);
  if (rc != FLR_OK) return rc;
  hipStream_t st = as_stream(stream);
  const int64_t R = P / 8;
  if (K > 1 && R > 0 && (!ws || (reinterpret_cast<uintptr_t>(ws) & 255) != 0)) return FLR_ERR_WORKSPACE;
  const int ntiles = K > 1 ? ntiles_of((int)K) : 0;
  const int t0 = (int)(part * ntiles / nparts), t1 = (int)((part + 1) * ntiles / nparts);
  float* A = reinterpret_cast<float*>(ws);
  if (K > 1 && R > 0 && t1 > t0 &&
      (rc = run_chains(X, K, R, ldx, taps, ntaps, any_dead ? dead : nullptr, gdead, nneg, 1, A, ws, ws_bytes, t0, t1,
                       st, static_cast<hipEvent_t>(after_rewrite))) != FLR_OK)
    return rc;
  // no chains ran (K < 2, no full step, no tiles here): X's dead slabs are free now
  if (after_rewrite && !(K > 1 && R > 0 && t1 > t0) &&
      hipEventRecord(static_cast<hipEvent_t>(after_rewrite), st) != hipSuccess)
    return FLR_ERR_HIP;
  // the tail coordinates' columns (identity outside the tap-major blocks)
  TailCols tc;
  for (int64_t u = 8 * R; u < 8 * R + 8; ++u) {
    int64_t c = u;
    for (int64_t b = 0; b < ntaps && u < P; ++b) {
      const int64_t off = taps[4 * b], co = taps[4 * b + 1], ci = taps[4 * b + 2], kk = taps[4 * b + 3];
      if (u < off || u >= off + co * ci * kk) continue;
      const int64_t rel = u - off, o = rel / (ci * kk), i = (rel / kk) % ci, t = rel % kk;
      c = off + (t * ci + i) * co + o;
    }
    tc.c[u - 8 * R] = c;
  }
  // the finish kernel reads the tail columns from X: none of them may be a dead tap
  for (int64_t u = 8 * R; any_dead && u < P; ++u)
    for (int64_t b = 0; b < ntaps; ++b) {
      const int64_t off = taps[4 * b], co = taps[4 * b + 1], ci = taps[4 * b + 2], kk = taps[4 * b + 3];
      if (u < off || u >= off + co * ci * kk) continue;
      const int64_t t = (u - off) % kk;
      if (t < 64 && ((dead[b] >> t) & 1)) return FLR_ERR_ARG;
    }
  const int64_t kk = K * K;
  hipLaunchKernelGGL(ref_finish_kernel, dim3((unsigned)((kk + 255) / 256)), dim3(256), 0, st, A, R > 0 ? 1 : 0, X, tc,
                     (int)K, P, ldx, R, t0, t1, D);
  return launch_status("ref_finish_kernel");
}

extern "C" int flr_pairwise_l2_reference_tap(const float* X, int64_t K, int64_t P, int64_t ldx,
                                             const int64_t* taps, int64_t ntaps, double* D, void* ws, size_t ws_bytes,
                                             int64_t part, int64_t nparts, void* stream) {
  return flr_pairwise_l2_reference_tap_dead(X, K, P, ldx, taps, ntaps, nullptr, nullptr, 0, D, ws, ws_bytes, part,
                                            nparts, nullptr, stream);
}

extern "C" int flr_pairwise_l2_reference(const float* X, int64_t K, int64_t P, int64_t ldx, double* D, void* ws,
                                         size_t ws_bytes, int64_t part, int64_t nparts, void* stream) {
  return flr_pairwise_l2_reference_tap(X, K, P, ldx, nullptr, 0, D, ws, ws_bytes, part, nparts, stream);
}

extern "C" int flr_pairwise_l2_reference_partial_tap(const float* X, int64_t K, int64_t steps, int64_t ldx,
                                                     const int64_t* taps, int64_t ntaps, int first, void* ws,
                                                     size_t ws_bytes, void* stream) {
  if (K < 1 || steps < 0 || ldx < 8 * steps || (K > 1 && steps > 0 && !X)) return FLR_ERR_ARG;
  if (ntaps < 0 || (ntaps > 0 && !taps)) return FLR_ERR_ARG;
  for (int64_t b = 0, end = 0; b < ntaps; ++b) {  // ascending, disjoint, wholly inside the slice's chain steps
    const int64_t off = taps[4 * b], co = taps[4 * b + 1], ci = taps[4 * b + 2], kk = taps[4 * b + 3];
    if (off < end || co < 1 || ci < 1 || kk < 1 || kk > TAP_ROWS || co > INT32_MAX || ci > INT32_MAX ||
        off + co * ci * kk > 8 * steps)
      return FLR_ERR_ARG;
    end = off + co * ci * kk;
  }
  if (K > (1 << 15)) return FLR_ERR_UNSUPPORTED;
  int rc = check_rows(X, K, 8 * steps, ldx);
  if (rc != FLR_OK) return rc;
  if (!ws || (reinterpret_cast<uintptr_t>(ws) & 255) != 0 || ws_bytes < a_bytes(K)) return FLR_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  float* A = reinterpret_cast<float*>(ws);
  if (K < 2) return FLR_OK;
  if (steps == 0) {  // nothing to add; a first call still starts every chain at 0
    if (first && hipMemsetAsync(A, 0, (size_t)8 * K * K * 4, st) != hipSuccess)
      return launch_status("reference distances: zero the chains");
    return FLR_OK;
  }
  return run_chains(X, K, steps, ldx, taps, ntaps, nullptr, nullptr, 0, first, A, ws, ws_bytes, 0, ntiles_of((int)K),
                    st);
}

extern "C" int flr_pairwise_l2_reference_partial(const float* X, int64_t K, int64_t steps, int64_t ldx, int first,
                                                 void* ws, size_t ws_bytes, void* stream) {
  return flr_pairwise_l2_reference_partial_tap(X, K, steps, ldx, nullptr, 0, first, ws, ws_bytes, stream);
}

extern "C" int flr_pairwise_l2_reference_finish(const float* Xtail, int64_t K, int64_t ntail, int64_t ldx,
                                                int chains, const void* ws, double* D, void* stream) {
  if (K < 1 || ntail < 0 || ntail > 7 || ldx < ntail || !D || (K > 1 && ntail > 0 && !Xtail) ||
      (K > 1 && chains && !ws))
    return FLR_ERR_ARG;
  if (K > (1 << 15)) return FLR_ERR_UNSUPPORTED;
  TailCols tc;
  for (int u = 0; u < 8; ++u) tc.c[u] = u;
  const int64_t kk = K * K;
  hipLaunchKernelGGL(ref_finish_kernel, dim3((unsigned)((kk + 255) / 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float*>(ws), chains ? 1 : 0, Xtail, tc, (int)K, ntail, ldx, (int64_t)0, 0,
                     K > 1 ? ntiles_of((int)K) : 0, D);
  return launch_status("ref_finish_kernel");
}
