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
  const int64_t per_step = K * 8 * 4;
  const int64_t nseg = (per_step * Rc + XC_CAP - 1) / XC_CAP;
  const int64_t Rs = ((R + nseg - 1) / nseg + XC_GROUP - 1) / XC_GROUP * XC_GROUP;
  return n + (size_t)(per_step * Rs + XC_SLACK);
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
  const int64_t per_step = K * 8 * 4;
  if (ws_bytes < na + (size_t)XC_SLACK) return FLR_ERR_WORKSPACE;
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
