// a9 — Krum pairwise l2 distances on gfx950.
//
// Replaces KrumDefense._compute_distances (src/defenses/krum.py:73-99), which
// loops over K(K-1)/2 pairs calling torch.norm(flat_i - flat_j).item().
//
// Engine (MFMA path, flr_pairwise_l2):
//   ||x_i - x_j||^2 = G_ii + G_jj - 2 G_ij with G the Gram matrix of the
//   CENTRED client matrix y = x - x_pivot (distances are translation
//   invariant, so subtracting any per-coordinate constant is exact; centring
//   removes the cancellation that makes a raw-weight Gram useless).  The pivot
//   is the medoid of a strided 2048-coordinate sample (prepass kernels below):
//   a central client, robust to < 50 % outliers, so benign pairs keep a
//   cancellation factor (|y_i|^2+|y_j|^2)/|y_i-y_j|^2 of about 2.  y is split into bf16 hi + lo
//   (y = hi + lo + O(2^-17 |y|)) and G_ij = sum (hi_i+lo_i)(hi_j+lo_j) is
//   formed by four v_mfma_f32_32x32x16_bf16 products (each bf16*bf16 product is
//   exact in fp32, accumulation fp32).  The diagonal G_ii comes from the same
//   hi+lo values on the VALU.  One workgroup streams a contiguous coordinate
//   segment of ALL rows of its group once from HBM (LDS-DMA, XOR-swizzled
//   256-B rows), so the kernel is HBM-bound: bytes = 4*K*P (+ partials).
//   Per-segment fp32 partials are reduced in fixed order in fp64.
//
// Direct path (flr_pairwise_l2_direct): exact fp32 differences on the VALU,
// one 32x32 client-block pair per workgroup.  Used to cross-check the MFMA
// path; VALU-bound (2 ops per pair-coordinate).
#include "flr_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace flr {
namespace pw {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int CW = 64;          // coordinates per chunk = 256 B per row
constexpr int THREADS = 256;    // 4 waves; wave w owns k-step w of the chunk
constexpr int SUPER = 128;      // rows of a diagonal group (4 client blocks)
constexpr int REC_TILES = 16;   // max tiles per group (the K > 128 cross groups: 4 x 4)
constexpr int REC_DIAG = 8 * 32;  // max rows per group
constexpr int REC = REC_TILES * 1024 + REC_DIAG;   // floats per partial record
constexpr int MAX_SEG = 512;
// Gram workgroups per full call (all slices and groups): one round of the
// 2-per-CU residency on 256 CUs (measured: 1024 costs 3.5 % in the larger
// record write + reduction); 1/G of them per GPU when sharded.
constexpr int TARGET_BLOCKS = 512;

// Far clusters.  The centred Gram's error on a pair is about 1e-7 of
// |y_i|^2 + |y_j|^2 (y = x - x_pivot), so a pair whose distance is tiny next to
// its distance from the pivot — two members of a cluster far from the medoid,
// e.g. the sign-flipped attackers of a trained round (|x| ~ 1e3 |x_i - x_j|)
// — cancels catastrophically.  The pivot prepass estimates each pair's
// cancellation factor (|y_i|^2 + |y_j|^2) / |y_i - y_j|^2 from the exact sample
// distances; rows in any pair above COND_FLAG (lowest index first, at most
// RMAX, see below) get their mutual distances from exact fp32 differences over the
// whole vector instead ("refine" records, kept per canonical slice next to the
// Gram records so the sharded composition stays bit-identical).
// Up to RMAX flagged rows are refined (4 blocks of 32 rows: every row at
// K <= 128).  More flagged rows than that (K > 128 only, e.g. over 128
// duplicated clients) is an overflow: the pivot record counts it and every
// off-diagonal distance of that call is NaN — loud, never silently inaccurate
// (KrumDefense.publish raises on it).
constexpr int RMAX = 128;                   // refined rows per call
constexpr int RNB = RMAX / 32;              // row blocks of the refine list
constexpr int RNBP = RNB * (RNB + 1) / 2;   // block pairs (a <= b)
constexpr int RHDR = 2 + RMAX;              // refine header: count, row list, total flagged (as doubles)
constexpr int RBLK = RHDR + RMAX * RMAX;    // fp64 per slice: header + [RMAX][RMAX] sums
constexpr int PREC = 3 + RMAX;              // pivot record (int32): pivot, count, rows, total flagged
constexpr double COND_FLAG = 16.0;
constexpr int RSEG_MAX = 160;               // refine segments per slice (x 8 slices: 1280 workgroups, ~5 per CU)
constexpr int MAXK_PIVOT = 1024;

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// K > 128 cross groups: 2 blocks of super-block I against CROSS_NJ blocks of J.
// CROSS_NJ = 4 (NL = 6, 96 KB of LDS, one workgroup per CU): 56 ms at K = 512,
// P = 3.3e7.  CROSS_NJ = 2 (NL = 4, 64 KB, two per CU, so one wave's bf16 split
// can overlap the other's MFMAs) measured 67 ms: the extra split work (one block
// per tile instead of 0.75) costs more than the overlap gains.
//
// Round 3: CROSS_NI = 4 (the default): all four blocks of I against the four of
// J — one cross group per super-block pair, 16 tiles, NL = 8 (128 KB of LDS,
// one workgroup per CU).  Each chunk's bf16 split per wave then feeds 64 MFMAs
// per 8 blocks instead of 32 per 6, and the cross stage streams each pair's 256
// rows once (4x the matrix over all groups, diagonal included) instead of
// 5.5x.  FLR_GRAM_CROSS_NI=2 at build time: the 2 x 4 groups (A/B).
#ifndef FLR_GRAM_CROSS_NI
#define FLR_GRAM_CROSS_NI 4
#endif
constexpr int CROSS_NI = FLR_GRAM_CROSS_NI;
constexpr int CROSS_NJ = 4;
constexpr int CROSS_NL = CROSS_NI + CROSS_NJ;
constexpr int CROSS_PER_PAIR = (4 / CROSS_NI) * (4 / CROSS_NJ);  // cross groups per super-block pair

// Tile enumeration.  DIAG: every (a <= b) over NL loaded blocks, a-major.
// CROSS: a in {0..CROSS_NI-1} (rows of super-block I), b in {CROSS_NI..NL-1} (rows of J).
template <int NL, bool CROSS>
struct TileSet {
  static constexpr int N = CROSS ? CROSS_NI * (NL - CROSS_NI) : NL * (NL + 1) / 2;
  __host__ __device__ static constexpr int a(int t) {
    if (CROSS) return t / (NL - CROSS_NI);
    int r = t;
    for (int i = 0; i < NL; ++i) {
      if (r < NL - i) return i;
      r -= NL - i;
    }
    return -1;
  }
  __host__ __device__ static constexpr int b(int t) {
    if (CROSS) return CROSS_NI + t % (NL - CROSS_NI);
    int r = t;
    for (int i = 0; i < NL; ++i) {
      if (r < NL - i) return i + r;
      r -= NL - i;
    }
    return -1;
  }
};

__host__ __device__ inline int diag_tile_index(int nl, int a, int b) {
  // index of (a, b), a <= b, in TileSet<nl, false> order
  int t = 0;
  for (int i = 0; i < a; ++i) t += nl - i;
  return t + (b - a);
}

// LDS fragment reads as ONE asm statement (reads + lgkmcnt(0) together, outputs
// early-clobber): hipcc cannot see them, so it does not put its conservative
// vmcnt(0) (for the in-flight LDS-DMA into the other buffer) in front of them.
// Block b of the image sits at +8192 B * b; a0/a1 are the byte addresses of this
// lane's two 16-B slots in block 0.
#define FLR_DSR(n, o) "ds_read_b128 %" #n ", %" #o
template <int NL>
__device__ __forceinline__ void lds_read_blocks(uint32_t a0, uint32_t a1, f32x4 (&v)[NL][2]) {
  if constexpr (NL == 1) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]) : "v"(a0), "v"(a1) : "memory");
  } else if constexpr (NL == 2) {
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\t"
                 "ds_read_b128 %2, %4 offset:8192\n\tds_read_b128 %3, %5 offset:8192\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[1][0]), "=&v"(v[1][1]) : "v"(a0), "v"(a1) : "memory");
  } else if constexpr (NL == 3) {
    asm volatile("ds_read_b128 %0, %6\n\tds_read_b128 %1, %7\n\t"
                 "ds_read_b128 %2, %6 offset:8192\n\tds_read_b128 %3, %7 offset:8192\n\t"
                 "ds_read_b128 %4, %6 offset:16384\n\tds_read_b128 %5, %7 offset:16384\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[1][0]), "=&v"(v[1][1]), "=&v"(v[2][0]), "=&v"(v[2][1])
                 : "v"(a0), "v"(a1) : "memory");
  } else if constexpr (NL == 4) {
    asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\t"
                 "ds_read_b128 %2, %8 offset:8192\n\tds_read_b128 %3, %9 offset:8192\n\t"
                 "ds_read_b128 %4, %8 offset:16384\n\tds_read_b128 %5, %9 offset:16384\n\t"
                 "ds_read_b128 %6, %8 offset:24576\n\tds_read_b128 %7, %9 offset:24576\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[1][0]), "=&v"(v[1][1]), "=&v"(v[2][0]), "=&v"(v[2][1]),
                   "=&v"(v[3][0]), "=&v"(v[3][1])
                 : "v"(a0), "v"(a1) : "memory");
  } else if constexpr (NL == 8) {
    asm volatile("ds_read_b128 %0, %16\n\tds_read_b128 %1, %17\n\t"
                 "ds_read_b128 %2, %16 offset:8192\n\tds_read_b128 %3, %17 offset:8192\n\t"
                 "ds_read_b128 %4, %16 offset:16384\n\tds_read_b128 %5, %17 offset:16384\n\t"
                 "ds_read_b128 %6, %16 offset:24576\n\tds_read_b128 %7, %17 offset:24576\n\t"
                 "ds_read_b128 %8, %16 offset:32768\n\tds_read_b128 %9, %17 offset:32768\n\t"
                 "ds_read_b128 %10, %16 offset:40960\n\tds_read_b128 %11, %17 offset:40960\n\t"
                 "ds_read_b128 %12, %16 offset:49152\n\tds_read_b128 %13, %17 offset:49152\n\t"
                 "ds_read_b128 %14, %16 offset:57344\n\tds_read_b128 %15, %17 offset:57344\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[1][0]), "=&v"(v[1][1]), "=&v"(v[2][0]), "=&v"(v[2][1]),
                   "=&v"(v[3][0]), "=&v"(v[3][1]), "=&v"(v[4][0]), "=&v"(v[4][1]), "=&v"(v[5][0]), "=&v"(v[5][1]),
                   "=&v"(v[6][0]), "=&v"(v[6][1]), "=&v"(v[7][0]), "=&v"(v[7][1])
                 : "v"(a0), "v"(a1) : "memory");
  } else {
    static_assert(NL == 6, "unsupported block count");
    asm volatile("ds_read_b128 %0, %12\n\tds_read_b128 %1, %13\n\t"
                 "ds_read_b128 %2, %12 offset:8192\n\tds_read_b128 %3, %13 offset:8192\n\t"
                 "ds_read_b128 %4, %12 offset:16384\n\tds_read_b128 %5, %13 offset:16384\n\t"
                 "ds_read_b128 %6, %12 offset:24576\n\tds_read_b128 %7, %13 offset:24576\n\t"
                 "ds_read_b128 %8, %12 offset:32768\n\tds_read_b128 %9, %13 offset:32768\n\t"
                 "ds_read_b128 %10, %12 offset:40960\n\tds_read_b128 %11, %13 offset:40960\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[1][0]), "=&v"(v[1][1]), "=&v"(v[2][0]), "=&v"(v[2][1]),
                   "=&v"(v[3][0]), "=&v"(v[3][1]), "=&v"(v[4][0]), "=&v"(v[4][1]), "=&v"(v[5][0]), "=&v"(v[5][1])
                 : "v"(a0), "v"(a1) : "memory");
  }
}

struct GroupDesc {
  int blk[8];
};

// Group -> list of global client blocks it loads.
__device__ __forceinline__ GroupDesc group_desc(int g, int K, bool cross) {
  GroupDesc d;
  const int nb = cdiv(K, 32);
  if (K <= SUPER) {
    for (int i = 0; i < 8; ++i) d.blk[i] = i;
    (void)nb;
    return d;
  }
  const int nsb = cdiv(K, SUPER);
  if (!cross) {
    for (int i = 0; i < 8; ++i) d.blk[i] = 4 * g + i;
    return d;
  }
  const int q = (g - nsb) / CROSS_PER_PAIR, w = (g - nsb) % CROSS_PER_PAIR;
  const int hi = w / (4 / CROSS_NJ), hj = w % (4 / CROSS_NJ);
  int I = 0, rem = q;
  while (rem >= nsb - 1 - I) { rem -= nsb - 1 - I; ++I; }
  const int J = I + 1 + rem;
  for (int i = 0; i < CROSS_NI; ++i) d.blk[i] = 4 * I + CROSS_NI * hi + i;
  for (int i = 0; i < CROSS_NJ; ++i) d.blk[CROSS_NI + i] = 4 * J + CROSS_NJ * hj + i;
  return d;
}

// Canonical coordinate slices: the NCH full chunks of the whole client vector
// are cut into FLR_PW_SLICES contiguous slices, slice q = chunks
// [q*NCH/NS, (q+1)*NCH/NS).  Segment records are kept per slice and the
// slices are summed in slice order, so a GPU that holds only a few slices'
// coordinates (the coordinate-sharded exchange) computes exactly the records
// the single-GPU call computes for them.
__host__ __device__ inline int64_t slice_chunk(int64_t nch, int q) { return nch * q / FLR_PW_SLICES; }

template <int NL, bool CROSS, int TERMS, int ABLATE = 0, bool NTL = false>
// NL = 6 (96 KB of LDS) is limited to one workgroup per CU: give it the whole
// register file (with the 2-per-CU bound it spilled to scratch).
__global__ __launch_bounds__(THREADS, NL >= 6 ? 1 : 2) void gram_partials_kernel(
    const float* __restrict__ X, int K, int64_t ldx, int64_t nch_total, int q_base, int64_t chunk0,
    int group_base, int ngroups, const int* __restrict__ pivot_ptr, float* __restrict__ partials, int nseg,
    int seg_stride) {
  using TS = TileSet<NL, CROSS>;
  constexpr int NT = TS::N;
  constexpr int ROWS = 32 * NL;
  constexpr int BUF = ROWS * CW;  // floats per staging buffer
  extern __shared__ __attribute__((aligned(16))) float lds[];

  const int g = group_base + blockIdx.y;
  const int seg = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int h = lane >> 5, r = lane & 31;
  const GroupDesc gd = group_desc(g, K, CROSS);

  // Round-robin chunks within the slice: at any moment the slice's blocks read
  // one contiguous span of nseg*256 B of every row (DRAM-page friendly), not
  // nseg scattered 256-B runs.  Chunk indices are local to X (X's column 0 is
  // global chunk chunk0).
  const int q = q_base + (int)blockIdx.z;
  const int c_begin = (int)(slice_chunk(nch_total, q) - chunk0) + seg;
  const int c_end = (int)(slice_chunk(nch_total, q + 1) - chunk0);
  const int c_step = nseg;

  // Per-lane DMA source rows: instruction q of this wave covers LDS rows
  // 4*inst .. 4*inst+3, inst = wave*2*NL + q; this lane feeds row inst*4+lane/16.
  const float* src_row[2 * NL];
#pragma unroll
  for (int q = 0; q < 2 * NL; ++q) {
    const int inst = wave * 2 * NL + q;
    const int lrow = inst * 4 + (lane >> 4);
    int grow = 32 * gd.blk[lrow >> 5] + (lrow & 31);
    grow = grow < K ? grow : K - 1;  // padded rows duplicate the last client
    const int slot = (lane & 15) ^ (lrow & 15);  // XOR swizzle on the source
    src_row[q] = X + (int64_t)grow * ldx + 4 * slot;
  }

  // centre values for this lane's 8 coordinates of the wave's k-step
  const int pivot = __builtin_amdgcn_readfirstlane(*pivot_ptr);
  const float* cen_src = X + (int64_t)pivot * ldx + 16 * wave + 8 * h;
  auto load_cen = [&](int chunk, float (&c)[8]) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(cen_src + (int64_t)chunk * CW);
    const f32x4 b = *reinterpret_cast<const f32x4*>(cen_src + (int64_t)chunk * CW + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = a[j];
      c[4 + j] = b[j];
    }
  };

  auto stage = [&](int chunk, float* buf) {
#pragma unroll
    for (int q = 0; q < 2 * NL; ++q) {
      const int inst = wave * 2 * NL + q;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src_row[q] + (int64_t)chunk * CW),
          (__attribute__((address_space(3))) void*)(buf + inst * 256), 16, 0, NTL ? 2 : 0);
    }
  };

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  float dsum[NL];
#pragma unroll
  for (int b = 0; b < NL; ++b) dsum[b] = 0.f;

  int cur = 0;
  float cen[8], cen_next[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cen[j] = cen_next[j] = 0.f;
  if (c_begin < c_end) {
    stage(c_begin, lds);
    load_cen(c_begin, cen);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int c = c_begin; c < c_end; c += c_step) {
    float* buf = lds + cur * BUF;
    if (c + c_step < c_end && ABLATE != 2) {
      stage(c + c_step, lds + (cur ^ 1) * BUF);
      load_cen(c + c_step, cen_next);
    }
    if constexpr (ABLATE == 1) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      cur ^= 1;
      continue;
    }

    // ---- this wave's k-step: coordinates 16*wave + 8h + j of the chunk ----
    float raw[NL][8];
    {
      // row r of every block has the same swizzle (32*b + r = r mod 16)
      const int s0 = 4 * wave + 2 * h;
      const int p0 = s0 ^ (r & 15), p1 = (s0 + 1) ^ (r & 15);
      const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(buf) + (uint32_t)(r * CW * 4);
      f32x4 v[NL][2];
      lds_read_blocks<NL>(base + 16u * p0, base + 16u * p1, v);
#pragma unroll
      for (int b = 0; b < NL; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          raw[b][j] = v[b][0][j];
          raw[b][4 + j] = v[b][1][j];
        }
    }
    bf16x8 hi[NL], lo[NL], lo2[NL];
#pragma unroll
    for (int b = 0; b < NL; ++b) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float y = raw[b][j] - cen[j];
        const __bf16 hb = (__bf16)y;
        const float r1 = y - (float)hb;
        const __bf16 lb = (__bf16)r1;
        hi[b][j] = hb;
        lo[b][j] = lb;
        if constexpr (TERMS == 3) lo2[b][j] = (__bf16)(r1 - (float)lb);
        dsum[b] = __builtin_fmaf(y, y, dsum[b]);
      }
    }
    static_for<0, NT>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int a = TS::a(t), bb = TS::b(t);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[a], hi[bb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[a], lo[bb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo[a], hi[bb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo[a], lo[bb], acc[t], 0, 0, 0);
      if constexpr (TERMS == 3) {
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[a], lo2[bb], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo2[a], hi[bb], acc[t], 0, 0, 0);
      }
    });

    // next chunk landed (this wave's DMA + centre loads), then every wave is
    // done reading `cur` before anyone restages it.  sched_barrier keeps the
    // register-only MFMA/VALU work of this chunk in front of the wait.
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    cur ^= 1;
#pragma unroll
    for (int j = 0; j < 8; ++j) cen[j] = cen_next[j];
  }

  // ---- epilogue: reduce the 4 waves in fixed order, write the record ----
  float* rec = partials + (((int64_t)blockIdx.z * ngroups + g) * seg_stride + seg) * REC;
  float* red = lds;
  static_for<0, NT>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
#pragma unroll
    for (int e = 0; e < 16; ++e) red[wave * 1024 + e * 64 + lane] = acc[t][e];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      rec[t * 1024 + e] = ((red[e] + red[1024 + e]) + red[2048 + e]) + red[3072 + e];
    }
    __syncthreads();
  });
#pragma unroll
  for (int b = 0; b < NL; ++b) red[(wave * 2 + h) * ROWS + 32 * b + r] = dsum[b];
  __syncthreads();
  for (int row = tid; row < ROWS; row += THREADS) {
    float s = red[row];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += red[k * ROWS + row];
    rec[REC_TILES * 1024 + row] = s;
  }
}

// Sum the per-segment records of every group in fixed order (fp64), in two
// stages: stage 1 (grid.z = RSPLIT) sums a contiguous run of segments per
// split with 4 waves x 4 independent accumulators; stage 2 adds the splits.
constexpr int RSPLIT = 8;
__global__ __launch_bounds__(256) void reduce_records_kernel(const float* __restrict__ partials,
                                                              int seg_stride, int ngroups, int ngroups_diag,
                                                              int nseg_diag, int nseg_cross,
                                                              double* __restrict__ stage1) {
  __shared__ double red[4][64];
  const int g = blockIdx.y, z = blockIdx.z;
  const int nseg = (g % ngroups) < ngroups_diag ? nseg_diag : nseg_cross;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int s0 = (int)((int64_t)nseg * z / RSPLIT), s1 = (int)((int64_t)nseg * (z + 1) / RSPLIT);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (e < REC) {
    const float* p = partials + (int64_t)g * seg_stride * REC + e;
    int k = s0 + w;
    for (; k + 12 < s1; k += 16) {
      a0 += (double)p[(int64_t)k * REC];
      a1 += (double)p[(int64_t)(k + 4) * REC];
      a2 += (double)p[(int64_t)(k + 8) * REC];
      a3 += (double)p[(int64_t)(k + 12) * REC];
    }
    for (; k < s1; k += 4) a0 += (double)p[(int64_t)k * REC];
  }
  red[w][threadIdx.x & 63] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && e < REC)
    stage1[((int64_t)g * RSPLIT + z) * REC + e] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// nrec = slices x groups records (slice-major); gsum rows are glen doubles per
// slice (the groups' records, then the slice's refine block).
__global__ void reduce_splits_kernel(const double* __restrict__ stage1, int nrec, int ngroups, int64_t glen,
                                     double* __restrict__ gsum) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)nrec * REC) return;
  const int g = (int)(idx / REC), e = (int)(idx % REC);
  double s = 0.0;
  for (int z = 0; z < RSPLIT; ++z) s += stage1[((int64_t)g * RSPLIT + z) * REC + e];
  gsum[(int64_t)(g / ngroups) * glen + (int64_t)(g % ngroups) * REC + e] = s;
}

// ---- refine: exact differences for the flagged rows (see COND_FLAG) ----
// grid (nseg, RNBP block pairs (a <= b) of the row list, slices).  Each
// workgroup sums (x_i - x_j)^2 over its segment of the slice's chunks for the
// 32 x 32 pairs of its block pair.  The 32 rows of each block are staged per
// 64-coordinate chunk in LDS ([row][64 + 4]: conflict-free ds_read_b128 under
// the lane map below); a diagonal block pair stages them once and reads both
// operands from that image.  Wave w takes coordinates 16w .. 16w+15 of every
// chunk; lane (bi = lane >> 3, bj = lane & 7) the 4 x 4 pairs (bi + 8u, bj + 8v),
// reading 4-coordinate runs of its 8 rows as float4 (two LDS reads per 4 pairs
// per coordinate pair of rows, instead of four scalar reads per 4 pairs):
// fp32 sums over the 16 coordinates, fp64 across chunks, the four waves'
// partials added in wave order at the end.
typedef float f32x2 __attribute__((ext_vector_type(2)));
// block pair index -> (a, b), a <= b, a-major: (0,0) (0,1) .. (0,RNB-1) (1,1) ..
__host__ __device__ inline int bp_a(int pr) {
  int a = 0;
  while (pr >= RNB - a) { pr -= RNB - a; ++a; }
  return a;
}
__host__ __device__ inline int bp_b(int pr) {
  int a = 0;
  while (pr >= RNB - a) { pr -= RNB - a; ++a; }
  return a + pr;
}
// Staging (round 4): RSC chunks (256 coordinates = 1 KB per row) per stage,
// fetched by LDS-DMA (one global_load_lds_dwordx4 per row: no VGPR round trip,
// no per-chunk barrier), double buffered, the next stage in flight during this
// one's compute.  Row images are unpadded 1-KB rows with the 16-B slots
// XOR-swizzled by (row & 7) on the SOURCE address (the DMA writes lane-
// linearly), so the 8 rows of a ds_read_b128 lane group hit 8 distinct bank
// groups.  Per chunk the arithmetic is the same as before (wave w: coordinates
// 16w .. 16w+15 of every chunk, fp32 over those 16, fp64 across chunks in
// chunk order): the records are bit-identical to the register-staged form.
// Diagonal block pairs stage 32 rows (64 KB of LDS, two workgroups per CU),
// off-diagonal pairs 64 (128 KB): separate launches.
constexpr int RSC = 4;                 // chunks per stage
constexpr int RSW = RSC * CW;          // floats per staged row (1 KB)
template <bool DIAG>
__global__ __launch_bounds__(256) void refine_partials_kernel(const float* __restrict__ X, int64_t ldx,
                                                              int64_t nch_total, int q_base, int64_t chunk0,
                                                              const int* __restrict__ prec, int nseg,
                                                              double* __restrict__ rpart) {
  constexpr int NR = DIAG ? 32 : 64;   // staged rows: block a (and block b)
  extern __shared__ __attribute__((aligned(16))) float rl[];  // [2][NR][RSW]
  __shared__ double red[1024];
  const int c = prec[1];
  int a, b, pr;
  if constexpr (DIAG) {  // blockIdx.y = a
    a = b = (int)blockIdx.y;
    pr = 0;
    for (int t = 0; t < a; ++t) pr += RNB - t;
  } else {  // blockIdx.y = the off-diagonal pairs (a < b) in a-major order
    int r = (int)blockIdx.y;
    a = 0;
    while (r >= RNB - 1 - a) { r -= RNB - 1 - a; ++a; }
    b = a + 1 + r;
    pr = 0;
    for (int t = 0; t < a; ++t) pr += RNB - t;
    pr += b - a;
  }
  if (32 * b >= c) return;  // an empty block of the row list (uniform: the whole workgroup leaves)
  const int seg = blockIdx.x;
  const int q = q_base + (int)blockIdx.z;
  const int64_t s0 = slice_chunk(nch_total, q) - chunk0, s1 = slice_chunk(nch_total, q + 1) - chunk0;
  const int64_t c_begin = s0 + (s1 - s0) * seg / nseg, c_end = s0 + (s1 - s0) * (seg + 1) / nseg;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int bi = lane >> 3, bj = lane & 7;
  // staged rows of this wave: rows wave + 4 i (i < NR / 4); row t < 32 is list
  // position 32a + t, row 32 + t position 32b + t (past the count: row 0)
  const float* src[NR / 4];
#pragma unroll
  for (int i = 0; i < NR / 4; ++i) {
    const int t = wave + 4 * i;
    const int pos = t < 32 ? 32 * a + t : 32 * b + (t - 32);
    src[i] = X + (int64_t)prec[2 + (pos < c ? pos : 0)] * ldx;
  }
  const int64_t nst = (c_end - c_begin + RSC - 1) / RSC;
  auto stage = [&](int64_t st, float* buf) {
#pragma unroll
    for (int i = 0; i < NR / 4; ++i) {
      const int t = wave + 4 * i;
      // lane l fills LDS slot l of row t with the row's global slot l ^ (t & 7)
      int64_t ch0 = c_begin + st * RSC;
      const int gslot = lane ^ (t & 7);
      int64_t ch = ch0 + (gslot >> 4);
      ch = ch < c_end ? ch : c_begin;  // past the segment: any valid chunk (not computed)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src[i] + ch * CW + 4 * (gslot & 15)),
          (__attribute__((address_space(3))) void*)(buf + t * RSW), 16, 0, 0);
    }
  };
  // Compact mapping (diagonal block pairs with at most 28 rows, e.g. the 25
  // sign-flipped clients of C3): only the 4 x 4 sub-blocks (p <= q) of the upper
  // triangle over the valid rows are computed, two lanes per sub-block (8 of the
  // wave's 16 coordinates each) — 28 sub-blocks for 25 rows instead of the full
  // mapping's 32 x 32 pair slots, both triangles and the padding rows (the kernel
  // is VALU-bound: 0.58 ms at C3 with the full mapping).  Otherwise lane (bi, bj)
  // takes the strided 4 x 4 block (bi + 8u, bj + 8v) over the wave's 16 coordinates.
  const int ca = DIAG ? std::min(32, c - 32 * a) : 32;
  const int np = (ca + 3) / 4;
  const bool compact = DIAG && np * (np + 1) / 2 <= 32;  // uniform
  int t_p = 0, t_q = 0;
  bool t_ok = true;
  if (compact) {
    int t = lane >> 1, pp = 0;
    while (pp < np && t >= np - pp) { t -= np - pp; ++pp; }
    t_ok = pp < np;
    t_p = t_ok ? pp : 0;
    t_q = t_ok ? pp + t : 0;
  }
  const int half = lane & 1;
  auto arow = [&](int u) { return compact ? 4 * t_p + u : bi + 8 * u; };
  auto brow = [&](int v) { return compact ? 4 * t_q + v : bj + 8 * v; };
  double d[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) d[u][v] = 0.0;
  if (nst > 0) stage(0, rl);
  for (int64_t st = 0; st < nst; ++st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage st landed (every wave's DMA); stage st-1's buffer is free
    float* buf = rl + (st & 1) * NR * RSW;
    if (st + 1 < nst) stage(st + 1, rl + ((st + 1) & 1) * NR * RSW);
    const float* Ab = buf;
    const float* Bb = DIAG ? buf : buf + 32 * RSW;
#pragma unroll
    for (int cc = 0; cc < RSC; ++cc) {
      if (c_begin + st * RSC + cc >= c_end) break;  // uniform
      // pairs (u, 2w) and (u, 2w+1) share one packed accumulator: v_pk_add_f32 /
      // v_pk_fma_f32 do both pairs' sub + fma, each pair's own fp32 chain unchanged
      f32x2 sacc[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w2 = 0; w2 < 2; ++w2) sacc[u][w2] = f32x2{0.f, 0.f};
      auto k4_step = [&](int k4) {
        const int slot = 16 * cc + 4 * wave + k4;  // 16-B slot of coordinates 16 wave + 4 k4 .. +3 of chunk cc
        f32x4 av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ra = arow(u), rb = brow(u);
          av[u] = *reinterpret_cast<const f32x4*>(Ab + ra * RSW + 4 * (slot ^ (ra & 7)));
          bv[u] = *reinterpret_cast<const f32x4*>(Bb + rb * RSW + 4 * (slot ^ (rb & 7)));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int w2 = 0; w2 < 2; ++w2) {
              const f32x2 a2 = {av[u][e], av[u][e]};
              const f32x2 b2 = {bv[2 * w2][e], bv[2 * w2 + 1][e]};
              const f32x2 df = a2 - b2;
              sacc[u][w2] = __builtin_elementwise_fma(df, df, sacc[u][w2]);
            }
      };
      if (compact) {
        k4_step(2 * half);
        k4_step(2 * half + 1);
      } else {
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) k4_step(k4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) d[u][v] += (double)sacc[u][v >> 1][v & 1];
    }
  }
  if (compact) {
    // the eight partials of a pair (wave w, half h) added in (w, h) order into
    // red, the record's [32][32] image (entries of no sub-block stay 0)
    for (int e = tid; e < 1024; e += 256) red[e] = 0.0;
    __syncthreads();
    for (int ph = 0; ph < 8; ++ph) {
      if (t_ok && wave == (ph >> 1) && half == (ph & 1))
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) red[(4 * t_p + u) * 32 + 4 * t_q + v] += d[u][v];
      __syncthreads();
    }
    double* rec = rpart + (((int64_t)blockIdx.z * RNBP + pr) * nseg + seg) * 1024;
    for (int e = tid; e < 1024; e += 256) rec[e] = red[e];
    return;
  }
  // the four waves' partials, added in wave order (one 8-KB exchange per wave)
  for (int w = 1; w < 4; ++w) {
    if (wave == w)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) red[(bi + 8 * u) * 32 + bj + 8 * v] = d[u][v];
    __syncthreads();
    if (wave == 0)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) d[u][v] += red[(bi + 8 * u) * 32 + bj + 8 * v];
    __syncthreads();
  }
  if (wave == 0) {
    double* rec = rpart + (((int64_t)blockIdx.z * RNBP + pr) * nseg + seg) * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) rec[(bi + 8 * u) * 32 + bj + 8 * v] = d[u][v];
  }
}

// Per slice: the segments summed in order into the slice's refine block
// (gsum + z * glen + ngroups * REC): header (count, rows) then [RMAX][RMAX].
__global__ __launch_bounds__(256) void refine_reduce_kernel(const double* __restrict__ rpart, int nseg,
                                                            const int* __restrict__ prec, int ngroups,
                                                            int64_t glen, double* __restrict__ gsum) {
  const int z = blockIdx.y, pr = blockIdx.x;
  double* blk = gsum + (int64_t)z * glen + (int64_t)ngroups * REC;
  const int c = prec[1];
  if (pr == 0)  // header: count, the RMAX row slots, the total flagged count
    for (int t = threadIdx.x; t < RHDR; t += 256) blk[t] = t == 0 ? (double)c : (double)prec[1 + t];
  const int a = bp_a(pr), b = bp_b(pr);
  if (32 * b >= c) return;
  for (int e = threadIdx.x; e < 1024; e += 256) {
    const double* p = rpart + ((int64_t)z * RNBP + pr) * nseg * 1024 + e;
    double s = 0.0;
#pragma unroll 16
    for (int k = 0; k < nseg; ++k) s += p[(int64_t)k * 1024];  // independent loads, 16 in flight
    blk[RHDR + (32 * a + (e >> 5)) * RMAX + 32 * b + (e & 31)] = s;
  }
}

// Rows to refine, from the exact sample distances Ds and the pivot (one
// workgroup): row i is flagged when some j has
//   Ds[i][j]^2 * COND_FLAG < Ds[i][p]^2 + Ds[j][p]^2.
// The first RMAX flagged rows in index order go to prec[2..], their count to
// prec[1], the number of flagged rows (may exceed RMAX) to prec[2 + RMAX].
__global__ __launch_bounds__(256) void flag_rows_kernel(const double* __restrict__ Ds, int K, int* __restrict__ prec) {
  __shared__ unsigned char flag[MAXK_PIVOT];
  const int p = prec[0];
  for (int i = threadIdx.x; i < K; i += 256) {
    const double dip = Ds[(int64_t)i * K + p];
    int f = 0;
    for (int j = 0; j < K && !f; ++j) {
      if (j == i) continue;
      const double dij = Ds[(int64_t)i * K + j], djp = Ds[(int64_t)j * K + p];
      f = dij * dij * COND_FLAG < dip * dip + djp * djp;
    }
    flag[i] = (unsigned char)f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0, total = 0;
    for (int i = 0; i < K; ++i)
      if (flag[i]) {
        if (c < RMAX) prec[2 + c++] = i;
        ++total;
      }
    prec[1] = c;
    for (int t = c; t < RMAX; ++t) prec[2 + t] = 0;
    prec[2 + RMAX] = total;
  }
}

// Exact-difference contribution of the coordinates that do not fill a chunk.
__global__ void tail_d2_kernel(const float* __restrict__ X, int K, int64_t ldx, int64_t p0,
                               int64_t p1, double* __restrict__ tail) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)K * K) return;
  const int i = (int)(idx / K), j = (int)(idx % K);
  double s = 0.0;
  if (i != j) {
    const float* xi = X + (int64_t)i * ldx;
    const float* xj = X + (int64_t)j * ldx;
    for (int64_t p = p0; p < p1; ++p) {
      const float d = xi[p] - xj[p];
      s += (double)d * (double)d;
    }
  }
  tail[idx] = s;
}

__device__ __forceinline__ int tile_entry(int row, int col) {
  // inverse of the 32x32 MFMA C/D map: row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  const int reg = (row & 3) + 4 * (row >> 3);
  const int lane = col + 32 * ((row >> 2) & 1);
  return reg * 64 + lane;
}

// D from the per-slice group sums, adding the slices in slice order.
__global__ void assemble_kernel(const double* __restrict__ gsum, int ngroups, int64_t glen,
                                const double* __restrict__ tail, int K, double* __restrict__ D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)K * K) return;
  int i = (int)(idx / K), j = (int)(idx % K);
  // more flagged rows than the refine list holds (K > RMAX only): every entry
  // NaN, the diagonal included — the marker KrumDefense checks (a NaN client
  // update never makes the diagonal NaN); loud, not inaccurate
  const double* hdr = gsum + (int64_t)ngroups * REC;  // slice 0's header (every slice holds the same)
  const int c = (int)hdr[0];
  if ((int)hdr[1 + RMAX] > c) {
    D[idx] = __builtin_nan("");
    return;
  }
  if (i == j) {
    D[idx] = 0.0;
    return;
  }
  if (i > j) {
    const int tmp = i; i = j; j = tmp;
  }
  int g, lb_i, lb_j, t;
  const int ri = i & 31, rj = j & 31;
  if (K <= SUPER) {
    const int nl = cdiv(K, 32);
    g = 0;
    lb_i = i >> 5;
    lb_j = j >> 5;
    t = diag_tile_index(nl, lb_i, lb_j);
  } else {
    const int nsb = cdiv(K, SUPER);
    const int I = i / SUPER, J = j / SUPER;
    const int bi = (i % SUPER) >> 5, bj = (j % SUPER) >> 5;
    if (I == J) {
      g = I;
      lb_i = bi;
      lb_j = bj;
      t = diag_tile_index(4, bi, bj);
    } else {
      int q = 0;
      for (int a = 0; a < I; ++a) q += nsb - 1 - a;
      q += J - I - 1;
      g = nsb + CROSS_PER_PAIR * q + (bi / CROSS_NI) * (4 / CROSS_NJ) + bj / CROSS_NJ;
      lb_i = bi % CROSS_NI;
      lb_j = CROSS_NI + bj % CROSS_NJ;
      t = lb_i * CROSS_NJ + bj % CROSS_NJ;
    }
  }
  // a refined pair (both rows in the refine list): the exact-difference sums
  int pi = -1, pj = -1;
  for (int u = 0; u < c; ++u) {
    const int row = (int)hdr[1 + u];
    pi = row == i ? u : pi;
    pj = row == j ? u : pj;
  }
  double d2;
  if (pi >= 0 && pj >= 0) {
    const int lo = pi < pj ? pi : pj, hi = pi < pj ? pj : pi;
    d2 = 0.0;
    for (int q = 0; q < FLR_PW_SLICES; ++q) d2 += gsum[(int64_t)q * glen + (int64_t)ngroups * REC + RHDR + lo * RMAX + hi];
    d2 += tail[idx];
  } else {
    double gij = 0.0, gii = 0.0, gjj = 0.0;
    for (int q = 0; q < FLR_PW_SLICES; ++q) {
      const double* rec = gsum + (int64_t)q * glen + (int64_t)g * REC;
      gij += rec[t * 1024 + tile_entry(ri, rj)];
      gii += rec[REC_TILES * 1024 + 32 * lb_i + ri];
      gjj += rec[REC_TILES * 1024 + 32 * lb_j + rj];
    }
    d2 = gii + gjj - 2.0 * gij + tail[idx];
  }
  if (d2 < 0.0) d2 = 0.0;
  D[idx] = (double)(float)sqrt(d2);
}

// ---- pivot prepass: medoid of a strided coordinate sample ----
// Xs[i][s] = X[i][s*stride] (row-major, ld = SAMPLE); the sample's exact
// distances come from the direct kernel below; pivot = argmin_i sum_j Ds[i][j].
constexpr int SAMPLE = 2048;
constexpr int SAMPLE_NSEG = 8;

// Xs[i][s] = X[i][s*stride - 64*chunk0] for the sample positions s*stride that
// fall in X's global chunk range [chunk0, chunk1); 0 for the others (the
// per-rank samples of the sharded path are then combined by an exact sum).
__global__ void sample_gather_kernel(const float* __restrict__ X, int K, int64_t ldx, int S, int64_t stride,
                                     int64_t chunk0, int64_t chunk1, float* __restrict__ Xs) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)K * S) return;
  const int i = (int)(idx / S), s = (int)(idx % S);
  const int64_t pos = (int64_t)s * stride - chunk0 * CW;
  Xs[idx] = (pos >= 0 && pos < (chunk1 - chunk0) * CW) ? X[(int64_t)i * ldx + pos] : 0.f;
}

// One workgroup: rowsum_i = sum_j Ds[i][j] (fp64, j order), then argmin
// (lowest index on ties).
__global__ __launch_bounds__(256) void pivot_kernel(const double* __restrict__ Ds, int K, int* __restrict__ pivot) {
  __shared__ double bv[256];
  __shared__ int bi[256];
  double v = __builtin_huge_val();
  int ix = 0x7fffffff;
  // rows with a non-finite sample distance to at most half the others: a
  // client that sent NaN / inf (its whole row non-finite) is never the pivot,
  // and the others' sums skip its column (a NaN pivot made every
  // off-diagonal distance NaN, so Krum's order fell back to the identity)
  for (int i = threadIdx.x; i < K; i += 256) {
    double r = 0.0;
    int bad = 0;
    for (int j = 0; j < K; ++j) {
      const double d = Ds[(int64_t)i * K + j];
      if (__builtin_isfinite(d))
        r += d;
      else
        ++bad;
    }
    if (2 * bad <= K - 1 && r < v) { v = r; ix = i; }
  }
  bv[threadIdx.x] = v;
  bi[threadIdx.x] = ix;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double v2 = bv[threadIdx.x + o];
      const int i2 = bi[threadIdx.x + o];
      if (v2 < bv[threadIdx.x] || (v2 == bv[threadIdx.x] && i2 < bi[threadIdx.x])) {
        bv[threadIdx.x] = v2;
        bi[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *pivot = bi[0] == 0x7fffffff ? 0 : bi[0];
}

struct Plan {
  int64_t nchunks;   // full 64-coordinate chunks of the whole vector
  int nseg;          // record stride per (slice, group) = max(nseg_diag, nseg_cross)
  int nseg_diag;     // segments per (slice, DIAG group)
  int nseg_cross;    // segments per (slice, CROSS group)
  int ngroups_diag;  // groups launched with the DIAG kernel
  int ngroups_cross; // groups launched with the CROSS kernel
  int nl_diag;       // loaded blocks per DIAG group
  int ngroups() const { return ngroups_diag + ngroups_cross; }
};

// Depends on (K, P) only — never on how the slices are spread over GPUs — so
// every segment record is the same whichever GPU computes it.
inline Plan make_plan(int64_t K, int64_t P) {
  Plan p;
  p.nchunks = P / CW;
  if (K <= SUPER) {
    p.ngroups_diag = 1;
    p.ngroups_cross = 0;
    p.nl_diag = cdiv((int)K, 32);
  } else {
    const int nsb = cdiv((int)K, SUPER);
    p.ngroups_diag = nsb;
    p.ngroups_cross = nsb * (nsb - 1) / 2 * CROSS_PER_PAIR;
    p.nl_diag = 4;
  }
  const int64_t min_slice = p.nchunks / FLR_PW_SLICES;
  const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(min_slice, MAX_SEG));
  if (K <= SUPER) {
    const int target = std::max(1, TARGET_BLOCKS / (FLR_PW_SLICES * p.ngroups()));
    p.nseg = p.nseg_diag = (int)std::min<int64_t>(cap, target);
    p.nseg_cross = 0;
    return p;
  }
  // K > 128: the DIAG and CROSS groups are separate launches, so each gets its
  // own segment count, chosen to minimise the number of residency rounds per
  // unit of work: ceil(units * n / slots) / n (units = groups x slices; slots =
  // 2 workgroups per CU for the 64 KB stages, 1 for the 96 KB NL = 6 cross stage).
  auto pick = [&](int units, int slots) {
    int best = 1;
    for (int n = 2; n <= std::min<int64_t>(cap, 64); ++n) {
      // rounds(n) / n < rounds(best) / best
      const int64_t rn = ((int64_t)units * n + slots - 1) / slots, rb = ((int64_t)units * best + slots - 1) / slots;
      if (rn * best < rb * n) best = n;
    }
    return best;
  };
  p.nseg_diag = pick(p.ngroups_diag * FLR_PW_SLICES, 2 * 256);
  p.nseg_cross = pick(p.ngroups_cross * FLR_PW_SLICES, CROSS_NL >= 6 ? 256 : 512);
  p.nseg = std::max(p.nseg_diag, p.nseg_cross);
  return p;
}

inline int direct_npairs(int64_t K) {
  const int nb = cdiv((int)K, 32);
  return nb * (nb + 1) / 2;
}

inline int64_t sample_len(int64_t P) { return std::min<int64_t>(SAMPLE, (P / CW) * CW); }

// fp64 per slice of gsum: the groups' Gram records, then the slice's refine block
inline size_t gsum_doubles(int64_t K) {
  return (size_t)make_plan(K, (int64_t)CW * FLR_PW_SLICES).ngroups() * REC + RBLK;
}
// refine segments per slice: depends on P only (the same records at every GPU count)
inline int refine_nseg(int64_t P) {
  const int64_t min_slice = (P / CW) / FLR_PW_SLICES;
  return (int)std::max<int64_t>(1, std::min<int64_t>(min_slice, RSEG_MAX));
}

// Workspace carve-up (every piece 256-B aligned).  `nsl` = slices computed by
// this call (FLR_PW_SLICES for the whole-vector call).
struct Layout {
  size_t partials, stage1, gsum, tail, xs, spart, ds, pivot, rpart, total;
};
inline Layout layout(int64_t K, int64_t P, int nsl = FLR_PW_SLICES) {
  const Plan p = make_plan(K, P);
  Layout l;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += align_up(bytes, 256); return o; };
  l.partials = take((size_t)nsl * p.ngroups() * p.nseg * REC * sizeof(float));
  l.stage1 = take((size_t)nsl * p.ngroups() * RSPLIT * REC * sizeof(double));
  l.gsum = take((size_t)FLR_PW_SLICES * gsum_doubles(K) * sizeof(double));
  l.tail = take((size_t)K * K * sizeof(double));
  l.xs = take((size_t)K * SAMPLE * sizeof(float));
  l.spart = take((size_t)direct_npairs(K) * SAMPLE_NSEG * 1024 * sizeof(float));
  l.ds = take((size_t)K * K * sizeof(double));
  l.pivot = take(PREC * sizeof(int));
  l.rpart = take((size_t)nsl * RNBP * refine_nseg(P) * 1024 * sizeof(double));
  l.total = off;
  return l;
}

// Wrong-result ablations (timing only: FLR_GRAM_ABLATE=1 skips the MFMAs, =2
// the loads) exist only in a tools build (make ABLATION=1 -> -DFLR_ABLATION);
// the shipped library has no switch that changes results.
inline int gram_ablate() {
#ifdef FLR_ABLATION
  static const int a = [] {
    const char* e = flr::knob("FLR_GRAM_ABLATE");
    return e ? atoi(e) : 0;
  }();
  return a;
#else
  return 0;
#endif
}

// bf16 terms per value: 3 (hi+mid+lo, 6 MFMA products) removes the split's
// representation error, which dominates below ~1M coordinates; above that the
// fp32 accumulation dominates and 2 terms (4 products) measure the same error
// at 2/3 of the kernel time.  FLR_GRAM_TERMS=2|3 overrides.  P is the WHOLE
// vector's length (the same choice on every GPU of a sharded call).
inline int gram_terms(int64_t P) {
  const char* e = flr::knob("FLR_GRAM_TERMS");
  if (e && (e[0] == '2' || e[0] == '3')) return e[0] - '0';
  return P < (int64_t(1) << 20) ? 3 : 2;
}

struct GramArgs {
  const float* X;
  int K;
  int64_t ldx, P, chunk0;
  int q0, nsl;
  const int* pivot;
  float* partials;
};

template <int NL, bool CROSS>
int launch_gram(const GramArgs& a, const Plan& p, int group_base, int ngroups, hipStream_t st) {
  const size_t lds = (size_t)2 * 32 * NL * CW * sizeof(float);
  const int nseg = CROSS ? p.nseg_cross : p.nseg_diag;
  dim3 grid(nseg, ngroups, a.nsl);
#define FLR_GRAM_LAUNCH(T, AB, ...)                                                                      \
  hipLaunchKernelGGL((gram_partials_kernel<NL, CROSS, T, AB, ##__VA_ARGS__>), grid, dim3(THREADS), lds, st, a.X, \
                     a.K, a.ldx, p.nchunks, a.q0, a.chunk0, group_base, p.ngroups(), a.pivot, a.partials, nseg, p.nseg)
  if (gram_terms(a.P) == 3) {
    FLR_GRAM_LAUNCH(3, 0);
    return launch_status("gram_partials_kernel");
  }
#ifdef FLR_ABLATION
  if constexpr (NL == 4 && !CROSS) {
    if (gram_ablate() == 1) {
      FLR_GRAM_LAUNCH(2, 1);
      return launch_status("gram_partials_kernel");
    }
    if (gram_ablate() == 2) {
      FLR_GRAM_LAUNCH(2, 2);
      return launch_status("gram_partials_kernel");
    }
  }
#endif
  // every row in one group (K <= 32 NL, no cross stage): each chunk of X is read
  // once, so the DMA streams it non-temporally: C3 (K = 128) 1.044 -> 0.93 ms,
  // 0.72 -> 0.81 of 8 TB/s.  Where groups re-read rows (K > 128) the default policy
  // keeps their L2 / MALL hits (non-temporal there: C5 +9 %, C4 -1 %;
  // profiles/r3_gram_nt.txt).  FLR_GRAM_NT=0: default policy everywhere, 2:
  // non-temporal everywhere (A/B)
  {
    const char* e = flr::knob("FLR_GRAM_NT");
    const int mode = e ? atoi(e) : 1;
    if (mode == 2 || (mode == 1 && !CROSS && a.K <= 32 * NL)) {
      FLR_GRAM_LAUNCH(2, 0, true);
      return launch_status("gram_partials_kernel");
    }
  }
  FLR_GRAM_LAUNCH(2, 0);
#undef FLR_GRAM_LAUNCH
  return launch_status("gram_partials_kernel");
}

// ----------------------------- direct path -----------------------------
constexpr int DCW = 64;

__global__ __launch_bounds__(256) void direct_partials_kernel(const float* __restrict__ X, int K,
                                                              int64_t P, int64_t ldx, int nseg,
                                                              float* __restrict__ partials) {
  __shared__ float A[32][DCW + 1];
  __shared__ float B[32][DCW + 1];
  // blockIdx.y -> block pair (a <= b)
  const int nb = cdiv(K, 32);
  int pr = blockIdx.y, a = 0;
  while (pr >= nb - a) { pr -= nb - a; ++a; }
  const int b = a + pr;
  const int seg = blockIdx.x;
  const int nch = (int)((P + DCW - 1) / DCW);
  const int c_begin = (int)((int64_t)nch * seg / nseg), c_end = (int)((int64_t)nch * (seg + 1) / nseg);
  const int tid = threadIdx.x;
  const int ia = 2 * (tid >> 4), jb = 2 * (tid & 15);
  float s00 = 0.f, s01 = 0.f, s10 = 0.f, s11 = 0.f;
  for (int c = c_begin; c < c_end; ++c) {
    const int64_t p0 = (int64_t)c * DCW;
    for (int e = tid; e < 32 * DCW; e += 256) {
      const int rr = e / DCW, cc = e % DCW;
      const int64_t p = p0 + cc;
      int ga = 32 * a + rr, gb = 32 * b + rr;
      ga = ga < K ? ga : K - 1;
      gb = gb < K ? gb : K - 1;
      A[rr][cc] = p < P ? X[(int64_t)ga * ldx + p] : 0.f;
      B[rr][cc] = p < P ? X[(int64_t)gb * ldx + p] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int cc = 0; cc < DCW; ++cc) {
      const float a0 = A[ia][cc], a1 = A[ia + 1][cc], b0 = B[jb][cc], b1 = B[jb + 1][cc];
      float d;
      d = a0 - b0; s00 = __builtin_fmaf(d, d, s00);
      d = a0 - b1; s01 = __builtin_fmaf(d, d, s01);
      d = a1 - b0; s10 = __builtin_fmaf(d, d, s10);
      d = a1 - b1; s11 = __builtin_fmaf(d, d, s11);
    }
    __syncthreads();
  }
  float* rec = partials + ((int64_t)blockIdx.y * nseg + seg) * 1024;
  rec[ia * 32 + jb] = s00;
  rec[ia * 32 + jb + 1] = s01;
  rec[(ia + 1) * 32 + jb] = s10;
  rec[(ia + 1) * 32 + jb + 1] = s11;
}

__global__ void direct_assemble_kernel(const float* __restrict__ partials, int K, int nseg,
                                       double* __restrict__ D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)K * K) return;
  int i = (int)(idx / K), j = (int)(idx % K);
  if (i == j) {
    D[idx] = 0.0;
    return;
  }
  if (i > j) {
    const int tmp = i; i = j; j = tmp;
  }
  const int nb = cdiv(K, 32);
  const int a = i >> 5, b = j >> 5;
  int pr = 0;
  for (int x = 0; x < a; ++x) pr += nb - x;
  pr += b - a;
  const float* rec = partials + (int64_t)pr * nseg * 1024 + (i & 31) * 32 + (j & 31);
  double s = 0.0;
  for (int k = 0; k < nseg; ++k) s += (double)rec[(int64_t)k * 1024];
  D[idx] = (double)(float)sqrt(s);
}

inline int direct_nseg(int64_t K, int64_t P) {
  const int nb = cdiv((int)K, 32);
  const int npairs = nb * (nb + 1) / 2;
  const int nch = (int)((P + DCW - 1) / DCW);
  return std::max(1, std::min(nch, std::max(1, 1024 / npairs)));
}

}  // namespace pw
}  // namespace flr

using namespace flr;
using namespace flr::pw;

namespace {

// Pivot = medoid of the sample Xs [K][S] (exact differences, direct kernel).
int pivot_phase(const float* Xs, int K, int S, float* spart, double* Ds, int* pivot, hipStream_t st) {
  int rc;
  const int nblk = (int)(((int64_t)K * K + 255) / 256);
  const int snseg = std::min(SAMPLE_NSEG, cdiv(S, DCW));
  hipLaunchKernelGGL(direct_partials_kernel, dim3(snseg, direct_npairs(K)), dim3(256), 0, st, Xs, K,
                     (int64_t)S, (int64_t)S, snseg, spart);
  if ((rc = launch_status("direct_partials_kernel(sample)")) != FLR_OK) return rc;
  hipLaunchKernelGGL(direct_assemble_kernel, dim3(nblk), dim3(256), 0, st, spart, K, snseg, Ds);
  if ((rc = launch_status("direct_assemble_kernel(sample)")) != FLR_OK) return rc;
  hipLaunchKernelGGL(pivot_kernel, dim3(1), dim3(256), 0, st, Ds, K, pivot);
  if ((rc = launch_status("pivot_kernel")) != FLR_OK) return rc;
  hipLaunchKernelGGL(flag_rows_kernel, dim3(1), dim3(256), 0, st, Ds, K, pivot);
  return launch_status("flag_rows_kernel");
}

// Centred-Gram records of slices [q0, q0 + nsl), reduced per (slice, group)
// in fixed order into gsum [nsl][ngroups][REC] (fp64).
int gram_phase(const GramArgs& a, double* stage1, double* gsum, double* rpart, hipStream_t st, void* ev_begin,
               void* ev_end) {
  const Plan p = make_plan(a.K, a.P);
  int rc;
  if (ev_begin && hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), st) != hipSuccess) return FLR_ERR_HIP;
  if (a.K <= SUPER) {
    switch (p.nl_diag) {
      case 1: rc = launch_gram<1, false>(a, p, 0, 1, st); break;
      case 2: rc = launch_gram<2, false>(a, p, 0, 1, st); break;
      case 3: rc = launch_gram<3, false>(a, p, 0, 1, st); break;
      default: rc = launch_gram<4, false>(a, p, 0, 1, st); break;
    }
  } else {
    rc = launch_gram<4, false>(a, p, 0, p.ngroups_diag, st);
    if (rc == FLR_OK) rc = launch_gram<CROSS_NL, true>(a, p, p.ngroups_diag, p.ngroups_cross, st);
  }
  if (rc != FLR_OK) return rc;
  if (ev_end && hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), st) != hipSuccess) return FLR_ERR_HIP;
  const int nrec = a.nsl * p.ngroups();  // (slice, group) pairs, slice-major
  hipLaunchKernelGGL(reduce_records_kernel, dim3(cdiv(REC, 64), nrec, RSPLIT), dim3(256), 0, st, a.partials,
                     p.nseg, p.ngroups(), p.ngroups_diag, p.nseg_diag, p.nseg_cross, stage1);
  if ((rc = launch_status("reduce_records_kernel")) != FLR_OK) return rc;
  const int64_t glen = (int64_t)gsum_doubles(a.K);
  hipLaunchKernelGGL(reduce_splits_kernel, dim3(cdiv(nrec * REC, 256)), dim3(256), 0, st, stage1, nrec,
                     p.ngroups(), glen, gsum);
  if ((rc = launch_status("reduce_splits_kernel")) != FLR_OK) return rc;
  // the flagged rows' exact-difference records of these slices (workgroups of an
  // empty row-list block leave at once)
  const int rseg = refine_nseg(a.P);
  hipLaunchKernelGGL(refine_partials_kernel<true>, dim3(rseg, RNB, a.nsl), dim3(256), 2 * 32 * RSW * sizeof(float),
                     st, a.X, a.ldx, p.nchunks, a.q0, a.chunk0, a.pivot, rseg, rpart);
  if ((rc = launch_status("refine_partials_kernel<diag>")) != FLR_OK) return rc;
  hipLaunchKernelGGL(refine_partials_kernel<false>, dim3(rseg, RNBP - RNB, a.nsl), dim3(256),
                     2 * 64 * RSW * sizeof(float), st, a.X, a.ldx, p.nchunks, a.q0, a.chunk0, a.pivot, rseg, rpart);
  if ((rc = launch_status("refine_partials_kernel<cross>")) != FLR_OK) return rc;
  hipLaunchKernelGGL(refine_reduce_kernel, dim3(RNBP, a.nsl), dim3(256), 0, st, rpart, rseg, a.pivot, p.ngroups(),
                     glen, gsum);
  return launch_status("refine_reduce_kernel");
}

bool aligned16(const void* p, int64_t ld) { return ((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (ld % 4 == 0); }

}  // namespace

extern "C" size_t flr_pairwise_l2_workspace(int64_t K, int64_t P) {
  if (K < 1 || P < 0) return 0;
  return layout(K, P).total;
}

extern "C" int flr_pairwise_l2(const float* X, int64_t K, int64_t P, int64_t ldx, double* D,
                               void* workspace, size_t workspace_bytes, void* stream) {
  return flr_pairwise_l2_ex(X, K, P, ldx, D, workspace, workspace_bytes, stream, nullptr, nullptr);
}

extern "C" int flr_pairwise_l2_ex(const float* X, int64_t K, int64_t P, int64_t ldx, double* D,
                                  void* workspace, size_t workspace_bytes, void* stream, void* ev_begin,
                                  void* ev_end) {
  if (K < 1 || P < 0 || ldx < P || !D || (K > 1 && P > 0 && !X)) return FLR_ERR_ARG;
  if (K > MAXK_PIVOT) return FLR_ERR_UNSUPPORTED;
  const Layout L = layout(K, P);
  if (!workspace || workspace_bytes < L.total || (reinterpret_cast<uintptr_t>(workspace) & 255))
    return FLR_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  const Plan p = make_plan(K, P);
  char* w = static_cast<char*>(workspace);
  double* gsum = reinterpret_cast<double*>(w + L.gsum);
  double* tail = reinterpret_cast<double*>(w + L.tail);
  float* Xs = reinterpret_cast<float*>(w + L.xs);
  int* pivot = reinterpret_cast<int*>(w + L.pivot);

  // The DMA path reads 16-B pieces: it needs 16-B aligned rows.
  const bool aligned = aligned16(X, ldx);
  const int64_t p_main = aligned ? p.nchunks * CW : 0;
  const int K32 = (int)K;
  const int nblk = (int)((K * K + 255) / 256);
  int rc = FLR_OK;
  if (p_main > 0) {
    // 1. pivot: medoid of a strided sample of the main region (exact differences)
    const int S = (int)sample_len(P);
    hipLaunchKernelGGL(sample_gather_kernel, dim3((unsigned)cdiv(K32 * S, 256)), dim3(256), 0, st, X, K32, ldx,
                       S, p_main / S, (int64_t)0, p.nchunks, Xs);
    if ((rc = launch_status("sample_gather_kernel")) != FLR_OK) return rc;
    rc = pivot_phase(Xs, K32, S, reinterpret_cast<float*>(w + L.spart), reinterpret_cast<double*>(w + L.ds), pivot,
                     st);
    if (rc != FLR_OK) return rc;
    // 2.-3. centred Gram records of every canonical slice, fixed-order fp64 sums
    const GramArgs a{X, K32, ldx, P, 0, 0, FLR_PW_SLICES, pivot, reinterpret_cast<float*>(w + L.partials)};
    rc = gram_phase(a, reinterpret_cast<double*>(w + L.stage1), gsum, reinterpret_cast<double*>(w + L.rpart), st,
                    ev_begin, ev_end);
    if (rc != FLR_OK) return rc;
  } else {  // no full chunk: the tail is everything (and the refine list empty)
    if (hipMemsetAsync(gsum, 0, (size_t)FLR_PW_SLICES * gsum_doubles(K) * sizeof(double), st) != hipSuccess)
      return FLR_ERR_HIP;
  }
  // 4. exact contribution of the trailing partial chunk, then D (slices in order)
  hipLaunchKernelGGL(tail_d2_kernel, dim3(nblk), dim3(256), 0, st, X, K32, ldx, p_main, P, tail);
  if ((rc = launch_status("tail_d2_kernel")) != FLR_OK) return rc;
  hipLaunchKernelGGL(assemble_kernel, dim3(nblk), dim3(256), 0, st, gsum, p.ngroups(), (int64_t)gsum_doubles(K),
                     tail, K32, D);
  return launch_status("assemble_kernel");
}

/* ---- phases of the coordinate-sharded call ---- */

extern "C" int flr_pw_slice_chunks(int64_t P, int64_t q, int64_t* chunk_begin, int64_t* chunk_end) {
  if (P < 0 || q < 0 || q >= FLR_PW_SLICES || !chunk_begin || !chunk_end) return FLR_ERR_ARG;
  *chunk_begin = slice_chunk(P / CW, (int)q);
  *chunk_end = slice_chunk(P / CW, (int)q + 1);
  return FLR_OK;
}

extern "C" int64_t flr_pairwise_sample_len(int64_t P) { return P < 0 ? 0 : sample_len(P); }

extern "C" size_t flr_pairwise_gsum_len(int64_t K) { return K < 1 ? 0 : gsum_doubles(K); }

extern "C" int64_t flr_pairwise_pivot_len(void) { return PREC; }

extern "C" size_t flr_pairwise_sliced_workspace(int64_t K, int64_t P, int64_t nslices) {
  if (K < 1 || P < 0 || nslices < 1 || nslices > FLR_PW_SLICES) return 0;
  return layout(K, P, (int)nslices).total;
}

extern "C" int flr_pairwise_sample(const float* X, int64_t K, int64_t ldx, int64_t P, int64_t chunk0,
                                   int64_t chunk1, float* Xs, void* stream) {
  const int64_t nch = P / CW;
  if (K < 1 || K > MAXK_PIVOT || P < CW || !Xs || chunk0 < 0 || chunk1 < chunk0 || chunk1 > nch) return FLR_ERR_ARG;
  if (chunk1 > chunk0 && (!X || ldx < (chunk1 - chunk0) * CW)) return FLR_ERR_ARG;
  const int S = (int)sample_len(P);
  hipLaunchKernelGGL(sample_gather_kernel, dim3((unsigned)cdiv((int)K * S, 256)), dim3(256), 0, as_stream(stream), X,
                     (int)K, ldx, S, nch * CW / S, chunk0, chunk1, Xs);
  return launch_status("sample_gather_kernel");
}

extern "C" int flr_pairwise_pivot(const float* Xs, int64_t K, int64_t P, int* pivot, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (K < 1 || K > MAXK_PIVOT || P < CW || !Xs || !pivot) return FLR_ERR_ARG;
  const Layout L = layout(K, P, 1);
  if (!workspace || workspace_bytes < L.total || (reinterpret_cast<uintptr_t>(workspace) & 255))
    return FLR_ERR_WORKSPACE;
  char* w = static_cast<char*>(workspace);
  return pivot_phase(Xs, (int)K, (int)sample_len(P), reinterpret_cast<float*>(w + L.spart),
                     reinterpret_cast<double*>(w + L.ds), pivot, as_stream(stream));
}

extern "C" int flr_pairwise_gram_slices(const float* X, int64_t K, int64_t ldx, int64_t P, int64_t q0, int64_t q1,
                                        const int* pivot, double* gsum, void* workspace, size_t workspace_bytes,
                                        void* stream, void* ev_begin, void* ev_end) {
  if (K < 1 || K > MAXK_PIVOT || P < 0 || q0 < 0 || q1 <= q0 || q1 > FLR_PW_SLICES || !pivot || !gsum)
    return FLR_ERR_ARG;
  const int64_t nch = P / CW;
  const int64_t c0 = slice_chunk(nch, (int)q0), c1 = slice_chunk(nch, (int)q1);
  if (c1 > c0 && (!X || ldx < (c1 - c0) * CW || !aligned16(X, ldx))) return FLR_ERR_ARG;
  const Layout L = layout(K, P, (int)(q1 - q0));
  if (!workspace || workspace_bytes < L.total || (reinterpret_cast<uintptr_t>(workspace) & 255))
    return FLR_ERR_WORKSPACE;
  char* w = static_cast<char*>(workspace);
  const GramArgs a{X, (int)K, ldx, P, c0, (int)q0, (int)(q1 - q0), pivot, reinterpret_cast<float*>(w + L.partials)};
  return gram_phase(a, reinterpret_cast<double*>(w + L.stage1), gsum, reinterpret_cast<double*>(w + L.rpart),
                    as_stream(stream), ev_begin, ev_end);
}

extern "C" int flr_pairwise_tail(const float* X, int64_t K, int64_t ldx, int64_t p0, int64_t p1, double* tail,
                                 void* stream) {
  if (K < 1 || p0 < 0 || p1 < p0 || !tail || (p1 > p0 && (!X || ldx < p1))) return FLR_ERR_ARG;
  hipLaunchKernelGGL(tail_d2_kernel, dim3((unsigned)((K * K + 255) / 256)), dim3(256), 0, as_stream(stream), X,
                     (int)K, ldx, p0, p1, tail);
  return launch_status("tail_d2_kernel");
}

extern "C" int flr_pairwise_finish(const double* gsum, const double* tail, int64_t K, double* D, void* stream) {
  if (K < 1 || K > MAXK_PIVOT || !gsum || !tail || !D) return FLR_ERR_ARG;
  hipLaunchKernelGGL(assemble_kernel, dim3((unsigned)((K * K + 255) / 256)), dim3(256), 0, as_stream(stream), gsum,
                     make_plan(K, (int64_t)CW * FLR_PW_SLICES).ngroups(), (int64_t)gsum_doubles(K), tail, (int)K, D);
  return launch_status("assemble_kernel");
}

extern "C" size_t flr_pairwise_l2_direct_workspace(int64_t K, int64_t P) {
  if (K < 1 || P < 0) return 0;
  return (size_t)direct_npairs(K) * direct_nseg(K, P) * 1024 * sizeof(float);
}

extern "C" int flr_pairwise_l2_direct(const float* X, int64_t K, int64_t P, int64_t ldx, double* D,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  if (K < 1 || P < 0 || ldx < P || !D || (K > 1 && P > 0 && !X)) return FLR_ERR_ARG;
  if (K > (1 << 16)) return FLR_ERR_UNSUPPORTED;
  const size_t need = flr_pairwise_l2_direct_workspace(K, P);
  if (!workspace || workspace_bytes < need) return FLR_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  const int nb = cdiv((int)K, 32);
  const int npairs = nb * (nb + 1) / 2;
  const int nseg = direct_nseg(K, P);
  float* partials = static_cast<float*>(workspace);
  hipLaunchKernelGGL(direct_partials_kernel, dim3(nseg, npairs), dim3(256), 0, st, X, (int)K, P, ldx,
                     nseg, partials);
  int rc = launch_status("direct_partials_kernel");
  if (rc != FLR_OK) return rc;
  const int64_t kk = K * K;
  hipLaunchKernelGGL(direct_assemble_kernel, dim3((int)((kk + 255) / 256)), dim3(256), 0, st, partials,
                     (int)K, nseg, D);
  return launch_status("direct_assemble_kernel");
}
