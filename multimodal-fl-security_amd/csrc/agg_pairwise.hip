// a9 — Krum pairwise l2 distances on gfx950.
//
// Replaces KrumDefense._compute_distances (src/defenses/krum.py:73-99), which
// loops over K(K-1)/2 pairs calling torch.norm(flat_i - flat_j).item().
//
// Engine (MFMA path, flr_pairwise_l2):
//   ||x_i - x_j||^2 = G_ii + G_jj - 2 G_ij with G the Gram matrix of the
//   per-coordinate CENTRED client matrix y = x - c (c = mean over the group's
//   rows for that coordinate; distances are translation invariant, so any
//   per-coordinate constant is exact, and centring removes the cancellation
//   that makes a raw-weight Gram useless).  y is split into bf16 hi + lo
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
#include <type_traits>

namespace flr {
namespace pw {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int CW = 64;          // coordinates per chunk = 256 B per row
constexpr int THREADS = 256;    // 4 waves; wave w owns k-step w of the chunk
constexpr int SUPER = 128;      // rows of a diagonal group (4 client blocks)
constexpr int REC_TILES = 10;   // max tiles per group
constexpr int REC_DIAG = 6 * 32;
constexpr int REC = REC_TILES * 1024 + REC_DIAG;   // floats per partial record
constexpr int MAX_SEG = 512;

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// Tile enumeration.  DIAG: every (a <= b) over NL loaded blocks, a-major.
// CROSS (NL = 6): a in {0,1} (rows of super-block I), b in {2..5} (rows of J).
template <int NL, bool CROSS>
struct TileSet {
  static constexpr int N = CROSS ? 8 : NL * (NL + 1) / 2;
  __host__ __device__ static constexpr int a(int t) {
    if (CROSS) return t / 4;
    int r = t;
    for (int i = 0; i < NL; ++i) {
      if (r < NL - i) return i;
      r -= NL - i;
    }
    return -1;
  }
  __host__ __device__ static constexpr int b(int t) {
    if (CROSS) return 2 + t % 4;
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

// Sum over the 32 lanes of each half-wave; every lane ends with the same value
// (each step pairs lanes symmetrically, so fp addition order is identical).
__device__ __forceinline__ float half_wave_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // xor 1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // xor 2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)); // half mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)); // mirror
  v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));                     // xor 16
  return v;
}

struct GroupDesc {
  int blk[6];
};

// Group -> list of global client blocks it loads.
__device__ __forceinline__ GroupDesc group_desc(int g, int K, bool cross) {
  GroupDesc d;
  const int nb = cdiv(K, 32);
  if (K <= SUPER) {
    for (int i = 0; i < 6; ++i) d.blk[i] = i;
    (void)nb;
    return d;
  }
  const int nsb = cdiv(K, SUPER);
  if (!cross) {
    for (int i = 0; i < 6; ++i) d.blk[i] = 4 * g + i;
    return d;
  }
  const int q = (g - nsb) >> 1, h = (g - nsb) & 1;
  int I = 0, rem = q;
  while (rem >= nsb - 1 - I) { rem -= nsb - 1 - I; ++I; }
  const int J = I + 1 + rem;
  d.blk[0] = 4 * I + 2 * h;
  d.blk[1] = 4 * I + 2 * h + 1;
  for (int i = 0; i < 4; ++i) d.blk[2 + i] = 4 * J + i;
  return d;
}

template <int NL, bool CROSS>
__global__ __launch_bounds__(THREADS, 2) void gram_partials_kernel(
    const float* __restrict__ X, int K, int64_t ldx, int nchunks, int group_base,
    float* __restrict__ partials, int nseg) {
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

  const int c_begin = (int)((int64_t)nchunks * seg / nseg);
  const int c_end = (int)((int64_t)nchunks * (seg + 1) / nseg);

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

  auto stage = [&](int chunk, float* buf) {
#pragma unroll
    for (int q = 0; q < 2 * NL; ++q) {
      const int inst = wave * 2 * NL + q;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src_row[q] + (int64_t)chunk * CW),
          (__attribute__((address_space(3))) void*)(buf + inst * 256), 16, 0, 0);
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

  const float inv_rows = 1.0f / (float)ROWS;
  int cur = 0;
  if (c_begin < c_end) stage(c_begin, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int c = c_begin; c < c_end; ++c) {
    float* buf = lds + cur * BUF;
    if (c + 1 < c_end) stage(c + 1, lds + (cur ^ 1) * BUF);

    // ---- this wave's k-step: coordinates 16*wave + 8h + j of the chunk ----
    float raw[NL][8];
#pragma unroll
    for (int b = 0; b < NL; ++b) {
      const int lrow = 32 * b + r;
      const int s0 = 4 * wave + 2 * h;
      const int p0 = s0 ^ (lrow & 15), p1 = (s0 + 1) ^ (lrow & 15);
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(buf + lrow * CW + 4 * p0);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(buf + lrow * CW + 4 * p1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        raw[b][j] = v0[j];
        raw[b][4 + j] = v1[j];
      }
    }
    float cen[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = raw[0][j];
#pragma unroll
      for (int b = 1; b < NL; ++b) s += raw[b][j];
      cen[j] = half_wave_sum(s) * inv_rows;
    }
    bf16x8 hi[NL], lo[NL];
#pragma unroll
    for (int b = 0; b < NL; ++b) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float y = raw[b][j] - cen[j];
        const __bf16 hb = (__bf16)y;
        const float hf = (float)hb;
        const __bf16 lb = (__bf16)(y - hf);
        hi[b][j] = hb;
        lo[b][j] = lb;
        const float v = hf + (float)lb;
        dsum[b] = __builtin_fmaf(v, v, dsum[b]);
      }
    }
    static_for<0, NT>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int a = TS::a(t), bb = TS::b(t);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[a], hi[bb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[a], lo[bb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo[a], hi[bb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo[a], lo[bb], acc[t], 0, 0, 0);
    });

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: reduce the 4 waves in fixed order, write the record ----
  float* rec = partials + ((int64_t)blockIdx.y * nseg + seg) * REC;
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

// Sum the per-segment records of every group in fixed order (fp64).
// Thread (w, lane): entry blockIdx.x*64 + lane, segments s = w (mod 4).
__global__ __launch_bounds__(256) void reduce_records_kernel(const float* __restrict__ partials,
                                                              int nseg, double* __restrict__ gsum) {
  __shared__ double red[4][64];
  const int g = blockIdx.y;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  double s = 0.0;
  if (e < REC) {
    const float* p = partials + (int64_t)g * nseg * REC + e;
    for (int k = w; k < nseg; k += 4) s += (double)p[(int64_t)k * REC];
  }
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && e < REC)
    gsum[(int64_t)g * REC + e] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
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

__global__ void assemble_kernel(const double* __restrict__ gsum, const double* __restrict__ tail,
                                int K, double* __restrict__ D) {
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
      g = nsb + 2 * q + (bi >> 1);
      lb_i = bi & 1;
      lb_j = 2 + bj;
      t = lb_i * 4 + bj;
    }
  }
  const double* rec = gsum + (int64_t)g * REC;
  const double gij = rec[t * 1024 + tile_entry(ri, rj)];
  const double gii = rec[REC_TILES * 1024 + 32 * lb_i + ri];
  const double gjj = rec[REC_TILES * 1024 + 32 * lb_j + rj];
  double d2 = gii + gjj - 2.0 * gij + tail[idx];
  if (d2 < 0.0) d2 = 0.0;
  D[idx] = (double)(float)sqrt(d2);
}

struct Plan {
  int nchunks;       // full 64-coordinate chunks
  int nseg;          // segments per group
  int ngroups_diag;  // groups launched with the DIAG kernel
  int ngroups_cross; // groups launched with the CROSS kernel
  int nl_diag;       // loaded blocks per DIAG group
  int ngroups() const { return ngroups_diag + ngroups_cross; }
};

inline Plan make_plan(int64_t K, int64_t P) {
  Plan p;
  p.nchunks = (int)(P / CW);
  if (K <= SUPER) {
    p.ngroups_diag = 1;
    p.ngroups_cross = 0;
    p.nl_diag = cdiv((int)K, 32);
  } else {
    const int nsb = cdiv((int)K, SUPER);
    p.ngroups_diag = nsb;
    p.ngroups_cross = nsb * (nsb - 1);  // two half-groups per super-block pair
    p.nl_diag = 4;
  }
  const int target = std::max(1, 2 * 256 / std::max(1, p.ngroups()));
  p.nseg = std::max(1, std::min(p.nchunks, std::min(MAX_SEG, target)));
  return p;
}

inline size_t ws_partials(const Plan& p) { return (size_t)p.ngroups() * p.nseg * REC * sizeof(float); }
inline size_t ws_gsum(const Plan& p) { return (size_t)p.ngroups() * REC * sizeof(double); }

template <int NL, bool CROSS>
int launch_gram(const float* X, int K, int64_t ldx, const Plan& p, int group_base, int ngroups,
                float* partials, hipStream_t st) {
  const size_t lds = (size_t)2 * 32 * NL * CW * sizeof(float);
  dim3 grid(p.nseg, ngroups);
  hipLaunchKernelGGL((gram_partials_kernel<NL, CROSS>), grid, dim3(THREADS), lds, st, X, K, ldx,
                     p.nchunks, group_base, partials + (size_t)group_base * p.nseg * REC, p.nseg);
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

extern "C" size_t flr_pairwise_l2_workspace(int64_t K, int64_t P) {
  if (K < 1 || P < 0) return 0;
  const Plan p = make_plan(K, P);
  return align_up(ws_partials(p), 256) + align_up(ws_gsum(p), 256) +
         align_up((size_t)K * K * sizeof(double), 256);
}

extern "C" int flr_pairwise_l2(const float* X, int64_t K, int64_t P, int64_t ldx, double* D,
                               void* workspace, size_t workspace_bytes, void* stream) {
  if (K < 1 || P < 0 || ldx < P || !D || (K > 1 && P > 0 && !X)) return FLR_ERR_ARG;
  if (K > (1 << 16)) return FLR_ERR_UNSUPPORTED;
  const size_t need = flr_pairwise_l2_workspace(K, P);
  if (!workspace || workspace_bytes < need || (reinterpret_cast<uintptr_t>(workspace) & 255))
    return FLR_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  const Plan p = make_plan(K, P);
  char* w = static_cast<char*>(workspace);
  float* partials = reinterpret_cast<float*>(w);
  double* gsum = reinterpret_cast<double*>(w + align_up(ws_partials(p), 256));
  double* tail = reinterpret_cast<double*>(w + align_up(ws_partials(p), 256) + align_up(ws_gsum(p), 256));

  // The DMA path reads 16-B pieces: needs 16-B aligned rows.
  const bool aligned = ((reinterpret_cast<uintptr_t>(X) & 15) == 0) && (ldx % 4 == 0);
  const int64_t p_main = aligned ? (int64_t)p.nchunks * CW : 0;
  const int K32 = (int)K;
  int rc = FLR_OK;
  if (p_main > 0) {
    if (K <= SUPER) {
      switch (p.nl_diag) {
        case 1: rc = launch_gram<1, false>(X, K32, ldx, p, 0, 1, partials, st); break;
        case 2: rc = launch_gram<2, false>(X, K32, ldx, p, 0, 1, partials, st); break;
        case 3: rc = launch_gram<3, false>(X, K32, ldx, p, 0, 1, partials, st); break;
        default: rc = launch_gram<4, false>(X, K32, ldx, p, 0, 1, partials, st); break;
      }
    } else {
      rc = launch_gram<4, false>(X, K32, ldx, p, 0, p.ngroups_diag, partials, st);
      if (rc == FLR_OK)
        rc = launch_gram<6, true>(X, K32, ldx, p, p.ngroups_diag, p.ngroups_cross, partials, st);
    }
    if (rc != FLR_OK) return rc;
    dim3 rgrid(cdiv(REC, 64), p.ngroups());
    hipLaunchKernelGGL(reduce_records_kernel, rgrid, dim3(256), 0, st, partials, p.nseg, gsum);
    if ((rc = launch_status("reduce_records_kernel")) != FLR_OK) return rc;
  } else {
    if (hipMemsetAsync(gsum, 0, ws_gsum(p), st) != hipSuccess) return FLR_ERR_HIP;
  }
  const int64_t kk = K * K;
  const int nblk = (int)((kk + 255) / 256);
  hipLaunchKernelGGL(tail_d2_kernel, dim3(nblk), dim3(256), 0, st, X, K32, ldx, p_main, P, tail);
  if ((rc = launch_status("tail_d2_kernel")) != FLR_OK) return rc;
  hipLaunchKernelGGL(assemble_kernel, dim3(nblk), dim3(256), 0, st, gsum, tail, K32, D);
  return launch_status("assemble_kernel");
}

extern "C" size_t flr_pairwise_l2_direct_workspace(int64_t K, int64_t P) {
  if (K < 1 || P < 0) return 0;
  const int nb = cdiv((int)K, 32);
  const int npairs = nb * (nb + 1) / 2;
  return (size_t)npairs * direct_nseg(K, P) * 1024 * sizeof(float);
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
