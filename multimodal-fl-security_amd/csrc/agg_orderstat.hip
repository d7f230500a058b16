// a12 / a13 — coordinate-wise trimmed mean and lower median on gfx950.
//
// Replaces TrimmedMeanDefense.aggregate (src/defenses/trimmed_mean.py:48-90)
// and MedianDefense.aggregate / _coordinate_wise_median (:92-103, 141-166).
// The reference stacks the K client tensors, runs torch.sort(dim=0), slices
// rows [t, K-t) and calls .mean(dim=0) (trimmed) or torch.median(dim=0)
// (lower median = sorted row (K-1)/2).
//
// Engine: one lane per coordinate.  The lane loads its K values (each load
// instruction reads 256 contiguous bytes of one client row), sorts them in
// registers with Batcher's odd-even merge network (padded to a power of two
// with +inf; 1471 compare-exchanges at K = 128, all register-resident), then
// reads the order statistics with compile-time register indices.  The
// trimmed sum restates torch's CPU outer-reduction order (cascade_sum:
// 16-row blocks folded through 4 levels, then divided by R), which makes it
// bit-identical to torch on the vectorised columns.
//
// NaN: torch.sort orders NaN after +inf and torch.median(dim=0) returns NaN
// for a column holding any NaN.  The min/max compare-exchanges below would
// instead drop a NaN (fminf/fmaxf return the other operand), so a wave that
// loaded any NaN (one ballot; never in practice) maps each NaN to +inf and
// counts them: the top n_nan ranks of torch's order are then exactly the
// NaN, the median is NaN when n_nan > 0, and the trimmed mean is NaN when
// n_nan > t (a NaN survives the trim).
#include "flr_common.h"

#include <type_traits>

namespace flr {
namespace ostat {

constexpr int THREADS = 256;

__device__ __forceinline__ void cas(float& a, float& b) {
  const float lo = fminf(a, b), hi = fmaxf(a, b);
  a = lo;
  b = hi;
}

template <int LO, int N, int R>
__device__ __forceinline__ void oem_merge(float* v) {
  constexpr int M = R * 2;
  if constexpr (M < N) {
    oem_merge<LO, N, M>(v);
    oem_merge<LO + R, N, M>(v);
#pragma unroll
    for (int i = LO + R; i + R < LO + N; i += M) cas(v[i], v[i + R]);
  } else {
    cas(v[LO], v[LO + R]);
  }
}

template <int LO, int N>
__device__ __forceinline__ void oem_sort(float* v) {
  if constexpr (N > 1) {
    constexpr int M = N / 2;
    oem_sort<LO, M>(v);
    oem_sort<LO + M, M>(v);
    oem_merge<LO, N, 1>(v);
  }
}

// Maps NaN to +inf in place and returns this lane's NaN count; the scan runs
// only in a wave that loaded a NaN (wave-uniform branch).
template <int N>
__device__ __forceinline__ int nan_to_inf(float* v) {
  bool any = false;
#pragma unroll
  for (int k = 0; k < N; ++k) any |= __builtin_isnan(v[k]);
  int n = 0;
  if (__any(any)) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const bool isn = __builtin_isnan(v[k]);
      n += isn ? 1 : 0;
      v[k] = isn ? __builtin_huge_valf() : v[k];
    }
  }
  return n;
}

template <int N>
__device__ __forceinline__ void reg_fence(float* v) {
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" : "+v"(v[k]));
}

// MODE 0: trimmed mean over ranks [t, K-t); MODE 1: lower median.
// 3 waves/SIMD: the NP = 128 network fits the 168 VGPRs available.
template <int NP, int MODE>
__global__ __launch_bounds__(THREADS, 3) void orderstat_kernel(const float* __restrict__ X, int K, int64_t P,
                                                            int64_t ldx, int t, float* __restrict__ out,
                                                            const int32_t* __restrict__ rows, uint32_t rmax) {
  const int64_t p = (int64_t)blockIdx.x * THREADS + threadIdx.x;
  if (p >= P) return;
  float v[NP];
  if (rows) {  // a row subset (e.g. the Multi-Krum selection); the index loads are wave-uniform
#pragma unroll
    for (int k = 0; k < NP; ++k) v[k] = k < K ? X[(int64_t)min((uint32_t)rows[k], rmax) * ldx + p] : __builtin_huge_valf();
  } else {
#pragma unroll
    for (int k = 0; k < NP; ++k) v[k] = k < K ? X[(int64_t)k * ldx + p] : __builtin_huge_valf();
  }
  // Empty asm fences pin all NP values in VGPRs at the phase boundaries, so
  // the compiler cannot stretch load, sort and sum live ranges into one
  // another: without them ROCm 7.2 spilled 237-283 VGPRs of the NP = 128
  // trimmed mean to scratch (5.7 ms at C3's K = 128, P = 11.8 M, against
  // 1.6 ms for the median); with them 5 (the output address and NaN count,
  // stored once).
  reg_fence<NP>(v);
  const int nnan = nan_to_inf<NP>(v);
  oem_sort<0, NP>(v);
  if constexpr (MODE == 0) reg_fence<NP>(v);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (MODE == 1) {
    const int med = (K - 1) / 2;
    float r = v[0];
#pragma unroll
    for (int k = 1; k < NP; ++k) r = (k == med) ? v[k] : r;
    out[p] = nnan > 0 ? __builtin_nanf("") : r;
  } else {
    // t, R wave-uniform (SGPRs): the rank tests are scalar compares and uniform
    // branches, no per-rank lane masks
    const int tu = __builtin_amdgcn_readfirstlane(t);
    const int R = __builtin_amdgcn_readfirstlane(K - 2 * tu);
    const int nfull = R & ~15;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int pos = k - tu;
      if ((unsigned)pos < (unsigned)R) {
        a0 = add_rn(a0, v[k]);
        if (pos < nfull && ((pos + 1) & 15) == 0) {
          a1 = add_rn(a1, a0);
          a0 = 0.f;
        }
      }
      // NP <= 128: a block end i = pos + 1 is at most 128, never a multiple of
      // 256, so the level-2/3 folds (i & 0xF0 == 0, i & 0xF00 == 0) never fire.
      static_assert(NP <= 128, "level-2 cascade folds not implemented");
    }
    a0 = add_rn(a0, a1);
    a0 = add_rn(a0, a2);
    a0 = add_rn(a0, a3);
    out[p] = nnan > t ? __builtin_nanf("") : div_rn(a0, (float)R);
  }
}


// ---- K > 128: one coordinate spread over L = 2 or 4 adjacent lanes ------------
// Lane g of the group holds clients [128g, 128g+128) (padding +inf).  Each lane
// first sorts its 128 registers with the same odd-even merge network as the
// single-lane kernel (all directions compile-time, 2 VALU ops per compare).
// Sorted lanes are then merged pairwise by bitonic merges:
//   flip step: lane g's register i meets register 127-i of the partner lane
//              (DPP quad permutation), the lower lane keeps the min, the upper
//              the max -- one v_med3_f32 against a lane-constant -inf / +inf;
//   (L = 4) a cross-lane half-cleaner between lanes g and g^1, same register;
//   then a 7-stage in-lane half-cleaner (j = 64..1, ascending everywhere).
// Rank e then sits in lane e/128, register e%128.  About half the VALU work of a
// full 512-wide bitonic sort.  SPLIT (K = 128 * L: every register a client): the same network with
// the in-lane sort's 32-register quarters screened and sorted in turn, so ≈ 1600 of
// its ≈ 5250 compare-exchange instructions run while later quarters' loads are
// still in flight (C5 trimmed mean 23.7 -> 23.3 ms, median 19.9 -> 19.2; C4 10.1 ->
// 9.8 and 8.5 -> 8.0; halves gave 23.4 / 19.4 / 9.9 / 8.2).  Trimmed sums follow
// torch's cascade in rank order across the group's lanes (below): bit-identical
// to torch on the vectorised columns, as the single-lane kernel.
template <int CTRL>
__device__ __forceinline__ float dpp_swap(float x) {
  // all lanes valid (quad permutation, full masks): no "old" operand to initialise
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}

// med3(a, b, -inf) = min(a, b); med3(a, b, +inf) = max(a, b)
template <int CTRL>
__device__ __forceinline__ void merge_flip(float* v, float bound) {
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const float wa = dpp_swap<CTRL>(v[127 - i]);
    const float wb = dpp_swap<CTRL>(v[i]);
    v[i] = __builtin_amdgcn_fmed3f(v[i], wa, bound);
    v[127 - i] = __builtin_amdgcn_fmed3f(v[127 - i], wb, bound);
  }
}

template <int CTRL>
__device__ __forceinline__ void merge_cross(float* v, float bound) {
#pragma unroll
  for (int i = 0; i < 128; ++i) v[i] = __builtin_amdgcn_fmed3f(v[i], dpp_swap<CTRL>(v[i]), bound);
}

__device__ __forceinline__ void half_clean_lane(float* v) {
#pragma unroll
  for (int j = 64; j >= 1; j >>= 1) {
#pragma unroll
    for (int i = 0; i < 128; ++i)
      if ((i & j) == 0) cas(v[i], v[i + j]);
  }
}

template <int L, int MODE, bool SPLIT, bool ROWS>
__global__ __launch_bounds__(THREADS) void orderstat_multilane_kernel(const float* __restrict__ X, int K,
                                                                         int64_t P, int64_t ldx, int t,
                                                                         float* __restrict__ out,
                                                                         const int32_t* __restrict__ rows,
                                                                         uint32_t rmax) {
  const int64_t gidx = (int64_t)blockIdx.x * THREADS + threadIdx.x;
  const int64_t p = gidx / L;
  const int g = (int)(gidx % L);
  const bool active = p < P;  // inactive lanes still join the exchanges
  const int64_t pc = active ? p : 0;
  float v[128];
  if constexpr (ROWS) {
    // a row subset (e.g. the Multi-Krum selection): the workgroup stages the clamped
    // indices in LDS once (padding entries repeat row 0), so a lane's 128 loads issue
    // back to back instead of each waiting on its own index load
    __shared__ int32_t srow[128 * L];
    for (int i = threadIdx.x; i < 128 * L; i += THREADS) srow[i] = (int32_t)min((uint32_t)rows[i < K ? i : 0], rmax);
    __syncthreads();
    const int32_t* rg = srow + 128 * g;
    const float* __restrict__ col = X + pc;
#pragma unroll
    for (int i = 0; i < 128; ++i) v[i] = col[(int64_t)rg[i] * ldx];
    if constexpr (!SPLIT) {
#pragma unroll
      for (int i = 0; i < 128; ++i) v[i] = 128 * g + i < K ? v[i] : __builtin_huge_valf();
    }
  } else if constexpr (SPLIT) {
    const float* __restrict__ base = X + (int64_t)(128 * g) * ldx + pc;
#pragma unroll
    for (int i = 0; i < 128; ++i) v[i] = base[(int64_t)i * ldx];
  } else {
    const float* __restrict__ base = X + (int64_t)(128 * g) * ldx + pc;
    if (K >= 128 * L) {  // wave-uniform: every register holds a client
#pragma unroll
      for (int i = 0; i < 128; ++i) v[i] = base[(int64_t)i * ldx];
    } else {
#pragma unroll
      for (int i = 0; i < 128; ++i) v[i] = 128 * g + i < K ? base[(int64_t)i * ldx] : __builtin_huge_valf();
    }
  }
  int nnan;
  if constexpr (SPLIT) {
    // every lane holds K / L clients here (K = 128 * L): the in-lane sort's quarters
    // are screened and sorted as their loads land; the ordered fences put each later
    // quarter's load wait behind the sorts before it (vmcnt counts at most 63, so the
    // first wait covers two quarters)
    nnan = nan_to_inf<32>(v);
    oem_sort<0, 32>(v);
    reg_fence<32>(v);
    reg_fence<32>(v + 32);
    nnan += nan_to_inf<32>(v + 32);
    oem_sort<32, 32>(v);
    oem_merge<0, 64, 1>(v);
    reg_fence<64>(v);
    reg_fence<32>(v + 64);
    nnan += nan_to_inf<32>(v + 64);
    oem_sort<64, 32>(v);
    reg_fence<32>(v + 64);
    reg_fence<32>(v + 96);
    nnan += nan_to_inf<32>(v + 96);
    oem_sort<96, 32>(v);
    oem_merge<64, 64, 1>(v);
    oem_merge<0, 128, 1>(v);
  } else {
    nnan = nan_to_inf<128>(v);
    oem_sort<0, 128>(v);
  }
  if (__any(nnan > 0)) {  // the coordinate's total over its L lanes (adjacent lanes)
    nnan += __shfl_xor(nnan, 1, 64);
    if constexpr (L == 4) nnan += __shfl_xor(nnan, 2, 64);
  }
  const float inf = __builtin_huge_valf();
  // Rank pruning for the median: after the last merge's cross-lane stages every
  // lane holds exactly its 128 ranks (unsorted).  When the median is the top
  // rank of a lane (med % 128 == 127: K = 255/256 over 2 lanes, 511/512 over
  // 4) it is that lane's maximum, so the final in-lane half-cleaner (7 stages
  // of 64 compare-exchanges) becomes one 127-step max.  Wave-uniform (K).
  const int medk = (K - 1) / 2;
  const bool top = MODE == 1 && (medk & 127) == 127;
  // pairs (0,1), (2,3): quad permutation [1,0,3,2]
  merge_flip<0xB1>(v, (g & 1) ? inf : -inf);
  if constexpr (L == 4) {
    half_clean_lane(v);
    // (0,1) against (2,3): flip partners g^3 = quad permutation [3,2,1,0]
    merge_flip<0x1B>(v, g < 2 ? -inf : inf);
    merge_cross<0xB1>(v, (g & 1) ? inf : -inf);
  }
  if (!top) half_clean_lane(v);
  __builtin_amdgcn_sched_barrier(0);
  float r = 0.f;
  if constexpr (MODE == 1) {
    const int med = medk;
    const int loc = med - 128 * g;
    if (top) {
      float mx = v[0];
#pragma unroll
      for (int i = 1; i < 128; ++i) mx = fmaxf(mx, v[i]);
      if (active && g == med / 128) out[p] = nnan > 0 ? __builtin_nanf("") : mx;
      return;
    }
#pragma unroll
    for (int i = 0; i < 128; ++i) r = (i == loc) ? v[i] : r;
    if (active && g == med / 128) out[p] = nnan > 0 ? __builtin_nanf("") : r;  // the lane that owns rank med
  } else {
    // torch's outer-reduction cascade (multi_row_sum, level step 16: the block
    // sums folded into a1 every 16 ranks, a1 into a2 every 256) over the ranks
    // [t, K - t) in rank order, which run through the group's lanes in lane
    // order: pass s continues the cascade over lane s's registers from the state
    // lane s - 1 left (broadcast in the group), so every add is torch's add in
    // torch's order (bit-identical on the vectorised columns, like the
    // single-lane kernel).  Every lane runs every pass (wave-uniform work: L x
    // 128 conditional adds against the ~5000-instruction sort)
    const int tu = __builtin_amdgcn_readfirstlane(t);
    const int R = __builtin_amdgcn_readfirstlane(K - 2 * tu);
    const int nfull = R & ~15;
    static_assert(128 * L <= 4096, "the level-3 fold (4096 ranks) is not implemented");
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    const int gbase = (int)(threadIdx.x & 63) & ~(L - 1);
#pragma unroll
    for (int s = 0; s < L; ++s) {
      float b0 = a0, b1 = a1, b2 = a2;
#pragma unroll
      for (int i = 0; i < 128; ++i) {
        const int pos = 128 * g + i - tu;
        const bool in = (unsigned)pos < (unsigned)R;
        b0 = in ? add_rn(b0, v[i]) : b0;
        const bool f1 = in && pos < nfull && ((pos + 1) & 15) == 0;
        const bool f2 = f1 && ((pos + 1) & 0xF0) == 0;
        b1 = f1 ? add_rn(b1, b0) : b1;
        b0 = f1 ? 0.f : b0;
        b2 = f2 ? add_rn(b2, b1) : b2;
        b1 = f2 ? 0.f : b1;
      }
      a0 = __shfl(b0, gbase + s, 64);
      a1 = __shfl(b1, gbase + s, 64);
      a2 = __shfl(b2, gbase + s, 64);
    }
    float tot = add_rn(a0, a1);
    tot = add_rn(tot, a2);
    if (active && g == 0) out[p] = nnan > t ? __builtin_nanf("") : div_rn(tot, (float)(K - 2 * t));
  }
}

template <int L, int MODE>
void launch_ml(bool full, bool has_rows, const float* X, int K, int64_t P, int64_t ldx, int t, float* out,
               const int32_t* rows, uint32_t rmax, hipStream_t st) {
  const dim3 grid((unsigned)((L * P + THREADS - 1) / THREADS));
  auto k = full ? (has_rows ? orderstat_multilane_kernel<L, MODE, true, true>
                            : orderstat_multilane_kernel<L, MODE, true, false>)
                : (has_rows ? orderstat_multilane_kernel<L, MODE, false, true>
                            : orderstat_multilane_kernel<L, MODE, false, false>);
  hipLaunchKernelGGL(k, grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out, rows, rmax);
}

template <int MODE>
int launch(const float* X, int K, int64_t P, int64_t ldx, int t, float* out, hipStream_t st,
           const int32_t* rows = nullptr, int64_t nrows = 0) {
  // a row index outside [0, nrows) is clamped into range: no out-of-bounds read
  // (the result is then unspecified; flr.h states the precondition)
  const uint32_t rmax = (uint32_t)(nrows > 0 ? nrows - 1 : 0);
  const dim3 grid((unsigned)((P + THREADS - 1) / THREADS));
  if (K <= 8)
    hipLaunchKernelGGL((orderstat_kernel<8, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out, rows, rmax);
  else if (K <= 16)
    hipLaunchKernelGGL((orderstat_kernel<16, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out, rows, rmax);
  else if (K <= 32)
    hipLaunchKernelGGL((orderstat_kernel<32, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out, rows, rmax);
  else if (K <= 64)
    hipLaunchKernelGGL((orderstat_kernel<64, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out, rows, rmax);
  else if (K <= 128)
    hipLaunchKernelGGL((orderstat_kernel<128, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out, rows, rmax);
  else if (K <= 512) {
    // K = 128 * L (every register a client): the split-load form; a row subset: the
    // LDS-staged index form
    const bool full = K == 256 || K == 512;
    if (K <= 256)
      launch_ml<2, MODE>(full, rows != nullptr, X, K, P, ldx, t, out, rows, rmax, st);
    else
      launch_ml<4, MODE>(full, rows != nullptr, X, K, P, ldx, t, out, rows, rmax, st);
  }
  else
    return FLR_ERR_UNSUPPORTED;
  return launch_status("orderstat_kernel");
}

}  // namespace ostat
}  // namespace flr

using namespace flr;

extern "C" int flr_trimmed_mean(const float* X, int64_t K, int64_t P, int64_t ldx, int64_t t, float* out,
                                void* stream) {
  if (K < 1 || P < 0 || ldx < P || t < 0 || K - 2 * t < 1 || !X || !out) return FLR_ERR_ARG;
  if (P == 0) return FLR_OK;
  return ostat::launch<0>(X, (int)K, P, ldx, (int)t, out, as_stream(stream));
}

extern "C" int flr_median_lower(const float* X, int64_t K, int64_t P, int64_t ldx, float* out, void* stream) {
  if (K < 1 || P < 0 || ldx < P || !X || !out) return FLR_ERR_ARG;
  if (P == 0) return FLR_OK;
  return ostat::launch<1>(X, (int)K, P, ldx, 0, out, as_stream(stream));
}

extern "C" int flr_trimmed_mean_rows(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows,
                                     int64_t m, int64_t t, float* out, void* stream) {
  if (K < 1 || m < 1 || m > K || P < 0 || ldx < P || t < 0 || m - 2 * t < 1 || !X || !out || !rows)
    return FLR_ERR_ARG;
  if (P == 0) return FLR_OK;
  return ostat::launch<0>(X, (int)m, P, ldx, (int)t, out, as_stream(stream), rows, K);
}

extern "C" int flr_median_lower_rows(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows,
                                     int64_t m, float* out, void* stream) {
  if (K < 1 || m < 1 || m > K || P < 0 || ldx < P || !X || !out || !rows) return FLR_ERR_ARG;
  if (P == 0) return FLR_OK;
  return ostat::launch<1>(X, (int)m, P, ldx, 0, out, as_stream(stream), rows, K);
}
