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

// MODE 0: trimmed mean over ranks [t, K-t); MODE 1: lower median.
template <int NP, int MODE>
// 3 waves/SIMD: the NP=128 network needs ~150 VGPRs; the bound stops the
// trimmed sum from pushing the kernel over the 168-VGPR occupancy step.
__global__ __launch_bounds__(THREADS, 3) void orderstat_kernel(const float* __restrict__ X, int K, int64_t P,
                                                            int64_t ldx, int t, float* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * THREADS + threadIdx.x;
  if (p >= P) return;
  float v[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) v[k] = k < K ? X[(int64_t)k * ldx + p] : __builtin_huge_valf();
  oem_sort<0, NP>(v);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (MODE == 1) {
    const int med = (K - 1) / 2;
    float r = v[0];
#pragma unroll
    for (int k = 1; k < NP; ++k) r = (k == med) ? v[k] : r;
    out[p] = r;
  } else {
    const int R = K - 2 * t;
    const int nfull = R & ~15;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int pos = k - t;
      // branch-free (selects keep the live ranges short; t, R are wave-uniform)
      const bool in = (unsigned)pos < (unsigned)R;
      const float n0 = add_rn(a0, v[k]);
      a0 = in ? n0 : a0;
      const bool blk = in && pos < nfull && ((pos + 1) & 15) == 0;
      const int i = pos + 1;
      const bool l2 = blk && (i & 0xF0) == 0;
      const bool l3 = l2 && (i & 0xF00) == 0;
      const float n1 = add_rn(a1, a0);
      a1 = blk ? n1 : a1;
      a0 = blk ? 0.f : a0;
      const float n2 = add_rn(a2, a1);
      a2 = l2 ? n2 : a2;
      a1 = l2 ? 0.f : a1;
      const float n3 = add_rn(a3, a2);
      a3 = l3 ? n3 : a3;
      a2 = l3 ? 0.f : a2;
    }
    a0 = add_rn(a0, a1);
    a0 = add_rn(a0, a2);
    a0 = add_rn(a0, a3);
    out[p] = div_rn(a0, (float)R);
  }
}


// ---- K > 128: one coordinate spread over L = 2 or 4 adjacent lanes ------------
// Lane g of the group holds clients [128g, 128g+128) (padding +inf) and the
// group runs a full bitonic sort over N = 128 L elements, element e = 128g + i
// in register i of lane g: stages with j < 128 compare registers of one lane
// (direction known at compile time while k <= 128, per lane above), stages with
// j >= 128 exchange register i with lane g ^ (j/128).  Rank e then sits in lane
// e/128, register e%128.  Trimmed sums are per-lane sequential in rank order,
// combined in lane order (deterministic; 1e-5 vs torch, not bit-exact).
template <int K2, int J>
__device__ __forceinline__ void bitonic_reg_stage(float* v, bool asc_lane) {
  // k = K2, j = J < 128: pairs (i, i ^ J) inside the lane
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    const int p = i ^ J;
    if (p > i) {
      const float a = v[i], b = v[p];
      const float lo = fminf(a, b), hi = fmaxf(a, b);
      bool asc;
      if constexpr (K2 < 128) asc = (i & K2) == 0;  // (128g + i) & K2 == i & K2
      else asc = asc_lane;                          // K2 >= 128: set by the lane index
      v[i] = asc ? lo : hi;
      v[p] = asc ? hi : lo;
    }
  }
}

template <int K2, int J>
__device__ __forceinline__ void bitonic_lane_stage(float* v, int g) {
  constexpr int JL = J / 128;
  const bool lower = (g & JL) == 0;
  const bool asc = ((g * 128) & K2) == 0;
  const bool keep_min = lower == asc;
  // partner lane = lane ^ JL (JL = 1 or 2): a DPP quad permutation, so the
  // exchange is one VALU op per register (no LDS round trip, short live range)
  constexpr int CTRL = JL == 1 ? 0xB1 : 0x4E;
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    const float w = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[i]), CTRL, 0xF, 0xF, false));
    v[i] = keep_min ? fminf(v[i], w) : fmaxf(v[i], w);
  }
}

template <int K2, int J, int N>
__device__ __forceinline__ void bitonic_stages_j(float* v, int g) {
  if constexpr (J >= 1) {
    if constexpr (J >= 128) bitonic_lane_stage<K2, J>(v, g);
    else bitonic_reg_stage<K2, J>(v, ((g * 128) & K2) == 0);
    bitonic_stages_j<K2, J / 2, N>(v, g);
  }
}

template <int K2, int N>
__device__ __forceinline__ void bitonic_sort_all(float* v, int g) {
  if constexpr (K2 <= N) {
    bitonic_stages_j<K2, K2 / 2, N>(v, g);
    bitonic_sort_all<K2 * 2, N>(v, g);
  }
}

template <int L, int MODE>
__global__ __launch_bounds__(THREADS) void orderstat_multilane_kernel(const float* __restrict__ X, int K,
                                                                         int64_t P, int64_t ldx, int t,
                                                                         float* __restrict__ out) {
  const int64_t gidx = (int64_t)blockIdx.x * THREADS + threadIdx.x;
  const int64_t p = gidx / L;
  const int g = (int)(gidx % L);
  const bool active = p < P;  // inactive lanes still join the shuffles
  const int64_t pc = active ? p : 0;
  float v[128];
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    const int k = 128 * g + i;
    v[i] = k < K ? X[(int64_t)k * ldx + pc] : __builtin_huge_valf();
  }
  bitonic_sort_all<2, 128 * L>(v, g);
  __builtin_amdgcn_sched_barrier(0);
  float r = 0.f;
  if constexpr (MODE == 1) {
    const int med = (K - 1) / 2;
    const int loc = med - 128 * g;
#pragma unroll
    for (int i = 0; i < 128; ++i) r = (i == loc) ? v[i] : r;
    if (active && g == med / 128) out[p] = r;  // the lane that owns rank med
  } else {
    const int lo = t, hi = K - t;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 128; ++i) {
      const int e = 128 * g + i;
      acc = (e >= lo && e < hi) ? add_rn(acc, v[i]) : acc;
    }
    // combine lanes in order 0..L-1 (lane 0 ends with the total)
    float tot = acc;
    if constexpr (L >= 2) {
      const float a1 = __shfl_down(acc, 1, 64);
      tot = add_rn(acc, a1);  // lanes 0: acc0 + acc1 ; lane 2: acc2 + acc3
      if constexpr (L == 4) {
        const float t2 = __shfl_down(tot, 2, 64);
        tot = add_rn(tot, t2);
      }
    }
    if (active && g == 0) out[p] = div_rn(tot, (float)(K - 2 * t));
  }
}

template <int MODE>
int launch(const float* X, int K, int64_t P, int64_t ldx, int t, float* out, hipStream_t st) {
  const dim3 grid((unsigned)((P + THREADS - 1) / THREADS));
  if (K <= 8)
    hipLaunchKernelGGL((orderstat_kernel<8, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out);
  else if (K <= 16)
    hipLaunchKernelGGL((orderstat_kernel<16, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out);
  else if (K <= 32)
    hipLaunchKernelGGL((orderstat_kernel<32, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out);
  else if (K <= 64)
    hipLaunchKernelGGL((orderstat_kernel<64, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out);
  else if (K <= 128)
    hipLaunchKernelGGL((orderstat_kernel<128, MODE>), grid, dim3(THREADS), 0, st, X, K, P, ldx, t, out);
  else if (K <= 256)
    hipLaunchKernelGGL((orderstat_multilane_kernel<2, MODE>), dim3((unsigned)((2 * P + THREADS - 1) / THREADS)),
                       dim3(THREADS), 0, st, X, K, P, ldx, t, out);
  else if (K <= 512)
    hipLaunchKernelGGL((orderstat_multilane_kernel<4, MODE>), dim3((unsigned)((4 * P + THREADS - 1) / THREADS)),
                       dim3(THREADS), 0, st, X, K, P, ldx, t, out);
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
