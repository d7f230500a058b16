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
