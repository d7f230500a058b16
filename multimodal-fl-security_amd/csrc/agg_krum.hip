// a10 — Krum score + selection on the device.
//
// Replaces KrumDefense._krum_score and the selection in aggregate
// (src/defenses/krum.py:101-131, 149-176):
//   sorted = np.sort(distances[i]); score = np.sum(sorted[1 : m + 1])
//   order  = np.argsort(scores)
// np.sum over a contiguous float64 slice is numpy's pairwise summation
// (8 accumulators for n <= 128, recursive halving above); it is restated
// exactly here, so scores are bit-identical to numpy given the same D.
// np.argsort's default quicksort is not stable; exact score ties are broken
// here by the lower client index (documented divergence, tests flag ties).
// NaN as numpy orders it: np.sort and np.argsort put NaN after +inf, so a
// NaN distance lands in a row's last ranks and a NaN score (a client that sent
// NaN) is ranked last — rejected, not selected.  Every order slot is written.
#include "flr_common.h"

namespace flr {
namespace krum {

constexpr int MAXK = 1024;

// a sorts after b in numpy's order (NaN after everything, NaNs equal)
__device__ __forceinline__ bool np_after(double a, double b) { return a > b || (a != a && b == b); }
__device__ __forceinline__ bool np_equal(double a, double b) { return a == b || (a != a && b != b); }

// numpy pairwise_sum_DOUBLE (numpy/_core/src/umath/loops_utils.h.src), exact.
template <int DEPTH>
__device__ double np_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128 || DEPTH == 0) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  if constexpr (DEPTH > 0) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sum<DEPTH - 1>(a, n2) + np_pairwise_sum<DEPTH - 1>(a + n2, n - n2);
  }
  return 0.0;
}

// One workgroup per client row: bitonic sort of the row in LDS, then the
// numpy pairwise sum of ranks 1..m.
__global__ __launch_bounds__(256) void score_kernel(const double* __restrict__ D, int K, int m,
                                                    double* __restrict__ scores) {
  __shared__ double s[MAXK];
  const int i = blockIdx.x;
  int np2 = 1;
  while (np2 < K) np2 <<= 1;
  for (int j = threadIdx.x; j < np2; j += blockDim.x)
    s[j] = j < K ? D[(int64_t)i * K + j] : __builtin_nan("");  // pads sort with the NaNs, after every value
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int idx = threadIdx.x; idx < np2; idx += blockDim.x) {
        const int ixj = idx ^ j;
        if (ixj > idx) {
          const double a = s[idx], b = s[ixj];
          const bool up = (idx & k) == 0;
          if ((up && np_after(a, b)) || (!up && np_after(b, a))) {
            s[idx] = b;
            s[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) scores[i] = 0.0 + np_pairwise_sum<4>(s + 1, m);
}

// Stable rank: order[rank(i)] = i.
__global__ __launch_bounds__(1024) void order_kernel(const double* __restrict__ scores, int K,
                                                     int32_t* __restrict__ order) {
  __shared__ double s[MAXK];
  for (int j = threadIdx.x; j < K; j += blockDim.x) s[j] = scores[j];
  __syncthreads();
  for (int i = threadIdx.x; i < K; i += blockDim.x) {
    const double si = s[i];
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const double sj = s[j];
      rank += np_after(si, sj) || (np_equal(sj, si) && j < i);
    }
    order[rank] = i;
  }
}

}  // namespace krum
}  // namespace flr

using namespace flr;

extern "C" int flr_krum_select(const double* D, int64_t K, int64_t f, double* scores,
                               int32_t* order, void* stream) {
  if (K < 1 || f < 0 || !D || !scores || !order) return FLR_ERR_ARG;
  if (K < 2 * f + 3) return FLR_ERR_KRUM_N;
  if (K > krum::MAXK) return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  const int m = (int)(K - f - 2);
  hipLaunchKernelGGL(krum::score_kernel, dim3((int)K), dim3(256), 0, st, D, (int)K, m, scores);
  int rc = launch_status("krum score_kernel");
  if (rc != FLR_OK) return rc;
  hipLaunchKernelGGL(krum::order_kernel, dim3(1), dim3(1024), 0, st, scores, (int)K, order);
  return launch_status("krum order_kernel");
}
