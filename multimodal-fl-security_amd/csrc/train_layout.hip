// a1 / a8 / a15 — round-boundary layout moves of the training state.
//
// load_global (run_experiments.py:203, every client starts from the global
// model): broadcast one parameter block to all K clients' blocks.
// export (run_experiments.py:238-240 + krum.py:55-57, the update list
// flattened in parameters() order): the parameter-major training blocks ->
// rows of the client-major client matrix, and for tap-major conv weights the
// [KH*KW][Cin][Cout] -> [Cout][Cin][KH*KW] permutation back to torch order.
// All HBM-bound copies: 16-B accesses where alignment allows; the transpose
// goes through a [taps][16][64] LDS tile so both sides are coalesced.
#include "flr_common.h"

#include <algorithm>

namespace flr {
namespace layout {

constexpr int THREADS = 256;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// dst[k * dstride + i] = src[i], i < n, k < K  (grid: chunks x K); rows
// k < nneg get -src (the sign-flip attackers' copy of an untrained range)
template <bool VEC>
__global__ __launch_bounds__(THREADS) void broadcast_kernel(const float* __restrict__ src, int64_t n,
                                                            float* __restrict__ dst, int64_t dstride, int nneg) {
  float* d = dst + (int64_t)blockIdx.y * dstride;
  const float sg = (int)blockIdx.y < nneg ? -1.f : 1.f;
  if constexpr (VEC) {
    const int64_t nv = n / 4;
    for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < nv; i += (int64_t)gridDim.x * THREADS)
      reinterpret_cast<f32x4*>(d)[i] = reinterpret_cast<const f32x4*>(src)[i] * sg;
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) d[4 * nv + threadIdx.x] = src[4 * nv + threadIdx.x] * sg;
  } else {
    for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS)
      d[i] = src[i] * sg;
  }
}

// dst[k * dstride + i] = src[k * sstride + i]
// rows k < nneg are written negated (the sign-flip attackers' submission,
// model_poisoning.py:274-276, folded into the export pass)
template <bool VEC>
__global__ __launch_bounds__(THREADS) void copy_rows_kernel(const float* __restrict__ src, int64_t sstride,
                                                            int64_t n, float* __restrict__ dst, int64_t dstride,
                                                            int nneg) {
  const float* s = src + (int64_t)blockIdx.y * sstride;
  float* d = dst + (int64_t)blockIdx.y * dstride;
  const float sg = (int)blockIdx.y < nneg ? -1.f : 1.f;
  if constexpr (VEC) {
    const int64_t nv = n / 4;
    for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < nv; i += (int64_t)gridDim.x * THREADS)
      reinterpret_cast<f32x4*>(d)[i] = reinterpret_cast<const f32x4*>(s)[i] * sg;
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) d[4 * nv + threadIdx.x] = s[4 * nv + threadIdx.x] * sg;
  } else {
    for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS)
      d[i] = s[i] * sg;
  }
}

// Tap-major [k][t][ci][co] (KK taps) -> torch order [k][co][ci][t] at
// dst + k * dstride.  One workgroup = (16 ci) x (64 co) x all taps of one
// client: loads walk co (coalesced), stores walk (ci, t) for each co (a
// contiguous run of 16 * KK floats).
constexpr int TCI = 16, TCO = 64, MAXKK = 9;
template <bool VEC>
__global__ __launch_bounds__(THREADS) void tap_to_ref_kernel(const float* __restrict__ wt, int KK, int Cin, int Cout,
                                                             float* __restrict__ dst, int64_t dstride, int nneg) {
  __shared__ float tile[MAXKK * TCI][TCO + 1];
  const int k = blockIdx.z;
  const float sg = k < nneg ? -1.f : 1.f;
  const int ci0 = blockIdx.y * TCI, co0 = blockIdx.x * TCO;
  const float* src = wt + (int64_t)k * KK * Cin * Cout;
  float* out = dst + (int64_t)k * dstride;
  const int run = TCI * KK;  // (ci, t) pairs per co
  if constexpr (VEC) {  // full tile (Cin % 16 == 0, Cout % 64 == 0), 16-B aligned rows
    for (int e = threadIdx.x; e < KK * TCI * (TCO / 4); e += THREADS) {
      const int c4 = e % (TCO / 4), r = e / (TCO / 4);  // r = t * TCI + ci
      const int t = r / TCI, ci = r % TCI;
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + ((int64_t)t * Cin + ci0 + ci) * Cout + co0 + 4 * c4);
#pragma unroll
      for (int q = 0; q < 4; ++q) tile[r][4 * c4 + q] = v[q] * sg;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < TCO * (run / 4); e += THREADS) {
      const int co = e / (run / 4), q0 = 4 * (e % (run / 4));  // q = ci * KK + t
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = tile[((q0 + q) % KK) * TCI + (q0 + q) / KK][co];
      *reinterpret_cast<f32x4*>(out + ((int64_t)(co0 + co) * Cin + ci0) * KK + q0) = v;
    }
  } else {
    for (int e = threadIdx.x; e < KK * TCI * TCO; e += THREADS) {
      const int co = e % TCO, r = e / TCO;
      const int t = r / TCI, ci = r % TCI;
      float v = 0.f;
      if (ci0 + ci < Cin && co0 + co < Cout) v = src[((int64_t)t * Cin + ci0 + ci) * Cout + co0 + co] * sg;
      tile[r][co] = v;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < TCO * run; e += THREADS) {
      const int co = e / run, q = e % run;
      const int ci = q / KK, t = q % KK;
      if (ci0 + ci < Cin && co0 + co < Cout)
        out[((int64_t)(co0 + co) * Cin + ci0 + ci) * KK + t] = tile[t * TCI + ci][co];
    }
  }
}

inline unsigned grid_x(int64_t work) {
  int64_t g = (work + THREADS - 1) / THREADS;
  return (unsigned)(g < 1 ? 1 : (g > 256 ? 256 : g));
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace layout
}  // namespace flr

using namespace flr;

extern "C" int flr_broadcast_rows(const float* src, int64_t n, float* dst, int64_t K, int64_t dst_stride,
                                  void* stream) {
  return flr_broadcast_rows_neg(src, n, dst, K, dst_stride, 0, stream);
}

extern "C" int flr_broadcast_rows_neg(const float* src, int64_t n, float* dst, int64_t K, int64_t dst_stride,
                                      int64_t nneg, void* stream) {
  if (!src || !dst || n < 0 || K < 1 || K > 65535 || dst_stride < n || nneg < 0) return FLR_ERR_ARG;
  const int ng = (int)std::min<int64_t>(nneg, K);
  if (n == 0) return FLR_OK;
  const bool vec = layout::al16(src) && layout::al16(dst) && dst_stride % 4 == 0;
  const dim3 grid(layout::grid_x(vec ? n / 4 : n), (unsigned)K);
  if (vec)
    hipLaunchKernelGGL(layout::broadcast_kernel<true>, grid, dim3(layout::THREADS), 0, as_stream(stream), src, n, dst,
                       dst_stride, ng);
  else
    hipLaunchKernelGGL(layout::broadcast_kernel<false>, grid, dim3(layout::THREADS), 0, as_stream(stream), src, n,
                       dst, dst_stride, ng);
  return launch_status("broadcast_rows");
}

extern "C" int flr_copy_rows(const float* src, int64_t src_stride, int64_t n, float* dst, int64_t dst_stride,
                             int64_t K, void* stream) {
  return flr_copy_rows_neg(src, src_stride, n, dst, dst_stride, K, 0, stream);
}

extern "C" int flr_copy_rows_neg(const float* src, int64_t src_stride, int64_t n, float* dst, int64_t dst_stride,
                                 int64_t K, int64_t nneg, void* stream) {
  if (!src || !dst || n < 0 || K < 1 || K > 65535 || src_stride < n || dst_stride < n || nneg < 0) return FLR_ERR_ARG;
  if (n == 0) return FLR_OK;
  const bool vec = layout::al16(src) && layout::al16(dst) && src_stride % 4 == 0 && dst_stride % 4 == 0;
  const dim3 grid(layout::grid_x(vec ? n / 4 : n), (unsigned)K);
  if (vec)
    hipLaunchKernelGGL(layout::copy_rows_kernel<true>, grid, dim3(layout::THREADS), 0, as_stream(stream), src,
                       src_stride, n, dst, dst_stride, (int)std::min<int64_t>(nneg, K));
  else
    hipLaunchKernelGGL(layout::copy_rows_kernel<false>, grid, dim3(layout::THREADS), 0, as_stream(stream), src,
                       src_stride, n, dst, dst_stride, (int)std::min<int64_t>(nneg, K));
  return launch_status("copy_rows");
}

extern "C" int flr_tap_major_to_torch(const float* w_t, int64_t K, int64_t KK, int64_t Cin, int64_t Cout, float* dst,
                                      int64_t dst_stride, void* stream) {
  return flr_tap_major_to_torch_neg(w_t, K, KK, Cin, Cout, dst, dst_stride, 0, stream);
}

extern "C" int flr_tap_major_to_torch_neg(const float* w_t, int64_t K, int64_t KK, int64_t Cin, int64_t Cout,
                                          float* dst, int64_t dst_stride, int64_t nneg, void* stream) {
  if (!w_t || !dst || K < 1 || K > 65535 || KK < 1 || KK > layout::MAXKK || Cin < 1 || Cout < 1 ||
      dst_stride < KK * Cin * Cout || nneg < 0)
    return FLR_ERR_ARG;
  const int ng = (int)std::min<int64_t>(nneg, K);
  const dim3 grid((unsigned)cdiv((int)Cout, layout::TCO), (unsigned)cdiv((int)Cin, layout::TCI), (unsigned)K);
  const bool vec = Cin % layout::TCI == 0 && Cout % layout::TCO == 0 && layout::al16(w_t) && layout::al16(dst) &&
                   dst_stride % 4 == 0 && (layout::TCI * KK) % 4 == 0;
  if (vec)
    hipLaunchKernelGGL(layout::tap_to_ref_kernel<true>, grid, dim3(layout::THREADS), 0, as_stream(stream), w_t,
                       (int)KK, (int)Cin, (int)Cout, dst, dst_stride, ng);
  else
    hipLaunchKernelGGL(layout::tap_to_ref_kernel<false>, grid, dim3(layout::THREADS), 0, as_stream(stream), w_t,
                       (int)KK, (int)Cin, (int)Cout, dst, dst_stride, ng);
  return launch_status("tap_major_to_torch");
}
