// Microbenchmark: per-step cost of the reference-exact chain step
//   acc = fma(d, d, acc), d = fl(x_j - x_i), x_i wave-uniform
// with x_i delivered by: 0 nothing (x_i in VGPRs already: lower bound),
// 1 v_mov_b64_dpp row_newbcast per 2 steps + v_pk_add_f32,
// 2 v_readlane x2 into an SGPR pair per 2 steps + v_pk_add_f32 (SGPR operand),
// 3 v_sub_f32_dpp per step (the current kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pks(f32x2 v, f32x2 x) {
  f32x2 r;
  asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(v), "v"(x));
  return r;
}
__device__ __forceinline__ f32x2 pkss(f32x2 v, f32x2 x) {
  f32x2 r;
  asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(v), "s"(x));
  return r;
}
template <int S> __device__ __forceinline__ f32x2 bc64(double x) {
  long long y = __builtin_amdgcn_update_dpp(__builtin_bit_cast(long long, x), __builtin_bit_cast(long long, x),
                                            0x150 + (S & 15), 0xf, 0xf, true);
  return __builtin_bit_cast(f32x2, y);
}
template <int S> __device__ __forceinline__ float bc32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + (S & 15), 0xf, 0xf, false));
}

template <int MODE, int... S>
__device__ __forceinline__ float run(double xd, f32x2 xv, const float (&xs)[32], const f32x2 (&v)[16], float acc,
                                     std::integer_sequence<int, S...>) {
  f32x2 d[16];
  if constexpr (MODE == 0) {
    ((d[S] = pks(v[S], xv)), ...);
  } else if constexpr (MODE == 1) {
    ((d[S] = pks(v[S], bc64<S>(xd))), ...);
  } else if constexpr (MODE == 2) {
    ((d[S] = pkss(v[S], f32x2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv[0]), 2 * S)),
                              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv[1]), 2 * S + 1))})), ...);
  } else if constexpr (MODE == 3) {
    ((d[S] = f32x2{bc32<2 * S>(xv[0]) - v[S][0], bc32<2 * S + 1>(xv[1]) - v[S][1]}), ...);
  } else if constexpr (MODE == 4) {  // plain v_sub_f32, x_i in a VGPR
    ((d[S] = f32x2{v[S][0] - xv[0], v[S][1] - xv[1]}), ...);
  } else {  // MODE 5: plain v_sub_f32 with an SGPR operand (x_i uniform)
    ((d[S] = f32x2{v[S][0] - xs[2 * S], v[S][1] - xs[2 * S + 1]}), ...);
  }
  ((acc = __builtin_fmaf(d[S][1], d[S][1], __builtin_fmaf(d[S][0], d[S][0], acc))), ...);
  return acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void k(const float* in, float* out, int iters) {
  f32x2 v[16];
  for (int i = 0; i < 16; ++i) v[i] = f32x2{in[(threadIdx.x + i) & 255], in[(threadIdx.x + 2 * i) & 255]} * 1e-3f;
  f32x2 xv = {in[threadIdx.x & 255], in[(threadIdx.x + 1) & 255]};
  double xd = __builtin_bit_cast(double, xv);
  float xs[32];
  for (int i = 0; i < 32; ++i) xs[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[i])));
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    acc = run<MODE>(xd, xv, xs, v, acc, std::make_integer_sequence<int, 16>{});
    asm volatile("" : "+v"(xv), "+v"(xd));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
void run_mode(int wps, float* in, float* out) {
  const int iters = 4096;
  dim3 grid(256 * wps);
  hipLaunchKernelGGL((k<MODE>), grid, dim3(256), 0, 0, in, out, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k<MODE>), grid, dim3(256), 0, 0, in, out, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double steps = (double)iters * 32;
  printf("mode %d waves/SIMD %d: %.3f ms, %.2f ns per chain step (%.1f cyc @2.4GHz)\n", MODE, wps, ms,
         ms * 1e6 / steps, ms * 1e6 / steps * 2.4);
}

int main() {
  float *in, *out;
  (void)hipMalloc(&in, 4096);
  (void)hipMalloc(&out, 256 * 8 * 256 * 4);
  (void)hipMemset(in, 0, 4096);
  for (int wps : {1, 2}) {
    run_mode<0>(wps, in, out);
    run_mode<1>(wps, in, out);
    run_mode<2>(wps, in, out);
    run_mode<3>(wps, in, out);
    run_mode<4>(wps, in, out);
    run_mode<5>(wps, in, out);
  }
  return 0;
}
