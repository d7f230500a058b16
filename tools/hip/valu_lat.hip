// Microbenchmark: dependent v_fma_f32 chain latency on gfx950 (one lane-chain per
// lane, NC independent chains interleaved per lane), with and without a DPP
// subtraction feeding each fma; waves per SIMD set by the grid.  Prints ns per
// step of one chain and cycles at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>

template <int S> __device__ __forceinline__ float bc(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + (S & 15), 0xf, 0xf, false));
}

template <int NC, int DPP, int... S>
__device__ __forceinline__ void steps(float (&acc)[NC], float xv, const float (&v)[32], std::integer_sequence<int, S...>) {
  if constexpr (DPP) {
    float d[32];
    ((d[S] = bc<S>(xv) - v[S]), ...);
    ((acc[S % NC] = __builtin_fmaf(d[S], d[S], acc[S % NC])), ...);
  } else {
    ((acc[S % NC] = __builtin_fmaf(v[S], v[S], acc[S % NC])), ...);
  }
}

template <int NC, int DPP>
__global__ __launch_bounds__(256) void k(const float* in, float* out, int iters) {
  float v[32];
  for (int i = 0; i < 32; ++i) v[i] = in[(threadIdx.x + i) & 255] * 1e-3f;
  float xv = in[threadIdx.x & 255];
  float acc[NC];
  for (int c = 0; c < NC; ++c) acc[c] = 0.f;
  for (int it = 0; it < iters; ++it) {
    steps<NC, DPP>(acc, xv, v, std::make_integer_sequence<int, 32>{});
    asm volatile("" : "+v"(xv));
  }
  float s = 0.f;
  for (int c = 0; c < NC; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NC, int DPP>
void run(int wps, float* in, float* out) {
  const int iters = 4096;
  dim3 grid(256 * wps / 4 * 4 / 4);  // 256 CUs x wps waves per SIMD: blocks of 4 waves
  grid.x = 256 * wps;
  hipLaunchKernelGGL((k<NC, DPP>), grid, dim3(256), 0, 0, in, out, iters);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((k<NC, DPP>), grid, dim3(256), 0, 0, in, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double steps_per_chain = (double)iters * 32 / NC;
  const double ns = ms * 1e6 / steps_per_chain;
  printf("chains/lane %d dpp %d waves/SIMD %d: %.3f ms, %.2f ns per chain step (%.1f cyc @2.4GHz), %.1f cyc per lane-step\n",
         NC, DPP, wps, ms, ns, ns * 2.4, ns * 2.4 / NC);
}

int main() {
  float *in, *out;
  hipMalloc(&in, 4096);
  hipMalloc(&out, 256 * 8 * 256 * 4);
  hipMemset(in, 0, 4096);
  for (int wps : {1, 2, 4}) {
    run<1, 0>(wps, in, out);
    run<2, 0>(wps, in, out);
    run<4, 0>(wps, in, out);
    run<1, 1>(wps, in, out);
    run<2, 1>(wps, in, out);
    run<4, 1>(wps, in, out);
  }
  return 0;
}
