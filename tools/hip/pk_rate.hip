// Microbenchmark (round 6): what a SIMD sustains on the reference-exact chain
// step (acc = fma(d, d, acc), d = fl(x_i - x_j)) in the scalar form the chain
// kernel runs (v_sub_f32_dpp + v_fmac_f32 per chain step) against the packed
// form of a 2 x 2 pair block per lane (v_mov_b64_dpp row_newbcast of the
// (x_i, x_i') pair, two v_pk_add_f32 with op_sel broadcasting x_j and x_j',
// two v_pk_fma_f32: four chain steps), plus bare v_fma_f32 / v_pk_fma_f32
// streams.  Independent accumulators, 1 and 2 waves per SIMD.  Prints cycles
// (at the event-measured time x 2.4 GHz) per wave instruction and per chain
// step of one lane.  Timing only: operands are constants.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

#define REP4(X) X X X X
#define REP16(X) REP4(X) REP4(X) REP4(X) REP4(X)

// mode 0: scalar chain form, 4 independent chains per lane, 16 steps each
// mode 1: packed 2x2 form, 4 chains per lane, 16 steps (5 instructions / step)
// mode 2: 64 v_fma_f32 over 8 accumulators
// mode 3: 64 v_pk_fma_f32 over 8 accumulator pairs
// mode 4: 64 v_pk_add_f32 with op_sel broadcast
// mode 5: 64 v_mov_b64_dpp row_newbcast
template <int MODE>
__global__ __launch_bounds__(256) void k(const float* in, float* out, int iters) {
  const int l = threadIdx.x & 255;
  float x0 = in[l] * 1e-3f, x1 = in[(l + 1) & 255] * 1e-3f;
  f32x2 xs = {x0, x1}, xi = {x1, x0}, jj = {x0 + 1.f, x1 + 2.f};
  f32x2 a0 = {0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0, d0, d1;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, t0, t1, t2, t3;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
      asm volatile("s_nop 1\n\t" REP16(
                       "v_sub_f32_dpp %[t0], %[x0], %[x1] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                       "v_sub_f32_dpp %[t1], %[x0], %[x1] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                       "v_fmac_f32 %[s0], %[t2], %[t2]\n\t"
                       "v_fmac_f32 %[s1], %[t3], %[t3]\n\t"
                       "v_sub_f32_dpp %[t2], %[x1], %[x0] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                       "v_sub_f32_dpp %[t3], %[x1], %[x0] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                       "v_fmac_f32 %[s2], %[t0], %[t0]\n\t"
                       "v_fmac_f32 %[s3], %[t1], %[t1]\n\t")
                   : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [t0] "=&v"(t0), [t1] "=&v"(t1),
                     [t2] "+v"(t2), [t3] "+v"(t3)
                   : [x0] "v"(x0), [x1] "v"(x1));
    } else if constexpr (MODE == 1) {
      asm volatile("s_nop 1\n\t" REP16(
                       "v_mov_b64_dpp %[xi], %[xs] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                       "v_pk_fma_f32 %[a0], %[d0], %[d0], %[a0]\n\t"
                       "v_pk_add_f32 %[d0], %[xi], %[jj] op_sel:[0,0] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
                       "v_pk_fma_f32 %[a1], %[d1], %[d1], %[a1]\n\t"
                       "v_pk_add_f32 %[d1], %[xi], %[jj] op_sel:[0,1] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]\n\t")
                   : [a0] "+v"(a0), [a1] "+v"(a1), [d0] "+v"(d0), [d1] "+v"(d1), [xi] "=&v"(xi)
                   : [xs] "v"(xs), [jj] "v"(jj));
    } else if constexpr (MODE == 2) {
      asm volatile(REP4(REP4("v_fmac_f32 %[s0], %[x0], %[x1]\n\tv_fmac_f32 %[s1], %[x0], %[x1]\n\t"
                             "v_fmac_f32 %[s2], %[x0], %[x1]\n\tv_fmac_f32 %[s3], %[x0], %[x1]\n\t"))
                   : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3)
                   : [x0] "v"(x0), [x1] "v"(x1));
    } else if constexpr (MODE == 3) {
      asm volatile(REP4(REP4("v_pk_fma_f32 %[a0], %[xs], %[jj], %[a0]\n\tv_pk_fma_f32 %[a1], %[xs], %[jj], %[a1]\n\t"
                             "v_pk_fma_f32 %[a2], %[xs], %[jj], %[a2]\n\tv_pk_fma_f32 %[a3], %[xs], %[jj], %[a3]\n\t"))
                   : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
                   : [xs] "v"(xs), [jj] "v"(jj));
    } else if constexpr (MODE == 4) {
      asm volatile(REP4(REP4(
                       "v_pk_add_f32 %[a0], %[xs], %[jj] op_sel:[0,0] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
                       "v_pk_add_f32 %[a1], %[xs], %[jj] op_sel:[0,1] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]\n\t"
                       "v_pk_add_f32 %[a2], %[xs], %[jj] op_sel:[0,0] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
                       "v_pk_add_f32 %[a3], %[xs], %[jj] op_sel:[0,1] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]\n\t"))
                   : [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3)
                   : [xs] "v"(xs), [jj] "v"(jj));
    } else {
      asm volatile("s_nop 1\n\t" REP4(REP4("v_mov_b64_dpp %[a0], %[xs] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                                           "v_mov_b64_dpp %[a1], %[xs] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                                           "v_mov_b64_dpp %[a2], %[jj] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                                           "v_mov_b64_dpp %[a3], %[jj] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"))
                   : [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3)
                   : [xs] "v"(xs), [jj] "v"(jj));
    }
  }
  const float r = s0 + s1 + s2 + s3 + a0[0] + a1[1] + a2[0] + a3[1] + a4[0] + a5[0] + a6[0] + a7[0] + d0[0] + d1[1] +
                  xi[0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// instructions per loop trip and chain steps per lane per trip
static const int kInstr[6] = {128, 80, 64, 64, 64, 64};
static const int kSteps[6] = {64, 64, 0, 0, 0, 0};

template <int MODE>
void run_mode(int wps, float* in, float* out) {
  const int iters = 8192;
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
  const double cyc = ms * 1e-3 * 2.4e9;  // per SIMD: wps waves share it
  const double per_instr = cyc / ((double)iters * kInstr[MODE] * wps);
  printf("{\"mode\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.2f", MODE, wps, ms,
         per_instr);
  if (kSteps[MODE])
    printf(", \"simd_cycles_per_lane_chain_step\": %.3f", cyc / ((double)iters * kSteps[MODE] * wps));
  printf("}\n");
}

int main() {
  float *in, *out;
  (void)hipMalloc(&in, 4096);
  (void)hipMalloc(&out, 256 * 4 * 256 * 4);
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
