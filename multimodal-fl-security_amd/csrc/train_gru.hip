// a3 — the text encoder's GRU recurrence (gate math) for all clients of a GPU.
//
// Reference layer: nn.GRU(embed, hidden, num_layers=1, batch_first=True), the
// second modality branch of the late-fusion model (BASELINE configs C2/C3;
// fusion structure src/models/cub200_cnn.py:88-117), trained per client in
// run_experiments.py:216-235.  torch's GRU cell (gate order r, z, n):
//   r = sigmoid(i_r + h_r)       z = sigmoid(i_z + h_z)
//   n = tanh(i_n + r * h_n)      h' = (h - n) * z + n
// with i = x W_ih^T + b_ih (whole sequence, one GEMM outside) and
// h_* = h W_hh^T + b_hh (one batched GEMM per step, outside).  These kernels
// are the per-step pointwise part: ONE launch per step forward and one per
// step backward replace torch's ~30 strided elementwise launches per step.
//
// Layouts (fp32, per GPU, K clients x B samples, hidden H, T steps):
//   gi    [K][B][T][3H]   input projections (the GEMM's natural output)
//   gh    [K][B][3H]      this step's hidden projections (bias included)
//   hseq  [K][T+1][B][H]  h_0 .. h_T (h_0 = 0), so hseq[k, 0:T] is the
//                         contiguous [T*B][H] operand of the dW_hh GEMM
//   gates [K][T][B][4][H] r, z, n, h_n saved for backward
//   dgh   [K][T][B][3H]   d(h W_hh^T + b_hh) per step, for dW_hh / db_hh
//   dgi   [K][B][T][3H]   d(gi)
#include "flr_common.h"

#include <stdlib.h>
#include <string.h>

namespace flr {
namespace gru {

constexpr int THREADS = 256;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

struct Dims {
  int K, B, T, H, t;
  int wshared;  // 1: every client reads the one packed W_hh copy (the first local step)
};

__device__ __forceinline__ void decompose(const Dims& d, int64_t idx, int& k, int& b, int& j) {
  j = (int)(idx % d.H);
  const int64_t kb = idx / d.H;
  b = (int)(kb % d.B);
  k = (int)(kb / d.B);
}

__global__ __launch_bounds__(THREADS) void fwd_step_kernel(const float* __restrict__ gi, const float* __restrict__ gh,
                                                           float* __restrict__ hseq, float* __restrict__ gates,
                                                           const Dims d) {
  const int64_t idx = (int64_t)blockIdx.x * THREADS + threadIdx.x;
  if (idx >= (int64_t)d.K * d.B * d.H) return;
  int k, b, j;
  decompose(d, idx, k, b, j);
  const int H = d.H;
  const int64_t kb = (int64_t)k * d.B + b;
  const float* gir = gi + (kb * d.T + d.t) * 3 * H;
  const float* ghr = gh + kb * 3 * H;
  const int64_t hrow = (((int64_t)k * (d.T + 1) + d.t) * d.B + b) * H;
  const float hp = hseq[hrow + j];
  const float r = sigm(gir[j] + ghr[j]);
  const float z = sigm(gir[H + j] + ghr[H + j]);
  const float hn = ghr[2 * H + j];
  const float n = tanhf(gir[2 * H + j] + r * hn);
  hseq[hrow + (int64_t)d.B * H + j] = (hp - n) * z + n;  // h_{t+1}
  float* g = gates + (((int64_t)k * d.T + d.t) * d.B + b) * 4 * H;
  g[j] = r;
  g[H + j] = z;
  g[2 * H + j] = n;
  g[3 * H + j] = hn;
}

// dh: dL/dh_{t+1} [K][B][H]; writes dgh[:, t], dgi[:, :, t] and
// dh_direct = dL/dh_t through the z-gate path (the W_hh path is the caller's GEMM).
__global__ __launch_bounds__(THREADS) void bwd_step_kernel(const float* __restrict__ dh,
                                                           const float* __restrict__ gates,
                                                           const float* __restrict__ hseq, float* __restrict__ dgh,
                                                           float* __restrict__ dgi, float* __restrict__ dh_direct,
                                                           const Dims d) {
  const int64_t idx = (int64_t)blockIdx.x * THREADS + threadIdx.x;
  if (idx >= (int64_t)d.K * d.B * d.H) return;
  int k, b, j;
  decompose(d, idx, k, b, j);
  const int H = d.H;
  const int64_t kb = (int64_t)k * d.B + b;
  const int64_t srow = ((int64_t)k * d.T + d.t) * d.B + b;
  const float* g = gates + srow * 4 * H;
  const float r = g[j], z = g[H + j], n = g[2 * H + j], hn = g[3 * H + j];
  const float hp = hseq[(((int64_t)k * (d.T + 1) + d.t) * d.B + b) * H + j];
  const float dy = dh[idx];
  const float dz = dy * (hp - n);
  const float dn = dy * (1.0f - z);
  const float dnp = dn * (1.0f - n * n);
  const float dr = dnp * hn;
  const float drp = dr * (r * (1.0f - r));
  const float dzp = dz * (z * (1.0f - z));
  float* o = dgh + srow * 3 * H;
  o[j] = drp;
  o[H + j] = dzp;
  o[2 * H + j] = dnp * r;
  float* q = dgi + (kb * d.T + d.t) * 3 * H;
  q[j] = drp;
  q[H + j] = dzp;
  q[2 * H + j] = dnp;
  dh_direct[idx] = dy * z;
}

// ---- fused per-step kernels: the recurrence GEMM with the gate math in its
// epilogue.  One wave per (client, 32 hidden units); B <= 32 batch rows are the
// MFMA's 32 rows.  fp32 operands split into three bf16 terms, six products per
// 16-deep k-step on v_mfma_f32_32x32x16_bf16 (the bf16x6 form of the batched
// GEMM: per-product error a few 2^-24 |a b|).  The forward reads W_hh rows
// ([3H][H], k-contiguous); the backward reads W_hh^T ([H][3H], transposed once
// per optimizer step by flr_gru_transpose) so both operands load k-contiguous.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a = (__bf16)v[j];
    const float r1 = v[j] - (float)a;
    const __bf16 b = (__bf16)r1;
    hi[j] = a;
    mid[j] = b;
    lo[j] = (__bf16)(r1 - (float)b);
  }
}

// Raw buffer loads: an out-of-range byte offset returns 0 with no branch, so a
// wave's loads of several k-steps stay in flight together (a per-lane branch
// would join through register moves that wait on each load).
using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned SENT = 0x80000000u;  // past every buffer here (< 2 GB)

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int64_t nfloats) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane((int)(nfloats * 4));
  void* base = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
}

// 8 floats of a row starting at k0; zeros for an invalid row or past R.  V8: R
// and k0 are multiples of 8, so k0 < R covers all 8.
template <bool V8>
__device__ __forceinline__ void bload8(rsrc_t r, bool ok, int row_off, int k0, int R, float (&v)[8]) {
  if constexpr (V8) {
    const unsigned off = (ok && k0 < R) ? (unsigned)(row_off + k0) * 4u : SENT;
    const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    const f32x4 y = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16u, 0, 0));
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const unsigned off = (ok && k0 + e < R) ? (unsigned)(row_off + k0 + e) * 4u : SENT;
      v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
    }
  }
}

// Packed weights (flr_gru_pack): for a 32-row block `blk` and k-step s, the 64
// lanes' 8-float B fragments as two contiguous 1 KB halves,
//   wp[((blk * S + s) * 2 + q) * 256 + lane * 4 + e] = W[blk row (lane & 31)][16 s + 8 (lane >> 5) + 4 q + e]
// zero-padded, so one b128 per half reads 1 KB contiguous across the wave.
__device__ __forceinline__ void pload8(rsrc_t r, bool in, int blk, int S, int s, int lane, float (&v)[8]) {
  const unsigned off = in ? (unsigned)(((blk * S + s) * 2) * 256 + lane * 4) * 4u : SENT;
  const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  const f32x4 y = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off + 1024u, 0, 0));
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
}

__device__ __forceinline__ f32x16 mfma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                        const bf16x8& bm, const bf16x8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
  return c;
}

// Workgroup -> (client, 32-unit block).  Workgroups go round-robin over the 8
// XCDs by linear id; remap so one client's unit blocks share an XCD (and its L2:
// they all read the same h_t / dgh_t rows).
__device__ __forceinline__ void block_coords(int nub, int& k, int& ub) {
  const int n = gridDim.x, L = blockIdx.x;
  const int idx = (n % 8 == 0) ? (L % 8) * (n / 8) + L / 8 : L;
  k = idx / nub;
  ub = idx % nub;
}

// The k-steps (16 deep) are split over the NW waves of a workgroup in contiguous
// ranges; each wave issues the loads of G k-steps before their MFMAs, and the
// NW partial accumulators are summed in wave order through LDS (deterministic).
// Every loop bound is wave-uniform: the MFMA needs all 64 lanes.  The epilogue's
// operands (16 x 64 elements over the workgroup) are loaded before the GEMM.
__device__ __forceinline__ float bload1(rsrc_t r, bool ok, int64_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, ok ? (unsigned)off * 4u : SENT, 0, 0));
}

// forward step t: gh = h_t W_hh^T + b_hh for the units [j0, j0+32) of all three
// gates, then the gate math of fwd_step_kernel for those units.
// SEQ: the waves' partial sums added in wave order through ONE LDS slot (wave w
// adds its partials to the slot in turn: the same sums in the same order as
// the NW-slot form, bit-identical), 12 KB instead of 96 KB of LDS, and the
// kernel held to 128 VGPRs, so two workgroups share a CU and one's W_hh
// stream overlaps the other's reduction and gate math (the NW-slot form runs
// one workgroup per CU: 1024 workgroups in four serial rounds at C3).
template <bool V8, int NW, int G, bool SEQ = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(SEQ ? 4 : 1))) void fwd_fused_kernel(const float* __restrict__ gi,
                                                            const float* __restrict__ whhP,
                                                            const float* __restrict__ bhh, float* __restrict__ hseq,
                                                            float* __restrict__ gates, const Dims d, int nub) {
  constexpr int EPT = 16 / NW;  // epilogue elements per thread
  __shared__ float red[SEQ ? 1 : NW][3][16][64];
  int k, ub;
  block_coords(nub, k, ub);
  const int j0 = ub * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const int B = d.B, H = d.H;
  const rsrc_t rh = make_rsrc(hseq + ((int64_t)k * (d.T + 1) + d.t) * B * H, (int64_t)B * H);
  const int S = (H + 15) / 16, per = (S + NW - 1) / NW;
  const rsrc_t rw = make_rsrc(whhP + (d.wshared ? 0 : (int64_t)k * 3 * nub * S * 512), (int64_t)3 * nub * S * 512);
  const rsrc_t rg = make_rsrc(gi + (int64_t)k * B * d.T * 3 * H, (int64_t)B * d.T * 3 * H);
  const rsrc_t rbias = make_rsrc(bhh + (int64_t)k * 3 * H, (int64_t)3 * H);
  // epilogue operands: element p = tid + 64 NW i -> (e, ln) of the MFMA tile
  float pgi[EPT][3], php[EPT], pbh[EPT][3];
  auto load_epi = [&]() {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int p = threadIdx.x + 64 * NW * i, e = p >> 6, ln = p & 63;
      const int b = (e & 3) + 8 * (e >> 2) + 4 * (ln >> 5), j = j0 + (ln & 31);
      const bool ok = b < B && j < H;
      const int64_t go = ((int64_t)b * d.T + d.t) * 3 * H + j;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        pgi[i][g] = bload1(rg, ok, go + g * H);
        pbh[i][g] = bload1(rbias, ok, g * H + j);
      }
      php[i] = bload1(rh, ok, (int64_t)b * H + j);
    }
  };
  // SEQ: the epilogue operands are loaded after the MFMAs (their latency under the
  // ordered reduction), keeping them out of the loads' register peak
  if constexpr (!SEQ) load_epi();
  const bool aok = l32 < B;
  f32x16 acc[3];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[g][e] = 0.f;
  const int s1 = min(S, (wave + 1) * per);
  for (int s = wave * per; s < s1; s += G) {
    float a[G][8], b[G][3][8];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const bool in = s + q < s1;
      const int k0 = (s + q) * 16 + 8 * h;
      bload8<V8>(rh, aok && in, l32 * H, k0, H, a[q]);
#pragma unroll
      for (int g = 0; g < 3; ++g) pload8(rw, in, g * nub + ub, S, s + q, lane, b[q][g]);
    }
    __builtin_amdgcn_sched_barrier(0);  // every load of the group issued before the first MFMA
#pragma unroll
    for (int q = 0; q < G; ++q) {
      bf16x8 ah, am, al;
      split3(a[q], ah, am, al);
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        bf16x8 bh, bm, bl;
        split3(b[q][g], bh, bm, bl);
        acc[g] = mfma6(ah, am, al, bh, bm, bl, acc[g]);
      }
    }
  }
  if constexpr (SEQ) {
    load_epi();
    for (int w = 0; w < NW; ++w) {
      if (wave == w)
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int e = 0; e < 16; ++e) red[0][g][e][lane] = w == 0 ? acc[g][e] : red[0][g][e][lane] + acc[g][e];
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int e = 0; e < 16; ++e) red[wave][g][e][lane] = acc[g][e];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int p = threadIdx.x + 64 * NW * i, e = p >> 6, ln = p & 63;
    const int b = (e & 3) + 8 * (e >> 2) + 4 * (ln >> 5), j = j0 + (ln & 31);
    if (b >= B || j >= H) continue;
    float v[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      float x = red[0][g][e][ln];
      if constexpr (!SEQ)
#pragma unroll
        for (int w = 1; w < NW; ++w) x += red[w][g][e][ln];
      v[g] = x;
    }
    const int64_t hrw = (((int64_t)k * (d.T + 1) + d.t) * B + b) * H;
    const float ghr = pbh[i][0] + v[0], ghz = pbh[i][1] + v[1], hn = pbh[i][2] + v[2];
    const float r = sigm(pgi[i][0] + ghr);
    const float z = sigm(pgi[i][1] + ghz);
    const float n = tanhf(pgi[i][2] + r * hn);
    hseq[hrw + (int64_t)B * H + j] = (php[i] - n) * z + n;  // h_{t+1}
    float* gg = gates + (((int64_t)k * d.T + d.t) * B + b) * 4 * H;
    gg[j] = r;
    gg[H + j] = z;
    gg[2 * H + j] = n;
    gg[3 * H + j] = hn;
  }
}

// backward step t >= 1: dh_t = dh_direct + dgh_t W_hh for the units [i0, i0+32)
// (W_hh^T rows), then the element backward of step t - 1 for those units
// (d.t = t - 1).  dh_direct is read and rewritten in place by the same thread.
template <bool V8, int NW, int G, bool SEQ = false>  // SEQ: as fwd_fused_kernel's
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(SEQ ? 6 : 1))) void bwd_fused_kernel(const float* __restrict__ whhTP,
                                                            const float* __restrict__ gates,
                                                            const float* __restrict__ hseq, float* __restrict__ dgh,
                                                            float* __restrict__ dgi, float* __restrict__ dh_direct,
                                                            float* __restrict__ dh0, const Dims d, int nub) {
  constexpr int EPT = 16 / NW;
  __shared__ float red[SEQ ? 1 : NW][16][64];
  int k, ub;
  block_coords(nub, k, ub);
  const int i0 = ub * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const int B = d.B, H = d.H, R = 3 * H;
  const int t = d.t + 1;  // this launch's GEMM step
  const rsrc_t ra = make_rsrc(dgh + ((int64_t)k * d.T + t) * B * R, (int64_t)B * R);
  const int S = (R + 15) / 16, per = (S + NW - 1) / NW;
  const rsrc_t rb = make_rsrc(whhTP + (d.wshared ? 0 : (int64_t)k * nub * S * 512), (int64_t)nub * S * 512);
  const rsrc_t rdd = make_rsrc(dh_direct + (int64_t)k * B * H, (int64_t)B * H);
  // epilogue operands: dh_direct, and step t-1's gates and h_{t-1} when d.t >= 0
  const bool elem = d.t >= 0;
  const int tg = elem ? d.t : 0;
  const rsrc_t rgt = make_rsrc(gates + ((int64_t)k * d.T + tg) * B * 4 * H, (int64_t)B * 4 * H);
  const rsrc_t rhp = make_rsrc(hseq + ((int64_t)k * (d.T + 1) + tg) * B * H, (int64_t)B * H);
  float pdd[EPT], pg[EPT][4], php[EPT];
  auto load_epi = [&]() {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int p = threadIdx.x + 64 * NW * i, e = p >> 6, ln = p & 63;
      const int b = (e & 3) + 8 * (e >> 2) + 4 * (ln >> 5), j = i0 + (ln & 31);
      const bool ok = b < B && j < H;
      pdd[i] = bload1(rdd, ok, (int64_t)b * H + j);
#pragma unroll
      for (int q = 0; q < 4; ++q) pg[i][q] = bload1(rgt, ok && elem, (int64_t)b * 4 * H + q * H + j);
      php[i] = bload1(rhp, ok && elem, (int64_t)b * H + j);
    }
  };
  if constexpr (!SEQ) load_epi();
  const bool aok = l32 < B;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  const int s1 = min(S, (wave + 1) * per);
  for (int s = wave * per; s < s1; s += G) {
    float a[G][8], b[G][8];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const bool in = s + q < s1;
      const int k0 = (s + q) * 16 + 8 * h;
      bload8<V8>(ra, aok && in, l32 * R, k0, R, a[q]);
      pload8(rb, in, ub, S, s + q, lane, b[q]);
    }
    __builtin_amdgcn_sched_barrier(0);  // every load of the group issued before the first MFMA
#pragma unroll
    for (int q = 0; q < G; ++q) {
      bf16x8 ah, am, al, bh, bm, bl;
      split3(a[q], ah, am, al);
      split3(b[q], bh, bm, bl);
      acc = mfma6(ah, am, al, bh, bm, bl, acc);
    }
  }
  if constexpr (SEQ) {
    load_epi();
    for (int w = 0; w < NW; ++w) {
      if (wave == w)
#pragma unroll
        for (int e = 0; e < 16; ++e) red[0][e][lane] = w == 0 ? acc[e] : red[0][e][lane] + acc[e];
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[wave][e][lane] = acc[e];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int p = threadIdx.x + 64 * NW * i, e = p >> 6, ln = p & 63;
    const int b = (e & 3) + 8 * (e >> 2) + 4 * (ln >> 5), j = i0 + (ln & 31);
    if (b >= B || j >= H) continue;
    float x = red[0][e][ln];
    if constexpr (!SEQ)
#pragma unroll
      for (int w = 1; w < NW; ++w) x += red[w][e][ln];
    const int64_t kb = (int64_t)k * B + b;
    const int64_t idx = kb * H + j;
    const float dy = pdd[i] + x;  // dL/dh_t
    if (dh0) dh0[idx] = dy;
    if (!elem) continue;
    // step t-1's element backward (bwd_step_kernel's math)
    const float r = pg[i][0], z = pg[i][1], n = pg[i][2], hn = pg[i][3];
    const float dz = dy * (php[i] - n);
    const float dn = dy * (1.0f - z);
    const float dnp = dn * (1.0f - n * n);
    const float dr = dnp * hn;
    const float drp = dr * (r * (1.0f - r));
    const float dzp = dz * (z * (1.0f - z));
    const int64_t srow = ((int64_t)k * d.T + d.t) * B + b;
    float* o = dgh + srow * 3 * H;
    o[j] = drp;
    o[H + j] = dzp;
    o[2 * H + j] = dnp * r;
    float* q = dgi + (kb * d.T + d.t) * 3 * H;
    q[j] = drp;
    q[H + j] = dzp;
    q[2 * H + j] = dnp;
    dh_direct[idx] = dy * z;
  }
}

// Pack a client's weight into the fused kernels' fragment order (pload8).  The
// packed operand is the [NG * H][C] matrix of rows (g, r) and columns c with
//   TRANS = 0: element = w[(g H + r) C + c]   (W_hh, [3H][H]: NG = 3, C = H)
//   TRANS = 1: element = w[c H + r]           (W_hh^T of a [C][H] W_hh: NG = 1, C = 3H)
// Row blocks of 32 per group (the last one zero-padded), k-steps of 16 (padded).
// One workgroup per (client, row block, 128-column chunk) through an LDS tile.
template <int TRANS>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ w, int NG, int H, int C,
                                                   float* __restrict__ wp) {
  __shared__ float tile[32][129];
  const int k = blockIdx.z, blk = blockIdx.y, c0 = blockIdx.x * 128;
  const int nub = (H + 31) / 32, S = (C + 15) / 16;
  const int g = blk / nub, r0 = (blk % nub) * 32;
  const float* src = w + (int64_t)k * NG * H * C;
  for (int e = threadIdx.x; e < 32 * 128; e += 256) {
    int r, c;
    if (TRANS) { c = e >> 5; r = e & 31; } else { r = e >> 7; c = e & 127; }
    const bool ok = r0 + r < H && c0 + c < C;
    const int64_t off = TRANS ? (int64_t)(c0 + c) * H + r0 + r : ((int64_t)g * H + r0 + r) * C + c0 + c;
    tile[r][c] = ok ? src[off] : 0.f;
  }
  __syncthreads();
  float* dst = wp + ((int64_t)k * NG * nub + blk) * S * 512;
  for (int o = threadIdx.x; o < 8 * 512; o += 256) {  // the 8 k-steps of this chunk
    const int sl = o >> 9, q = (o >> 8) & 1, lane = (o >> 2) & 63, e = o & 3;
    const int s = c0 / 16 + sl;
    if (s < S) dst[(int64_t)s * 512 + q * 256 + lane * 4 + e] = tile[lane & 31][sl * 16 + 8 * (lane >> 5) + 4 * q + e];
  }
}

inline bool dims_ok(int64_t K, int64_t B, int64_t T, int64_t H, int64_t t) {
  return K > 0 && B > 0 && T > 0 && H > 0 && t >= 0 && t < T && K * B * H < (int64_t)1 << 31;
}

}  // namespace gru
}  // namespace flr

using namespace flr;

extern "C" int flr_gru_fwd_step(const float* gi, const float* gh, float* hseq, float* gates, int64_t K, int64_t B,
                                int64_t T, int64_t H, int64_t t, void* stream) {
  if (!gi || !gh || !hseq || !gates || !gru::dims_ok(K, B, T, H, t)) return FLR_ERR_ARG;
  const gru::Dims d{(int)K, (int)B, (int)T, (int)H, (int)t};
  const int64_t n = K * B * H;
  hipLaunchKernelGGL(gru::fwd_step_kernel, dim3((unsigned)((n + gru::THREADS - 1) / gru::THREADS)),
                     dim3(gru::THREADS), 0, as_stream(stream), gi, gh, hseq, gates, d);
  return launch_status("gru fwd step");
}

extern "C" int flr_gru_bwd_step(const float* dh, const float* gates, const float* hseq, float* dgh, float* dgi,
                                float* dh_direct, int64_t K, int64_t B, int64_t T, int64_t H, int64_t t,
                                void* stream) {
  if (!dh || !gates || !hseq || !dgh || !dgi || !dh_direct || !gru::dims_ok(K, B, T, H, t)) return FLR_ERR_ARG;
  const gru::Dims d{(int)K, (int)B, (int)T, (int)H, (int)t};
  const int64_t n = K * B * H;
  hipLaunchKernelGGL(gru::bwd_step_kernel, dim3((unsigned)((n + gru::THREADS - 1) / gru::THREADS)),
                     dim3(gru::THREADS), 0, as_stream(stream), dh, gates, hseq, dgh, dgi, dh_direct, d);
  return launch_status("gru bwd step");
}

namespace flr {
namespace gru {
// (waves per workgroup, k-steps per load group); FLR_GRU_FW / FLR_GRU_BW = "NW,G" for A/B timing
// (tools/gru_bench.py); default 8 waves x 2 k-steps for both (C3: fwd 29 us, bwd 27 us per step)
inline int cfg_index(const char* env, int dflt) {
  static const char* names[] = {"4,4", "8,2", "2,8", "8,2s", "8,6", "4,12", "16,3", "", "8,2s"};
  const char* v = flr::knob(env);
  if (v)
    for (int i = 0; i < 9; ++i)
        if (names[i][0] && !strcmp(v, names[i])) return i;
  return dflt;
}
template <bool V8>
inline void launch_fwd(int cfg, dim3 grid, hipStream_t st, const float* gi, const float* whh, const float* bhh,
                       float* hseq, float* gates, const Dims& d, int nub) {
  switch (cfg) {
    case 0: hipLaunchKernelGGL((fwd_fused_kernel<V8, 4, 4>), grid, dim3(256), 0, st, gi, whh, bhh, hseq, gates, d, nub); break;
    case 2: hipLaunchKernelGGL((fwd_fused_kernel<V8, 2, 8>), grid, dim3(128), 0, st, gi, whh, bhh, hseq, gates, d, nub); break;
    case 3: hipLaunchKernelGGL((fwd_fused_kernel<V8, 8, 1, true>), grid, dim3(512), 0, st, gi, whh, bhh, hseq, gates, d, nub); break;
    default: hipLaunchKernelGGL((fwd_fused_kernel<V8, 8, 2>), grid, dim3(512), 0, st, gi, whh, bhh, hseq, gates, d, nub);
  }
}
template <bool V8>
inline void launch_bwd(int cfg, dim3 grid, hipStream_t st, const float* whhT, const float* gates, const float* hseq,
                       float* dgh, float* dgi, float* dh_direct, float* dh0, const Dims& d, int nub) {
  switch (cfg) {
    case 5: hipLaunchKernelGGL((bwd_fused_kernel<V8, 4, 12>), grid, dim3(256), 0, st, whhT, gates, hseq, dgh, dgi, dh_direct, dh0, d, nub); break;
    case 6: hipLaunchKernelGGL((bwd_fused_kernel<V8, 16, 3>), grid, dim3(1024), 0, st, whhT, gates, hseq, dgh, dgi, dh_direct, dh0, d, nub); break;
    case 4: hipLaunchKernelGGL((bwd_fused_kernel<V8, 8, 6>), grid, dim3(512), 0, st, whhT, gates, hseq, dgh, dgi, dh_direct, dh0, d, nub); break;
    case 3: hipLaunchKernelGGL((bwd_fused_kernel<V8, 8, 2, true>), grid, dim3(512), 0, st, whhT, gates, hseq, dgh, dgi, dh_direct, dh0, d, nub); break;
    default: hipLaunchKernelGGL((bwd_fused_kernel<V8, 8, 2>), grid, dim3(512), 0, st, whhT, gates, hseq, dgh, dgi, dh_direct, dh0, d, nub);
  }
}
}  // namespace gru
}  // namespace flr

extern "C" int flr_gru_fwd_fused(const float* gi, const float* whh, const float* bhh, float* hseq, float* gates,
                                 int64_t K, int64_t B, int64_t T, int64_t H, int64_t t, void* stream) {
  return flr_gru_fwd_fused_ex(gi, whh, 0, bhh, hseq, gates, K, B, T, H, t, stream);
}

extern "C" int flr_gru_fwd_fused_ex(const float* gi, const float* whh, int shared_w, const float* bhh, float* hseq,
                                    float* gates, int64_t K, int64_t B, int64_t T, int64_t H, int64_t t,
                                    void* stream) {
  if (!gi || !whh || !bhh || !hseq || !gates || !gru::dims_ok(K, B, T, H, t) || B > 32 || K > 65535)
    return FLR_ERR_ARG;
  const gru::Dims d{(int)K, (int)B, (int)T, (int)H, (int)t, shared_w ? 1 : 0};
  const int nub = (int)((H + 31) / 32);
  const int cfg = gru::cfg_index("FLR_GRU_FW", 1);  // read per call: captured launches keep theirs
  if (H % 8 == 0)
    gru::launch_fwd<true>(cfg, dim3((unsigned)(K * nub)), as_stream(stream), gi, whh, bhh, hseq, gates, d, nub);
  else
    gru::launch_fwd<false>(cfg, dim3((unsigned)(K * nub)), as_stream(stream), gi, whh, bhh, hseq, gates, d, nub);
  return launch_status("gru fwd fused");
}

extern "C" int flr_gru_bwd_fused(const float* whhT, const float* gates, const float* hseq, float* dgh, float* dgi,
                                 float* dh_direct, float* dh0, int64_t K, int64_t B, int64_t T, int64_t H, int64_t t,
                                 void* stream) {
  return flr_gru_bwd_fused_ex(whhT, 0, gates, hseq, dgh, dgi, dh_direct, dh0, K, B, T, H, t, stream);
}

extern "C" int flr_gru_bwd_fused_ex(const float* whhT, int shared_w, const float* gates, const float* hseq,
                                    float* dgh, float* dgi, float* dh_direct, float* dh0, int64_t K, int64_t B,
                                    int64_t T, int64_t H, int64_t t, void* stream) {
  if (!whhT || !gates || !hseq || !dgh || !dgi || !dh_direct || !gru::dims_ok(K, B, T, H, t) || t < 1 || B > 32 ||
      K > 65535)
    return FLR_ERR_ARG;
  const gru::Dims d{(int)K, (int)B, (int)T, (int)H, (int)(t - 1), shared_w ? 1 : 0};
  const int nub = (int)((H + 31) / 32);
  const int cfg = gru::cfg_index("FLR_GRU_BW", 1);
  if (H % 8 == 0)
    gru::launch_bwd<true>(cfg, dim3((unsigned)(K * nub)), as_stream(stream), whhT, gates, hseq, dgh, dgi, dh_direct,
                          dh0, d, nub);
  else
    gru::launch_bwd<false>(cfg, dim3((unsigned)(K * nub)), as_stream(stream), whhT, gates, hseq, dgh, dgi, dh_direct,
                           dh0, d, nub);
  return launch_status("gru bwd fused");
}

extern "C" int flr_gru_pack(const float* w, int64_t K, int64_t NG, int64_t H, int64_t C, int trans, float* wp,
                            void* stream) {
  if (!w || !wp || K < 1 || K > 65535 || NG < 1 || H < 1 || C < 1 || (trans && NG != 1) ||
      K * NG * H * C >= (int64_t)1 << 31)
    return FLR_ERR_ARG;
  const dim3 grid((unsigned)((C + 127) / 128), (unsigned)(NG * ((H + 31) / 32)), (unsigned)K);
  if (trans)
    hipLaunchKernelGGL(gru::pack_kernel<1>, grid, dim3(256), 0, as_stream(stream), w, (int)NG, (int)H, (int)C, wp);
  else
    hipLaunchKernelGGL(gru::pack_kernel<0>, grid, dim3(256), 0, as_stream(stream), w, (int)NG, (int)H, (int)C, wp);
  return launch_status("gru pack");
}
