// a3 (text branch) and the C4/C5 encoder layers on gfx950: embedding lookup
// with a deterministic scatter-add backward, LayerNorm with a fused residual
// add, and multi-head self-attention forward/backward, each batched over the
// clients of a GPU (client k's rows are a contiguous run of `rows_per_client`).
//
// Replaces nn.Embedding / nn.LayerNorm / the scaled-dot-product attention of
// the ViT-S image and BERT-mini text encoders (BASELINE.json configs[3-4]; the
// reference has no such model, its fusion head is cub200_cnn.py:88-93) and the
// GRU branch's embedding (the a3 row).  fp32 throughout; every reduction has a
// fixed order, so a client's result never depends on the launch it shares.
#include "flr_common.h"

#include <algorithm>

namespace flr {
namespace xf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// fill
// ---------------------------------------------------------------------------
__global__ void fill_kernel(float* __restrict__ p, int64_t n, float v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const int64_t n4 = n / 4;
    f32x4* q = reinterpret_cast<f32x4*>(p);
    for (int64_t j = i; j < n4; j += stride) q[j] = f32x4{v, v, v, v};
    for (int64_t j = 4 * n4 + i; j < n; j += stride) p[j] = v;
  } else {
    for (int64_t j = i; j < n; j += stride) p[j] = v;
  }
}

// ---------------------------------------------------------------------------
// embedding forward: out[k][n] = ((w0[ids0] + w1[ids1]) + w2[ids2])
// one wave per output row; E % 4 == 0 rows move as 16-B vectors
// ---------------------------------------------------------------------------
struct EmbTab {
  const float* w;
  int64_t w_k;     // client stride of the table
  const int64_t* ids;
  int64_t ids_k;   // client stride of the ids (0: shared by every client)
  int64_t V;       // rows (ids outside [0, V) produce NaN: the caller validates)
};

__global__ __launch_bounds__(256) void embed_fwd_kernel(EmbTab t0, EmbTab t1, EmbTab t2, int ntab, int K, int64_t N,
                                                        int E, float* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (int64_t)K * N) return;
  const int k = (int)(row / N);
  const int64_t n = row - (int64_t)k * N;
  const float* src[3];
  bool bad = false;
  EmbTab tabs[3] = {t0, t1, t2};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    src[j] = nullptr;
    if (j < ntab) {
      const int64_t id = tabs[j].ids[k * tabs[j].ids_k + n];
      bad |= id < 0 || id >= tabs[j].V;
      src[j] = tabs[j].w + k * tabs[j].w_k + (bad ? 0 : id) * E;
    }
  }
  float* dst = out + row * E;
  if (bad) {
    for (int e = lane; e < E; e += 64) dst[e] = __builtin_nanf("");
    return;
  }
  for (int e = lane; e < E; e += 64) {
    float v = src[0][e];
    if (ntab > 1) v = add_rn(v, src[1][e]);
    if (ntab > 2) v = add_rn(v, src[2][e]);
    dst[e] = v;
  }
}

// ---------------------------------------------------------------------------
// embedding backward, deterministic: dtable[k][id] = sum over the positions n
// holding id, in position order, starting from 0 — torch's CPU
// embedding_dense_backward (index_add over the indices in order).
// 1. per client, sort keys id * N + n in LDS (bitonic, padded to a power of
//    two with 0xFFFFFFFF); 2. one wave per sorted position that starts a run of
//    equal ids sums the run's rows and writes the table row (overwrite).  Rows
//    no position touches are left alone (the caller zero-fills dtable).
// ---------------------------------------------------------------------------
constexpr int SORT_MAX = 4096;

__global__ __launch_bounds__(1024) void embed_sort_kernel(const int64_t* __restrict__ ids, int64_t ids_k, int N,
                                                          int NP, int64_t V, uint32_t* __restrict__ keys) {
  __shared__ uint32_t s[SORT_MAX];
  const int k = blockIdx.x;
  for (int i = threadIdx.x; i < NP; i += blockDim.x) {
    uint32_t key = 0xFFFFFFFFu;
    if (i < N) {
      int64_t id = ids[k * ids_k + i];
      id = id < 0 || id >= V ? V : id;  // out-of-range ids sort last and are skipped
      key = (uint32_t)(id * N + i);
    }
    s[i] = key;
  }
  __syncthreads();
  for (int size = 2; size <= NP; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < NP / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t a = s[lo], b = s[hi];
        if ((a > b) == up) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < N; i += blockDim.x) keys[(int64_t)k * N + i] = s[i];
}

__global__ __launch_bounds__(256) void embed_scatter_kernel(const uint32_t* __restrict__ keys, int K, int N, int64_t V,
                                                            const float* __restrict__ dout, int E,
                                                            float* __restrict__ dtab, int64_t dtab_k) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= (int64_t)K * N) return;
  const int k = (int)(w / N);
  const int j = (int)(w - (int64_t)k * N);
  const uint32_t* kk = keys + (int64_t)k * N;
  const uint32_t key = kk[j];
  const uint32_t id = key / (uint32_t)N;
  if (id >= V) return;
  if (j > 0 && kk[j - 1] / (uint32_t)N == id) return;  // not the head of its run
  int end = j + 1;
  while (end < N && kk[end] / (uint32_t)N == id) ++end;
  const float* src = dout + (int64_t)k * N * E;
  float* dst = dtab + k * dtab_k + (int64_t)id * E;
  for (int e0 = 0; e0 < E; e0 += 64 * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int q = j; q < end; ++q) {
      const int n = (int)(kk[q] % (uint32_t)N);
      const float* r = src + (int64_t)n * E;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + lane + 64 * u;
        if (e < E) acc[u] = add_rn(acc[u], r[e]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + lane + 64 * u;
      if (e < E) dst[e] = acc[u];
    }
  }
}

// ---------------------------------------------------------------------------
// LayerNorm, one wave per row (D <= 1024, D % 4 == 0 for the vector path):
//   s = x [+ r];  y = (s - mean) * rstd * gamma + beta,  rstd = 1/sqrt(var + eps)
// (biased variance, as nn.LayerNorm).  Row i belongs to client i / rpc.
// ---------------------------------------------------------------------------
constexpr int LN_MAXV = 4;  // float4 per lane: D <= 64 * 4 * 4 = 1024

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ r, int64_t ldr,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float* __restrict__ y, int64_t ldy, float* __restrict__ s_out,
                                                     int64_t lds, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int64_t rows, int D, int rpc,
                                                     float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int k = (int)(row / rpc);
  const int nv = D / 4;
  f32x4 v[LN_MAXV];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int q = lane + 64 * c;
    v[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (q < nv) {
      f32x4 a = *reinterpret_cast<const f32x4*>(x + row * ldx + 4 * q);
      if (r) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(r + row * ldr + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = add_rn(a[e], b[e]);
        if (s_out) *reinterpret_cast<f32x4*>(s_out + row * lds + 4 * q) = a;
      }
      v[c] = a;
      sum += (a[0] + a[1]) + (a[2] + a[3]);
    }
  }
  const float mean = wave_sum(sum) / (float)D;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    if (lane + 64 * c < nv) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[c][e] - mean;
        sq = __builtin_fmaf(d, d, sq);
      }
    }
  }
  const float var = wave_sum(sq) / (float)D;
  const float rstd = 1.f / __fsqrt_rn(var + eps);
  const float* g = gamma + (int64_t)k * D;
  const float* b = beta + (int64_t)k * D;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int q = lane + 64 * c;
    if (q < nv) {
      const f32x4 gg = *reinterpret_cast<const f32x4*>(g + 4 * q);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b + 4 * q);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[c][e] - mean) * rstd * gg[e] + bb[e];
      *reinterpret_cast<f32x4*>(y + row * ldy + 4 * q) = o;
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// backward: xh = (s - mean) rstd, gy = gamma dy,
//   ds = rstd (gy - mean(gy) - xh mean(gy xh)) [+ dskip]
// dgamma = sum_rows dy xh, dbeta = sum_rows dy: per (client, chunk of
// LN_CHUNK rows) partials in fixed order, then ln_reduce_kernel over chunks.
constexpr int LN_CHUNK = 64;

__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, int64_t lddy,
                                                     const float* __restrict__ s, int64_t lds,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const float* __restrict__ dskip, int64_t ldk,
                                                     float* __restrict__ dx, int64_t lddx, int rpc, int D,
                                                     int nchunk, float* __restrict__ part) {
  // grid: (nchunk, K); wave w handles rows w, w + 4, ... of the chunk
  __shared__ float red[4][2][1024];
  const int k = blockIdx.y, ch = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nv = D / 4;
  const float* g = gamma + (int64_t)k * D;
  f32x4 gg[LN_MAXV], pg[LN_MAXV], pb[LN_MAXV];
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int q = lane + 64 * c;
    gg[c] = q < nv ? *reinterpret_cast<const f32x4*>(g + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    pg[c] = pb[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int r0 = ch * LN_CHUNK, r1 = std::min(rpc, r0 + LN_CHUNK);
  for (int lr = r0 + wave; lr < r1; lr += 4) {
    const int64_t row = (int64_t)k * rpc + lr;
    const float mean = mean_in[row], rstd = rstd_in[row];
    f32x4 xh[LN_MAXV], gy[LN_MAXV];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      const int q = lane + 64 * c;
      xh[c] = gy[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < nv) {
        const f32x4 sv = *reinterpret_cast<const f32x4*>(s + row * lds + 4 * q);
        const f32x4 d = *reinterpret_cast<const f32x4*>(dy + row * lddy + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[c][e] = (sv[e] - mean) * rstd;
          gy[c][e] = gg[c][e] * d[e];
          a += gy[c][e];
          b = __builtin_fmaf(gy[c][e], xh[c][e], b);
          pg[c][e] = __builtin_fmaf(d[e], xh[c][e], pg[c][e]);
          pb[c][e] += d[e];
        }
      }
    }
    const float ma = wave_sum(a) / (float)D, mb = wave_sum(b) / (float)D;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      const int q = lane + 64 * c;
      if (q < nv) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rstd * (gy[c][e] - ma - xh[c][e] * mb);
        if (dskip) {
          const f32x4 sk = *reinterpret_cast<const f32x4*>(dskip + row * ldk + 4 * q);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = add_rn(o[e], sk[e]);
        }
        *reinterpret_cast<f32x4*>(dx + row * lddx + 4 * q) = o;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int q = lane + 64 * c;
    if (q < nv) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[wave][0][4 * q + e] = pg[c][e];
        red[wave][1][4 * q + e] = pb[c][e];
      }
    }
  }
  __syncthreads();
  float* pp = part + ((int64_t)k * nchunk + ch) * 2 * D;
  for (int i = threadIdx.x; i < 2 * D; i += 256) {
    const int which = i / D, col = i - which * D;
    pp[i] = ((red[0][which][col] + red[1][which][col]) + red[2][which][col]) + red[3][which][col];
  }
}

__global__ void ln_reduce_kernel(const float* __restrict__ part, int nchunk, int D, float* __restrict__ dgamma,
                                 float* __restrict__ dbeta) {
  const int k = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * D) return;
  const float* p = part + (int64_t)k * nchunk * 2 * D + i;
  float acc = 0.f;
  for (int c = 0; c < nchunk; ++c) acc += p[(int64_t)c * 2 * D];
  if (i < D) dgamma[(int64_t)k * D + i] = acc;
  else dbeta[(int64_t)k * D + i - D] = acc;
}

// ---------------------------------------------------------------------------
// multi-head self-attention, one workgroup per (client * batch row, head),
// T <= ATT_MAXT tokens, head width 64, fp32 on the VALU.
// qkv rows [rows][3D]: q at h*64, k at D + h*64, v at 2D + h*64 (the fused
// in-projection's output).  ctx rows [rows][D] (heads concatenated),
// lse [(kb * H + h) * T + i].
//   S = Q K^T / 8,  P = softmax_row(S),  O = P V
// LDS regions of T4 = roundup(T, 4) rows x LDR floats (LDR >= max(64, T4),
// LDR / 4 odd: 16-B rows, conflict-free ds_read_b128 for 16 distinct rows);
// rows T..T4-1 hold zeros, so the 4-deep inner loops need no bounds.
// Thread (ti, tj) = (tid / 16, tid % 16): score rows ti + 16a, columns
// tj + 16c (a, c < NT); output rows ti + 16a, columns 4 tj .. 4 tj + 3.
// Rows >= T are clamped to T - 1 on read and never written.
// ---------------------------------------------------------------------------
constexpr int DH = 64;
constexpr int ATT_MAXT = 96;

__host__ __device__ inline int att_t4(int T) { return (T + 3) & ~3; }
// row stride 4m with m odd: 16 lanes reading 16 distinct rows with ds_read_b128
// hit 16 distinct 4-bank groups of the 64 banks (conflict-free)
__host__ __device__ inline int att_ldr(int T) {
  const int x = att_t4(T) > DH ? att_t4(T) : DH;
  return ((x / 4) & 1) ? x : x + 4;
}

// s[a][c] = sum_d A[ra][d] * B[rc][d] over d < 64 (16-B LDS reads)
template <int NA, int NC>
__device__ __forceinline__ void att_dot(const float* A, const float* Bm, int ldr, const int (&ra)[NA],
                                        const int (&rc)[NC], float (&s)[NA][NC]) {
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int c = 0; c < NC; ++c) s[a][c] = 0.f;
#pragma unroll 2
  for (int d = 0; d < DH; d += 4) {
    f32x4 av[NA], bv[NC];
#pragma unroll
    for (int a = 0; a < NA; ++a) av[a] = *reinterpret_cast<const f32x4*>(A + ra[a] * ldr + d);
#pragma unroll
    for (int c = 0; c < NC; ++c) bv[c] = *reinterpret_cast<const f32x4*>(Bm + rc[c] * ldr + d);
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[a][c] = __builtin_fmaf(av[a][e], bv[c][e], s[a][c]);
  }
}

// o[a][0..3] = sum_j L[ra][j] * R[j][4 tj .. 4 tj + 3] over j < T4 (L's columns
// j >= T and R's rows j >= T are zero)
template <int NT>
__device__ __forceinline__ void att_mat(const float* L, const float* R, int ldr, int T4, const int (&ra)[NT], int tj,
                                        f32x4 (&o)[NT]) {
#pragma unroll
  for (int a = 0; a < NT; ++a) o[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < T4; j += 4) {
    f32x4 lv[NT], rv[4];
#pragma unroll
    for (int a = 0; a < NT; ++a) lv[a] = *reinterpret_cast<const f32x4*>(L + ra[a] * ldr + j);
#pragma unroll
    for (int q = 0; q < 4; ++q) rv[q] = *reinterpret_cast<const f32x4*>(R + (j + q) * ldr + 4 * tj);
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) o[a][e] = __builtin_fmaf(lv[a][q], rv[q][e], o[a][e]);
  }
}

__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// NS heads' [T][64] row blocks (row stride ld[s], column offset folded into
// src[s]) into LDS regions [T4][ldr]; rows T..T4-1 zeroed.  Every global load
// is issued before the first LDS store: at two workgroups per CU nothing else
// hides a serial chain of HBM latencies.
template <int NS, int THR>
__device__ __forceinline__ void att_load(float* const (&dst)[NS], const float* const (&src)[NS],
                                         const int64_t (&ld)[NS], int T, int ldr) {
  constexpr int ATT_LOAD_IT = (((ATT_MAXT + 3) & ~3) * 16 + THR - 1) / THR;
  const int T4 = att_t4(T);
  f32x4 v[NS][ATT_LOAD_IT];
#pragma unroll
  for (int it = 0; it < ATT_LOAD_IT; ++it) {
    const int e = threadIdx.x + THR * it;
    const int i = e >> 4, q = e & 15;
#pragma unroll
    for (int k = 0; k < NS; ++k)
      v[k][it] = i < T ? *reinterpret_cast<const f32x4*>(src[k] + i * ld[k] + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int it = 0; it < ATT_LOAD_IT; ++it) {
    const int e = threadIdx.x + THR * it;
    const int i = e >> 4, q = e & 15;
    if (e < T4 * 16) {
#pragma unroll
      for (int k = 0; k < NS; ++k) *reinterpret_cast<f32x4*>(dst[k] + i * ldr + 4 * q) = v[k][it];
    }
  }
}

template <int N>
__device__ __forceinline__ void att_rows(int T, int t, int step, int (&r)[N]) {
#pragma unroll
  for (int a = 0; a < N; ++a) r[a] = min(t + step * a, T - 1);
}

// THR threads per (sequence, head): thread (ti, tj) = (tid / 16, tid % 16) owns
// score rows ti + RS a (RS = THR / 16, a < NA) and columns tj + 16 c (c < NT);
// every score, softmax sum and output element is computed by one thread in the
// same order whatever THR is (bit-identical); 512 threads put four waves on each
// SIMD at two workgroups per CU instead of two (att_threads).
template <int NT, int THR>
struct AttShape {
  static constexpr int RS = THR / 16;
  static constexpr int NA = (NT * 16 + RS - 1) / RS;
};

template <int NT, int THR>
__global__ __launch_bounds__(THR) void att_fwd_kernel(const float* __restrict__ qkv, float* __restrict__ ctx,
                                                      float* __restrict__ lse, int T, int H) {
  constexpr int RS = AttShape<NT, THR>::RS, NA = AttShape<NT, THR>::NA;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int ldr = att_ldr(T), T4 = att_t4(T);
  const int region = T4 * ldr;
  float* Qs = sm;  // later: P [T4][ldr]
  float* Ks = Qs + region;
  float* Vs = Ks + region;
  const int h = blockIdx.x, kb = blockIdx.y;
  const int D = H * DH;
  const int64_t row0 = (int64_t)kb * T;
  const float* base = qkv + row0 * 3 * D + h * DH;
  {
    float* const dst[3] = {Qs, Ks, Vs};
    const float* const src[3] = {base, base + D, base + 2 * D};
    const int64_t ld[3] = {3 * D, 3 * D, 3 * D};
    att_load<3, THR>(dst, src, ld, T, ldr);
  }
  __syncthreads();
  const int tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
  int ra[NA], rc[NT];
  att_rows<NA>(T, ti, RS, ra);
  att_rows<NT>(T, tj, 16, rc);
  float s[NA][NT];
  att_dot<NA, NT>(Qs, Ks, ldr, ra, rc, s);
  __syncthreads();  // Q is dead: its region takes P
  float* Ps = Qs;
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = ti + RS * a;
    float m = -__builtin_huge_valf();
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      s[a][c] = s[a][c] * 0.125f;  // / sqrt(64): exact
      if (tj + 16 * c < T) m = fmaxf(m, s[a][c]);
    }
    m = group16_max(m);
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const float p = tj + 16 * c < T ? expf(s[a][c] - m) : 0.f;
      s[a][c] = p;
      sum += p;
    }
    sum = group16_sum(sum);
    const float inv = 1.f / sum;
    if (i < T) {
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        const int j = tj + 16 * c;
        if (j < T4) Ps[i * ldr + j] = s[a][c] * inv;  // columns T..T4-1: 0
      }
      if (tj == 0) lse[((int64_t)kb * H + h) * T + i] = m + logf(sum);
    }
  }
  __syncthreads();
  f32x4 o[NA];
  att_mat<NA>(Ps, Vs, ldr, T4, ra, tj, o);
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = ti + RS * a;
    if (i < T) *reinterpret_cast<f32x4*>(ctx + (row0 + i) * D + h * DH + 4 * tj) = o[a];
  }
}

// backward: P = exp(S / 8 - lse); dV = P^T dO; dP = dO V^T;
// Drow_i = sum_d dO[i][d] O[i][d]; dS = P (dP - Drow) / 8;
// dQ = dS K; dK = dS^T Q.  dqkv rows [rows][3D] (overwritten).
// Four LDS regions: Q, K, V (-> P^T -> dS), dO (-> dS^T).
template <int NT, int THR>
__global__ __launch_bounds__(THR) void att_bwd_kernel(const float* __restrict__ qkv, const float* __restrict__ ctx,
                                                      const float* __restrict__ dctx, const float* __restrict__ lse,
                                                      float* __restrict__ dqkv, int T, int H) {
  constexpr int RS = AttShape<NT, THR>::RS, NA = AttShape<NT, THR>::NA;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int ldr = att_ldr(T), T4 = att_t4(T);
  const int region = T4 * ldr;
  float* Qs = sm;
  float* Ks = Qs + region;
  float* Vs = Ks + region;
  float* dOs = Vs + region;
  const int h = blockIdx.x, kb = blockIdx.y;
  const int D = H * DH;
  const int64_t row0 = (int64_t)kb * T;
  const float* base = qkv + row0 * 3 * D + h * DH;
  const int tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
  int ra[NA], rc[NT];
  att_rows<NA>(T, ti, RS, ra);
  att_rows<NT>(T, tj, 16, rc);
  // Drow for rows ti + RS a (16 lanes split the 64 columns, 4 each) and the
  // rows' lse: loads issued ahead of the LDS fill
  f32x4 gv[NA], ov[NA];
  float lrow[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int64_t off = (row0 + ra[a]) * D + h * DH + 4 * tj;
    gv[a] = *reinterpret_cast<const f32x4*>(dctx + off);
    ov[a] = *reinterpret_cast<const f32x4*>(ctx + off);
    lrow[a] = lse[((int64_t)kb * H + h) * T + ra[a]];
  }
  {
    float* const dst[4] = {Qs, Ks, Vs, dOs};
    const float* const src[4] = {base, base + D, base + 2 * D, dctx + row0 * D + h * DH};
    const int64_t ld[4] = {3 * D, 3 * D, 3 * D, D};
    att_load<4, THR>(dst, src, ld, T, ldr);
  }
  float drow[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_fmaf(gv[a][e], ov[a][e], acc);
    drow[a] = group16_sum(acc);
  }
  __syncthreads();
  float p[NA][NT], dp[NA][NT];
  att_dot<NA, NT>(Qs, Ks, ldr, ra, rc, p);
  att_dot<NA, NT>(dOs, Vs, ldr, ra, rc, dp);
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int c = 0; c < NT; ++c) p[a][c] = tj + 16 * c < T ? expf(p[a][c] * 0.125f - lrow[a]) : 0.f;
  __syncthreads();  // V is dead: its region takes P^T
  float* Pt = Vs;
  for (int e = tid; e < T4 * ldr; e += THR) Pt[e] = 0.f;
  __syncthreads();
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = ti + RS * a;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const int j = tj + 16 * c;
      if (i < T && j < T) Pt[j * ldr + i] = p[a][c];
    }
  }
  __syncthreads();
  float* dq = dqkv + row0 * 3 * D + h * DH;
  {  // dV[j][4tj..] = sum_i P^T[j][i] dO[i][4tj..]
    f32x4 o[NA];
    att_mat<NA>(Pt, dOs, ldr, T4, ra, tj, o);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int j = ti + RS * a;
      if (j < T) *reinterpret_cast<f32x4*>(dq + (int64_t)j * 3 * D + 2 * D + 4 * tj) = o[a];
    }
  }
  __syncthreads();  // P^T and dO are dead: dS into V's region, dS^T into dO's
  float* dS = Vs;
  float* dSt = dOs;
  for (int e = tid; e < T4 * ldr; e += THR) {
    dS[e] = 0.f;
    dSt[e] = 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = ti + RS * a;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const int j = tj + 16 * c;
      if (i < T && j < T) {
        const float v = p[a][c] * (dp[a][c] - drow[a]) * 0.125f;
        dS[i * ldr + j] = v;
        dSt[j * ldr + i] = v;
      }
    }
  }
  __syncthreads();
  {
    f32x4 oq[NA], ok[NA];
    att_mat<NA>(dS, Ks, ldr, T4, ra, tj, oq);   // dQ[i] = sum_j dS[i][j] K[j]
    att_mat<NA>(dSt, Qs, ldr, T4, ra, tj, ok);  // dK[j] = sum_i dS^T[j][i] Q[i]
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int r = ti + RS * a;
      if (r < T) {
        *reinterpret_cast<f32x4*>(dq + (int64_t)r * 3 * D + 4 * tj) = oq[a];
        *reinterpret_cast<f32x4*>(dq + (int64_t)r * 3 * D + D + 4 * tj) = ok[a];
      }
    }
  }
}

// out = dy * act'(aux) [* mul] elementwise (the backward of an activation
// whose producing GEMM is not fused with it); modes as flr_bgemm_ex's D* modes.
__global__ void act_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ aux,
                               const float* __restrict__ mul, int act, float* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = dy[i];
    const float a = aux[i];
    if (act == FLR_ACT_DRELU) {
      v = a > 0.f ? v : 0.f;
    } else if (act == FLR_ACT_DGELU) {
      const float cdf = 0.5f * (1.f + erff(a * 0.70710678118654752440f));
      v = v * (cdf + a * (expf(-0.5f * a * a) * 0.39894228040143267794f));
    } else if (act == FLR_ACT_DTANH) {
      v = v * (1.f - a * a);
    }
    if (mul) v = v * mul[i];
    out[i] = v;
  }
}

inline size_t att_fwd_lds(int T) { return (size_t)3 * att_t4(T) * att_ldr(T) * sizeof(float); }
inline size_t att_bwd_lds(int T) { return (size_t)4 * att_t4(T) * att_ldr(T) * sizeof(float); }

}  // namespace xf
}  // namespace flr

using namespace flr;

extern "C" int flr_fill(float* p, int64_t n, float value, void* stream) {
  if (n < 0 || (n > 0 && !p)) return FLR_ERR_ARG;
  if (n == 0) return FLR_OK;
  const int64_t blocks = std::min<int64_t>((n / 4 + 255) / 256 + 1, 16384);
  hipLaunchKernelGGL(xf::fill_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p, n, value);
  return launch_status("fill_kernel");
}

namespace flr {
namespace xf {
// x0[k][b][t] = (t == 0 ? cls[k] : tok[k][b*P + t - 1]) + pos[k][t]  (rows of D)
__global__ void vit_tokens_kernel(const float* __restrict__ tok, const float* __restrict__ cls,
                                  const float* __restrict__ pos, float* __restrict__ x0, int B, int P, int D,
                                  int64_t total4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int d4 = D / 4, T = P + 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
    const int q = (int)(i % d4);
    const int64_t row = i / d4;  // (k, b, t)
    const int t = (int)(row % T);
    const int64_t kb = row / T;
    const int k = (int)(kb / B), b = (int)(kb % B);
    const f32x4 a = t == 0 ? reinterpret_cast<const f32x4*>(cls + (int64_t)k * D)[q]
                           : reinterpret_cast<const f32x4*>(tok + (((int64_t)k * B + b) * P + t - 1) * D)[q];
    const f32x4 pp = reinterpret_cast<const f32x4*>(pos + ((int64_t)k * T + t) * D)[q];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = add_rn(a[e], pp[e]);
    reinterpret_cast<f32x4*>(x0)[i] = o;
  }
}
}  // namespace xf
}  // namespace flr

extern "C" int flr_vit_tokens(const float* tok, const float* cls, const float* pos, int64_t K, int64_t B, int64_t P,
                              int64_t D, float* x0, void* stream) {
  if (!tok || !cls || !pos || !x0 || K < 1 || B < 1 || P < 1 || D < 4 || D % 4) return FLR_ERR_ARG;
  const int64_t total4 = K * B * (P + 1) * D / 4;
  const int64_t blocks = std::min<int64_t>((total4 + 255) / 256, 16384);
  hipLaunchKernelGGL(xf::vit_tokens_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), tok, cls, pos,
                     x0, (int)B, (int)P, (int)D, total4);
  return launch_status("vit_tokens_kernel");
}

extern "C" int flr_act_bwd(const float* dy, const float* aux, const float* mul, int act, float* out, int64_t n,
                           void* stream) {
  if (n < 0 || (n > 0 && (!dy || !aux || !out)) || act < FLR_ACT_DRELU || act > FLR_ACT_DTANH) return FLR_ERR_ARG;
  if (n == 0) return FLR_OK;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
  hipLaunchKernelGGL(xf::act_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), dy, aux, mul, act,
                     out, n);
  return launch_status("act_bwd_kernel");
}

extern "C" int flr_embedding_fwd(const float* w0, int64_t w0_k, int64_t V0, const int64_t* ids0, int64_t ids0_k,
                                 const float* w1, int64_t w1_k, int64_t V1, const int64_t* ids1, int64_t ids1_k,
                                 const float* w2, int64_t w2_k, int64_t V2, const int64_t* ids2, int64_t ids2_k,
                                 int64_t K, int64_t N, int64_t E, float* out, void* stream) {
  if (!w0 || !ids0 || !out || K < 1 || K > 65535 || N < 1 || E < 1 || V0 < 1) return FLR_ERR_ARG;
  if ((w1 && (!ids1 || V1 < 1)) || (w2 && (!w1 || !ids2 || V2 < 1))) return FLR_ERR_ARG;
  const int ntab = w2 ? 3 : (w1 ? 2 : 1);
  const xf::EmbTab t0{w0, w0_k, ids0, ids0_k, V0}, t1{w1, w1_k, ids1, ids1_k, V1}, t2{w2, w2_k, ids2, ids2_k, V2};
  const int64_t rows = K * N;
  hipLaunchKernelGGL(xf::embed_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, as_stream(stream), t0,
                     ntab > 1 ? t1 : t0, ntab > 2 ? t2 : t0, ntab, (int)K, N, (int)E, out);
  return launch_status("embed_fwd_kernel");
}

extern "C" size_t flr_embedding_bwd_workspace(int64_t K, int64_t N) {
  if (K < 1 || N < 1) return 0;
  return align_up((size_t)K * N * sizeof(uint32_t), 256);
}

extern "C" int flr_embedding_bwd(const float* dout, const int64_t* ids, int64_t ids_k, int64_t K, int64_t N,
                                 int64_t V, int64_t E, float* dtable, int64_t dtable_k, int zero_fill,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  if (!dout || !ids || !dtable || K < 1 || K > 65535 || N < 1 || E < 1 || V < 1) return FLR_ERR_ARG;
  if (N > xf::SORT_MAX || (V + 1) * N >= (int64_t(1) << 32) - 1) return FLR_ERR_UNSUPPORTED;
  if (!workspace || workspace_bytes < flr_embedding_bwd_workspace(K, N)) return FLR_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  int rc;
  if (zero_fill) {
    if (dtable_k == V * E) {
      if ((rc = flr_fill(dtable, K * V * E, 0.f, stream)) != FLR_OK) return rc;
    } else {
      for (int64_t k = 0; k < K; ++k)
        if ((rc = flr_fill(dtable + k * dtable_k, V * E, 0.f, stream)) != FLR_OK) return rc;
    }
  }
  int NP = 1;
  while (NP < N) NP <<= 1;
  uint32_t* keys = static_cast<uint32_t*>(workspace);
  hipLaunchKernelGGL(xf::embed_sort_kernel, dim3((unsigned)K), dim3(1024), 0, st, ids, ids_k, (int)N, NP, V, keys);
  if ((rc = launch_status("embed_sort_kernel")) != FLR_OK) return rc;
  const int64_t waves = K * N;
  hipLaunchKernelGGL(xf::embed_scatter_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, keys, (int)K,
                     (int)N, V, dout, (int)E, dtable, dtable_k);
  return launch_status("embed_scatter_kernel");
}

extern "C" int flr_layernorm_fwd(const float* x, int64_t ldx, const float* residual, int64_t ldr, const float* gamma,
                                 const float* beta, float* y, int64_t ldy, float* s_out, int64_t lds, float* mean,
                                 float* rstd, int64_t rows, int64_t D, int64_t rows_per_client, float eps,
                                 void* stream) {
  if (!x || !gamma || !beta || !y || !mean || !rstd || rows < 1 || D < 4 || D % 4 || D > 1024) return FLR_ERR_ARG;
  if (rows_per_client < 1 || rows % rows_per_client || (s_out && !residual)) return FLR_ERR_ARG;
  if (ldx % 4 || ldy % 4 || (residual && ldr % 4) || (s_out && lds % 4)) return FLR_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(xf::ln_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, as_stream(stream), x, ldx,
                     residual, ldr, gamma, beta, y, ldy, s_out, lds, mean, rstd, rows, (int)D, (int)rows_per_client,
                     eps);
  return launch_status("ln_fwd_kernel");
}

extern "C" size_t flr_layernorm_bwd_workspace(int64_t K, int64_t rows_per_client, int64_t D) {
  if (K < 1 || rows_per_client < 1 || D < 1) return 0;
  const int64_t nchunk = (rows_per_client + xf::LN_CHUNK - 1) / xf::LN_CHUNK;
  return align_up((size_t)K * nchunk * 2 * D * sizeof(float), 256);
}

extern "C" int flr_layernorm_bwd(const float* dy, int64_t lddy, const float* s, int64_t lds, const float* gamma,
                                 const float* mean, const float* rstd, const float* dskip, int64_t ldk, float* dx,
                                 int64_t lddx, float* dgamma, float* dbeta, int64_t K, int64_t rows_per_client,
                                 int64_t D, void* workspace, size_t workspace_bytes, void* stream) {
  if (!dy || !s || !gamma || !mean || !rstd || !dx || !dgamma || !dbeta) return FLR_ERR_ARG;
  if (K < 1 || K > 65535 || rows_per_client < 1 || D < 4 || D % 4 || D > 1024) return FLR_ERR_ARG;
  if (lddy % 4 || lds % 4 || lddx % 4 || (dskip && ldk % 4)) return FLR_ERR_UNSUPPORTED;
  if (!workspace || workspace_bytes < flr_layernorm_bwd_workspace(K, rows_per_client, D)) return FLR_ERR_WORKSPACE;
  const int nchunk = (int)((rows_per_client + xf::LN_CHUNK - 1) / xf::LN_CHUNK);
  float* part = static_cast<float*>(workspace);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(xf::ln_bwd_kernel, dim3((unsigned)nchunk, (unsigned)K), dim3(256), 0, st, dy, lddy, s, lds, gamma,
                     mean, rstd, dskip, ldk, dx, lddx, (int)rows_per_client, (int)D, nchunk, part);
  int rc = launch_status("ln_bwd_kernel");
  if (rc != FLR_OK) return rc;
  hipLaunchKernelGGL(xf::ln_reduce_kernel, dim3((unsigned)((2 * D + 255) / 256), (unsigned)K), dim3(256), 0, st, part,
                     nchunk, (int)D, dgamma, dbeta);
  return launch_status("ln_reduce_kernel");
}

namespace {
// 512 threads per (sequence, head) for T > 80 (AttShape; T = 96: fwd 28.2 -> 15.4 us,
// bwd 35.8 -> 32.3 at KB = 64, H = 2, bit-identical).  At T = 65 (ViT-S/4) the 512-thread
// form computes 96 score rows instead of 80 and measured slower (fwd 263 -> 293 us, bwd
// 492 -> 678 at KB = 1024, H = 6), so T <= 80 stays on 256.  FLR_ATT_THREADS=256 / 512
// forces a form (A/B, read per launch; tools/att_bench.py).
inline int att_threads(int NT) {
  const char* e = flr::knob("FLR_ATT_THREADS");
  if (e && atoi(e) == 256) return 256;
  if (e && atoi(e) == 512) return 512;
  return NT >= 6 ? 512 : 256;
}
template <int NT>
int att_fwd_launch(const float* qkv, float* ctx, float* lse, int64_t KB, int T, int H, hipStream_t st) {
  const dim3 grid((unsigned)H, (unsigned)KB);
  if (att_threads(NT) == 512)
    hipLaunchKernelGGL((xf::att_fwd_kernel<NT, 512>), grid, dim3(512), xf::att_fwd_lds(T), st, qkv, ctx, lse, T, H);
  else
    hipLaunchKernelGGL((xf::att_fwd_kernel<NT, 256>), grid, dim3(256), xf::att_fwd_lds(T), st, qkv, ctx, lse, T, H);
  return launch_status("att_fwd_kernel");
}
template <int NT>
int att_bwd_launch(const float* qkv, const float* ctx, const float* dctx, const float* lse, float* dqkv, int64_t KB,
                   int T, int H, hipStream_t st) {
  const dim3 grid((unsigned)H, (unsigned)KB);
  if (att_threads(NT) == 512)
    hipLaunchKernelGGL((xf::att_bwd_kernel<NT, 512>), grid, dim3(512), xf::att_bwd_lds(T), st, qkv, ctx, dctx, lse,
                       dqkv, T, H);
  else
    hipLaunchKernelGGL((xf::att_bwd_kernel<NT, 256>), grid, dim3(256), xf::att_bwd_lds(T), st, qkv, ctx, dctx, lse,
                       dqkv, T, H);
  return launch_status("att_bwd_kernel");
}
}  // namespace

extern "C" int flr_attention_fwd(const float* qkv, int64_t KB, int64_t T, int64_t H, int64_t head_dim, float* ctx,
                                 float* lse, void* stream) {
  if (!qkv || !ctx || !lse || KB < 1 || KB > 65535 || T < 1 || H < 1 || H > 65535) return FLR_ERR_ARG;
  if (head_dim != xf::DH || T > xf::ATT_MAXT) return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  const int t = (int)T, h = (int)H;
  switch ((t + 15) / 16) {
    case 1: return att_fwd_launch<1>(qkv, ctx, lse, KB, t, h, st);
    case 2: return att_fwd_launch<2>(qkv, ctx, lse, KB, t, h, st);
    case 3: return att_fwd_launch<3>(qkv, ctx, lse, KB, t, h, st);
    case 4: return att_fwd_launch<4>(qkv, ctx, lse, KB, t, h, st);
    case 5: return att_fwd_launch<5>(qkv, ctx, lse, KB, t, h, st);
    default: return att_fwd_launch<6>(qkv, ctx, lse, KB, t, h, st);
  }
}

extern "C" int flr_attention_bwd(const float* qkv, const float* ctx, const float* dctx, const float* lse,
                                 int64_t KB, int64_t T, int64_t H, int64_t head_dim, float* dqkv, void* stream) {
  if (!qkv || !ctx || !dctx || !lse || !dqkv || KB < 1 || KB > 65535 || T < 1 || H < 1 || H > 65535)
    return FLR_ERR_ARG;
  if (head_dim != xf::DH || T > xf::ATT_MAXT) return FLR_ERR_UNSUPPORTED;
  hipStream_t st = as_stream(stream);
  const int t = (int)T, h = (int)H;
  switch ((t + 15) / 16) {
    case 1: return att_bwd_launch<1>(qkv, ctx, dctx, lse, dqkv, KB, t, h, st);
    case 2: return att_bwd_launch<2>(qkv, ctx, dctx, lse, dqkv, KB, t, h, st);
    case 3: return att_bwd_launch<3>(qkv, ctx, dctx, lse, dqkv, KB, t, h, st);
    case 4: return att_bwd_launch<4>(qkv, ctx, dctx, lse, dqkv, KB, t, h, st);
    case 5: return att_bwd_launch<5>(qkv, ctx, dctx, lse, dqkv, KB, t, h, st);
    default: return att_bwd_launch<6>(qkv, ctx, dctx, lse, dqkv, KB, t, h, st);
  }
}
