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

namespace flr {
namespace gru {

constexpr int THREADS = 256;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

struct Dims {
  int K, B, T, H, t;
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
