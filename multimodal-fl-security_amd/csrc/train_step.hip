// a5 / a6 / a7 — cross-entropy and the fused clip + SGD-momentum step, for all
// clients of a GPU at once (client matrix layout, one row per client).
//
// Reference (per client, experiments/run_experiments.py:206-235):
//   loss = CrossEntropyLoss()(model(x), y)                        (mean over batch)
//   loss.backward(); clip_grad_norm_(params, 1.0); optimizer.step()
//   optimizer = SGD(lr, momentum=0.9, weight_decay=wd), re-created per client
//   per round, so the momentum buffer starts as a copy of the first gradient.
// torch.optim.SGD (single-tensor path): g += wd*p; buf = g (first step) else
// buf = momentum*buf + g; p += -lr*buf.  clip_grad_norm_: total = ||grads||_2,
// coef = min(1, max_norm / (total + 1e-6)), g *= coef.
#include "flr_common.h"

#include <algorithm>

namespace flr {
namespace train {

constexpr int THREADS = 256;
constexpr int NBLK = 32;   // norm partial blocks per client row (>= 8 float4 per lane at C3's unfused blocks)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// partial[k][b] = sum of g^2 over block b of row k (fp64 for a stable norm).
__global__ __launch_bounds__(THREADS) void sumsq_kernel(const float* __restrict__ G, int64_t P, int64_t ldg,
                                                        double* __restrict__ partial) {
  __shared__ double red[THREADS / 64];
  const int k = blockIdx.y, b = blockIdx.x;
  const float* g = G + (int64_t)k * ldg;
  const int64_t p0 = P * b / NBLK, p1 = P * (b + 1) / NBLK;
  double acc = 0.0;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += THREADS) {
    const double v = (double)g[p];
    acc += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < THREADS / 64; ++w) s += red[w];
    partial[(int64_t)k * NBLK + b] = s;
  }
}

// coef[k] = min(1, max_norm / (||g_k|| + 1e-6)) in fp32 (torch computes it in
// the gradient dtype); norms_out[k] = ||g_k||.
// partial [nparts][K][NBLK] (the blocked step's launches over block chunks),
// summed part by part in fixed order.
__global__ void clip_coef_kernel(const double* __restrict__ partial, int K, float max_norm,
                                 float* __restrict__ coef, float* __restrict__ norms_out, int nparts = 1) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int c = 0; c < nparts; ++c)
    for (int b = 0; b < NBLK; ++b) s += partial[((int64_t)c * K + k) * NBLK + b];
  const float total = (float)sqrt(s);
  float c = __fdiv_rn(max_norm, __fadd_rn(total, 1e-6f));
  coef[k] = c < 1.0f ? c : 1.0f;
  if (norms_out) norms_out[k] = total;
}

// The whole optimizer step, one pass: g' = coef*g (+wd*p); buf; p.
__global__ __launch_bounds__(THREADS) void sgd_kernel(float* __restrict__ X, const float* __restrict__ G,
                                                      float* __restrict__ M, int64_t P, int64_t ld,
                                                      const float* __restrict__ coef, float lr, float mom,
                                                      float wd, int first) {
  const int k = blockIdx.y;
  const float c = coef ? coef[k] : 1.0f;
  float* x = X + (int64_t)k * ld;
  const float* g = G + (int64_t)k * ld;
  float* m = M + (int64_t)k * ld;
  const float nlr = -lr;
  for (int64_t p = (int64_t)blockIdx.x * THREADS + threadIdx.x; p < P; p += (int64_t)gridDim.x * THREADS) {
    const float xp = x[p];
    float gp = g[p] * c;
    if (wd != 0.0f) gp = __builtin_fmaf(wd, xp, gp);
    const float b = first ? gp : m[p] * mom + gp;  // buf.mul_(mom).add_(g): two roundings
    m[p] = b;
    x[p] = __builtin_fmaf(nlr, b, xp);
  }
}

// Cross-entropy over rows of logits [R, C] (R = K*B), labels int64 [R].
// loss_row[r] = logsumexp - logit[label]; dlogits = (softmax - onehot) * scale
// with scale = 1/B (mean over each client's batch).  One wave per row.
__global__ __launch_bounds__(THREADS) void ce_kernel(const float* __restrict__ logits, const int64_t* __restrict__ labels,
                                                     int R, int C, float scale, float* __restrict__ loss_row,
                                                     float* __restrict__ dlogits) {
  const int r = blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float* z = logits + (int64_t)r * C;
  float mx = -__builtin_huge_valf();
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, z[c]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += expf(z[c] - mx);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
  const float lse = mx + logf(se);
  const int64_t y = labels[r];
  if (lane == 0) loss_row[r] = lse - z[y];
  float* dz = dlogits + (int64_t)r * C;
  for (int c = lane; c < C; c += 64) {
    const float sm = expf(z[c] - lse);
    dz[c] = (sm - (c == y ? 1.0f : 0.0f)) * scale;
  }
}

// loss[k] = mean over the client's B rows (sequential, fp32).
__global__ void ce_mean_kernel(const float* __restrict__ loss_row, int K, int B, float* __restrict__ loss) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += loss_row[(int64_t)k * B + b];
  loss[k] = s / (float)B;
}

// out[c] = (sum_r X[r][c]) / R with a sequential fp64 sum — the client's
// reported loss, sum(loss.item() per batch) / len (fl_client.py:143-149).
__global__ void mean_rows_kernel(const float* __restrict__ X, int R, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int r = 0; r < R; ++r) s += (double)X[(int64_t)r * C + c];
  out[c] = (float)(s / (double)R);
}

__global__ void scale_rows_kernel(float* __restrict__ d, const float* __restrict__ gk, int K, int B, int C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)K * B * C) return;
  d[i] *= gk[i / ((int64_t)B * C)];
}


// ---- parameter-major ("blocked") variants -------------------------------
// Training keeps each parameter as its own contiguous [K][n_j] block (so a
// grouped convolution's weight view is free and autograd's gradient tensors
// are used in place).  A client's flattened index e in [0, P) lives in block
// j with pre[j] <= e < pre[j+1], at x[j] + k*cs[j] + (e - pre[j]), where the
// client stride cs[j] is n[j] for a whole parameter and larger for a sub-slab
// (the live kernel taps of a tap-major conv weight; the dead taps' slabs are
// left out of the step altogether).
constexpr int MAXB = 80;        // blocks per launch (the table is a kernel argument, < 4 KB)
constexpr int MAX_PARTS = 8;    // launches per step: up to 640 parameter blocks
struct BlockTable {
  float* x[MAXB];
  const float* g[MAXB];
  float* m[MAXB];
  int64_t pre[MAXB + 1];
  int32_t cs[MAXB];   // client stride of block j (elements)
  int32_t xo[MAXB];   // last step with an output matrix: block j's offset in an output row
  uint8_t vec[MAXB];  // bit 0: block j may use 16-B accesses (n % 4 == 0, all three bases 16-B aligned);
                      // bit 1: its squares arrive as producer partials (extra_sq): sumsq skips it;
                      // bit 2: the first step reads its parameters from the shared x_src + xo[j]
  int nb;
};

// Visits e in [lo, hi) of a block whose client segment starts 256-B aligned
// when n % 4 == 0: scalar head up to a 4-element boundary, float4 body, scalar
// tail.  f1(e) handles one element, f4(e) four consecutive ones.
template <class F1, class F4>
__device__ __forceinline__ void visit_range(int64_t lo, int64_t hi, int64_t pre, bool vec, F1 f1, F4 f4) {
  if (!vec) {
    for (int64_t e = lo + threadIdx.x; e < hi; e += THREADS) f1(e);
    return;
  }
  int64_t vlo = pre + ((lo - pre + 3) & ~(int64_t)3);
  if (vlo > hi) vlo = hi;
  const int64_t vhi = pre + ((hi - pre) & ~(int64_t)3);
  for (int64_t e = lo + threadIdx.x; e < vlo; e += THREADS) f1(e);
  for (int64_t e = vlo + 4 * (int64_t)threadIdx.x; e < vhi; e += 4 * THREADS) f4(e);
  for (int64_t e = (vhi > vlo ? vhi : vlo) + threadIdx.x; e < hi; e += THREADS) f1(e);
}

__global__ __launch_bounds__(THREADS) void sumsq_blocked_kernel(const BlockTable tb, int64_t P,
                                                                double* __restrict__ partial, int64_t ld = NBLK) {
  __shared__ double red[THREADS / 64];
  const int k = blockIdx.y, b = blockIdx.x;
  const int64_t p0 = P * b / NBLK, p1 = P * (b + 1) / NBLK;
  double acc = 0.0;
  for (int j = 0; j < tb.nb; ++j) {
    const int64_t lo = p0 > tb.pre[j] ? p0 : tb.pre[j];
    const int64_t hi = p1 < tb.pre[j + 1] ? p1 : tb.pre[j + 1];
    if (lo >= hi || (tb.vec[j] & 2)) continue;
    const float* g = tb.g[j] + (int64_t)k * tb.cs[j] - tb.pre[j];
    auto f1 = [&](int64_t e) {
      const double v = (double)g[e];
      acc += v * v;
    };
    if (!(tb.vec[j] & 1)) {
      for (int64_t e = lo + threadIdx.x; e < hi; e += THREADS) f1(e);
      continue;
    }
    // visit_range's order, with 8 float4 loads in flight per lane before they are summed
    const int64_t pre = tb.pre[j];
    int64_t vlo = pre + ((lo - pre + 3) & ~(int64_t)3);
    if (vlo > hi) vlo = hi;
    const int64_t vhi = pre + ((hi - pre) & ~(int64_t)3);
    for (int64_t e = lo + threadIdx.x; e < vlo; e += THREADS) f1(e);
    int64_t e = vlo + 4 * (int64_t)threadIdx.x;
    for (; e + 7 * 4 * THREADS < vhi; e += 8 * 4 * THREADS) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(g + e + u * 4 * THREADS);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc += (double)v[u][q] * (double)v[u][q];
    }
    for (; e < vhi; e += 4 * THREADS) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(g + e);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += (double)v[q] * (double)v[q];
    }
    for (int64_t t = (vhi > vlo ? vhi : vlo) + threadIdx.x; t < hi; t += THREADS) f1(t);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < THREADS / 64; ++w) s += red[w];
    partial[(int64_t)k * ld + b] = s;
  }
}

// clip_coef_kernel plus producer partials extra[k][0, n_extra) (e.g. the conv
// weight-gradient epilogues' sums of squares): one workgroup per client sums
// the nparts*NBLK blocked partials and the extra ones, thread t taking
// indices t, t+256, ... in order, then a fixed tree over the threads.
__global__ __launch_bounds__(THREADS) void clip_coef_ex_kernel(const double* __restrict__ partial, int K,
                                                               float max_norm, float* __restrict__ coef,
                                                               float* __restrict__ norms_out, int nparts,
                                                               const double* __restrict__ extra, int64_t n_extra) {
  __shared__ double red[THREADS];
  const int k = blockIdx.x, t = threadIdx.x;
  const int nb = nparts * NBLK;
  double s = 0.0;
  for (int64_t i = t; i < nb + n_extra; i += THREADS)
    s += i < nb ? partial[((int64_t)(i / NBLK) * K + k) * NBLK + i % NBLK] : extra[(int64_t)k * n_extra + (i - nb)];
  red[t] = s;
  __syncthreads();
  for (int o = THREADS / 2; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) {
    const float total = (float)sqrt(red[0]);
    const float c = __fdiv_rn(max_norm, __fadd_rn(total, 1e-6f));
    coef[k] = c < 1.0f ? c : 1.0f;
    if (norms_out) norms_out[k] = total;
  }
}

// grid (NSGD, K): workgroup b of client k updates flattened range [P*b/NSGD, P*(b+1)/NSGD).
// flags: bit 0 = the optimizer's first step (buf = g, the old buffer is not
// read); bit 1 = its last step (the new buffer is not written: the optimizer
// is discarded after the client's local update, run_experiments.py:206-211).
// The float4 body keeps two groups of (x, g, m) loads in flight per lane.
// xout (last step only): the updated parameters go to the client matrix row
// xout + k*xout_ld + xo[j] instead of back to x (the training copy is
// reloaded from the global model next round anyway), negated for rows
// k < nneg (the sign-flip attackers' submission, model_poisoning.py:274-276).
constexpr int NSGD = 256;
// U float4 groups per lane in flight per iteration (FLR_SGD_U = 2 | 4 | 8; 8 measured
// 0.43 ms per C3 round faster than 2)
template <int U>
__global__ __launch_bounds__(THREADS) void sgd_blocked_kernel(const BlockTable tb, int64_t P,
                                                              const float* __restrict__ coef, float lr, float mom,
                                                              float wd, int flags, float* __restrict__ xout,
                                                              int64_t xout_ld, int nneg,
                                                              const float* __restrict__ xsrc) {
  const int k = blockIdx.y, b = blockIdx.x;
  const bool first = flags & 1, last = flags & 2;
  const float c = coef ? coef[k] : 1.0f;
  const float nlr = -lr;
  const bool redirect = last && xout != nullptr;
  const float sg = (redirect && k < nneg) ? -1.f : 1.f;
  const int64_t nsgd = gridDim.x;  // NSGD, or fewer for a small parameter group
  const int64_t p0 = P * b / nsgd, p1 = P * (b + 1) / nsgd;
  auto upd = [&](float xp, float gr, float mp, float& mo, float& xo) {
    float gp = gr * c;
    if (wd != 0.0f) gp = __builtin_fmaf(wd, xp, gp);
    const float bb = first ? gp : mp * mom + gp;  // buf.mul_(mom).add_(g): two roundings
    mo = bb;
    xo = __builtin_fmaf(nlr, bb, xp);
  };
  for (int j = 0; j < tb.nb; ++j) {
    const int64_t lo = p0 > tb.pre[j] ? p0 : tb.pre[j];
    const int64_t hi = p1 < tb.pre[j + 1] ? p1 : tb.pre[j + 1];
    if (lo >= hi) continue;
    const int64_t base = (int64_t)k * tb.cs[j] - tb.pre[j];
    float* x = tb.x[j] + base;
    const float* g = tb.g[j] + base;
    float* m = tb.m[j] + base;
    float* xd = redirect ? xout + (int64_t)k * xout_ld + tb.xo[j] - tb.pre[j] : x;
    // the first step of a round may read every client's parameters from one
    // shared copy (the global model they all start from)
    const float* xr = (first && xsrc && (tb.vec[j] & 4)) ? xsrc + tb.xo[j] - tb.pre[j] : x;
    auto one = [&](int64_t e) {
      float mo, xo;
      upd(xr[e], g[e], first ? 0.f : m[e], mo, xo);
      if (!last) m[e] = mo;
      xd[e] = xo * sg;
    };
    auto four = [&](const f32x4& xv, const f32x4& gv, const f32x4& mv, int64_t e) {
      f32x4 mo, xo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float a, bq;
        upd(xv[q], gv[q], mv[q], a, bq);
        mo[q] = a;
        xo[q] = bq;
      }
      if (!last) *reinterpret_cast<f32x4*>(m + e) = mo;
      *reinterpret_cast<f32x4*>(xd + e) = xo * sg;
    };
    if (!(tb.vec[j] & 1)) {
      for (int64_t e = lo + threadIdx.x; e < hi; e += THREADS) one(e);
      continue;
    }
    const int64_t pre = tb.pre[j];
    int64_t vlo = pre + ((lo - pre + 3) & ~(int64_t)3);
    if (vlo > hi) vlo = hi;
    const int64_t vhi = pre + ((hi - pre) & ~(int64_t)3);
    for (int64_t e = lo + threadIdx.x; e < vlo; e += THREADS) one(e);
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    int64_t e = vlo + 4 * (int64_t)threadIdx.x;
    for (; e + (U - 1) * 4 * THREADS < vhi; e += U * 4 * THREADS) {  // U float4 groups per lane in flight
      f32x4 xv[U], gv[U], mv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t eu = e + u * 4 * THREADS;
        xv[u] = *reinterpret_cast<const f32x4*>(xr + eu);
        gv[u] = *reinterpret_cast<const f32x4*>(g + eu);
        mv[u] = first ? z : *reinterpret_cast<const f32x4*>(m + eu);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) four(xv[u], gv[u], mv[u], e + u * 4 * THREADS);
    }
    for (; e < vhi; e += 4 * THREADS) {
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr + e), g0 = *reinterpret_cast<const f32x4*>(g + e);
      four(x0, g0, first ? z : *reinterpret_cast<const f32x4*>(m + e), e);
    }
    for (int64_t t = (vhi > vlo ? vhi : vlo) + threadIdx.x; t < hi; t += THREADS) one(t);
  }
}

}  // namespace train
}  // namespace flr

using namespace flr;

namespace flr {
// The clip norm's sum-of-squares partials of a set of gradient blocks (block j:
// g_blocks[j] + k * client_stride[j], numel[j] values per client), NBLK per
// client at out[k * out_ld + b] — the same pass and order as the optimizer's
// own (sumsq_blocked_kernel), launched early on a side stream by a trainer
// whose blocks' gradients are final before the backward ends; the optimizer
// then takes them as extra partials (block_normed set for those blocks).
int clip_sumsq_blocks(const float* const* g_blocks, const int64_t* numel, const int64_t* client_stride,
                      int64_t nblocks, int64_t K, double* out, int64_t out_ld, int nslots, hipStream_t st) {
  if (nslots != train::NBLK || nblocks < 1 || nblocks > train::MAXB || K < 1 || !out || out_ld < train::NBLK)
    return FLR_ERR_ARG;
  train::BlockTable tb;
  tb.nb = (int)nblocks;
  tb.pre[0] = 0;
  for (int q = 0; q < tb.nb; ++q) {
    const int64_t cs = client_stride[q];
    if (!g_blocks[q] || numel[q] < 0 || cs < numel[q] || cs >= ((int64_t)1 << 31)) return FLR_ERR_ARG;
    tb.x[q] = nullptr;
    tb.g[q] = g_blocks[q];
    tb.m[q] = nullptr;
    tb.pre[q + 1] = tb.pre[q] + numel[q];
    tb.cs[q] = (int32_t)cs;
    tb.vec[q] = (numel[q] % 4 == 0 && cs % 4 == 0 && (reinterpret_cast<uintptr_t>(g_blocks[q]) & 15) == 0) ? 1 : 0;
    tb.xo[q] = 0;
  }
  hipLaunchKernelGGL(train::sumsq_blocked_kernel, dim3(train::NBLK, (unsigned)K), dim3(train::THREADS), 0, st, tb,
                     tb.pre[tb.nb], out, out_ld);
  return launch_status("sumsq_blocked_kernel");
}
}  // namespace flr

extern "C" size_t flr_clip_sgd_workspace(int64_t K) {
  return align_up((size_t)train::MAX_PARTS * K * train::NBLK * sizeof(double), 256) +
         align_up((size_t)K * sizeof(float), 256);
}

extern "C" int flr_clip_sgd_step(float* X, const float* G, float* M, int64_t K, int64_t P, int64_t ld, float lr,
                                 float momentum, float weight_decay, float max_norm, int first_step,
                                 float* norms_out, void* workspace, size_t workspace_bytes, void* stream) {
  if (K < 1 || P < 0 || ld < P || !X || !G || !M) return FLR_ERR_ARG;
  if (max_norm > 0 && (!workspace || workspace_bytes < flr_clip_sgd_workspace(K))) return FLR_ERR_WORKSPACE;
  if (P == 0) return FLR_OK;
  hipStream_t st = as_stream(stream);
  float* coef = nullptr;
  int rc;
  if (max_norm > 0) {
    double* partial = static_cast<double*>(workspace);
    coef = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                    align_up((size_t)train::MAX_PARTS * K * train::NBLK * sizeof(double), 256));
    hipLaunchKernelGGL(train::sumsq_kernel, dim3(train::NBLK, (unsigned)K), dim3(train::THREADS), 0, st, G, P, ld,
                       partial);
    if ((rc = launch_status("sumsq_kernel")) != FLR_OK) return rc;
    hipLaunchKernelGGL(train::clip_coef_kernel, dim3(cdiv((int)K, 64)), dim3(64), 0, st, partial, (int)K, max_norm,
                       coef, norms_out);
    if ((rc = launch_status("clip_coef_kernel")) != FLR_OK) return rc;
  }
  const int64_t per_row = (P + train::THREADS - 1) / train::THREADS;
  const unsigned gx = (unsigned)(per_row < 1024 ? per_row : 1024);
  hipLaunchKernelGGL(train::sgd_kernel, dim3(gx, (unsigned)K), dim3(train::THREADS), 0, st, X, G, M, P, ld, coef, lr,
                     momentum, weight_decay, first_step);
  return launch_status("sgd_kernel");
}

extern "C" int flr_cross_entropy(const float* logits, const int64_t* labels, int64_t K, int64_t B, int64_t C,
                                 float* loss, float* dlogits, float* loss_rows, void* stream) {
  if (K < 1 || B < 1 || C < 1 || !logits || !labels || !loss || !dlogits || !loss_rows) return FLR_ERR_ARG;
  hipStream_t st = as_stream(stream);
  const int R = (int)(K * B);
  hipLaunchKernelGGL(train::ce_kernel, dim3(cdiv(R, train::THREADS / 64)), dim3(train::THREADS), 0, st, logits,
                     labels, R, (int)C, 1.0f / (float)B, loss_rows, dlogits);
  int rc = launch_status("ce_kernel");
  if (rc != FLR_OK) return rc;
  hipLaunchKernelGGL(train::ce_mean_kernel, dim3(cdiv((int)K, 64)), dim3(64), 0, st, loss_rows, (int)K, (int)B, loss);
  return launch_status("ce_mean_kernel");
}

extern "C" int flr_mean_rows(const float* X, int64_t R, int64_t C, float* out, void* stream) {
  if (!X || !out || R < 1 || C < 1) return FLR_ERR_ARG;
  hipLaunchKernelGGL(train::mean_rows_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, as_stream(stream), X,
                     (int)R, (int)C, out);
  return launch_status("mean_rows_kernel");
}

extern "C" int flr_scale_client_rows(float* d, const float* gk, int64_t K, int64_t B, int64_t C, void* stream) {
  if (K < 1 || B < 1 || C < 1 || !d || !gk) return FLR_ERR_ARG;
  const int64_t n = K * B * C;
  hipLaunchKernelGGL(train::scale_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), d,
                     gk, (int)K, (int)B, (int)C);
  return launch_status("scale_rows_kernel");
}

extern "C" int flr_clip_sgd_step_blocked(float* const* x_blocks, const float* const* g_blocks, float* const* m_blocks,
                                         const int64_t* block_numel, const int64_t* block_client_stride,
                                         int64_t nblocks, int64_t K, float lr,
                                         float momentum, float weight_decay, float max_norm, int first_step,
                                         float* norms_out, void* workspace, size_t workspace_bytes, void* stream) {
  return flr_clip_sgd_step_blocked_x(x_blocks, g_blocks, m_blocks, block_numel, block_client_stride, nblocks, K, lr,
                                     momentum, weight_decay, max_norm, first_step, nullptr, nullptr, 0, 0, nullptr,
                                     nullptr, 0, norms_out, workspace, workspace_bytes, stream);
}

extern "C" int flr_clip_sgd_step_blocked_x(float* const* x_blocks, const float* const* g_blocks,
                                           float* const* m_blocks, const int64_t* block_numel,
                                           const int64_t* block_client_stride, int64_t nblocks, int64_t K, float lr,
                                           float momentum, float weight_decay, float max_norm, int first_step,
                                           float* x_out, const int64_t* out_offsets, int64_t out_ld, int64_t nneg,
                                           const uint8_t* block_normed, const double* extra_sq, int64_t n_extra,
                                           float* norms_out, void* workspace, size_t workspace_bytes, void* stream) {
  return flr_clip_sgd_step_blocked_src(x_blocks, g_blocks, m_blocks, block_numel, block_client_stride, nblocks, K, lr,
                                       momentum, weight_decay, max_norm, first_step, x_out, out_offsets, out_ld, nneg,
                                       block_normed, extra_sq, n_extra, nullptr, nullptr, norms_out, workspace,
                                       workspace_bytes, stream);
}

extern "C" int flr_clip_sgd_step_blocked_src(float* const* x_blocks, const float* const* g_blocks,
                                             float* const* m_blocks, const int64_t* block_numel,
                                             const int64_t* block_client_stride, int64_t nblocks, int64_t K, float lr,
                                             float momentum, float weight_decay, float max_norm, int first_step,
                                             float* x_out, const int64_t* out_offsets, int64_t out_ld, int64_t nneg,
                                             const uint8_t* block_normed, const double* extra_sq, int64_t n_extra,
                                             const float* x_src, const int64_t* src_offsets, float* norms_out,
                                             void* workspace, size_t workspace_bytes, void* stream) {
  return flr_clip_sgd_step_phase(x_blocks, g_blocks, m_blocks, block_numel, block_client_stride, nblocks, K, lr,
                                 momentum, weight_decay, max_norm, first_step, x_out, out_offsets, out_ld, nneg,
                                 block_normed, extra_sq, n_extra, x_src, src_offsets, norms_out, FLR_SGD_PHASE_ALL,
                                 workspace, workspace_bytes, stream);
}

extern "C" int flr_clip_sgd_step_phase(float* const* x_blocks, const float* const* g_blocks, float* const* m_blocks,
                                       const int64_t* block_numel, const int64_t* block_client_stride,
                                       int64_t nblocks, int64_t K, float lr, float momentum, float weight_decay,
                                       float max_norm, int first_step, float* x_out, const int64_t* out_offsets,
                                       int64_t out_ld, int64_t nneg, const uint8_t* block_normed,
                                       const double* extra_sq, int64_t n_extra, const float* x_src,
                                       const int64_t* src_offsets, float* norms_out, int phase, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  if (phase < FLR_SGD_PHASE_NORM || phase > FLR_SGD_PHASE_ALL) return FLR_ERR_ARG;
  if (n_extra < 0 || (n_extra > 0 && !extra_sq)) return FLR_ERR_ARG;
  // the first step's shared parameter source: block j at x_src + src_offsets[j] (< 0: none)
  const float* xsrc = (first_step & 1) ? x_src : nullptr;
  if (xsrc && !src_offsets) return FLR_ERR_ARG;
  if (K < 1 || nblocks < 1 || nblocks > (int64_t)train::MAXB * train::MAX_PARTS || !x_blocks || !g_blocks ||
      !m_blocks || !block_numel)
    return FLR_ERR_ARG;
  // the output matrix is written on the last step only
  float* xout = (first_step & 2) ? x_out : nullptr;
  if (xout && (!out_offsets || out_ld < 1 || nneg < 0)) return FLR_ERR_ARG;
  if (max_norm > 0 && (!workspace || workspace_bytes < flr_clip_sgd_workspace(K))) return FLR_ERR_WORKSPACE;
  // the blocks in launches of at most MAXB (the table travels as a kernel argument)
  const int nparts = (int)((nblocks + train::MAXB - 1) / train::MAXB);
  train::BlockTable tbs[train::MAX_PARTS];
  int64_t P = 0;
  for (int c = 0; c < nparts; ++c) {
    train::BlockTable& tb = tbs[c];
    const int j0 = c * train::MAXB, j1 = (int)std::min<int64_t>(nblocks, (int64_t)j0 + train::MAXB);
    tb.nb = j1 - j0;
    tb.pre[0] = 0;
    for (int q = 0; q < tb.nb; ++q) {
      const int j = j0 + q;
      if (!x_blocks[j] || !g_blocks[j] || !m_blocks[j] || block_numel[j] < 0) return FLR_ERR_ARG;
      tb.x[q] = x_blocks[j];
      tb.g[q] = g_blocks[j];
      tb.m[q] = m_blocks[j];
      tb.pre[q + 1] = tb.pre[q] + block_numel[j];
      const int64_t cs = block_client_stride ? block_client_stride[j] : block_numel[j];
      if (cs < block_numel[j] || cs >= ((int64_t)1 << 31)) return FLR_ERR_ARG;
      tb.cs[q] = (int32_t)cs;
      const uintptr_t al = reinterpret_cast<uintptr_t>(x_blocks[j]) | reinterpret_cast<uintptr_t>(g_blocks[j]) |
                           reinterpret_cast<uintptr_t>(m_blocks[j]);
      tb.vec[q] = (block_numel[j] % 4 == 0 && cs % 4 == 0 && (al & 15) == 0) ? 1 : 0;
      if (block_normed && block_normed[j]) tb.vec[q] |= 2;
      tb.xo[q] = 0;
      if (xout) {
        const int64_t o = out_offsets[j];
        if (o < 0 || o + block_numel[j] > out_ld || o >= ((int64_t)1 << 31)) return FLR_ERR_ARG;
        tb.xo[q] = (int32_t)o;
        // 16-B output accesses need the row segment 16-B aligned as well
        if (o % 4 != 0 || out_ld % 4 != 0 || (reinterpret_cast<uintptr_t>(xout) & 15) != 0) tb.vec[q] &= ~1;
      }
      if (xsrc && src_offsets[j] >= 0) {  // xo holds the source offset (one step both: they must agree)
        const int64_t o = src_offsets[j];
        if (o >= ((int64_t)1 << 31) || (xout && o != tb.xo[q])) return FLR_ERR_ARG;
        tb.xo[q] = (int32_t)o;
        tb.vec[q] |= 4;
        if (o % 4 != 0 || (reinterpret_cast<uintptr_t>(xsrc) & 15) != 0) tb.vec[q] &= ~1;
      }
    }
    P += tb.pre[tb.nb];
  }
  if (P == 0) return FLR_OK;
  // the optimizer's own sum-of-squares pass covers the blocks without producer
  // partials, re-packed into their own tables so its NBLK ranges split only them
  train::BlockTable sqt[train::MAX_PARTS];
  int nsq = 0;
  if (block_normed) {
    for (int c = 0; c < nparts; ++c)
      for (int q = 0; q < tbs[c].nb; ++q) {
        if (tbs[c].vec[q] & 2) continue;
        if (nsq == 0 || sqt[nsq - 1].nb == train::MAXB) {
          sqt[nsq].nb = 0;
          sqt[nsq].pre[0] = 0;
          ++nsq;
        }
        train::BlockTable& t = sqt[nsq - 1];
        const int r = t.nb++;
        t.x[r] = tbs[c].x[q];
        t.g[r] = tbs[c].g[q];
        t.m[r] = tbs[c].m[q];
        t.cs[r] = tbs[c].cs[q];
        t.vec[r] = tbs[c].vec[q];
        t.xo[r] = 0;
        t.pre[r + 1] = t.pre[r] + (tbs[c].pre[q + 1] - tbs[c].pre[q]);
      }
  } else {
    for (int c = 0; c < nparts; ++c) sqt[c] = tbs[c];
    nsq = nparts;
  }
  hipStream_t st = as_stream(stream);
  float* coef = nullptr;
  int rc;
  if (max_norm > 0) {
    coef = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                    align_up((size_t)train::MAX_PARTS * K * train::NBLK * sizeof(double), 256));
  }
  if (max_norm > 0 && (phase & FLR_SGD_PHASE_NORM)) {
    double* partial = static_cast<double*>(workspace);
    for (int c = 0; c < nsq; ++c) {
      hipLaunchKernelGGL(train::sumsq_blocked_kernel, dim3(train::NBLK, (unsigned)K), dim3(train::THREADS), 0, st,
                         sqt[c], sqt[c].pre[sqt[c].nb], partial + (int64_t)c * K * train::NBLK);
      if ((rc = launch_status("sumsq_blocked_kernel")) != FLR_OK) return rc;
    }
    if (n_extra > 0 || block_normed)
      hipLaunchKernelGGL(train::clip_coef_ex_kernel, dim3((unsigned)K), dim3(train::THREADS), 0, st, partial, (int)K,
                         max_norm, coef, norms_out, nsq, extra_sq, n_extra);
    else
      hipLaunchKernelGGL(train::clip_coef_kernel, dim3(cdiv((int)K, 64)), dim3(64), 0, st, partial, (int)K, max_norm,
                         coef, norms_out, nsq);
    if ((rc = launch_status("clip_coef_kernel")) != FLR_OK) return rc;
  }
  if (!(phase & FLR_SGD_PHASE_UPDATE)) return FLR_OK;
  static const int unroll = [] {
    const char* e = flr::knob("FLR_SGD_U");
    const int u = e ? atoi(e) : 0;
    return (u == 2 || u == 4 || u == 8) ? u : 8;
  }();
  for (int c = 0; c < nparts; ++c) {
    auto kern = unroll == 8 ? train::sgd_blocked_kernel<8>
                            : (unroll == 4 ? train::sgd_blocked_kernel<4> : train::sgd_blocked_kernel<2>);
    // workgroups per client: NSGD, fewer for a small group (each takes >= 8192 elements: one
    // iteration of the 8-deep float4 loop); the update is elementwise, so the split changes nothing
    const int64_t pc = tbs[c].pre[tbs[c].nb];
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(train::NSGD, (pc + 8191) / 8192));
    hipLaunchKernelGGL(kern, dim3(gx, (unsigned)K), dim3(train::THREADS), 0, st, tbs[c],
                       tbs[c].pre[tbs[c].nb], coef, lr, momentum, weight_decay, first_step & 3, xout, out_ld,
                       (int)std::min<int64_t>(nneg, K), xsrc);
    if ((rc = launch_status("sgd_blocked_kernel")) != FLR_OK) return rc;
  }
  return FLR_OK;
}
