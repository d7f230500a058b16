/* ORACLE (test infrastructure only) — the reference's per-pair Krum distance
 * `torch.norm(flat_i - flat_j).item()` (src/defenses/krum.py:95) restated as
 * plain C: the fp32 CPU accumulation of torch.norm probed on this image
 * (tests/test_oracle.py pins this file against torch.norm
 * itself on random vectors of many lengths):
 *   d = fl(a - b); 8 fp32 lanes, lane c = fma(d[8r+c], d[8r+c], lane c) over r;
 *   s = lane 0 + ... + lane 7 in order;
 *   tail (the P mod 8 last elements): while 4 or more remain, the next 4 as
 *   s = s + fl(d[t]*d[t]) (separate multiply and add), the last 0..3 as
 *   s = fma(d[t], d[t], s) — the compiled scalar tail loop of torch's norm
 *   kernel (probed: tools/diag_norm_host.py, tests/test_oracle.py);
 *   sqrt_f32(s).
 * Built by oracle/Makefile with -ffp-contract=off (no implicit contraction). */
#include <math.h>
#include <stdint.h>

float flr_oracle_norm_diff(const float* a, const float* b, int64_t n) {
  float lane[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t nf = n / 8 * 8;
  for (int64_t r = 0; r < nf; r += 8)
    for (int c = 0; c < 8; ++c) {
      const float d = a[r + c] - b[r + c];
      lane[c] = fmaf(d, d, lane[c]);
    }
  float s = lane[0];
  for (int c = 1; c < 8; ++c) s = s + lane[c];
  int64_t t = nf;
  if (t + 4 <= n)
    for (const int64_t e = t + 4; t < e; ++t) {
      const float d = a[t] - b[t];
      const float q = d * d;
      s = s + q;
    }
  for (; t < n; ++t) {
    const float d = a[t] - b[t];
    s = fmaf(d, d, s);
  }
  return sqrtf(s);
}

/* D[i][j] = (double)flr_oracle_norm_diff(row i, row j), D[i][i] = 0
 * (krum.py:89-97's matrix); pairs spread over OpenMP threads. */
void flr_oracle_norm_pairs(const float* X, int64_t K, int64_t P, int64_t ldx, double* D) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = 0; i < K; ++i) {
    D[i * K + i] = 0.0;
    for (int64_t j = i + 1; j < K; ++j) {
      const double v = (double)flr_oracle_norm_diff(X + i * ldx, X + j * ldx, P);
      D[i * K + j] = v;
      D[j * K + i] = v;
    }
  }
}
