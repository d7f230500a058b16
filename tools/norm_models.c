/* Diagnostic (not product): candidate fp32 accumulation models of CPU
 * torch.norm(a - b), to identify which one a host's torch build uses. */
#include <math.h>
#include <stdint.h>
static float lanesum(const float* l, int L, int tree) {
  if (!tree) { float s = l[0]; for (int c = 1; c < L; ++c) s = s + l[c]; return s; }
  float t[64]; for (int c = 0; c < L; ++c) t[c] = l[c];
  for (int w = L / 2; w >= 1; w /= 2) for (int c = 0; c < w; ++c) t[c] = t[c] + t[c + w];
  return t[0];
}
/* L lanes x U unrolled accumulators (each L lanes); accumulators combined
 * acc0 + acc1 + ... (lane-wise, in order) then lanes summed (seq or tree);
 * tail: mul + add (tailfma=0) or fma (1) */
float norm_model(const float* a, const float* b, int64_t n, int L, int U, int tree, int tailfma) {
  float acc[8][64];
  for (int u = 0; u < U; ++u) for (int c = 0; c < L; ++c) acc[u][c] = 0.f;
  const int64_t step = (int64_t)L * U;
  const int64_t nf = n / step * step;
  for (int64_t r = 0; r < nf; r += step)
    for (int u = 0; u < U; ++u)
      for (int c = 0; c < L; ++c) { float d = a[r + u * L + c] - b[r + u * L + c]; acc[u][c] = fmaf(d, d, acc[u][c]); }
  /* remaining full L-vectors go into acc[0] */
  int64_t r = nf;
  for (; r + L <= n; r += L)
    for (int c = 0; c < L; ++c) { float d = a[r + c] - b[r + c]; acc[0][c] = fmaf(d, d, acc[0][c]); }
  for (int u = 1; u < U; ++u) for (int c = 0; c < L; ++c) acc[0][c] = acc[0][c] + acc[u][c];
  float s = lanesum(acc[0], L, tree);
  for (; r < n; ++r) { float d = a[r] - b[r]; if (tailfma) s = fmaf(d, d, s); else { float q = d * d; s = s + q; } }
  return sqrtf(s);
}
double norm_double(const float* a, const float* b, int64_t n) {
  double s = 0; for (int64_t r = 0; r < n; ++r) { float d = a[r] - b[r]; s += (double)d * d; } return sqrt(s);
}
/* 8 fma lanes, lanes summed in order, then the tail: while >= 4 remain, 4
 * elements as separate multiply + add; the last < 4 as fma (mode 0); other
 * splits for comparison (mode 1: groups of 4 as mul+add only for the first
 * group; mode 2: all mul+add; mode 3: all fma) */
float norm_model2(const float* a, const float* b, int64_t n, int mode) {
  float lane[8] = {0};
  const int64_t nf = n / 8 * 8;
  for (int64_t r = 0; r < nf; r += 8)
    for (int c = 0; c < 8; ++c) { float d = a[r + c] - b[r + c]; lane[c] = fmaf(d, d, lane[c]); }
  float s = lane[0];
  for (int c = 1; c < 8; ++c) s = s + lane[c];
  int64_t t = nf;
  if (mode == 0 || mode == 1)
    for (; t + 4 <= n; t += 4) {
      for (int k = 0; k < 4; ++k) { float d = a[t + k] - b[t + k]; float q = d * d; s = s + q; }
      if (mode == 1) { t += 4; break; }
    }
  for (; t < n; ++t) { float d = a[t] - b[t]; if (mode == 2) { float q = d * d; s = s + q; } else s = fmaf(d, d, s); }
  return sqrtf(s);
}
