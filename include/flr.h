/*
 * flr.h — C ABI of the MI355X-native federated-round engine (gfx950).
 *
 * Every entry point takes plain device pointers, element counts and a
 * hipStream_t passed as `void*` (NULL = the legacy default stream).  Nothing
 * here allocates: scratch space is caller-provided (query the size with the
 * matching *_workspace function).  Calls are stream-ordered and return as soon
 * as the work is enqueued.  Results are deterministic: fixed reduction order,
 * no float atomics, so 1/2/4/8-GPU runs give bit-identical outputs.
 *
 * Each function names the reference interface it replaces
 * (Shashank8834/multimodal-fl-security, paths relative to its repo root).
 *
 * Matrix convention ("client matrix"): X is K rows (clients, in global client
 * order) × P fp32 coordinates (the client's parameters flattened in
 * `model.parameters()` order, krum.py:55-57), row stride `ldx` elements.
 */
#ifndef FLR_H
#define FLR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define FLR_OK 0
#define FLR_ERR_ARG (-1)          /* invalid argument (shape, null pointer) */
#define FLR_ERR_HIP (-2)          /* a HIP runtime call or launch failed    */
#define FLR_ERR_UNSUPPORTED (-3)  /* shape outside what the kernels handle   */
#define FLR_ERR_WORKSPACE (-4)    /* workspace too small or misaligned       */
#define FLR_ERR_KRUM_N (-5)       /* n < 2f+3 (krum.py:153-157)             */

const char* flr_version(void);
/* "gfx950", or "gfx950 ablation" for the tools build (make ABLATION=1) that
 * adds the measured-slower and timing-only kernel forms. */
const char* flr_build_info(void);
/* The A/B switches (FLR_* names): the process environment's FLR_*
 * variables are read once, when the library loads; this sets (value NULL:
 * unsets) one afterwards, for an in-process A/B.  FLR_ERR_ARG unless the name
 * starts with FLR_. */
int flr_set_knob(const char* name, const char* value);
const char* flr_status_string(int status);
/* Last HIP error string recorded by a failing call on this thread. */
const char* flr_last_error(void);

/* ---- a9: Krum pairwise l2 ---------------------------------------------
 * Replaces KrumDefense._compute_distances (src/defenses/krum.py:73-99):
 *   D[i][j] = float32(||X_i - X_j||_2) stored as float64, D[i][i] = 0.
 * Engine: centred Gram matrix on MFMA (bf16 hi/lo split, fp32 accumulate),
 * fixed-order fp64 reduction of per-segment partials.  Any K >= 1.
 * Pairs the centring cannot condition (two rows close to each other but far
 * from the medoid pivot, e.g. a cluster of sign-flipped updates) are flagged
 * from the pivot sample and recomputed from exact fp32 differences (up to 128
 * such rows per call: every row at K <= 128).  More flagged rows than that
 * (K > 128 only) makes EVERY D entry NaN, the diagonal included — the marker
 * callers test (D[0][0] is NaN only then; NaN client rows leave the diagonal
 * 0): a loud failure, never a silently inaccurate distance.
 */
size_t flr_pairwise_l2_workspace(int64_t K, int64_t P);
int flr_pairwise_l2(const float* X, int64_t K, int64_t P, int64_t ldx,
                    double* D, void* workspace, size_t workspace_bytes,
                    void* stream);

/* Same, recording two caller-created hipEvent_t around the main MFMA kernel
 * launch(es) on `stream` (for live per-kernel timing); either may be NULL. */
int flr_pairwise_l2_ex(const float* X, int64_t K, int64_t P, int64_t ldx,
                       double* D, void* workspace, size_t workspace_bytes,
                       void* stream, void* ev_begin, void* ev_end);

/* Coordinate-sharded form of the same computation (the exchange mode where
 * GPU g holds ALL K clients but only a contiguous range of coordinates, see
 * DESIGN.md §2).  The full chunks (64 coordinates) of the vector are cut into
 * FLR_PW_SLICES canonical slices; flr_pairwise_l2 itself runs on exactly these
 * slices, so composing the phases below over any split of the slices gives
 * D bit-identical to flr_pairwise_l2 on the whole matrix:
 *   1. flr_pairwise_sample on every holder, then an exact SUM of the [K][S]
 *      samples (the positions a holder does not own are written as 0);
 *   2. flr_pairwise_pivot on the combined sample (replicated) -> the pivot
 *      record, flr_pairwise_pivot_len() int32 (pivot, refined-row count, rows);
 *   3. flr_pairwise_gram_slices for the holder's slices [q0, q1): X's column
 *      0 is the first coordinate of slice q0 (chunk flr_pw_slice_chunks(q0));
 *      gsum [q1-q0][flr_pairwise_gsum_len(K)] fp64;
 *   4. flr_pairwise_tail on the holder of the coordinates past the last full
 *      chunk (everyone else: p0 == p1, writes zeros), then an exact SUM;
 *   5. gather the gsum blocks of all slices in slice order ->
 *      [FLR_PW_SLICES][gsum_len]; flr_pairwise_finish -> D.
 * P is always the WHOLE vector's length. */
#define FLR_PW_SLICES 8
int flr_pw_slice_chunks(int64_t P, int64_t q, int64_t* chunk_begin, int64_t* chunk_end);
int64_t flr_pairwise_sample_len(int64_t P);
size_t flr_pairwise_gsum_len(int64_t K);
int64_t flr_pairwise_pivot_len(void);
size_t flr_pairwise_sliced_workspace(int64_t K, int64_t P, int64_t nslices);
int flr_pairwise_sample(const float* X, int64_t K, int64_t ldx, int64_t P, int64_t chunk0,
                        int64_t chunk1, float* Xs, void* stream);
int flr_pairwise_pivot(const float* Xs, int64_t K, int64_t P, int* pivot, void* workspace,
                       size_t workspace_bytes, void* stream);
int flr_pairwise_gram_slices(const float* X, int64_t K, int64_t ldx, int64_t P, int64_t q0,
                             int64_t q1, const int* pivot, double* gsum, void* workspace,
                             size_t workspace_bytes, void* stream, void* ev_begin,
                             void* ev_end);
int flr_pairwise_tail(const float* X, int64_t K, int64_t ldx, int64_t p0, int64_t p1,
                      double* tail, void* stream);
int flr_pairwise_finish(const double* gsum, const double* tail, int64_t K, double* D,
                        void* stream);

/* Reference-exact variant (pairwise_method="reference"):
 * D[i][j] bit-identical to the reference's fp32 torch.norm(flat_i - flat_j)
 * .item() (krum.py:89-97) — per pair, 8 fp32 chains of sequential
 * fma(d, d, chain) over every 8th coordinate d = fl(x_i - x_j), the chains
 * summed 0..7 in order, the P mod 8 tail added in order (a first group of 4
 * as separate multiply + add, the last 0..3 as fma), correctly rounded
 * sqrt_f32 (tail probed in tools/diag_norm_host.py;
 * oracle/norm_ref.c; the same bits under torch's AVX2 and AVX512 dispatch,
 * tests/test_oracle.py test_norm_ref_model_cpu_capability).  X in the reference's coordinate order (parameters()
 * order); rows 16-B aligned and ldx % 4 == 0 (else FLR_ERR_ARG).
 * Workspace (256-B aligned): flr_pairwise_l2_reference_workspace(K, P) bytes
 * — the chains' running sums plus one chain-major copy of a coordinate segment
 * (at most 8 GiB; a smaller workspace runs more, shorter segments, the same
 * result; segments hold whole multiples of 512 chain steps, zero-filled past
 * the last, plus 4 KB of prefetch slack: below K x 16 KiB + 4 KiB past the
 * sums, FLR_ERR_WORKSPACE).  part / nparts: this call computes the pairs of tile range
 * [part * T / nparts, (part + 1) * T / nparts), T =
 * flr_pairwise_l2_reference_tiles(K), and writes 0 for every other pair: the
 * nparts results summed (exact: one non-zero term per pair) are the whole D.
 * VALU-issue bound: each pair's 8 chains run the whole vector sequentially. */
size_t flr_pairwise_l2_reference_workspace(int64_t K, int64_t P);
int flr_pairwise_l2_reference_tiles(int64_t K);
int flr_pairwise_l2_reference(const float* X, int64_t K, int64_t P, int64_t ldx,
                              double* D, void* ws, size_t ws_bytes, int64_t part,
                              int64_t nparts, void* stream);
/* The same over a training-order client matrix: the ntaps blocks taps[4b ..
 * 4b+3] = {off, Cout, Cin, KK} (ascending, disjoint, inside [0, P)) hold a
 * convolution weight stored tap-major, column off + (t * Cin + ci) * Cout + co
 * for reference coordinate off + (co * Cin + ci) * KK + t (torch's
 * [Cout][Cin][kh][kw]); every other column is its own coordinate.  The
 * trainers' layout (flr_resnet_gru_reorder), so a round's matrix goes in as
 * written, no torch-order copy; ntaps = 0 is flr_pairwise_l2_reference. */
int flr_pairwise_l2_reference_tap(const float* X, int64_t K, int64_t P, int64_t ldx,
                                  const int64_t* taps, int64_t ntaps, double* D, void* ws,
                                  size_t ws_bytes, int64_t part, int64_t nparts, void* stream);
/* The same with dead taps: dead[b] bit t set = tap t of block b is not in X
 * (FLR_TC_DEFER_DEAD): its slab is read from gdead at the same training-order
 * offset, negated on rows k < nneg — the values flr_resnet_gru_fill_dead
 * writes, so D is bit-identical to the call on the filled X.  No dead column
 * may lie in the last P mod 8 (read from X): FLR_ERR_ARG.  after_rewrite
 * (a hipEvent_t, or NULL): recorded on the stream once the call has read
 * X for the last time (before the chain kernel of the last segment): the
 * dead slabs may be written from then on, beside the chains. */
int flr_pairwise_l2_reference_tap_dead(const float* X, int64_t K, int64_t P, int64_t ldx,
                                       const int64_t* taps, int64_t ntaps, const uint64_t* dead,
                                       const float* gdead, int64_t nneg, double* D, void* ws,
                                       size_t ws_bytes, int64_t part, int64_t nparts,
                                       void* after_rewrite, void* stream);
/* The same split over coordinate ranges held by different ranks (the
 * coordinate-sharded exchange): each range continues the chains where the
 * previous range left them.  _partial: `steps` chain steps of X (coordinates
 * 0 .. 8 steps - 1 of each row; a range starting at a multiple of 8 reference
 * coordinates) added to the running chain sums held in ws's first 8 K^2 floats
 * (first: start from 0; otherwise the previous range's ws sums, copied in);
 * ws as for flr_pairwise_l2_reference_workspace(K, 8 steps).  _finish: D from
 * the chain sums (chains = 0: none) and the last P mod 8 coordinates (Xtail,
 * ntail <= 7).  Each step is the same fp32 operation in the same order as in
 * the one-call form, so D is bit-identical to it. */
int flr_pairwise_l2_reference_partial(const float* X, int64_t K, int64_t steps, int64_t ldx,
                                      int first, void* ws, size_t ws_bytes, void* stream);
int flr_pairwise_l2_reference_finish(const float* Xtail, int64_t K, int64_t ntail, int64_t ldx,
                                     int chains, const void* ws, double* D, void* stream);
/* The same partial chains over a TRAINING-ORDER coordinate slice (a rank of
 * a training-order round at G > 1): taps {off, Cout, Cin, KK} name the
 * tap-major blocks inside the slice (offsets from X, each wholly inside
 * [0, 8 steps)), as flr_pairwise_l2_reference_tap; the slice must hold whole
 * blocks (the round engine aligns its rank boundaries to them). */
int flr_pairwise_l2_reference_partial_tap(const float* X, int64_t K, int64_t steps, int64_t ldx,
                                          const int64_t* taps, int64_t ntaps, int first, void* ws,
                                          size_t ws_bytes, void* stream);

/* Direct-difference VALU variant (same contract, exact fp32 differences);
 * a slower second implementation used to cross-check the MFMA path. */
size_t flr_pairwise_l2_direct_workspace(int64_t K, int64_t P);
int flr_pairwise_l2_direct(const float* X, int64_t K, int64_t P, int64_t ldx,
                           double* D, void* workspace, size_t workspace_bytes,
                           void* stream);

/* ---- a10: Krum score + selection --------------------------------------
 * Replaces KrumDefense._krum_score + the argsort in aggregate
 * (src/defenses/krum.py:101-131, 149-176):
 *   m = K - f - 2; scores[i] = numpy-pairwise-sum(sort(D[i])[1 : m+1]);
 *   order = argsort(scores) (ties broken by lower client index).
 * NaN in numpy's order: after every value in the row sort and in the argsort
 * (a client whose update is NaN gets a NaN score and the last ranks).
 * D: device fp64 K×K (row-major, ld = K). scores: device fp64 [K];
 * order: device int32 [K].  Returns FLR_ERR_KRUM_N if K < 2f+3.
 */
int flr_krum_select(const double* D, int64_t K, int64_t f, double* scores,
                    int32_t* order, void* stream);

/* ---- a11: Multi-Krum mean ---------------------------------------------
 * Replaces the Multi-Krum average (src/defenses/krum.py:182-192):
 *   out = (((0 + X[rows[0]]) + X[rows[1]]) + ...) / divisor   (fp32, in order)
 * rows: device int32 [m] (e.g. the first m entries of `order`); divisor is
 * the reference's multi_k (== m unless multi_k > K).
 * Precondition: every rows[i] in [0, K).  The indices are device-resident, so
 * this is not checked on the host; an out-of-range index is clamped into range
 * on the device (no out-of-bounds read) and the result is then unspecified.
 */
int flr_rows_mean(const float* X, int64_t K, int64_t P, int64_t ldx,
                  const int32_t* rows, int64_t m, int64_t divisor, float* out,
                  void* stream);
/* The same over a training-order matrix whose dead-tap ranges [dead_off[r],
 * + dead_n[r]) are not written (the round engine's FLR_DEFER_DEAD=2): row k's
 * value there is gdead's, negated for k < nneg, summed in the same order —
 * bit-identical to flr_rows_mean over the filled rows; X's dead ranges are not
 * read (the float4 groups wholly inside them).  16-B aligned rows and out. */
int flr_rows_mean_dead(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows,
                       int64_t m, int64_t divisor, const int64_t* dead_off, const int64_t* dead_n,
                       int64_t ndead, const float* gdead, int64_t nneg, float* out, void* stream);

/* ---- a14: FedAvg -------------------------------------------------------
 * Replaces NoDefense.aggregate (src/defenses/base_defense.py:80-97) and the
 * inline FedAvg of experiments/run_experiments.py:246-254:
 *   out = (sum_i fl(n_i * X_i)) / sum_i n_i     (fp32, client order)
 * num_examples: device int64 [K].
 */
int flr_fedavg(const float* X, int64_t K, int64_t P, int64_t ldx,
               const int64_t* num_examples, float* out, void* stream);

/* ---- a12: coordinate-wise trimmed mean ---------------------------------
 * Replaces TrimmedMeanDefense.aggregate (src/defenses/trimmed_mean.py:48-90)
 * for one fixed t (= max(1, int(K*trim_ratio)), computed by the caller):
 *   out[p] = mean(sort(X[:,p])[t : K-t])   (torch's cascade-sum order)
 * Requires K - 2t >= 1 (the caller falls back to the median otherwise).
 */
int flr_trimmed_mean(const float* X, int64_t K, int64_t P, int64_t ldx,
                     int64_t t, float* out, void* stream);

/* ---- a13: coordinate-wise lower median ---------------------------------
 * Replaces MedianDefense.aggregate / _coordinate_wise_median
 * (src/defenses/trimmed_mean.py:92-103, 141-166): torch.median(dim=0)[0]
 * = sort(X[:,p])[(K-1)/2]. Bit-exact (selection, no arithmetic).
 */
int flr_median_lower(const float* X, int64_t K, int64_t P, int64_t ldx,
                     float* out, void* stream);

/* The same two order statistics over the row subset rows[0..m) of X (device
 * int32 indices, m <= K <= 512): the coordinate-wise trimmed mean of the
 * Multi-Krum selection ("Krum + trimmed-mean", BASELINE.json configs[4]).
 * Precondition as flr_rows_mean: rows[i] in [0, K) (out-of-range indices are
 * clamped on the device, never read out of bounds; the result is unspecified). */
int flr_trimmed_mean_rows(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows, int64_t m,
                          int64_t t, float* out, void* stream);
int flr_median_lower_rows(const float* X, int64_t K, int64_t P, int64_t ldx, const int32_t* rows, int64_t m,
                          float* out, void* stream);

/* ---- a6 + a7: fused gradient clip + SGD-momentum step -----------------
 * Replaces, for every client row at once, clip_grad_norm_(params, max_norm)
 * + torch.optim.SGD(lr, momentum, weight_decay).step()
 * (experiments/run_experiments.py:206-211, 234-235; fl_client.py:123-141):
 *   coef_k = min(1, max_norm / (||G_k|| + 1e-6))   (skipped if max_norm <= 0)
 *   g = coef_k*G_k + wd*X_k;  M_k = first ? g : momentum*M_k + g;  X_k -= lr*M_k
 * X, G, M: device fp32 K×P (row stride ld), updated in place.  norms_out:
 * optional device fp32 [K] (pre-clip gradient norms).
 */
size_t flr_clip_sgd_workspace(int64_t K);
int flr_clip_sgd_step(float* X, const float* G, float* M, int64_t K, int64_t P,
                      int64_t ld, float lr, float momentum, float weight_decay,
                      float max_norm, int first_step, float* norms_out,
                      void* workspace, size_t workspace_bytes, void* stream);

/* Same step on the parameter-major training layout: block j holds block_numel[j]
 * elements per client at client stride block_client_stride[j] (NULL: the
 * blocks are whole parameters, stride = numel); x/g/m_blocks are host arrays
 * of nblocks device pointers (nblocks <= 768, run as launches of <= 96 blocks).  Client k's element e of block j
 * is at ptr_j + k*stride_j + e.  Elements not covered by any block (dead
 * kernel taps, whose gradient is identically zero) are neither read nor
 * updated; with weight_decay == 0 that is exactly the reference's update.
 * first_step is a flag word here: bit 0 = first step (as above), bit 1 = the
 * optimizer's last step (the momentum buffer is not written back: the
 * reference re-creates the optimizer per client per round,
 * run_experiments.py:206-211, so a last step's buffer is never read). */
int flr_clip_sgd_step_blocked(float* const* x_blocks, const float* const* g_blocks,
                              float* const* m_blocks, const int64_t* block_numel,
                              const int64_t* block_client_stride,
                              int64_t nblocks, int64_t K, float lr, float momentum,
                              float weight_decay, float max_norm, int first_step,
                              float* norms_out, void* workspace,
                              size_t workspace_bytes, void* stream);
/* The same step; on the LAST step (first_step bit 1) with x_out != NULL the
 * updated parameters are written to the client matrix instead of back to the
 * blocks: block j of client k lands at x_out + k*out_ld + out_offsets[j]
 * (the trainer's "training order" client matrix, run_experiments.py:238),
 * negated for clients k < nneg (sign-flip attackers, model_poisoning.py:
 * 274-276).  This folds the round's export pass into the optimizer.
 * Clip norm from producer partials: blocks with block_normed[j] != 0 are left
 * out of the optimizer's own sum-of-squares pass; their squares come as fp64
 * partials extra_sq[k*n_extra + i], i < n_extra (e.g. written by
 * flr_conv2d_bwd_weight_t_sq), summed per client in a fixed order. */
int flr_clip_sgd_step_blocked_x(float* const* x_blocks, const float* const* g_blocks,
                                float* const* m_blocks, const int64_t* block_numel,
                                const int64_t* block_client_stride, int64_t nblocks,
                                int64_t K, float lr, float momentum, float weight_decay,
                                float max_norm, int first_step, float* x_out,
                                const int64_t* out_offsets, int64_t out_ld, int64_t nneg,
                                const uint8_t* block_normed, const double* extra_sq,
                                int64_t n_extra, float* norms_out, void* workspace,
                                size_t workspace_bytes, void* stream);
/* flr_clip_sgd_step_blocked_x whose FIRST step reads every client's parameters
 * of block j from one shared vector, x_src + src_offsets[j] (the global model
 * all clients start from, so no per-client copy of it is loaded; offset < 0:
 * the block reads x_blocks[j]); the update still goes to x_blocks (or x_out on
 * a last step, where src_offsets[j] must equal out_offsets[j]).  x_src NULL:
 * flr_clip_sgd_step_blocked_x. */
int flr_clip_sgd_step_blocked_src(float* const* x_blocks, const float* const* g_blocks,
                                  float* const* m_blocks, const int64_t* block_numel,
                                  const int64_t* block_client_stride, int64_t nblocks, int64_t K,
                                  float lr, float momentum, float weight_decay, float max_norm,
                                  int first_step, float* x_out, const int64_t* out_offsets,
                                  int64_t out_ld, int64_t nneg, const uint8_t* block_normed,
                                  const double* extra_sq, int64_t n_extra, const float* x_src,
                                  const int64_t* src_offsets, float* norms_out, void* workspace,
                                  size_t workspace_bytes, void* stream);
/* flr_clip_sgd_step_blocked_src in two phases, so the update can overlap
 * other work (the native trainers run it on a side stream, parameter group by
 * parameter group, under the next local step's forward):
 *   FLR_SGD_PHASE_NORM   the clip norms and coefficients of ALL the blocks
 *                        passed (per-client, into the workspace; norms_out);
 *   FLR_SGD_PHASE_UPDATE the clip + momentum + parameter update of the blocks
 *                        passed (any subset, any order), reading the
 *                        coefficients a NORM phase left in the same workspace;
 *   FLR_SGD_PHASE_ALL    both (= flr_clip_sgd_step_blocked_src).
 * The update is elementwise: splitting it over calls changes no bit. */
#define FLR_SGD_PHASE_NORM 1
#define FLR_SGD_PHASE_UPDATE 2
#define FLR_SGD_PHASE_ALL 3
int flr_clip_sgd_step_phase(float* const* x_blocks, const float* const* g_blocks, float* const* m_blocks,
                            const int64_t* block_numel, const int64_t* block_client_stride,
                            int64_t nblocks, int64_t K, float lr, float momentum, float weight_decay,
                            float max_norm, int first_step, float* x_out, const int64_t* out_offsets,
                            int64_t out_ld, int64_t nneg, const uint8_t* block_normed,
                            const double* extra_sq, int64_t n_extra, const float* x_src,
                            const int64_t* src_offsets, float* norms_out, int phase, void* workspace,
                            size_t workspace_bytes, void* stream);

/* ---- a2: client-batched 2-D convolution (bias-free, as in the conv blocks)
 * Replaces nn.Conv2d forward/backward for every client of a GPU at once
 * (image branch, src/models/cub200_cnn.py:71-77 template).  Layouts:
 *   x  [K][Cin][B][H][W]   (client-channel major: for one (client, channel)
 *                           the B*H*W pixels the GEMM walks are contiguous)
 *   w  [K][Cout][Cin][KH][KW]
 *   y  [K][Cout][B][Ho][Wo], Ho = (H + 2 pad - KH) / stride + 1
 * fp32 in, fp32 accumulate: each operand split into three bf16 terms, six
 * products per k-step on v_mfma_f32_32x32x16_bf16 (per-product error a few
 * 2^-24 |a b|, the size of an fp32 product's rounding); FLR_GEMM=f32 selects
 * the exact-fp32 v_mfma_f32_32x32x2_f32.  bwd_data writes dx, bwd_weight
 * writes dw (both overwrite).  Kernel taps that only read zero padding are
 * skipped (their dw is written as exact zeros).  The workspace (optional,
 * size from flr_conv2d_workspace) enables deterministic split-K for long
 * reductions; without it the kernels run unsplit. */
size_t flr_conv2d_workspace(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W,
                            int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                            int64_t pad);
int flr_conv2d_fwd(const float* x, const float* w, float* y, int64_t K, int64_t B,
                   int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH,
                   int64_t KW, int64_t stride, int64_t pad, void* workspace,
                   size_t workspace_bytes, void* stream);
int flr_conv2d_bwd_data(const float* dy, const float* w, float* dx, int64_t K,
                        int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                        int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                        void* workspace, size_t workspace_bytes, void* stream);
int flr_conv2d_bwd_weight(const float* x, const float* dy, float* dw, int64_t K,
                          int64_t B, int64_t Cin, int64_t H, int64_t W,
                          int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                          int64_t pad, void* workspace, size_t workspace_bytes,
                          void* stream);
/* flr_conv2d_bwd_weight given the workspace of the flr_conv2d_fwd call that
 * consumed the same x (and has not been reused since): when that forward took
 * the explicit-im2col path (short reductions: the 7x7 stem), its column matrix
 * heads the workspace and the weight gradient reads it instead of rebuilding
 * it.  Otherwise identical to flr_conv2d_bwd_weight. */
int flr_conv2d_bwd_weight_reuse(const float* x, const float* dy, float* dw, int64_t K,
                                int64_t B, int64_t Cin, int64_t H, int64_t W,
                                int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                int64_t pad, void* workspace, size_t workspace_bytes,
                                void* stream);

/* ---- a5: cross-entropy forward + backward ------------------------------
 * Replaces nn.CrossEntropyLoss() (mean over each client's batch;
 * run_experiments.py:186, 232) for K clients × B rows × C classes:
 *   loss[k] = mean_b (logsumexp(z_kb) - z_kb[y_kb]);
 *   dlogits = (softmax(z) - onehot(y)) / B.
 * logits/dlogits: device fp32 [K*B, C]; labels: device int64 [K*B];
 * loss: device fp32 [K]; loss_rows: device fp32 [K*B] scratch.
 */
int flr_cross_entropy(const float* logits, const int64_t* labels, int64_t K,
                      int64_t B, int64_t C, float* loss, float* dlogits,
                      float* loss_rows, void* stream);
/* out[c] = (sum_r X[r][c]) / R, the sum sequential in fp64: each client's
 * reported training loss, the mean of its per-step losses (fl_client.py:143-149). */
int flr_mean_rows(const float* X, int64_t R, int64_t C, float* out, void* stream);
/* d[k, b, c] *= gk[k]  (chain rule for a per-client upstream gradient). */
int flr_scale_client_rows(float* d, const float* gk, int64_t K, int64_t B,
                          int64_t C, void* stream);

/* Tap-major variants (the training engine's conv layout when Cin and Cout are
 * multiples of 64): w_t / dw_t are [K][KH][KW][Cin][Cout] per client, i.e.
 * torch's [Cout][Cin][KH][KW] permuted (0, 2, 3, 1) per client.  Same
 * activations, outputs and semantics as flr_conv2d_fwd / _bwd_data /
 * _bwd_weight; FLR_ERR_UNSUPPORTED when the channel counts do not qualify
 * (flr_conv2d_tap_major_ok).  Workspace (optional, split-K) from
 * flr_conv2d_t_workspace. */
int flr_conv2d_tap_major_ok(int64_t Cin, int64_t Cout);
size_t flr_conv2d_t_workspace(int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W,
                              int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                              int64_t pad);
int flr_conv2d_fwd_t(const float* x, const float* w_t, float* y, int64_t K, int64_t B,
                     int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH,
                     int64_t KW, int64_t stride, int64_t pad, void* workspace,
                     size_t workspace_bytes, void* stream);
int flr_conv2d_bwd_data_t(const float* dy, const float* w_t, float* dx, int64_t K,
                          int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                          int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                          void* workspace, size_t workspace_bytes, void* stream);
/* dx = dgrad + add (one rounding per element; add in dx's layout, NULL: none):
 * the residual block's two input-gradient paths summed in the dgrad epilogue,
 * the value autograd's accumulation of the conv path and the shortcut path
 * gives (the reference's BasicBlock backward, torchvision resnet18).  add may
 * be dx itself (in-place accumulation, dx += dgrad): the stride-parity classes
 * no kernel tap reaches are then skipped (a strided 1x1 shortcut writes only
 * its one class instead of zeros over the other three). */
int flr_conv2d_bwd_data_t_add(const float* dy, const float* w_t, const float* add,
                              float* dx, int64_t K, int64_t B, int64_t Cin, int64_t H,
                              int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                              int64_t stride, int64_t pad, void* workspace,
                              size_t workspace_bytes, void* stream);
/* The forward and the input gradient with w_stride floats between clients'
 * weights (KH*KW*Cin*Cout: the per-client layout above; 0: every client reads
 * the one copy at w_t — the first local step, when every client still holds
 * the global model, needs no per-client copy of it). */
int flr_conv2d_fwd_t_ex(const float* x, const float* w_t, int64_t w_stride, float* y,
                        int64_t K, int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                        int64_t KH, int64_t KW, int64_t stride, int64_t pad, void* workspace,
                        size_t workspace_bytes, void* stream);
int flr_conv2d_bwd_data_t_ex(const float* dy, const float* w_t, int64_t w_stride,
                             const float* add, float* dx, int64_t K, int64_t B, int64_t Cin,
                             int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                             int64_t stride, int64_t pad, void* workspace,
                             size_t workspace_bytes, void* stream);
/* zero_dead_taps: write the dead taps' slabs of dw_t as zeros (1) or leave
 * them untouched (0: the caller never reads them, see
 * flr_clip_sgd_step_blocked). */
int flr_conv2d_bwd_weight_t(const float* x, const float* dy, float* dw_t, int64_t K,
                            int64_t B, int64_t Cin, int64_t H, int64_t W,
                            int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                            int64_t pad, int zero_dead_taps, void* workspace,
                            size_t workspace_bytes, void* stream);
/* The same weight gradient, plus the clip norm's partial sums of squares
 * (a6, run_experiments.py:234): fp64 sums over fixed parts of client k's
 * live-tap gradient at sq[k*sq_ld + i], i < the slot count
 * flr_conv2d_bwd_weight_t_sq_slots returns for the geometry (<= sq_ld).
 * The parts depend on the per-client shape only, never on K.  Needs the
 * full flr_conv2d_t_workspace (FLR_ERR_WORKSPACE otherwise). */
int64_t flr_conv2d_bwd_weight_t_sq_slots(int64_t K, int64_t B, int64_t Cin, int64_t H,
                                         int64_t W, int64_t Cout, int64_t KH, int64_t KW,
                                         int64_t stride, int64_t pad);
int flr_conv2d_bwd_weight_t_sq(const float* x, const float* dy, float* dw_t, int64_t K,
                               int64_t B, int64_t Cin, int64_t H, int64_t W,
                               int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                               int64_t pad, int zero_dead_taps, double* sq, int64_t sq_ld,
                               void* workspace, size_t workspace_bytes, void* stream);

/* ---- a1 / a8 / a15: round-boundary layout moves of the training state ----
 * flr_broadcast_rows: dst[k*dst_stride + i] = src[i] (load_global: every
 * client starts from the global model, run_experiments.py:203).
 * flr_copy_rows: dst[k*dst_stride + i] = src[k*src_stride + i] (parameter
 * block -> client-matrix columns, run_experiments.py:238 + krum.py:55-57).
 * flr_tap_major_to_torch: w_t [K][KK][Cin][Cout] -> torch order
 * [Cout][Cin][KK] at dst + k*dst_stride (KK <= 9). */
int flr_broadcast_rows(const float* src, int64_t n, float* dst, int64_t K,
                       int64_t dst_stride, void* stream);
/* flr_broadcast_rows with rows k < nneg written as -src (the attackers' copy
 * of a range the optimizer never updates, e.g. dead conv taps). */
int flr_broadcast_rows_neg(const float* src, int64_t n, float* dst, int64_t K,
                           int64_t dst_stride, int64_t nneg, void* stream);
int flr_copy_rows(const float* src, int64_t src_stride, int64_t n, float* dst,
                  int64_t dst_stride, int64_t K, void* stream);
int flr_tap_major_to_torch(const float* w_t, int64_t K, int64_t KK, int64_t Cin,
                           int64_t Cout, float* dst, int64_t dst_stride, void* stream);
/* The same two exports with rows k < nneg written negated: the sign-flip
 * attackers' submitted update (model_poisoning.py:274-276, applied after
 * training as malicious_client.py:103-115) folded into the export pass. */
int flr_copy_rows_neg(const float* src, int64_t src_stride, int64_t n, float* dst, int64_t dst_stride, int64_t K,
                      int64_t nneg, void* stream);
int flr_tap_major_to_torch_neg(const float* w_t, int64_t K, int64_t KK, int64_t Cin, int64_t Cout, float* dst,
                               int64_t dst_stride, int64_t nneg, void* stream);

/* ---- §8(f): per-client norms and weighted row combinations ---------------
 * Building blocks of GradientClippingDefense / NormBoundingDefense /
 * DPSGDDefense (src/defenses/differential_privacy.py:74-164, 223-334) and
 * GeometricMedianDefense (src/defenses/trimmed_mean.py:177-265).
 * flr_row_norms: out[i] = ||X_i - center||_2 (type 0) or ||.||_inf (type 1),
 * center optional [P]; differences rounded to fp32, squares summed in fp64 in
 * a fixed order.  Workspace: flr_row_norms_workspace(K) bytes.
 * flr_weighted_rows: out = (sum_j fl(fl(X[rows[j]] * scales[j]) * weights[j]))
 * / divisor, sequential in j (rows NULL = all K rows in order, m = K; scales
 * NULL = 1).  weights/scales are device float arrays of length m. */
size_t flr_row_norms_workspace(int64_t K);
int flr_row_norms(const float* X, int64_t K, int64_t P, int64_t ldx,
                  const float* center, int type, double* out, void* workspace,
                  size_t workspace_bytes, void* stream);
/* out[i] = X_i . v (fp64 sum of exact products); workspace as flr_row_norms.
 * FLTrust's torch.dot (src/defenses/fltrust.py:176). */
int flr_row_dots(const float* X, int64_t K, int64_t P, int64_t ldx, const float* v,
                 double* out, void* workspace, size_t workspace_bytes, void* stream);
int flr_weighted_rows(const float* X, int64_t K, int64_t P, int64_t ldx,
                      const int32_t* rows, int64_t m, const float* weights,
                      const float* scales, float divisor, float* out,
                      void* stream);

/* ---- a3: GRU recurrence, pointwise gate math per time step ----------------
 * Replaces the per-step cell of nn.GRU (torch gate order r, z, n;
 * h' = (h - n) * z + n), used by the text branch of the multimodal model.
 * Layouts: gi [K][B][T][3H], gh [K][B][3H] (= h_t W_hh^T + b_hh),
 * hseq [K][T+1][B][H], gates [K][T][B][4][H] (r, z, n, h_n),
 * dgh [K][T][B][3H], dgi [K][B][T][3H], dh / dh_direct [K][B][H].
 * fwd_step reads hseq[:, t] and writes hseq[:, t+1] and gates[:, t];
 * bwd_step takes dh = dL/dh_{t+1} and writes dgh[:, t], dgi[:, :, t] and
 * dh_direct (the z-gate path of dL/dh_t; the caller adds dgh[:, t] W_hh). */
int flr_gru_fwd_step(const float* gi, const float* gh, float* hseq, float* gates,
                     int64_t K, int64_t B, int64_t T, int64_t H, int64_t t,
                     void* stream);
int flr_gru_bwd_step(const float* dh, const float* gates, const float* hseq,
                     float* dgh, float* dgi, float* dh_direct, int64_t K,
                     int64_t B, int64_t T, int64_t H, int64_t t, void* stream);
/* Fused recurrence steps (B <= 32): one launch per time step instead of a
 * batched GEMM plus a gate kernel.  flr_gru_fwd_fused: gh = h_t W_hh^T + b_hh
 * (whhP = W_hh [K][3H][H] packed by flr_gru_pack(NG=3, C=H, trans=0), bhh
 * [K][3H]) and the gate math of flr_gru_fwd_step in the GEMM's epilogue.
 * flr_gru_bwd_fused (t >= 1): dh_t = dh_direct + dgh[:, t] W_hh (whhTP = W_hh^T
 * packed by flr_gru_pack(NG=1, C=3H, trans=1)), then flr_gru_bwd_step's math
 * for step t - 1 with dy = dh_t (dh_direct rewritten in place); dh0 (optional,
 * [K][B][H]) receives dh_t.  Same products as the batched GEMM (bf16x6 on MFMA,
 * fp32 accumulate), a different reduction order. */
int flr_gru_fwd_fused(const float* gi, const float* whhP, const float* bhh, float* hseq, float* gates, int64_t K,
                      int64_t B, int64_t T, int64_t H, int64_t t, void* stream);
int flr_gru_bwd_fused(const float* whhTP, const float* gates, const float* hseq, float* dgh, float* dgi,
                      float* dh_direct, float* dh0, int64_t K, int64_t B, int64_t T, int64_t H, int64_t t,
                      void* stream);
/* The fused steps with shared_w = 1: every client reads the ONE packed copy at
 * whh / whhT (flr_gru_pack with K = 1): the first local step, when all clients
 * still hold the global W_hh.  shared_w = 0: the calls above. */
int flr_gru_fwd_fused_ex(const float* gi, const float* whh, int shared_w, const float* bhh,
                         float* hseq, float* gates, int64_t K, int64_t B, int64_t T, int64_t H,
                         int64_t t, void* stream);
int flr_gru_bwd_fused_ex(const float* whhT, int shared_w, const float* gates, const float* hseq,
                         float* dgh, float* dgi, float* dh_direct, float* dh0, int64_t K,
                         int64_t B, int64_t T, int64_t H, int64_t t, void* stream);
/* Pack a per-client weight into the fused kernels' MFMA-fragment order: the
 * [NG*H][C] operand (trans = 0: w is [NG*H][C]; trans = 1, NG = 1: w is [C][H]
 * and the operand is its transpose) in 32-row blocks x 16-deep k-steps, each
 * (block, k-step) 512 floats (two 1 KB wave loads), zero-padded.  wp holds
 * K * NG * ceil(H/32) * ceil(C/16) * 512 floats. */
int flr_gru_pack(const float* w, int64_t K, int64_t NG, int64_t H, int64_t C, int trans, float* wp, void* stream);

/* ---- a2: per-client BatchNorm (train mode) + fused residual add / ReLU ----
 * Replaces nn.BatchNorm2d(train) [+ identity add] [+ ReLU] of the conv blocks.
 * x, y, residual: [B][KC][HW] (kc = client*C + channel; the engine's
 * [K][C][B][H][W] activations are passed as B = 1, HW = B*H*W), gamma/beta/mean/
 * invstd: [KC].  fwd: y = act(x*alpha + (beta - mean*alpha) [+ residual]),
 * alpha = gamma/sqrt(var + eps), batch statistics over B*HW, act = ReLU if
 * relu != 0.  bwd: g = dy * (y > 0) if relu else dy; writes dx, dgamma,
 * dbeta, and dresidual = g when dresidual != NULL. */
int flr_batchnorm_fwd(const float* x, const float* gamma, const float* beta,
                      const float* residual, float* y, float* mean, float* invstd,
                      int64_t B, int64_t KC, int64_t HW, float eps, int relu,
                      void* stream);
int flr_batchnorm_bwd(const float* dy, const float* x, const float* y,
                      const float* gamma, const float* mean, const float* invstd,
                      float* dx, float* dgamma, float* dbeta, float* dresidual,
                      int64_t B, int64_t KC, int64_t HW, int relu, void* stream);
/* The ResNet stem's BatchNorm + ReLU + 3x3/2 pad-1 max-pool as one kernel each
 * way (torchvision resnet18 stem: bn1 -> relu -> maxpool), per (client,
 * channel) plane of NI images of H x W: the same values as flr_batchnorm_fwd
 * (relu, no residual) followed by flr_maxpool2d_fwd, and as flr_maxpool2d_bwd
 * followed by flr_batchnorm_bwd (relu; the mask recomputed from x, beta and
 * the saved statistics), without the BN output / its gradient in HBM.
 * y_pool / dy_pool: [KC][NI][H/2][W/2], argmax: 1-byte window offsets as
 * flr_maxpool2d_fwd's.  Shapes: H = W = 16, NI = 16 or 32 (the stem at 32 x 32
 * inputs, batch 16 / 32); else FLR_ERR_UNSUPPORTED (use the two-kernel form). */
int flr_batchnorm_relu_maxpool_fwd(const float* x, const float* gamma, const float* beta,
                                   float* y_pool, uint8_t* argmax, float* mean, float* invstd,
                                   int64_t KC, int64_t NI, int64_t H, int64_t W, float eps,
                                   void* stream);
int flr_maxpool_relu_batchnorm_bwd(const float* dy_pool, const uint8_t* argmax, const float* x,
                                   const float* gamma, const float* beta, const float* mean,
                                   const float* invstd, float* dx, float* dgamma, float* dbeta,
                                   int64_t KC, int64_t NI, int64_t H, int64_t W, void* stream);

/* ---- a3 / a4: batched dense GEMM (text branch, late-fusion MLP) ------------
 * Replaces the nn.Linear / nn.GRU matrix products of the text branch and the
 * fusion head (src/models/cub200_cnn.py:80-93, 107-117 template) for every
 * client at once:
 *   C_k[m][n] = (bias_k[n] or add_k[m][n] or 0) + sum_r A_k(m, r) B_k(n, r)
 * A(m, r) at A + k*a_k + m*a_m + r*a_r (B, C likewise; any strides, so
 * transposed operands are views); bias: NULL or [batch][bias_k] row vectors;
 * add: NULL or a C-shaped addend (may alias C).  Same MFMA tiles as the
 * convolutions (three-term bf16 split, fp32 accumulate; FLR_GEMM=f32: exact-fp32
 * MFMA); split-K chosen from (M, N, R) alone, so every client's result is
 * independent of the batch count.  Workspace (optional, split-K partials): flr_bgemm_workspace.
 * flr_sum_rows: out[k][n] = sum_m X[k][m][n] (bias gradients; eight interleaved
 * partial sums in a fixed order, deterministic). */
size_t flr_bgemm_workspace(int64_t batch, int64_t M, int64_t N, int64_t R);
/* flr_bgemm with a fused epilogue, applied per output element after the
 * bias / addend (and after the split-K reduction):
 *   pre (optional, C-shaped) <- v;  v <- act(v);  v <- v * mul (optional);  C <- v
 * act: FLR_ACT_NONE, _RELU, _GELU (exact erf, torch's nn.GELU()), _TANH; the
 * backward modes multiply the incoming gradient v by the activation's
 * derivative at aux (C-shaped, required): _DRELU (aux > 0, aux = the ReLU
 * input or output), _DGELU (aux = the GELU input), _DTANH (aux = the tanh
 * output).  mul / aux / pre share C's strides.  The late-fusion head's
 * ReLU + dropout mask, the transformer MLP's GELU and BERT's pooler tanh run
 * here instead of as separate elementwise passes. */
#define FLR_ACT_NONE 0
#define FLR_ACT_RELU 1
#define FLR_ACT_GELU 2
#define FLR_ACT_TANH 3
#define FLR_ACT_DRELU 4
#define FLR_ACT_DGELU 5
#define FLR_ACT_DTANH 6
int flr_bgemm_ex(const float* A, int64_t a_k, int64_t a_m, int64_t a_r, const float* B, int64_t b_k, int64_t b_n,
                 int64_t b_r, float* C, int64_t c_k, int64_t c_m, int64_t c_n, const float* bias, int64_t bias_k,
                 const float* add, int act, const float* mul, const float* aux, float* pre, int64_t batch,
                 int64_t M, int64_t N, int64_t R, void* workspace, size_t workspace_bytes, void* stream);
int flr_bgemm(const float* A, int64_t a_k, int64_t a_m, int64_t a_r, const float* B,
              int64_t b_k, int64_t b_n, int64_t b_r, float* C, int64_t c_k, int64_t c_m,
              int64_t c_n, const float* bias, int64_t bias_k, const float* add,
              int64_t batch, int64_t M, int64_t N, int64_t R, void* workspace,
              size_t workspace_bytes, void* stream);
int flr_sum_rows(const float* X, int64_t x_k, int64_t x_m, int64_t batch, int64_t M,
                 int64_t N, float* out, int64_t out_k, void* stream);
/* The same sum over M > 256 rows as fixed 256-row chunks reduced in chunk order
 * (a chunking that depends on M alone); workspace flr_sum_rows_workspace (0:
 * one pass, as flr_sum_rows). */
size_t flr_sum_rows_workspace(int64_t batch, int64_t M, int64_t N);
int flr_sum_rows_ex(const float* X, int64_t x_k, int64_t x_m, int64_t batch, int64_t M, int64_t N, float* out,
                    int64_t out_k, void* workspace, size_t workspace_bytes, void* stream);

/* ---- a2: max pooling of the image branch (the stem's 3x3/2 pad-1 pool) ----
 * Replaces nn.MaxPool2d / F.max_pool2d on x [nplanes][H][W] (planes = B*K*C of
 * the grouped layout).  torch's CPU rule: first in-bounds element of the
 * row-major window scan with (v > max || isnan(v)) wins; argmax [nplanes][Ho][Wo]
 * holds its window offset kh*KW + kw.  bwd: dx[e] = sum of dy over the windows
 * whose argmax is e, in output raster order (overwrites dx). */
int flr_maxpool2d_fwd(const float* x, float* y, uint8_t* argmax, int64_t nplanes, int64_t H,
                      int64_t W, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                      void* stream);
int flr_maxpool2d_bwd(const float* dy, const uint8_t* argmax, float* dx, int64_t nplanes,
                      int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t stride,
                      int64_t pad, void* stream);

/* ---- §8(f): per-round evaluation of the global model (forward only) -------
 * Replaces evaluate_model / compute_attack_success_rate /
 * compute_label_flip_asr (src/utils/metrics.py:14-157).
 * flr_batchnorm_infer: model.eval() BatchNorm — running statistics instead of
 * batch statistics — with the optional residual add and ReLU of the training
 * kernel; x, residual, y [KC][HW] (one contiguous plane per (client, channel)),
 * gamma / beta / running_mean / running_var [KC].
 * flr_classify_rows: logits [R][C] -> pred[r] = first index of the maximum
 * (torch.max(outputs, 1); NaN counts as the maximum) and, with labels,
 * loss_rows[r] = logsumexp(z_r) - z_r[label].  counts (int64[5], accumulated:
 * the caller zeroes them) += {pred == label, pred == target, label == source,
 * label == source && pred == label, label == source && pred == target}.
 * labels may be NULL (then only counts[1] is updated). */
int flr_batchnorm_infer(const float* x, const float* gamma, const float* beta,
                        const float* running_mean, const float* running_var,
                        const float* residual, float* y, int64_t KC, int64_t HW, float eps,
                        int relu, void* stream);
int flr_classify_rows(const float* logits, const int64_t* labels, int64_t R, int64_t C,
                      int64_t target, int64_t source, int32_t* pred, float* loss_rows,
                      int64_t* counts, void* stream);

/* ---- a3 + C4/C5 encoders: embedding, LayerNorm, self-attention -------------
 * (csrc/train_xfmr.hip).  Every op is batched over the clients of a GPU;
 * client k's rows are the k-th run of rows_per_client rows (or N positions).
 *
 * flr_fill: p[0..n) = value (a kernel, so it replays inside HIP graphs).
 *
 * flr_embedding_fwd replaces nn.Embedding (the GRU branch's token embedding,
 * BERT's word / token-type / position embeddings summed in that order):
 *   out[k][n] = ((w0[k][ids0[k][n]] + w1[k][ids1[k][n]]) + w2[k][ids2[k][n]])
 * wj at wj + k*wj_k (row-major [Vj][E]), idsj at idsj + k*idsj_k (stride 0 =
 * the same ids for every client); w1 / w2 may be NULL.  An id outside
 * [0, Vj) yields a NaN row (the caller validates; nothing faults).
 * flr_embedding_bwd: dtable[k][v] = sum of dout[k][n] over the n with
 * ids[k][n] == v, in increasing n, from 0 — torch's CPU embedding backward
 * (index_add in index order), bit for bit.  zero_fill != 0 first zeroes the
 * whole [V][E] table of every client; rows no id touches are otherwise left
 * as they are.  N <= 4096; workspace flr_embedding_bwd_workspace(K, N).
 */
int flr_fill(float* p, int64_t n, float value, void* stream);
/* out[i] = dy[i] * act'(aux[i]) [* mul[i]] for the FLR_ACT_D* modes (the
 * activation backward where no GEMM epilogue can take it). */
int flr_act_bwd(const float* dy, const float* aux, const float* mul, int act, float* out, int64_t n, void* stream);
int flr_embedding_fwd(const float* w0, int64_t w0_k, int64_t V0, const int64_t* ids0, int64_t ids0_k,
                      const float* w1, int64_t w1_k, int64_t V1, const int64_t* ids1, int64_t ids1_k,
                      const float* w2, int64_t w2_k, int64_t V2, const int64_t* ids2, int64_t ids2_k,
                      int64_t K, int64_t N, int64_t E, float* out, void* stream);
size_t flr_embedding_bwd_workspace(int64_t K, int64_t N);
int flr_embedding_bwd(const float* dout, const int64_t* ids, int64_t ids_k, int64_t K, int64_t N, int64_t V,
                      int64_t E, float* dtable, int64_t dtable_k, int zero_fill, void* workspace,
                      size_t workspace_bytes, void* stream);

/* flr_layernorm_fwd replaces nn.LayerNorm(D, eps) over `rows` rows (row i at
 * x + i*ldx, gamma / beta [K][D] for client i / rows_per_client), with the
 * residual add of the encoder block fused in front:
 *   s = x [+ residual];  y = (s - mean) rstd gamma + beta,  rstd = 1/sqrt(var + eps)
 * (biased variance).  s_out (optional, needs residual) receives s; mean / rstd
 * [rows] are saved for the backward.  D % 4 == 0, D <= 1024.
 * flr_layernorm_bwd: ds = rstd (g dy - mean(g dy) - xh mean(g dy xh)) [+ dskip],
 * xh = (s - mean) rstd, written to dx; dgamma / dbeta [K][D] = the per-client
 * sums over rows of dy xh / dy (fixed-order partials over 64-row chunks).
 * Workspace flr_layernorm_bwd_workspace(K, rows_per_client, D). */
int flr_layernorm_fwd(const float* x, int64_t ldx, const float* residual, int64_t ldr, const float* gamma,
                      const float* beta, float* y, int64_t ldy, float* s_out, int64_t lds, float* mean, float* rstd,
                      int64_t rows, int64_t D, int64_t rows_per_client, float eps, void* stream);
size_t flr_layernorm_bwd_workspace(int64_t K, int64_t rows_per_client, int64_t D);
int flr_layernorm_bwd(const float* dy, int64_t lddy, const float* s, int64_t lds, const float* gamma,
                      const float* mean, const float* rstd, const float* dskip, int64_t ldk, float* dx, int64_t lddx,
                      float* dgamma, float* dbeta, int64_t K, int64_t rows_per_client, int64_t D, void* workspace,
                      size_t workspace_bytes, void* stream);

/* ViT token sequence: x0 [K][B][P+1][D], row t of sequence (k, b) =
 * (t == 0 ? cls[k] : tok[k][b*P + t - 1]) + pos[k][t]  (the class token and
 * the patch projections plus the learned position embedding).  D % 4 == 0,
 * 16-B aligned operands. */
int flr_vit_tokens(const float* tok, const float* cls, const float* pos, int64_t K, int64_t B, int64_t P, int64_t D,
                   float* x0, void* stream);

/* Multi-head self-attention core (no mask) for KB = clients x batch
 * sequences of T <= 96 tokens, H heads of width head_dim = 64:
 *   qkv [KB*T][3*H*64] = the fused in-projection's output (q | k | v, heads
 *   concatenated inside each);  S = q k^T / 8;  P = softmax(S);  ctx = P v
 *   ctx [KB*T][H*64];  lse [KB][H][T] = the softmax log-normalisers (saved).
 * flr_attention_bwd recomputes P from lse and writes dqkv [KB*T][3*H*64]
 * (dq | dk | dv).  fp32 on the VALU, one workgroup per (sequence, head). */
int flr_attention_fwd(const float* qkv, int64_t KB, int64_t T, int64_t H, int64_t head_dim, float* ctx, float* lse,
                      void* stream);
int flr_attention_bwd(const float* qkv, const float* ctx, const float* dctx, const float* lse, int64_t KB, int64_t T,
                      int64_t H, int64_t head_dim, float* dqkv, void* stream);

/* ---- a1: the client plugin's local update, one C entry --------------------
 * Replaces the simulation's per-client loop (run_experiments.py:193-240) and
 * FLClient.fit / _train (fl_client.py:76-149) for K clients of the C2/C3
 * model family (ResNet image trunk + embedding / 1-layer GRU text branch +
 * late-fusion head; the module layout of flr.models.multimodal.MultimodalNet)
 * without torch: every client starts from `global` (P floats in the
 * reference's parameters() order), runs `steps` local steps (forward, mean
 * cross-entropy, backward, clip_grad_norm_(max_norm) when max_norm > 0,
 * SGD(lr, momentum, weight_decay) re-created per client, so momentum starts at
 * the first gradient), and writes its parameters() vector to row k of X
 * (X + k*ld, ld >= P; rows k < nneg negated: the sign-flip attackers,
 * model_poisoning.py:274-276).  loss_out[k] = the mean of the client's
 * per-step losses (fl_client.py:143-149); norms_out (optional [K]) receives
 * the last step's pre-clip gradient norms.  Inputs, device, per step s:
 * images [steps][K][B][C][H][W] f32, tokens [steps][K][B][T] int64, labels
 * [steps][K][B] int64, dropout_masks NULL or [steps][K][B][fusion] f32 (the
 * inverted-dropout multipliers).  The same kernel schedule as the Python
 * trainer (flr.train.ClientBatchTrainer), so both give the same bits.  All
 * state lives in the workspace (flr_train_clients_workspace); image_size must
 * bring the trunk to a 1x1 map (32 for the four stride-2 stages).  The text
 * branch (embedding + GRU, forward and backward) and the convolutions' weight
 * gradients run on two per-device streams, forked from and joined to `stream`
 * by events inside the call (graph-capturable; created by
 * flr_train_clients_workspace, outside any capture): one training call per
 * device at a time.  FLR_TEXT_STREAM=0 / FLR_WGRAD_STREAM=0 keep that work on
 * `stream`; the results are the same bits either way. */
typedef struct flr_resnet_gru_spec {
  int64_t num_classes, image_size, in_channels;
  int64_t widths[4], blocks[4];  /* the four ResNet stages (BasicBlock) */
  int64_t vocab, seq_len, embed, hidden, fusion;
} flr_resnet_gru_spec;
int64_t flr_resnet_gru_num_params(const flr_resnet_gru_spec* spec);
size_t flr_train_clients_workspace(const flr_resnet_gru_spec* spec, int64_t K, int64_t B,
                                   int64_t steps);
int flr_train_clients(const flr_resnet_gru_spec* spec, const float* global, float* X,
                      int64_t ld, const float* images, const int64_t* tokens,
                      const int64_t* labels, const float* dropout_masks, int64_t steps,
                      int64_t K, int64_t B, float lr, float momentum, float weight_decay,
                      float max_norm, int64_t nneg, float* loss_out, float* norms_out,
                      void* workspace, size_t workspace_bytes, void* stream);
/* flags (flr_train_clients_ex):
 * FLR_TC_TRAIN_ORDER — `global` and X's rows are in TRAINING order: every
 *   tap-major conv weight (Cin, Cout multiples of 64) as [KH][KW][Cin][Cout]
 *   at its torch offset (flr_resnet_gru_reorder converts a P-vector either
 *   way).  The round engine's order (flr.round): Krum distances, row
 *   selections, coordinate-wise means and order statistics do not depend on a
 *   common coordinate permutation, so the last optimizer step writes X's rows
 *   directly (no export pass), the untrained dead-tap ranges are copied from
 *   `global`, and only the aggregated P-vector is permuted back.
 * FLR_TC_DEFER_DEAD (with FLR_TC_TRAIN_ORDER) — the dead-tap ranges are left
 *   unwritten; the caller writes them with flr_resnet_gru_fill_dead before
 *   anything reads them (the round engine: on a side stream beside the Krum
 *   chains, whose tap rewrite reads those taps from `global` itself,
 *   flr_pairwise_l2_reference_tap_dead).
 * Flag 0 is flr_train_clients. */
#define FLR_TC_TRAIN_ORDER 1u
#define FLR_TC_DEFER_DEAD 2u
int flr_train_clients_ex(const flr_resnet_gru_spec* spec, const float* global, float* X,
                         int64_t ld, const float* images, const int64_t* tokens,
                         const int64_t* labels, const float* dropout_masks, int64_t steps,
                         int64_t K, int64_t B, float lr, float momentum, float weight_decay,
                         float max_norm, int64_t nneg, float* loss_out, float* norms_out,
                         unsigned flags, void* workspace, size_t workspace_bytes, void* stream);
/* dst <- src (one P-vector) in training order (to_train = 1) or back in the
 * reference's parameters() order (0); src != dst. */
int flr_resnet_gru_reorder(const flr_resnet_gru_spec* spec, const float* src, float* dst,
                           int to_train, void* stream);
/* Parameters the optimizer updates: P minus the dead conv taps (taps that only
 * read zero padding at this image size; exact-zero gradients) when
 * weight_decay == 0, else P. */
int64_t flr_resnet_gru_live_params(const flr_resnet_gru_spec* spec, float weight_decay);
/* The dead-tap ranges of a training-order row ([off[r], off[r] + n[r]), whole
 * tap slabs of tap-major weights, ascending): their count, the first
 * min(count, cap) written (cap = 0: count only); -1 on a bad spec. */
int64_t flr_resnet_gru_dead_ranges(const flr_resnet_gru_spec* spec, float weight_decay, int64_t* off,
                                   int64_t* n, int64_t cap);
/* X's dead-tap ranges (rows 0 .. K-1, training order) <- gtrain's, rows
 * k < nneg negated: what flr_train_clients_ex writes last without
 * FLR_TC_DEFER_DEAD. */
int flr_resnet_gru_fill_dead(const flr_resnet_gru_spec* spec, float weight_decay, const float* gtrain,
                             float* X, int64_t ld, int64_t K, int64_t nneg, void* stream);

/* ---- a1 for the C4/C5 family: flr_train_vit_bert ---------------------------
 * The same client-plugin local update (run_experiments.py:193-240,
 * fl_client.py:76-149) for the ViT-S + BERT-mini late-fusion model
 * (flr.models.transformer.ViTBertNet: ViT patch embedding, class token,
 * position embedding, vit_depth pre-LN blocks, final LayerNorm; BERT word /
 * position / token-type embeddings, embedding LayerNorm, bert_depth post-LN
 * layers, tanh pooler; fc1 over [img | txt], ReLU, dropout mask, fc2), with no
 * torch: the kernel schedule of the Python trainer (flr.train.
 * ClientBatchTrainer), so both give the same bits.  Clients run in passes of
 * `chunk` clients (0: min(K, 32)); activations scale with the chunk, weights
 * (and momentum when steps > 1) with K.  Heads of width 64, <= 96 tokens per
 * sequence, widths <= 1024, B*seq_len <= 4096.  Inputs as flr_train_clients
 * (images [steps][K][B][C][S][S], tokens [steps][K][B][seq_len] int64 ids,
 * labels [steps][K][B], dropout_masks NULL or [steps][K][B][fusion]).  The
 * family has no training-layout change: X's rows are in parameters() order
 * with or without FLR_TC_TRAIN_ORDER, written by the last optimizer step.  The
 * ViT and BERT layers' weight and bias gradients run on the per-device
 * weight-gradient stream of flr_train_clients (created by
 * flr_train_vit_bert_workspace; forked and joined by events inside the call,
 * graph-capturable): one training call per device at a time;
 * FLR_WGRAD_STREAM=0 keeps them on `stream`, same bits. */
typedef struct flr_vit_bert_spec {
  int64_t num_classes, image_size, in_channels, patch;
  int64_t vit_dim, vit_depth, vit_heads, vit_mlp;
  int64_t vocab, seq_len, bert_dim, bert_depth, bert_heads, bert_ffn, bert_max_pos;
  int64_t fusion;
} flr_vit_bert_spec;
int64_t flr_vit_bert_num_params(const flr_vit_bert_spec* spec);
size_t flr_train_vit_bert_workspace(const flr_vit_bert_spec* spec, int64_t K, int64_t B, int64_t steps,
                                    int64_t chunk);
int flr_train_vit_bert(const flr_vit_bert_spec* spec, const float* global, float* X, int64_t ld,
                       const float* images, const int64_t* tokens, const int64_t* labels,
                       const float* dropout_masks, int64_t steps, int64_t K, int64_t B, float lr,
                       float momentum, float weight_decay, float max_norm, int64_t nneg, float* loss_out,
                       float* norms_out, unsigned flags, int64_t chunk, void* workspace,
                       size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FLR_H */
