// a1 — the client plugin's local update as ONE C entry: flr_train_clients.
//
// Replaces, for a batch of K clients of the C2/C3 model family (ResNet-18
// image trunk + embedding / 1-layer GRU text branch + late-fusion head), the
// per-client loop of the simulation (experiments/run_experiments.py:193-240:
// fresh model <- global, fresh SGD(lr, momentum, wd), per batch forward, mean
// cross-entropy, backward, clip_grad_norm_, step; update = parameters()) and
// FLClient.fit / _train (src/client/fl_client.py:76-149: loss = mean of the
// per-batch losses).  It is the same schedule of kernels the Python trainer
// (flr.train.ClientBatchTrainer + flr.nn's autograd functions) launches, run
// from C++ without torch: a non-torch caller (the reference's Flower client
// over ctypes / cgo / N-API) trains through the ABI alone.
//
// Training state lives in the caller's workspace (the ABI never allocates):
// per-parameter [K][n] blocks of weights, momentum and gradients in the
// training layout (tap-major [KH][KW][Cin][Cout] for the 64-multiple convs),
// every activation of a step, and the kernels' scratch.  The schedule is laid
// out once by a dry run (Net with base == nullptr) that only sums sizes.
#include "flr_common.h"
#include "side_stream.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

namespace flr {
int clip_sumsq_blocks(const float* const* g_blocks, const int64_t* numel, const int64_t* client_stride,
                      int64_t nblocks, int64_t K, double* out, int64_t out_ld, int nslots, hipStream_t st);
namespace tc {

constexpr int THREADS = 256;

// ximg[k][c][b][p] = images[k][b][c][p]: the engine's client-channel-major layout
__global__ void permute_images_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t K, int64_t B,
                                      int64_t C, int64_t HW) {
  const int64_t n = K * B * C * HW;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS) {
    const int64_t p = i % HW, r = i / HW;
    const int64_t b = r % B, r2 = r / B;
    const int64_t c = r2 % C, k = r2 / C;
    dst[i] = src[((k * B + b) * C + c) * HW + p];
  }
}

// out = a + b (one rounding: autograd's accumulation of two gradient paths)
__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out,
                           int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS)
    out[i] = __fadd_rn(a[i], b[i]);
}

// dst[t][ci][co] = src[co][ci][t]: one client's torch-order conv weight -> tap-major
__global__ void to_tap_major_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t Cout,
                                    int64_t Cin, int64_t KK) {
  const int64_t n = Cout * Cin * KK;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS) {
    const int64_t co = i % Cout, r = i / Cout;
    const int64_t ci = r % Cin, t = r / Cin;
    dst[i] = src[(co * Cin + ci) * KK + t];
  }
}

// dst[co][ci][t] = src[t][ci][co]: tap-major -> torch order (one vector)
__global__ void from_tap_major_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t Cout,
                                      int64_t Cin, int64_t KK) {
  const int64_t n = Cout * Cin * KK;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS) {
    const int64_t t = i % KK, r = i / KK;
    const int64_t ci = r % Cin, co = r / Cin;
    dst[i] = src[(t * Cin + ci) * Cout + co];
  }
}

// X's dead-tap ranges (training order) <- the global vector, every range of every
// row in ONE launch (grid: slices x K): range r = [off[r], off[r] + n[r]) of both
// g and each row; rows k < nneg negated.  g, X 16-B aligned and ld % 4 == 0 (the
// caller checks), so g + o and X + k ld + o share their alignment: a scalar head
// to the 16-B boundary, f32x4 body, scalar tail.  The body's stores are
// non-temporal (the 3.6 GB of C3 rows are not re-read before the Gram streams
// them from HBM): 926 -> 652 us per C3 round, 3.8 -> 5.5 TB/s
// (profiles/r3_dead_ranges_nt.txt; plain stores from the client matrix's SGD
// step measured no faster non-temporal).
constexpr int DEAD_MAX = 96;
struct DeadTable {
  int64_t off[DEAD_MAX];
  int64_t n[DEAD_MAX];
  int cnt;
};
__global__ __launch_bounds__(THREADS) void dead_ranges_kernel(const DeadTable t, const float* __restrict__ g,
                                                              float* __restrict__ X, int64_t ld, int nneg) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  float* d = X + (int64_t)blockIdx.y * ld;
  const float sg = (int)blockIdx.y < nneg ? -1.f : 1.f;
  const int64_t i0 = (int64_t)blockIdx.x * THREADS + threadIdx.x, stride = (int64_t)gridDim.x * THREADS;
  for (int r = 0; r < t.cnt; ++r) {
    const int64_t o = t.off[r], n = t.n[r];
    const int64_t head = std::min<int64_t>(n, (4 - (o & 3)) & 3);
    const int64_t nv = (n - head) / 4;
    if (i0 < head) d[o + i0] = g[o + i0] * sg;
    const f32x4* gs = reinterpret_cast<const f32x4*>(g + o + head);
    f32x4* ds = reinterpret_cast<f32x4*>(d + o + head);
    for (int64_t i = i0; i < nv; i += stride) __builtin_nontemporal_store(gs[i] * sg, ds + i);
    const int64_t tl = o + head + 4 * nv, nt = n - head - 4 * nv;
    if (i0 < nt) d[tl + i0] = g[tl + i0] * sg;
  }
}

inline unsigned grid_for(int64_t n) {
  const int64_t g = (n + THREADS - 1) / THREADS;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

struct Param {
  std::string name;
  std::vector<int64_t> shape;  // torch shape
  int64_t n = 0, off = 0;      // numel, offset in the torch-order vector
  bool tap = false;            // trained tap-major
  bool dead = false;           // has dead taps skipped by the optimizer (wd == 0)
  int sq_base = -1;            // fused clip-norm partial slots (tap-major convs)
  bool sq_early = false;       // its clip-norm partials taken early on the text stream (text branch, head)
  float *w = nullptr, *m = nullptr, *g = nullptr, *tmp = nullptr;
};

struct ConvOp {  // one convolution of the trunk
  int p;         // parameter index
  int64_t Cin, H, Cout, k, stride, pad, Ho;
  bool need_dx;
  void* fws = nullptr;  // the forward's workspace (generic convs: the weight gradient reuses it)
  size_t fws_n = 0;
};

struct BnOp {
  int pg, pb;  // gamma / beta parameter indices
  int64_t C, HW;
  float *mean = nullptr, *invstd = nullptr;
};

struct Block {
  ConvOp c1, c2, ds;
  BnOp b1, b2, bds;
  bool has_ds;
  // activations: conv outputs, BN outputs; gradients
  float *x_in, *y1, *a1, *y2, *out, *yd, *ad;
  float *d_y2, *d_a1, *d_y1, *d_xm, *d_res, *d_yd, *d_xd, *d_in;
  int64_t in_elems, out_elems;
};

class Net {
 public:
  Net(const flr_resnet_gru_spec& s, int64_t K, int64_t B, float wd, float clip, char* base)
      : s_(s), K_(K), B_(B), base_(base), wd_(wd), clip_(clip) {}

  int layout() {  // parameters, their blocks, every buffer; returns FLR_OK or a status
    const auto& s = s_;
    if (s.image_size < 1 || s.in_channels < 1 || s.num_classes < 1 || s.vocab < 1 || s.seq_len < 1 || s.embed < 1 ||
        s.hidden < 1 || s.fusion < 1 || K_ < 1 || B_ < 1)
      return FLR_ERR_ARG;
    for (int i = 0; i < 4; ++i)
      if (s.widths[i] < 1 || s.blocks[i] < 1) return FLR_ERR_ARG;
    T_ = s.seq_len;
    H_ = s.hidden;
    E_ = s.embed;
    F_ = s.fusion;
    C_ = s.num_classes;
    const int64_t w0 = s.widths[0];
    // ---- parameters() order of MultimodalNet (flr.models.multimodal) ----
    int pc1 = add_param("conv1.weight", {w0, s.in_channels, 7, 7});
    int pbw = add_param("bn1.weight", {w0}), pbb = add_param("bn1.bias", {w0});
    int64_t H = s.image_size;
    stem_ = ConvOp{pc1, s.in_channels, H, w0, 7, 2, 3, (H + 6 - 7) / 2 + 1, false};
    Hs_ = stem_.Ho;
    stem_bn_ = BnOp{pbw, pbb, w0, B_ * Hs_ * Hs_};
    Hp_ = (Hs_ + 2 - 3) / 2 + 1;  // the 3x3/2/1 max pool
    // the fused stem BN + ReLU + pool kernels' shapes (FLR_STEM_FUSED=0: the three-kernel form)
    {
      const char* e = flr::knob("FLR_STEM_FUSED");
      stem_fused_ = !(e && e[0] == '0') && Hs_ == 16 && (B_ == 16 || B_ == 32);
    }
    int64_t cin = w0, Hc = Hp_;
    for (int li = 0; li < 4; ++li) {
      const int64_t cout = s.widths[li];
      for (int b = 0; b < s.blocks[li]; ++b) {
        const int64_t st = (b == 0 && li > 0) ? 2 : 1;
        const std::string pre = "layers." + std::to_string(li) + "." + std::to_string(b) + ".";
        Block bk{};
        const int64_t Ho = (Hc + 2 - 3) / st + 1;
        bk.c1 = ConvOp{add_param(pre + "conv1.weight", {cout, cin, 3, 3}), cin, Hc, cout, 3, st, 1, Ho, true};
        bk.b1 = BnOp{add_param(pre + "bn1.weight", {cout}), add_param(pre + "bn1.bias", {cout}), cout, B_ * Ho * Ho};
        bk.c2 = ConvOp{add_param(pre + "conv2.weight", {cout, cout, 3, 3}), cout, Ho, cout, 3, 1, 1, Ho, true};
        bk.b2 = BnOp{add_param(pre + "bn2.weight", {cout}), add_param(pre + "bn2.bias", {cout}), cout, B_ * Ho * Ho};
        bk.has_ds = st != 1 || cin != cout;
        if (bk.has_ds) {
          bk.ds = ConvOp{add_param(pre + "downsample.0.weight", {cout, cin, 1, 1}), cin, Hc, cout, 1, st, 0,
                         (Hc - 1) / st + 1, true};
          bk.bds = BnOp{add_param(pre + "downsample.1.weight", {cout}), add_param(pre + "downsample.1.bias", {cout}),
                        cout, B_ * Ho * Ho};
        }
        bk.in_elems = K_ * cin * B_ * Hc * Hc;
        bk.out_elems = K_ * cout * B_ * Ho * Ho;
        blocks_.push_back(bk);
        cin = cout;
        Hc = Ho;
      }
    }
    if (Hc != 1) return FLR_ERR_UNSUPPORTED;  // global average pooling is the 1x1 map (32x32 inputs)
    Dimg_ = cin;
    p_emb_ = add_param("embedding.weight", {s.vocab, E_});
    p_wih_ = add_param("gru.weight_ih_l0", {3 * H_, E_});
    p_whh_ = add_param("gru.weight_hh_l0", {3 * H_, H_});
    p_bih_ = add_param("gru.bias_ih_l0", {3 * H_});
    p_bhh_ = add_param("gru.bias_hh_l0", {3 * H_});
    p_w1_ = add_param("fc1.weight", {F_, Dimg_ + H_});
    p_b1_ = add_param("fc1.bias", {F_});
    p_w2_ = add_param("fc2.weight", {C_, F_});
    p_b2_ = add_param("fc2.bias", {C_});
    P_ = 0;
    for (auto& p : ps_) {
      p.off = P_;
      P_ += p.n;
    }
    // forward segments and the parameters each needs first (side-stream optimizer
    // groups, side_stream.h): the stem, every residual block, the text branch, the head
    gthr_.clear();
    gthr_.push_back(std::max({pc1, pbw, pbb}) + 1);
    for (const auto& bk : blocks_) {
      int m = std::max({bk.c1.p, bk.b1.pg, bk.b1.pb, bk.c2.p, bk.b2.pg, bk.b2.pb});
      if (bk.has_ds) m = std::max({m, bk.ds.p, bk.bds.pg, bk.bds.pb});
      gthr_.push_back(std::max(m + 1, gthr_.back()));
    }
    gthr_.push_back(std::max({p_emb_, p_wih_, p_whh_, p_bih_, p_bhh_}) + 1);
    gthr_.push_back((int)ps_.size());
    gtext_ = (int)gthr_.size() - 2;
    ghead_ = (int)gthr_.size() - 1;
    gorder_.assign(1, gtext_);
    for (int g = 0; g < gtext_; ++g) gorder_.push_back(g);
    gorder_.push_back(ghead_);
    // tap-major convs and their dead taps (flr.train.ClientBatchTrainer)
    mark_conv(stem_);
    for (auto& bk : blocks_) {
      mark_conv(bk.c1);
      mark_conv(bk.c2);
      if (bk.has_ds) mark_conv(bk.ds);
    }
    // ---- training state ----
    for (auto& p : ps_) {
      p.w = alloc<float>(K_ * p.n);
      p.m = alloc<float>(K_ * p.n);
      p.g = alloc<float>(K_ * p.n);
      if (p.tap) p.tmp = alloc<float>(p.n);  // one client's weight, permuted once per load
    }
    // optimizer blocks: whole parameters, the live-tap runs of dead-tap convs
    for (size_t j = 0; j < ps_.size(); ++j) {
      Param& p = ps_[j];
      if (!p.dead) {
        add_block((int)j, 0, p.n, p.n);
        continue;
      }
      const int64_t slab = p.shape[0] * p.shape[1];
      const std::vector<int> live = live_taps(p);
      int t0 = live[0];
      for (size_t i = 0; i < live.size(); ++i) {
        const bool end = i + 1 == live.size() || live[i + 1] != live[i] + 1;
        if (end) {
          add_block((int)j, t0 * slab, (live[i] + 1 - t0) * slab, p.n);
          if (i + 1 < live.size()) t0 = live[i + 1];
        }
      }
    }
    // fused clip-norm partial slots, in parameter order
    nsq_ = 0;
    if (clip_ > 0)
      for (auto& p : ps_) {
        if (!p.tap) continue;
        const ConvOp* c = conv_of(p);
        const int64_t n = flr_conv2d_bwd_weight_t_sq_slots(K_, B_, c->Cin, c->H, c->H, c->Cout, c->k, c->k, c->stride,
                                                           c->pad);
        if (n < 0) return FLR_ERR_UNSUPPORTED;
        p.sq_base = (int)nsq_;
        nsq_ += n;
      }
    // the text branch's and the head's partials: their gradients are final once
    // the text backward ends, long before the trunk's, so their sum of squares
    // runs on the text stream there (clip_sumsq_blocks) instead of in the
    // optimizer's pass at the end of the backward; kEarlySlots slots after the convs'
    sq_early_base_ = -1;
    if (clip_ > 0) {
      sq_early_base_ = nsq_;
      nsq_ += kEarlySlots;
      for (int j : {p_emb_, p_wih_, p_whh_, p_bih_, p_bhh_, p_w1_, p_b1_, p_w2_, p_b2_}) ps_[j].sq_early = true;
    }
    sq_ = alloc<double>(K_ * std::max<int64_t>(1, nsq_));
    sgd_ws_n_ = flr_clip_sgd_workspace(K_);
    sgd_ws_ = alloc<char>(sgd_ws_n_);
    // ---- activations of one step ----
    const int64_t C0 = s.in_channels, HW0 = s.image_size * s.image_size;
    ximg_ = alloc<float>(K_ * C0 * B_ * HW0);
    const int64_t stem_el = K_ * w0 * B_ * Hs_ * Hs_;
    y0_ = alloc<float>(stem_el);
    a0_ = alloc<float>(stem_el);
    d_a0_ = alloc<float>(stem_el);
    d_y0_ = alloc<float>(stem_el);
    bn_stats(stem_bn_);
    const int64_t pool_el = K_ * w0 * B_ * Hp_ * Hp_;
    p0_ = alloc<float>(pool_el);
    d_p0_ = alloc<float>(pool_el);
    arg0_ = alloc<uint8_t>(pool_el);
    stem_.fws_n = flr_conv2d_workspace(K_, B_, C0, s.image_size, s.image_size, w0, 7, 7, 2, 3);
    stem_.fws = alloc<char>(stem_.fws_n);
    float* x = p0_;
    float* dx = d_p0_;
    for (auto& bk : blocks_) {
      bk.x_in = x;
      bk.d_in = dx;
      const int64_t oe = bk.out_elems;
      bk.y1 = alloc<float>(oe);
      bk.a1 = alloc<float>(oe);
      bk.y2 = alloc<float>(oe);
      bk.out = alloc<float>(oe);
      bk.d_y2 = alloc<float>(oe);
      bk.d_a1 = alloc<float>(oe);
      bk.d_y1 = alloc<float>(oe);
      bk.d_xm = alloc<float>(bk.in_elems);
      bk.d_res = alloc<float>(oe);
      bn_stats(bk.b1);
      bn_stats(bk.b2);
      if (bk.has_ds) {
        bk.yd = alloc<float>(oe);
        bk.ad = alloc<float>(oe);
        bk.d_yd = alloc<float>(oe);
        bk.d_xd = alloc<float>(bk.in_elems);
        bn_stats(bk.bds);
      }
      conv_ws(bk.c1);
      conv_ws(bk.c2);
      if (bk.has_ds) conv_ws(bk.ds);
      x = bk.out;
      dx = alloc<float>(oe);  // the gradient at this block's output (the next block's d_in)
    }
    d_x4_ = dx;  // dL/d(trunk output), [K][Dimg][B] (the 1x1 map)
    // text branch + head
    const int64_t N = B_ * T_;
    emb_ = alloc<float>(K_ * N * E_);
    gi_ = alloc<float>(K_ * N * 3 * H_);
    hseq_ = alloc<float>(K_ * (T_ + 1) * B_ * H_);
    gates_ = alloc<float>(K_ * T_ * B_ * 4 * H_);
    gh_ = alloc<float>(K_ * B_ * 3 * H_);
    whhP_ = alloc<float>(K_ * packed(3, H_, H_));
    whhT_ = alloc<float>(K_ * packed(1, H_, 3 * H_));
    h1_ = alloc<float>(K_ * B_ * F_);
    logits_ = alloc<float>(K_ * B_ * C_);
    dlogits_ = alloc<float>(K_ * B_ * C_);
    rows_ = alloc<float>(K_ * B_);
    loss_ = alloc<float>(K_);
    dpre_ = alloc<float>(K_ * B_ * F_);
    dh_ = alloc<float>(K_ * B_ * H_);
    dh2_ = alloc<float>(K_ * B_ * H_);
    dh_direct_ = alloc<float>(K_ * B_ * H_);
    dgh_ = alloc<float>(K_ * T_ * B_ * 3 * H_);
    dgi_ = alloc<float>(K_ * N * 3 * H_);
    demb_ = alloc<float>(K_ * N * E_);
    // scratch shared by the GEMMs / row sums / embedding backward (stream-ordered)
    size_t gw = 0;
    auto gmax = [&](int64_t M, int64_t Nn, int64_t R) { gw = std::max(gw, flr_bgemm_workspace(K_, M, Nn, R)); };
    gmax(N, 3 * H_, E_);                         // gi
    gmax(B_, 3 * H_, H_);                        // gh (unfused GRU)
    gmax(B_, F_, Dimg_);  gmax(B_, F_, H_);      // fc1
    gmax(B_, C_, F_);                            // fc2
    gmax(B_, F_, C_);  gmax(C_, F_, B_);         // head backward
    gmax(B_, Dimg_, F_);  gmax(F_, Dimg_, B_);
    gmax(B_, H_, F_);  gmax(F_, H_, B_);
    gmax(B_, H_, 3 * H_);                        // unfused GRU backward
    gmax(3 * H_, H_, T_ * B_);                   // dW_hh
    gmax(N, E_, 3 * H_);  gmax(3 * H_, E_, N);   // W_ih backward
    gws_n_ = gw;
    gws_ = alloc<char>(gws_n_);
    size_t rw = 0;
    for (int64_t M : {B_, T_ * B_, N}) rw = std::max(rw, flr_sum_rows_workspace(K_, M, std::max({F_, C_, 3 * H_})));
    rws_n_ = rw;
    rws_ = alloc<char>(rws_n_);
    ews_n_ = flr_embedding_bwd_workspace(K_, N);
    ews_ = alloc<char>(ews_n_);
    cws_ = alloc<char>(cws_n_);  // the largest convolution workspace (conv_ws)
    cws2_ = alloc<char>(cws_n_);  // the weight-gradient stream's own (split-K partials)
    cws3_ = alloc<char>(cws_n_);  // the text stream's, for the trunk's last weight gradients
    if (N > 4096) return FLR_ERR_UNSUPPORTED;
    return FLR_OK;
  }

  size_t bytes() const { return off_; }
  int64_t P() const { return P_; }

  // ---- the run ---------------------------------------------------------------
  int load_global(const float* global, hipStream_t st) {
    int rc;
    for (auto& p : ps_) {
      const float* src = global + p.off;
      if (p.tap) {
        const int64_t KK = p.shape[2] * p.shape[3];
        hipLaunchKernelGGL(to_tap_major_kernel, dim3(grid_for(p.n)), dim3(THREADS), 0, st, src, p.tmp, p.shape[0],
                           p.shape[1], KK);
        if ((rc = launch_status("train_clients: to tap-major")) != FLR_OK) return rc;
        src = p.tmp;
      }
      if ((rc = flr_broadcast_rows(src, p.n, p.w, K_, p.n, st)) != FLR_OK) return rc;
    }
    return FLR_OK;
  }

  // Training order (flr.train.ClientBatchTrainer.to_train_order): the P-vector
  // with every tap-major conv weight in its training layout [KH][KW][Cin][Cout]
  // at its torch offset.  load_global_train broadcasts only what the kernels
  // read (the dead-tap slabs stay out of the training state).
  int load_global_train(const float* gtrain, hipStream_t st) {
    int rc;
    gshared_ = shared_first_ ? gtrain : nullptr;
    for (const auto& b : blocks_opt_) {
      const Param& p = ps_[b.j];
      if (gshared_ && p.tap) continue;  // the first step reads the one copy in gtrain
      if ((rc = flr_broadcast_rows(gtrain + p.off + b.o, b.n, p.w + b.o, K_, b.cs, st)) != FLR_OK) return rc;
    }
    return FLR_OK;
  }

  // src (one P-vector) -> dst in the other order; to_train: torch -> training
  int reorder(const float* src, float* dst, bool to_train, hipStream_t st) {
    int rc;
    int64_t run0 = 0, run1 = 0;  // a run of consecutive plain parameters: one copy
    auto flush = [&]() {
      const int r = run1 > run0 ? flr_copy_rows(src + run0, run1 - run0, run1 - run0, dst + run0, run1 - run0, 1, st)
                                : (int)FLR_OK;
      run0 = run1;
      return r;
    };
    for (const auto& p : ps_) {
      if (!p.tap) {
        if (run1 != p.off && (rc = flush()) != FLR_OK) return rc;
        if (run1 == run0) run0 = run1 = p.off;
        run1 = p.off + p.n;
        continue;
      }
      if ((rc = flush()) != FLR_OK) return rc;
      run0 = run1 = p.off + p.n;
      {
        const int64_t KK = p.shape[2] * p.shape[3];
        if (to_train)
          hipLaunchKernelGGL(to_tap_major_kernel, dim3(grid_for(p.n)), dim3(THREADS), 0, st, src + p.off,
                             dst + p.off, p.shape[0], p.shape[1], KK);
        else
          hipLaunchKernelGGL(from_tap_major_kernel, dim3(grid_for(p.n)), dim3(THREADS), 0, st, src + p.off,
                             dst + p.off, p.shape[0], p.shape[1], KK);
        if ((rc = launch_status("train_clients: reorder")) != FLR_OK) return rc;
      }
    }
    return flush();
  }

  // the dead-tap ranges of a training-order row, ascending (dead_ranges' table)
  void dead_list(std::vector<std::pair<int64_t, int64_t>>& out) const {
    for (size_t j = 0; j < ps_.size(); ++j) {
      const Param& p = ps_[j];
      if (!p.dead) continue;
      int64_t e = 0;
      for (const auto& b : blocks_opt_) {
        if (b.j != (int)j) continue;
        if (b.o > e) out.push_back({p.off + e, b.o - e});
        e = b.o + b.n;
      }
      if (p.n > e) out.push_back({p.off + e, p.n - e});
    }
  }

  // X's dead-tap ranges (training order) <- gtrain, rows k < nneg negated: one
  // launch over the range table when it fits and the rows are 16-B aligned
  // (was one broadcast per range: 57 launches per C3 round), else per range.
  int dead_ranges(const float* gtrain, float* X, int64_t ld, int64_t nneg, hipStream_t st, int64_t gx = 0) {
    int rc;
    DeadTable t;
    t.cnt = 0;
    int64_t total = 0;
    bool fits = (reinterpret_cast<uintptr_t>(gtrain) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
                ld % 4 == 0 && K_ <= 65535;
    for (size_t j = 0; j < ps_.size() && fits; ++j) {
      const Param& p = ps_[j];
      if (!p.dead) continue;
      int64_t e = 0;
      auto add = [&](int64_t a) {
        if (a <= e) return;
        if (t.cnt == DEAD_MAX) { fits = false; return; }
        t.off[t.cnt] = p.off + e;
        t.n[t.cnt++] = a - e;
        total = std::max(total, a - e);
      };
      for (const auto& b : blocks_opt_) {
        if (b.j != (int)j) continue;
        add(b.o);
        e = b.o + b.n;
      }
      add(p.n);
    }
    if (fits) {
      if (t.cnt == 0) return FLR_OK;
      // gx > 0: that many workgroups per row (a fill beside other kernels, throttled)
      const int64_t g = gx > 0 ? gx : std::max<int64_t>(1, std::min<int64_t>(256, (total / 4 + THREADS - 1) / THREADS));
      hipLaunchKernelGGL(dead_ranges_kernel, dim3((unsigned)g, (unsigned)K_), dim3(THREADS), 0, st, t, gtrain, X, ld,
                         (int)std::min<int64_t>(nneg, K_));
      return launch_status("train_clients: dead ranges");
    }
    for (size_t j = 0; j < ps_.size(); ++j) {
      const Param& p = ps_[j];
      if (!p.dead) continue;
      int64_t e = 0;
      auto fill = [&](int64_t a) {
        if (a > e && (rc = flr_broadcast_rows_neg(gtrain + p.off + e, a - e, X + p.off + e, K_, ld, nneg, st)) !=
                         FLR_OK)
          return rc;
        return (int)FLR_OK;
      };
      for (const auto& b : blocks_opt_) {
        if (b.j != (int)j) continue;
        if ((rc = fill(b.o)) != FLR_OK) return rc;
        e = b.o + b.n;
      }
      if ((rc = fill(p.n)) != FLR_OK) return rc;
    }
    return FLR_OK;
  }

  // training order: the first step's tap-major conv weights are gshared_ (the
  // global vector, one copy for every client; FLR_SHARED_FIRST=0: broadcast)
  bool shared_first_ = true;
  const float* gshared_ = nullptr;
  bool first_ = false;
  // the last step writes X's rows (training order) instead of the weights
  float* xout_ = nullptr;
  int64_t xld_ = 0, xneg_ = 0;

  int step(const float* images, const int64_t* tokens, const int64_t* labels, const float* mask, bool first,
           bool last, float* loss_row, float lr, float mom, hipStream_t st) {
    int rc;
#define FLR_TRY(x) \
  if ((rc = (x)) != FLR_OK) return rc
    const auto& s = s_;
    const int64_t C0 = s.in_channels, HW0 = s.image_size * s.image_size, N = B_ * T_;
    first_ = first;
    // ---------------- forward ----------------
    hipLaunchKernelGGL(permute_images_kernel, dim3(grid_for(K_ * B_ * C0 * HW0)), dim3(THREADS), 0, st, images,
                       ximg_, K_, B_, C0, HW0);
    FLR_TRY(launch_status("train_clients: images"));
    // the text branch first: its recurrence is latency-bound, so the previous step's
    // side-stream update of the trunk (HBM-bound) runs under it (side_stream.h)
    const Param &emb = ps_[p_emb_], &wih = ps_[p_wih_], &whh = ps_[p_whh_], &bih = ps_[p_bih_],
                &bhh = ps_[p_bhh_], &w1 = ps_[p_w1_], &b1 = ps_[p_b1_], &w2 = ps_[p_w2_], &b2 = ps_[p_b2_];
    // the text branch on its own stream beside the trunk (text_stream, side_stream.h);
    // its workspaces (gws_, rws_, ews_) are not used by the trunk
    const bool conc = text_ != nullptr;
    const hipStream_t ts = conc ? text_->s : st;
    if (conc) FLR_TRY(fork(st, ts, 0));
    FLR_TRY(wait_group(gtext_, ts));
    FLR_TRY(flr_embedding_fwd(emb.w, s.vocab * E_, s.vocab, tokens, N, nullptr, 0, 0, nullptr, 0, nullptr, 0, 0,
                              nullptr, 0, K_, N, E_, emb_, ts));
    const int64_t H3 = 3 * H_;
    FLR_TRY(gemm(emb_, N * E_, E_, 1, wih.w, H3 * E_, E_, 1, gi_, N * H3, H3, 1, bih.w, H3, nullptr, N, H3, E_, ts));
    const bool fused = B_ <= 32;
    // first step in training order: one packed copy of the global W_hh for every client
    const bool wsh = first_ && gshared_ != nullptr;
    if (fused) {
      FLR_TRY(flr_fill(hseq_, K_ * (T_ + 1) * B_ * H_, 0.f, ts));
      FLR_TRY(flr_gru_pack(wsh ? gshared_ + whh.off : whh.w, wsh ? 1 : K_, 3, H_, H_, 0, whhP_, ts));
      for (int64_t t = 0; t < T_; ++t)
        FLR_TRY(flr_gru_fwd_fused_ex(gi_, whhP_, wsh ? 1 : 0, bhh.w, hseq_, gates_, K_, B_, T_, H_, t, ts));
    } else {
      FLR_TRY(flr_fill(hseq_, K_ * (T_ + 1) * B_ * H_, 0.f, ts));
      for (int64_t t = 0; t < T_; ++t) {
        FLR_TRY(gemm(hseq_ + t * B_ * H_, (T_ + 1) * B_ * H_, H_, 1, whh.w, H3 * H_, H_, 1, gh_, B_ * H3, H3, 1,
                     bhh.w, H3, nullptr, B_, H3, H_, ts));
        FLR_TRY(flr_gru_fwd_step(gi_, gh_, hseq_, gates_, K_, B_, T_, H_, t, ts));
      }
    }
    if (conc) FLR_TRY(fork(ts, st, 1));  // joined before the head (event recorded here, waited there)
    int seg = 0;  // the previous step's update of each trunk segment's parameters (side stream)
    FLR_TRY(wait_group(seg++, st));
    FLR_TRY(conv_fwd(stem_, ximg_, y0_, st));
    if (stem_fused_) {  // bn1 + relu + maxpool in one pass: the BN output never reaches HBM
      FLR_TRY(flr_batchnorm_relu_maxpool_fwd(y0_, ps_[stem_bn_.pg].w, ps_[stem_bn_.pb].w, p0_, arg0_, stem_bn_.mean,
                                             stem_bn_.invstd, K_ * s.widths[0], B_, Hs_, Hs_, 1e-5f, st));
    } else {
      FLR_TRY(bn_fwd(stem_bn_, y0_, nullptr, a0_, true, st));
      FLR_TRY(flr_maxpool2d_fwd(a0_, p0_, arg0_, K_ * s.widths[0] * B_, Hs_, Hs_, 3, 3, 2, 1, st));
    }
    // a block's shortcut (strided 1x1 conv + BN) on the weight-gradient stream, idle in
    // the forward, beside conv1 / bn1 / conv2; joined before bn2 adds it
    int fev = 0;
    for (auto& bk : blocks_) {
      const float* idt = bk.x_in;
      FLR_TRY(wait_group(seg++, st));
      const bool ds_side = bk.has_ds && wgs_ && fev + 2 <= WgradStream::NEV;
      if (bk.has_ds) {
        const hipStream_t dst = ds_side ? wgs_->s : st;
        if (ds_side && (hipEventRecord(wgs_->ev[fev], st) != hipSuccess ||
                        hipStreamWaitEvent(dst, wgs_->ev[fev], 0) != hipSuccess))
          return launch_status("train_clients: shortcut fork");
        FLR_TRY(conv_fwd(bk.ds, bk.x_in, bk.yd, dst, ds_side ? cws2_ : nullptr));
        FLR_TRY(bn_fwd(bk.bds, bk.yd, nullptr, bk.ad, false, dst));
        if (ds_side && hipEventRecord(wgs_->ev[fev + 1], dst) != hipSuccess)
          return launch_status("train_clients: shortcut event");
        idt = bk.ad;
      }
      FLR_TRY(conv_fwd(bk.c1, bk.x_in, bk.y1, st));
      FLR_TRY(bn_fwd(bk.b1, bk.y1, nullptr, bk.a1, true, st));
      FLR_TRY(conv_fwd(bk.c2, bk.a1, bk.y2, st));
      if (ds_side) {
        if (hipStreamWaitEvent(st, wgs_->ev[fev + 1], 0) != hipSuccess)
          return launch_status("train_clients: shortcut join");
        fev += 2;
      }
      FLR_TRY(bn_fwd(bk.b2, bk.y2, idt, bk.out, true, st));
    }
    const float* x4 = blocks_.back().out;  // [K][Dimg][B]: img[k][b][c] = x4[k][c][b]
    const float* hT = hseq_ + T_ * B_ * H_;  // [K][B][H] at client stride (T+1)*B*H
    const int64_t hk = (T_ + 1) * B_ * H_, DI = Dimg_ + H_;
    // fc1 over the column blocks [img | h] (never concatenated), ReLU + dropout mask in the epilogue
    if (conc && hipStreamWaitEvent(st, text_->ev[1], 0) != hipSuccess)
      return launch_status("train_clients: text-stream join");
    FLR_TRY(wait_group(ghead_, st));
    pending_ = false;  // every side-stream update of the previous step is joined
    FLR_TRY(flr_bgemm_ex(x4, Dimg_ * B_, 1, B_, w1.w, F_ * DI, DI, 1, h1_, B_ * F_, F_, 1, b1.w, F_, nullptr,
                         FLR_ACT_NONE, nullptr, nullptr, nullptr, K_, B_, F_, Dimg_, gws_, gws_n_, st));
    FLR_TRY(flr_bgemm_ex(hT, hk, H_, 1, w1.w + Dimg_, F_ * DI, DI, 1, h1_, B_ * F_, F_, 1, nullptr, 0, h1_,
                         FLR_ACT_RELU, mask, nullptr, nullptr, K_, B_, F_, H_, gws_, gws_n_, st));
    FLR_TRY(gemm(h1_, B_ * F_, F_, 1, w2.w, C_ * F_, F_, 1, logits_, B_ * C_, C_, 1, b2.w, C_, nullptr, B_, C_, F_,
                 st));
    FLR_TRY(flr_cross_entropy(logits_, labels, K_, B_, C_, loss_, dlogits_, rows_, st));
    FLR_TRY(flr_copy_rows(loss_, K_, K_, loss_row, K_, 1, st));
    // ---------------- backward ----------------
    // the weight-gradient stream: forks from here on (every side-stream update of
    // the previous step was joined before the head, so no update still reads p.g)
    WgradStream* wgs_save = wgs_;
    wev_ = 0;
    // head (ClientMLP.backward): dpre = dlogits W2 * relu'(h1) * mask
    FLR_TRY(flr_bgemm_ex(dlogits_, B_ * C_, C_, 1, w2.w, C_ * F_, 1, F_, dpre_, B_ * F_, F_, 1, nullptr, 0, nullptr,
                         FLR_ACT_DRELU, mask, h1_, nullptr, K_, B_, F_, C_, gws_, gws_n_, st));
    FLR_TRY(gemm(dlogits_, B_ * C_, 1, C_, h1_, B_ * F_, 1, F_, w2.g, C_ * F_, F_, 1, nullptr, 0, nullptr, C_, F_, B_,
                 st));
    FLR_TRY(rowsum(dlogits_, B_ * C_, C_, B_, C_, b2.g, st));
    // image column block: dL/d(trunk output) written straight into its [K][Dimg][B] layout
    FLR_TRY(gemm(dpre_, B_ * F_, F_, 1, w1.w, F_ * DI, 1, DI, d_x4_, Dimg_ * B_, 1, B_, nullptr, 0, nullptr, B_, Dimg_,
                 F_, st));
    FLR_TRY(gemm(dpre_, B_ * F_, 1, F_, x4, Dimg_ * B_, B_, 1, w1.g, F_ * DI, DI, 1, nullptr, 0, nullptr, F_, Dimg_, B_,
                 st));
    FLR_TRY(gemm(dpre_, B_ * F_, F_, 1, w1.w + Dimg_, F_ * DI, 1, DI, dh_, B_ * H_, H_, 1, nullptr, 0, nullptr, B_, H_,
                 F_, st));
    FLR_TRY(gemm(dpre_, B_ * F_, 1, F_, hT, hk, 1, H_, w1.g + Dimg_, F_ * DI, DI, 1, nullptr, 0, nullptr, F_, H_, B_,
                 st));
    FLR_TRY(rowsum(dpre_, B_ * F_, F_, B_, F_, b1.g, st));
    if (conc) FLR_TRY(fork(st, ts, 2));
    // GRU (ClientGRU.backward)
    if (fused) {
      FLR_TRY(flr_gru_pack(wsh ? gshared_ + whh.off : whh.w, wsh ? 1 : K_, 1, H_, H3, 1, whhT_, ts));
      FLR_TRY(flr_gru_bwd_step(dh_, gates_, hseq_, dgh_, dgi_, dh_direct_, K_, B_, T_, H_, T_ - 1, ts));
      for (int64_t t = T_ - 1; t > 0; --t)
        FLR_TRY(flr_gru_bwd_fused_ex(whhT_, wsh ? 1 : 0, gates_, hseq_, dgh_, dgi_, dh_direct_, nullptr, K_, B_, T_,
                                     H_, t, ts));
    } else {
      const float* dh = dh_;
      for (int64_t t = T_ - 1; t >= 0; --t) {
        FLR_TRY(flr_gru_bwd_step(dh, gates_, hseq_, dgh_, dgi_, dh_direct_, K_, B_, T_, H_, t, ts));
        if (t > 0) {
          float* out = dh == dh2_ ? dh_ : dh2_;
          FLR_TRY(gemm(dgh_ + t * B_ * H3, T_ * B_ * H3, H3, 1, whh.w, H3 * H_, 1, H_, out, B_ * H_, H_, 1, nullptr,
                       0, dh_direct_, B_, H_, H3, ts));
          dh = out;
        }
      }
    }
    FLR_TRY(gemm(dgh_, T_ * B_ * H3, 1, H3, hseq_, hk, 1, H_, whh.g, H3 * H_, H_, 1, nullptr, 0, nullptr, H3, H_,
                 T_ * B_, ts));
    FLR_TRY(rowsum(dgh_, T_ * B_ * H3, H3, T_ * B_, H3, bhh.g, ts));
    // W_ih (ClientLinear.backward), then the embedding
    FLR_TRY(gemm(dgi_, N * H3, H3, 1, wih.w, H3 * E_, 1, E_, demb_, N * E_, E_, 1, nullptr, 0, nullptr, N, E_, H3, ts));
    FLR_TRY(gemm(dgi_, N * H3, 1, H3, emb_, N * E_, 1, E_, wih.g, H3 * E_, E_, 1, nullptr, 0, nullptr, H3, E_, N, ts));
    FLR_TRY(rowsum(dgi_, N * H3, H3, N, H3, bih.g, ts));
    FLR_TRY(flr_embedding_bwd(demb_, tokens, N, K_, N, s.vocab, E_, emb.g, s.vocab * E_, 1, ews_, ews_n_, ts));
    if (sq_early_base_ >= 0) FLR_TRY(early_sumsq(ts));  // the head's gradients: on st before fork 2
    if (conc) FLR_TRY(fork(ts, st, 3));
    // trunk, last block first.  The first blocks' weight gradients come last,
    // behind the weight-gradient stream's backlog, when the text stream has long
    // been idle: they run there instead (FLR_WG_TEXT blocks; 0: off)
    const int wg_text = conc ? [] {
      const char* e = flr::knob("FLR_WG_TEXT");
      return e ? atoi(e) : 2;
    }() : 0;
    tev_ = 4;
    for (int bi = (int)blocks_.size() - 1; bi >= 0; --bi) {
      Block& bk = blocks_[bi];
      wg_on_text_ = bi < wg_text;
      const float* d_out = bi + 1 < (int)blocks_.size() ? blocks_[bi + 1].d_in : d_x4_;
      FLR_TRY(bn_bwd(bk.b2, d_out, bk.y2, bk.out, true, bk.d_y2, bk.d_res, st));
      FLR_TRY(conv_bwd(bk.c2, bk.a1, bk.d_y2, bk.d_a1, st));
      FLR_TRY(bn_bwd(bk.b1, bk.d_a1, bk.y1, bk.a1, true, bk.d_y1, nullptr, st));
      const float* other = bk.d_res;  // identity shortcut: the residual gradient itself
      if (bk.has_ds) {
        FLR_TRY(bn_bwd(bk.bds, bk.d_res, bk.yd, nullptr, false, bk.d_yd, nullptr, st));
        if (ps_[bk.c1.p].tap && ps_[bk.ds.p].tap && fuse_res_) {
          // d_in = dgrad(c1), then the strided 1x1 shortcut's dgrad added in place
          // (its epilogue: dx = dgrad(ds) + dx, the same one fp32 add); the parity
          // classes no shortcut tap reaches are skipped instead of written as zeros
          FLR_TRY(conv_bwd(bk.c1, bk.x_in, bk.d_y1, bk.d_in, st));
          FLR_TRY(conv_bwd(bk.ds, bk.x_in, bk.d_yd, bk.d_in, st, bk.d_in));
          continue;
        }
        FLR_TRY(conv_bwd(bk.ds, bk.x_in, bk.d_yd, bk.d_xd, st));
        other = bk.d_xd;
      }
      // d_in = dgrad(c1) + other: the two paths' sum (autograd's accumulation),
      // in the dgrad epilogue when c1 is tap-major, else one extra pass
      if (ps_[bk.c1.p].tap && fuse_res_) {
        FLR_TRY(conv_bwd(bk.c1, bk.x_in, bk.d_y1, bk.d_in, st, other));
      } else {
        FLR_TRY(conv_bwd(bk.c1, bk.x_in, bk.d_y1, bk.d_xm, st));
        hipLaunchKernelGGL(add_kernel, dim3(grid_for(bk.in_elems)), dim3(THREADS), 0, st, bk.d_xm, other, bk.d_in,
                           bk.in_elems);
        FLR_TRY(launch_status("train_clients: gradient sum"));
      }
    }
    if (stem_fused_) {
      FLR_TRY(flr_maxpool_relu_batchnorm_bwd(d_p0_, arg0_, y0_, ps_[stem_bn_.pg].w, ps_[stem_bn_.pb].w, stem_bn_.mean,
                                             stem_bn_.invstd, d_y0_, ps_[stem_bn_.pg].g, ps_[stem_bn_.pb].g,
                                             K_ * s.widths[0], B_, Hs_, Hs_, st));
    } else {
      FLR_TRY(flr_maxpool2d_bwd(d_p0_, arg0_, d_a0_, K_ * s.widths[0] * B_, Hs_, Hs_, 3, 3, 2, 1, st));
      FLR_TRY(bn_bwd(stem_bn_, d_a0_, y0_, a0_, true, d_y0_, nullptr, st));
    }
    wg_on_text_ = false;
    FLR_TRY(conv_bwd(stem_, ximg_, d_y0_, nullptr, st));
    if (conc && hipStreamWaitEvent(st, text_->ev[3], 0) != hipSuccess)
      return launch_status("train_clients: text-stream join");
    if (conc && tev_ > 4) {  // the weight gradients run on the text stream
      if (hipEventRecord(text_->ev[TextStream::NEV - 1], text_->s) != hipSuccess ||
          hipStreamWaitEvent(st, text_->ev[TextStream::NEV - 1], 0) != hipSuccess)
        return launch_status("train_clients: text-stream weight-gradient join");
    }
    if (wgs_ && wev_ > 0) {  // every weight gradient (and its clip-norm partials) before the clip
      if (wev_ >= WgradStream::NEV) return FLR_ERR_UNSUPPORTED;
      if (hipEventRecord(wgs_->ev[wev_], wgs_->s) != hipSuccess || hipStreamWaitEvent(st, wgs_->ev[wev_], 0) != hipSuccess)
        return launch_status("train_clients: weight-gradient join");
    }
    wgs_ = wgs_save;
    // ---------------- clip + SGD-momentum ----------------
    std::vector<float*> xb, mb;
    std::vector<const float*> gb;
    std::vector<int64_t> nb, cs;
    std::vector<uint8_t> normed;
    std::vector<int64_t> xoffs;  // the blocks' offsets in a training-order row
    for (const auto& b : blocks_opt_) {
      const Param& p = ps_[b.j];
      xoffs.push_back(p.off + b.o);
      xb.push_back(p.w + b.o);
      gb.push_back(p.g + b.o);
      mb.push_back(p.m + b.o);
      nb.push_back(b.n);
      cs.push_back(b.cs);
      normed.push_back(p.sq_base >= 0 || p.sq_early ? 1 : 0);
    }
    const bool fuse = clip_ > 0 && nsq_ > 0;
    // first step in training order: the tap-major blocks read the shared global copy
    std::vector<int64_t> soffs;
    const bool src = first && gshared_;
    if (src)
      for (const auto& b : blocks_opt_) soffs.push_back(ps_[b.j].tap ? ps_[b.j].off + b.o : -1);
    const int flags = int(first) | (int(last) << 1);
    // the last step writes X: nothing after it in the call to overlap; a model with
    // more parameter groups than the side stream has events updates on the caller's stream
    if (last || !side_ || (int)gthr_.size() + 1 > SideStream::NEV) {
      FLR_TRY(flr_clip_sgd_step_blocked_src(xb.data(), gb.data(), mb.data(), nb.data(), cs.data(),
                                            (int64_t)xb.size(), K_, lr, mom, wd_, clip_, flags, last ? xout_ : nullptr,
                                            last && xout_ ? xoffs.data() : nullptr, xld_, xneg_,
                                            fuse ? normed.data() : nullptr, fuse ? sq_ : nullptr, fuse ? nsq_ : 0,
                                            src ? gshared_ : nullptr, src ? soffs.data() : nullptr, norms_, sgd_ws_,
                                            sgd_ws_n_, st));
      return FLR_OK;
    }
    // the clip norms on this stream; the update on the side stream, one launch per
    // forward segment's parameter group, each followed by its event (wait_group)
    FLR_TRY(flr_clip_sgd_step_phase(xb.data(), gb.data(), mb.data(), nb.data(), cs.data(), (int64_t)xb.size(), K_, lr,
                                    mom, wd_, clip_, flags, nullptr, nullptr, 0, 0, fuse ? normed.data() : nullptr,
                                    fuse ? sq_ : nullptr, fuse ? nsq_ : 0, nullptr, nullptr, norms_,
                                    FLR_SGD_PHASE_NORM, sgd_ws_, sgd_ws_n_, st));
    const int ng = (int)gthr_.size();
    hipEvent_t fork = side_->ev[ng];
    if (hipEventRecord(fork, st) != hipSuccess || hipStreamWaitEvent(side_->s, fork, 0) != hipSuccess)
      return launch_status("train_clients: side-stream fork");
    // group g = the blocks of parameters [gthr_[g-1], gthr_[g]); launched in forward order
    // (text branch, stem, residual blocks, head), each followed by its event
    size_t nlaunched = 0;
    for (int g : gorder_) {
      const int jlo = g ? gthr_[g - 1] : 0;
      size_t i0 = 0;
      while (i0 < blocks_opt_.size() && blocks_opt_[i0].j < jlo) ++i0;
      size_t i1 = i0;
      while (i1 < blocks_opt_.size() && blocks_opt_[i1].j < gthr_[g]) ++i1;
      nlaunched += i1 - i0;
      if (i1 > i0) {
        auto sub = [&](auto& v) { return v.data() + i0; };
        FLR_TRY(flr_clip_sgd_step_phase(sub(xb), sub(gb), sub(mb), sub(nb), sub(cs), (int64_t)(i1 - i0), K_, lr, mom,
                                        wd_, clip_, flags, nullptr, nullptr, 0, 0, nullptr, nullptr, 0,
                                        src ? gshared_ : nullptr, src ? sub(soffs) : nullptr, nullptr,
                                        FLR_SGD_PHASE_UPDATE, sgd_ws_, sgd_ws_n_, side_->s));
      }
      if (hipEventRecord(side_->ev[g], side_->s) != hipSuccess) return launch_status("train_clients: side-stream event");
    }
    if (nlaunched != blocks_opt_.size()) return FLR_ERR_ARG;  // a block outside every group: parameters out of order
    pending_ = true;
#undef FLR_TRY
    return FLR_OK;
  }

  // the forward's wait for the previous step's side-stream update of group g
  // record event e on `from`; with e even, `to` waits on it now (a fork); odd
  // events are waited on later by the caller (a join)
  int fork(hipStream_t from, hipStream_t to, int e) {
    if (hipEventRecord(text_->ev[e], from) != hipSuccess) return launch_status("train_clients: text-stream event");
    if (!(e & 1) && hipStreamWaitEvent(to, text_->ev[e], 0) != hipSuccess)
      return launch_status("train_clients: text-stream fork");
    return FLR_OK;
  }

  // the clip-norm partials of the parameters marked sq_early (their optimizer
  // blocks) into sq_[k][sq_early_base_ ..]
  int early_sumsq(hipStream_t s) {
    std::vector<const float*> g;
    std::vector<int64_t> n, cs;
    for (const auto& b : blocks_opt_) {
      const Param& p = ps_[b.j];
      if (!p.sq_early) continue;
      g.push_back(p.g + b.o);
      n.push_back(b.n);
      cs.push_back(b.cs);
    }
    if (g.empty()) return FLR_ERR_ARG;
    return clip_sumsq_blocks(g.data(), n.data(), cs.data(), (int64_t)g.size(), K_, sq_ + sq_early_base_, nsq_,
                             kEarlySlots, s);
  }

  int wait_group(int g, hipStream_t st) {
    if (!pending_) return FLR_OK;
    if (hipStreamWaitEvent(st, side_->ev[g], 0) != hipSuccess) return launch_status("train_clients: side-stream join");
    return FLR_OK;
  }

  // client-matrix rows in torch order (export), rows k < nneg negated
  int export_rows(float* X, int64_t ld, int64_t nneg, hipStream_t st) {
    int rc;
    for (auto& p : ps_) {
      if (p.tap)
        rc = flr_tap_major_to_torch_neg(p.w, K_, p.shape[2] * p.shape[3], p.shape[1], p.shape[0], X + p.off, ld, nneg,
                                        st);
      else
        rc = flr_copy_rows_neg(p.w, p.n, p.n, X + p.off, ld, K_, nneg, st);
      if (rc != FLR_OK) return rc;
    }
    return FLR_OK;
  }

  float* norms_ = nullptr;  // optional [K] clip norms (the caller's)
  bool fuse_res_ = true;     // FLR_FUSED_RES=0: the separate gradient-sum pass (A/B)
  int64_t live_params() const {
    int64_t n = 0;
    for (const auto& b : blocks_opt_) n += b.n;
    return n;
  }

 private:
  struct OptBlock {
    int j;
    int64_t o, n, cs;
  };

  template <class T>
  T* alloc(int64_t n) {
    const size_t a = align_up(off_, 256);
    off_ = a + (size_t)std::max<int64_t>(n, 0) * sizeof(T);
    return base_ ? reinterpret_cast<T*>(base_ + a) : nullptr;
  }
  int add_param(const std::string& name, std::vector<int64_t> shape) {
    Param p;
    p.name = name;
    p.shape = std::move(shape);
    p.n = 1;
    for (int64_t d : p.shape) p.n *= d;
    ps_.push_back(p);
    return (int)ps_.size() - 1;
  }
  void add_block(int j, int64_t o, int64_t n, int64_t cs) { blocks_opt_.push_back(OptBlock{j, o, n, cs}); }
  static int64_t packed(int64_t ng, int64_t h, int64_t c) { return ng * ((h + 31) / 32) * ((c + 15) / 16) * 512; }

  void mark_conv(ConvOp& c) {
    conv_index_.push_back(&c);
    Param& p = ps_[c.p];
    p.tap = flr_conv2d_tap_major_ok(c.Cin, c.Cout) != 0;
    if (p.tap && wd_ == 0.f) p.dead = (int64_t)live_taps(p).size() < c.k * c.k;
  }
  const ConvOp* conv_of(const Param& p) const {
    for (const ConvOp* c : conv_index_)
      if (&ps_[c->p] == &p) return c;
    return nullptr;
  }
  // taps kh*k + kw that read a non-padding pixel (square map; flr.models.multimodal.live_taps)
  std::vector<int> live_taps(const Param& p) const {
    const ConvOp* c = conv_of(p);
    std::vector<int> rows, out;
    for (int64_t t = 0; t < c->k; ++t)
      for (int64_t o = 0; o < c->Ho; ++o) {
        const int64_t i = o * c->stride - c->pad + t;
        if (i >= 0 && i < c->H) {
          rows.push_back((int)t);
          break;
        }
      }
    for (int kh : rows)
      for (int kw : rows) out.push_back(kh * (int)c->k + kw);
    return out;
  }
  void bn_stats(BnOp& b) {
    b.mean = alloc<float>(K_ * b.C);
    b.invstd = alloc<float>(K_ * b.C);
  }
  void conv_ws(ConvOp& c) {
    const Param& p = ps_[c.p];
    const size_t n = p.tap ? flr_conv2d_t_workspace(K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad)
                           : flr_conv2d_workspace(K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad);
    if (!p.tap) {  // generic convs keep their forward workspace for the weight gradient
      c.fws_n = n;
      c.fws = alloc<char>(n);
    }
    cws_n_ = std::max(cws_n_, n);
  }

  // a tap-major conv weight: per client, or (first step, training order) the
  // one global copy every client reads with client stride 0
  const float* tap_w(const Param& p, int64_t& stride) const {
    const bool shared = first_ && gshared_;
    stride = shared ? 0 : p.n;
    return shared ? gshared_ + p.off : p.w;
  }
  int conv_fwd(const ConvOp& c, const float* x, float* y, hipStream_t st, char* wsp = nullptr) {
    const Param& p = ps_[c.p];
    if (p.tap) {
      int64_t wst;
      const float* w = tap_w(p, wst);
      return flr_conv2d_fwd_t_ex(x, w, wst, y, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad,
                                 wsp ? wsp : cws_, cws_n_, st);
    }
    return flr_conv2d_fwd(x, p.w, y, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad, c.fws, c.fws_n, st);
  }
  // dx (when wanted) then dw, as ClientConv2d[T].backward
  // With the weight-gradient stream (wgs_, wev_ < NEV), a tap-major conv's dW runs on
  // it with the second workspace, forked here (dy ready on st), the data gradient
  // on st.  The two write disjoint outputs; dy and x are not rewritten this step.
  int conv_bwd(const ConvOp& c, const float* x, const float* dy, float* dx, hipStream_t st,
               const float* add = nullptr) {
    const Param& p = ps_[c.p];
    int rc;
    if (p.tap) {
      int64_t wst;
      const float* w = tap_w(p, wst);
      hipStream_t ws = st;
      char* wsp = cws_;
      if (wg_on_text_ && text_ && tev_ < TextStream::NEV - 1) {
        if (hipEventRecord(text_->ev[tev_], st) != hipSuccess || hipStreamWaitEvent(text_->s, text_->ev[tev_], 0) != hipSuccess)
          return launch_status("train_clients: text-stream weight-gradient fork");
        ++tev_;
        ws = text_->s;
        wsp = cws3_;
      } else if (wgs_ && wev_ + 1 < WgradStream::NEV) {  // one event kept for the join
        if (hipEventRecord(wgs_->ev[wev_], st) != hipSuccess || hipStreamWaitEvent(wgs_->s, wgs_->ev[wev_], 0) != hipSuccess)
          return launch_status("train_clients: weight-gradient fork");
        ++wev_;
        ws = wgs_->s;
        wsp = cws2_;
      }
      if (dx && (rc = flr_conv2d_bwd_data_t_ex(dy, w, wst, add, dx, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k,
                                               c.stride, c.pad, cws_, cws_n_, st)) != FLR_OK)
        return rc;
      const int zero_dead = p.dead ? 0 : 1;
      if (p.sq_base >= 0)
        return flr_conv2d_bwd_weight_t_sq(x, dy, p.g, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad,
                                          zero_dead, sq_ + p.sq_base, std::max<int64_t>(1, nsq_), wsp, cws_n_, ws);
      return flr_conv2d_bwd_weight_t(x, dy, p.g, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad, zero_dead,
                                     wsp, cws_n_, ws);
    }
    if (dx && (rc = flr_conv2d_bwd_data(dy, p.w, dx, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad, cws_,
                                        cws_n_, st)) != FLR_OK)
      return rc;
    return flr_conv2d_bwd_weight_reuse(x, dy, p.g, K_, B_, c.Cin, c.H, c.H, c.Cout, c.k, c.k, c.stride, c.pad, c.fws,
                                       c.fws_n, st);
  }
  int bn_fwd(const BnOp& b, const float* x, const float* res, float* y, bool relu, hipStream_t st) {
    return flr_batchnorm_fwd(x, ps_[b.pg].w, ps_[b.pb].w, res, y, b.mean, b.invstd, 1, K_ * b.C, b.HW, 1e-5f,
                             relu ? 1 : 0, st);
  }
  int bn_bwd(const BnOp& b, const float* dy, const float* x, const float* y, bool relu, float* dx, float* dres,
             hipStream_t st) {
    return flr_batchnorm_bwd(dy, x, relu ? y : nullptr, ps_[b.pg].w, b.mean, b.invstd, dx, ps_[b.pg].g, ps_[b.pb].g,
                             dres, 1, K_ * b.C, b.HW, relu ? 1 : 0, st);
  }
  int gemm(const float* A, int64_t ak, int64_t am, int64_t ar, const float* Bm, int64_t bk, int64_t bn, int64_t br,
           float* C, int64_t ck, int64_t cm, int64_t cn, const float* bias, int64_t bias_k, const float* add,
           int64_t M, int64_t N, int64_t R, hipStream_t st) {
    return flr_bgemm(A, ak, am, ar, Bm, bk, bn, br, C, ck, cm, cn, bias, bias_k, add, K_, M, N, R, gws_, gws_n_, st);
  }
  int rowsum(const float* X, int64_t xk, int64_t xm, int64_t M, int64_t N, float* out, hipStream_t st) {
    return flr_sum_rows_ex(X, xk, xm, K_, M, N, out, N, rws_, rws_n_, st);
  }

  flr_resnet_gru_spec s_;
  int64_t K_, B_;
  char* base_;
  float wd_, clip_;
  size_t off_ = 0;
  std::vector<Param> ps_;
  std::vector<OptBlock> blocks_opt_;
  std::vector<Block> blocks_;
  std::vector<const ConvOp*> conv_index_;
  ConvOp stem_{};
  BnOp stem_bn_{};
  int64_t T_ = 0, H_ = 0, E_ = 0, F_ = 0, C_ = 0, Dimg_ = 0, P_ = 0, Hs_ = 0, Hp_ = 0, nsq_ = 0;
  int p_emb_ = 0, p_wih_ = 0, p_whh_ = 0, p_bih_ = 0, p_bhh_ = 0, p_w1_ = 0, p_b1_ = 0, p_w2_ = 0, p_b2_ = 0;
  double* sq_ = nullptr;
  std::vector<int> gthr_;  // optimizer group g: parameters [gthr_[g-1], gthr_[g]) (forward segments)
  std::vector<int> gorder_;  // the groups in forward order: text branch, stem, residual blocks, head
  int gtext_ = 0, ghead_ = 0;
  static constexpr int kEarlySlots = 32;  // clip_sumsq_blocks' partials per client (train_step.hip NBLK)
  int sq_early_base_ = -1;                // their first slot in sq_ (-1: none)
 public:
  SideStream* side_ = nullptr;  // the optimizer's side stream (nullptr: the update runs on the caller's stream)
  TextStream* text_ = nullptr;  // the text branch's stream (nullptr: the caller's stream)
  WgradStream* wgs_ = nullptr;  // the weight-gradient stream (nullptr: on the caller's stream)
  int wev_ = 0;                 // fork events used this step
  bool stem_fused_ = false;     // bn1 + relu + maxpool fused (flr_batchnorm_relu_maxpool_fwd / _bwd)
 private:
  bool pending_ = false;        // a side-stream update the next forward must wait for
  char *sgd_ws_ = nullptr, *gws_ = nullptr, *rws_ = nullptr, *ews_ = nullptr, *cws_ = nullptr, *cws2_ = nullptr,
       *cws3_ = nullptr;
  bool wg_on_text_ = false;  // this conv's dW on the text stream (the first FLR_WG_TEXT residual blocks)
  int tev_ = 4;              // text-stream fork events used by them this step
  size_t sgd_ws_n_ = 0, gws_n_ = 0, rws_n_ = 0, ews_n_ = 0, cws_n_ = 0;
  float *ximg_ = nullptr, *y0_ = nullptr, *a0_ = nullptr, *d_a0_ = nullptr, *d_y0_ = nullptr, *p0_ = nullptr,
        *d_p0_ = nullptr, *d_x4_ = nullptr;
  uint8_t* arg0_ = nullptr;
  float *emb_ = nullptr, *gi_ = nullptr, *hseq_ = nullptr, *gates_ = nullptr, *gh_ = nullptr, *whhP_ = nullptr,
        *whhT_ = nullptr, *h1_ = nullptr, *logits_ = nullptr, *dlogits_ = nullptr, *rows_ = nullptr, *loss_ = nullptr,
        *dpre_ = nullptr, *dh_ = nullptr, *dh2_ = nullptr, *dh_direct_ = nullptr, *dgh_ = nullptr, *dgi_ = nullptr,
        *demb_ = nullptr;
};

}  // namespace tc
}  // namespace flr

using namespace flr;

extern "C" int64_t flr_resnet_gru_num_params(const flr_resnet_gru_spec* spec) {
  if (!spec) return -1;
  tc::Net net(*spec, 1, 1, 0.f, 0.f, nullptr);
  if (net.layout() != FLR_OK) return -1;
  return net.P();
}

extern "C" size_t flr_train_clients_workspace(const flr_resnet_gru_spec* spec, int64_t K, int64_t B,
                                              int64_t steps) {
  if (!spec || K < 1 || B < 1 || steps < 1) return 0;
  side_stream(true);  // created here, before any capture of the training call
  text_stream(true);
  wgrad_stream(true);
  tc::Net net(*spec, K, B, 0.f, 1.f, nullptr);
  if (net.layout() != FLR_OK) return 0;
  return align_up(net.bytes(), 256) + align_up((size_t)steps * K * sizeof(float), 256) + 256;
}

extern "C" int flr_train_clients(const flr_resnet_gru_spec* spec, const float* global, float* X, int64_t ld,
                                 const float* images, const int64_t* tokens, const int64_t* labels,
                                 const float* dropout_masks, int64_t steps, int64_t K, int64_t B, float lr,
                                 float momentum, float weight_decay, float max_norm, int64_t nneg, float* loss_out,
                                 float* norms_out, void* workspace, size_t workspace_bytes, void* stream) {
  return flr_train_clients_ex(spec, global, X, ld, images, tokens, labels, dropout_masks, steps, K, B, lr, momentum,
                              weight_decay, max_norm, nneg, loss_out, norms_out, 0, workspace, workspace_bytes, stream);
}

extern "C" int flr_train_clients_ex(const flr_resnet_gru_spec* spec, const float* global, float* X, int64_t ld,
                                    const float* images, const int64_t* tokens, const int64_t* labels,
                                    const float* dropout_masks, int64_t steps, int64_t K, int64_t B, float lr,
                                    float momentum, float weight_decay, float max_norm, int64_t nneg, float* loss_out,
                                    float* norms_out, unsigned flags, void* workspace, size_t workspace_bytes,
                                    void* stream) {
  if (!spec || !global || !X || !images || !tokens || !labels || !loss_out || steps < 1 || K < 1 || B < 1 || nneg < 0)
    return FLR_ERR_ARG;
  if (flags & ~(unsigned)(FLR_TC_TRAIN_ORDER | FLR_TC_DEFER_DEAD)) return FLR_ERR_ARG;
  if ((flags & FLR_TC_DEFER_DEAD) && !(flags & FLR_TC_TRAIN_ORDER)) return FLR_ERR_ARG;
  if (!workspace || workspace_bytes < flr_train_clients_workspace(spec, K, B, steps)) return FLR_ERR_WORKSPACE;
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  tc::Net net(*spec, K, B, weight_decay, max_norm, base);
  int rc = net.layout();
  if (rc != FLR_OK) return rc;
  if (ld < net.P()) return FLR_ERR_ARG;
  float* step_loss = reinterpret_cast<float*>(base + align_up(net.bytes(), 256));
  net.norms_ = norms_out;
  static const bool fuse_res = [] {
    const char* e = flr::knob("FLR_FUSED_RES");
    return !(e && e[0] == '0');
  }();
  net.fuse_res_ = fuse_res;
  static const bool shared_first = [] {
    const char* e = flr::knob("FLR_SHARED_FIRST");
    return !(e && e[0] == '0');
  }();
  net.shared_first_ = shared_first;
  const bool train_order = (flags & FLR_TC_TRAIN_ORDER) != 0;
  hipStream_t st = as_stream(stream);
  net.side_ = side_stream(true, st);
  net.text_ = text_stream(true, st);
  net.wgs_ = wgrad_stream(true, st);
  if (train_order) {
    net.xout_ = X;
    net.xld_ = ld;
    net.xneg_ = nneg;
    rc = net.load_global_train(global, st);
  } else {
    rc = net.load_global(global, st);
  }
  if (rc != FLR_OK) return rc;
  const int64_t C0 = spec->in_channels, HW0 = spec->image_size * spec->image_size, T = spec->seq_len;
  for (int64_t s = 0; s < steps; ++s) {
    rc = net.step(images + s * K * B * C0 * HW0, tokens + s * K * B * T, labels + s * K * B,
                  dropout_masks ? dropout_masks + s * K * B * spec->fusion : nullptr, s == 0, s == steps - 1,
                  step_loss + s * K, lr, momentum, st);
    if (rc != FLR_OK) return rc;
  }
  if (!train_order) {
    rc = net.export_rows(X, ld, nneg, st);
  } else if (!(flags & FLR_TC_DEFER_DEAD)) {
    rc = net.dead_ranges(global, X, ld, nneg, st);
  }
  if (rc != FLR_OK) return rc;
  return flr_mean_rows(step_loss, steps, K, loss_out, st);
}

extern "C" int64_t flr_resnet_gru_dead_ranges(const flr_resnet_gru_spec* spec, float weight_decay, int64_t* off,
                                              int64_t* n, int64_t cap) {
  if (!spec || cap < 0 || (cap > 0 && (!off || !n))) return -1;
  tc::Net net(*spec, 1, 1, weight_decay, 0.f, nullptr);
  if (net.layout() != FLR_OK) return -1;
  std::vector<std::pair<int64_t, int64_t>> r;
  net.dead_list(r);
  for (int64_t i = 0; i < cap && i < (int64_t)r.size(); ++i) {
    off[i] = r[i].first;
    n[i] = r[i].second;
  }
  return (int64_t)r.size();
}

extern "C" int flr_resnet_gru_fill_dead(const flr_resnet_gru_spec* spec, float weight_decay, const float* gtrain,
                                        float* X, int64_t ld, int64_t K, int64_t nneg, void* stream) {
  if (!spec || !gtrain || !X || K < 1 || nneg < 0) return FLR_ERR_ARG;
  tc::Net net(*spec, K, 1, weight_decay, 0.f, nullptr);
  const int rc = net.layout();
  if (rc != FLR_OK) return rc;
  if (ld < net.P()) return FLR_ERR_ARG;
  // FLR_FILL_GRID: workgroups per row (0: the training phase's grid); 1 or 4
  // beside the Krum chains measured slower still (profiles/r6_dead/)
  static const int64_t gx = [] {
    const char* e = flr::knob("FLR_FILL_GRID");
    const int v = e ? atoi(e) : 0;
    return (int64_t)(v >= 0 && v <= 256 ? v : 0);
  }();
  return net.dead_ranges(gtrain, X, ld, nneg, as_stream(stream), gx);
}

extern "C" int flr_resnet_gru_reorder(const flr_resnet_gru_spec* spec, const float* src, float* dst, int to_train,
                                      void* stream) {
  if (!spec || !src || !dst || src == dst) return FLR_ERR_ARG;
  tc::Net net(*spec, 1, 1, 0.f, 0.f, nullptr);
  const int rc = net.layout();
  if (rc != FLR_OK) return rc;
  return net.reorder(src, dst, to_train != 0, as_stream(stream));
}

extern "C" int64_t flr_resnet_gru_live_params(const flr_resnet_gru_spec* spec, float weight_decay) {
  if (!spec) return -1;
  tc::Net net(*spec, 1, 1, weight_decay, 0.f, nullptr);
  if (net.layout() != FLR_OK) return -1;
  return net.live_params();
}
