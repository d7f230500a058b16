// a1 for the C4/C5 model family — the client plugin's local update as ONE C
// entry: flr_train_vit_bert.
//
// Replaces, for a batch of K clients of the ViT-S + BERT-mini late-fusion
// model (flr.models.transformer.ViTBertNet), the per-client loop of the
// simulation (experiments/run_experiments.py:193-240: fresh model <- global,
// fresh SGD(lr, momentum, wd), per batch forward, mean cross-entropy,
// backward, clip_grad_norm_, step; update = parameters()) and FLClient.fit /
// _train (src/client/fl_client.py:76-149: loss = mean of the per-batch
// losses).  The kernel schedule is the Python trainer's (flr.train.
// ClientBatchTrainer over flr.models.transformer.vit_bert_forward and the
// flr.nn autograd functions) run from C++ without torch, so both give the same
// bits: the same GEMMs (flr_bgemm_ex with its fused bias / GELU / ReLU + mask /
// tanh epilogues), LayerNorms, attention, embedding and row-sum kernels, the
// two-path gradient sums of autograd as one rounded add, and the chunking of
// the clients into passes of at most `chunk` clients (activations scale with
// the chunk; parameters, momentum and the client matrix with K).
//
// Training state lives in the caller's workspace (the ABI never allocates):
// per-parameter [K][n] blocks of weights (and momentum when steps > 1), a
// chunk's [chunk][n] gradient blocks, every activation of one pass, the
// kernels' scratch.  The layout is computed by a dry run (base == nullptr)
// that sums sizes; the scratch sizes come from a dry pass over the schedule.
#include "flr_common.h"
#include "side_stream.h"

#include <algorithm>
#include <string>
#include <vector>

namespace flr {
namespace tv {

constexpr int THREADS = 256;

inline unsigned grid_for(int64_t n) {
  const int64_t g = (n + THREADS - 1) / THREADS;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

// patches[kb][py*G + px][c*p*p + kh*p + kw] = img[kb][c][py*p + kh][px*p + kw]
// (flr.models.transformer.patchify: Conv2d(C, D, p, stride p)'s receptive
// fields flattened in its weight's (c, kh, kw) order)
__global__ void patchify_kernel(const float* __restrict__ img, float* __restrict__ out, int64_t KB, int64_t C,
                                int64_t S, int64_t p) {
  const int64_t G = S / p, NP = G * G, pp = p * p, Cpp = C * pp;
  const int64_t n = KB * NP * Cpp;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS) {
    const int64_t e = i % Cpp, r = i / Cpp;
    const int64_t patch = r % NP, kb = r / NP;
    const int64_t c = e / pp, kh = (e / p) % p, kw = e % p;
    const int64_t y = (patch / G) * p + kh, x = (patch % G) * p + kw;
    out[i] = img[((kb * C + c) * S + y) * S + x];
  }
}

// out = a + b (one rounding: autograd's accumulation of two gradient paths)
__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out,
                           int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS)
    out[i] = __fadd_rn(a[i], b[i]);
}

// BERT's shared id rows: token types 0, positions n % T (arange(T).repeat(B))
__global__ void bert_ids_kernel(int64_t* __restrict__ type_ids, int64_t* __restrict__ pos_ids, int64_t N,
                                int64_t T) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < N; i += (int64_t)gridDim.x * THREADS) {
    type_ids[i] = 0;
    pos_ids[i] = i % T;
  }
}

struct Param {
  std::string name;
  std::vector<int64_t> shape;
  int64_t n = 0, off = 0;  // numel, offset in the parameters() vector
  float *w = nullptr, *m = nullptr, *g = nullptr;
};

struct Layer {  // one encoder layer's parameter indices (EncoderLayer's registration order)
  int ln1w, ln1b, qkvw, qkvb, projw, projb, ln2w, ln2b, fc1w, fc1b, fc2w, fc2b;
};

// saved activations of one encoder layer (per pass of kc clients)
struct LayerAct {
  float *h = nullptr;    // ViT: LN1 output (qkv input); BERT: unused (the layer input is the previous y)
  float *s1 = nullptr;   // LN1's residual stream s (ViT i > 0; BERT: x + attn)
  float *qkv = nullptr, *ctx = nullptr, *lse = nullptr;
  float *s2 = nullptr;   // LN2's s
  float *y2 = nullptr;   // LN2 output: ViT the MLP input; BERT the layer output
  float *y1 = nullptr;   // BERT: LN1 output (the MLP input)
  float *pre = nullptr, *hm = nullptr;  // the MLP's GELU input and output
  float *mean1 = nullptr, *rstd1 = nullptr, *mean2 = nullptr, *rstd2 = nullptr;
};

class Net {
 public:
  Net(const flr_vit_bert_spec& s, int64_t K, int64_t B, int64_t KC, int64_t steps, char* base)
      : s_(s), K_(K), B_(B), KC_(KC), steps_(steps), base_(base) {}

  int layout() {
    const auto& s = s_;
    if (s.num_classes < 1 || s.image_size < 1 || s.in_channels < 1 || s.patch < 1 || s.vit_dim < 1 ||
        s.vit_depth < 1 || s.vit_heads < 1 || s.vit_mlp < 1 || s.vocab < 1 || s.seq_len < 1 || s.bert_dim < 1 ||
        s.bert_depth < 1 || s.bert_heads < 1 || s.bert_ffn < 1 || s.bert_max_pos < 1 || s.fusion < 1 || K_ < 1 ||
        B_ < 1 || KC_ < 1 || steps_ < 1)
      return FLR_ERR_ARG;
    if (s.image_size % s.patch) return FLR_ERR_UNSUPPORTED;
    Dv_ = s.vit_dim;
    Db_ = s.bert_dim;
    Mv_ = s.vit_mlp;
    Fb_ = s.bert_ffn;
    F_ = s.fusion;
    C_ = s.num_classes;
    Tb_ = s.seq_len;
    G_ = s.image_size / s.patch;
    NP_ = G_ * G_;
    Tv_ = NP_ + 1;
    Cpp_ = s.in_channels * s.patch * s.patch;
    // kernel limits: attention heads of 64 over <= 96 tokens, LayerNorm widths
    // multiple of 4 up to 1024, positions within the table, embedding rows
    if (Dv_ % s.vit_heads || Dv_ / s.vit_heads != 64 || Db_ % s.bert_heads || Db_ / s.bert_heads != 64 ||
        Tv_ > 96 || Tb_ > 96 || Dv_ > 1024 || Db_ > 1024 || Tb_ > s.bert_max_pos || B_ * Tb_ > 4096)
      return FLR_ERR_UNSUPPORTED;
    // ---- parameters() order of ViTBertNet (flr.models.transformer) ----
    p_cls_ = add_param("vit.cls_token", {1, 1, Dv_});
    p_pos_ = add_param("vit.pos_embed", {1, Tv_, Dv_});
    p_pew_ = add_param("vit.patch_embed.weight", {Dv_, Cpp_});
    p_peb_ = add_param("vit.patch_embed.bias", {Dv_});
    for (int64_t i = 0; i < s.vit_depth; ++i)
      vl_.push_back(add_layer("vit.blocks." + std::to_string(i) + ".", Dv_, Mv_));
    p_nw_ = add_param("vit.norm.weight", {Dv_});
    p_nb_ = add_param("vit.norm.bias", {Dv_});
    p_word_ = add_param("bert.word_embeddings.weight", {s.vocab, Db_});
    p_bpos_ = add_param("bert.position_embeddings.weight", {s.bert_max_pos, Db_});
    p_type_ = add_param("bert.token_type_embeddings.weight", {2, Db_});
    p_ew_ = add_param("bert.emb_ln.weight", {Db_});
    p_eb_ = add_param("bert.emb_ln.bias", {Db_});
    for (int64_t i = 0; i < s.bert_depth; ++i)
      bl_.push_back(add_layer("bert.layers." + std::to_string(i) + ".", Db_, Fb_));
    p_poolw_ = add_param("bert.pooler.weight", {Db_, Db_});
    p_poolb_ = add_param("bert.pooler.bias", {Db_});
    p_f1w_ = add_param("fc1.weight", {F_, Dv_ + Db_});
    p_f1b_ = add_param("fc1.bias", {F_});
    p_f2w_ = add_param("fc2.weight", {C_, F_});
    p_f2b_ = add_param("fc2.bias", {C_});
    P_ = 0;
    for (auto& p : ps_) {
      p.off = P_;
      P_ += p.n;
    }
    // ---- training state: weights (and momentum for multi-step updates) for
    // every client, gradients for one pass ----
    for (auto& p : ps_) {
      p.w = alloc<float>(K_ * p.n);
      p.m = steps_ > 1 ? alloc<float>(K_ * p.n) : nullptr;
      p.g = alloc<float>(KC_ * p.n);
    }
    sgd_ws_n_ = flr_clip_sgd_workspace(KC_);
    sgd_ws_ = alloc<char>(sgd_ws_n_);
    // ---- activations of one pass (KC clients) ----
    const int64_t Rv = B_ * Tv_, Rb = B_ * Tb_, KC = KC_;
    patches_ = alloc<float>(KC * B_ * NP_ * Cpp_);
    tok_ = alloc<float>(KC * B_ * NP_ * Dv_);
    x0_ = alloc<float>(KC * Rv * Dv_);
    va_.resize(vl_.size());
    for (size_t i = 0; i < vl_.size(); ++i) {
      LayerAct& a = va_[i];
      a.h = alloc<float>(KC * Rv * Dv_);
      a.s1 = i > 0 ? alloc<float>(KC * Rv * Dv_) : nullptr;
      a.qkv = alloc<float>(KC * Rv * 3 * Dv_);
      a.ctx = alloc<float>(KC * Rv * Dv_);
      a.lse = alloc<float>(KC * B_ * s.vit_heads * Tv_);
      a.s2 = alloc<float>(KC * Rv * Dv_);
      a.y2 = alloc<float>(KC * Rv * Dv_);
      a.pre = alloc<float>(KC * Rv * Mv_);
      a.hm = alloc<float>(KC * Rv * Mv_);
      stats(a, KC * Rv);
    }
    sf_ = alloc<float>(KC * Rv * Dv_);
    yf_ = alloc<float>(KC * Rv * Dv_);
    meanf_ = alloc<float>(KC * Rv);
    rstdf_ = alloc<float>(KC * Rv);
    va_tmp_ = alloc<float>(KC * Rv * Dv_);  // proj / MLP outputs (consumed by the next LayerNorm)
    type_ids_ = alloc<int64_t>(Rb);
    pos_ids_ = alloc<int64_t>(Rb);
    e_ = alloc<float>(KC * Rb * Db_);
    xe_ = alloc<float>(KC * Rb * Db_);
    meane_ = alloc<float>(KC * Rb);
    rstde_ = alloc<float>(KC * Rb);
    ba_.resize(bl_.size());
    for (size_t i = 0; i < bl_.size(); ++i) {
      LayerAct& a = ba_[i];
      a.qkv = alloc<float>(KC * Rb * 3 * Db_);
      a.ctx = alloc<float>(KC * Rb * Db_);
      a.lse = alloc<float>(KC * B_ * s.bert_heads * Tb_);
      a.s1 = alloc<float>(KC * Rb * Db_);
      a.y1 = alloc<float>(KC * Rb * Db_);
      a.pre = alloc<float>(KC * Rb * Fb_);
      a.hm = alloc<float>(KC * Rb * Fb_);
      a.s2 = alloc<float>(KC * Rb * Db_);
      a.y2 = alloc<float>(KC * Rb * Db_);
      stats(a, KC * Rb);
    }
    ba_tmp_ = alloc<float>(KC * Rb * Db_);
    txt_ = alloc<float>(KC * B_ * Db_);
    h1_ = alloc<float>(KC * B_ * F_);
    logits_ = alloc<float>(KC * B_ * C_);
    dlogits_ = alloc<float>(KC * B_ * C_);
    rows_ = alloc<float>(KC * B_);
    loss_ = alloc<float>(KC);
    // ---- backward scratch ----
    dpre_h_ = alloc<float>(KC * B_ * F_);
    dimg_ = alloc<float>(KC * B_ * Dv_);
    dtxt_ = alloc<float>(KC * B_ * Db_);
    dpre_p_ = alloc<float>(KC * B_ * Db_);
    dxp_ = alloc<float>(KC * B_ * Db_);
    for (float*& p : vd_) p = alloc<float>(KC * Rv * Dv_);
    vdq_ = alloc<float>(KC * Rv * 3 * Dv_);
    vdp_ = alloc<float>(KC * Rv * Mv_);
    // the weight-gradient stream's second copies: a ViT layer's side work reads them
    // while the next layer writes the first (vd_[6]: the third buffer of the dL/dr ring)
    vdq2_ = alloc<float>(KC * Rv * 3 * Dv_);
    vdp2_ = alloc<float>(KC * Rv * Mv_);
    vdx2b_ = alloc<float>(KC * Rv * Dv_);
    vdr3_ = alloc<float>(KC * Rv * Dv_);
    dtok_ = alloc<float>(KC * B_ * NP_ * Dv_);
    for (float*& p : bd_) p = alloc<float>(KC * Rb * Db_);
    bdq_ = alloc<float>(KC * Rb * 3 * Db_);
    bdp_ = alloc<float>(KC * Rb * Fb_);
    // the weight-gradient stream's second copies of what a BERT layer's side work reads
    bdq2_ = alloc<float>(KC * Rb * 3 * Db_);
    bdp2_ = alloc<float>(KC * Rb * Fb_);
    bdy2b_ = alloc<float>(KC * Rb * Db_);
    bd1b_ = alloc<float>(KC * Rb * Db_);
    // ---- kernel scratch, sized by a dry pass over the schedule ----
    dry_ = true;
    kc_ = KC_;
    int rc = pass(nullptr, nullptr, nullptr, nullptr, nullptr);
    dry_ = false;
    if (rc != FLR_OK) return rc;
    gws_ = alloc<char>(gws_n_);
    rws_ = alloc<char>(rws_n_);
    gws2_ = alloc<char>(gws_n_);  // the weight-gradient stream's own
    rws2_ = alloc<char>(rws_n_);
    lws_ = alloc<char>(lws_n_);
    ews_ = alloc<char>(ews_n_);
    return FLR_OK;
  }

  size_t bytes() const { return off_; }
  int64_t P() const { return P_; }

  int load_global(const float* global, hipStream_t st) {
    int rc;
    for (auto& p : ps_)
      if ((rc = flr_broadcast_rows(global + p.off, p.n, p.w, K_, p.n, st)) != FLR_OK) return rc;
    return FLR_OK;
  }

  // one local step of clients [c0, c0 + kc): forward, loss, backward, clip +
  // SGD-momentum; the last step writes the parameters to X's rows
  int step(const float* images, const int64_t* tokens, const int64_t* labels, const float* mask, int64_t c0,
           int64_t kc, bool first, bool last, float* loss_row, float lr, float mom, float wd, float clip, float* X,
           int64_t ld, int64_t nneg, float* norms, hipStream_t st) {
    c0_ = c0;
    kc_ = kc;
    st_ = st;
    int rc = pass(images, tokens, labels, mask, loss_row);
    if (rc != FLR_OK) return rc;
    std::vector<float*> xb, mb;
    std::vector<const float*> gb;
    std::vector<int64_t> nb, xoffs;
    for (const auto& p : ps_) {
      xb.push_back(p.w + c0 * p.n);
      gb.push_back(p.g);
      mb.push_back(p.m ? p.m + c0 * p.n : p.g);  // one step: the momentum buffer is neither read nor written
      nb.push_back(p.n);
      xoffs.push_back(p.off);
    }
    const int64_t neg = std::max<int64_t>(0, std::min(nneg, c0 + kc) - c0);
    return flr_clip_sgd_step_blocked_x(xb.data(), gb.data(), mb.data(), nb.data(), nullptr, (int64_t)xb.size(), kc,
                                       lr, mom, wd, clip, int(first) | (int(last) << 1),
                                       last ? X + c0 * ld : nullptr, last ? xoffs.data() : nullptr, ld, neg, nullptr,
                                       nullptr, 0, norms ? norms + c0 : nullptr, sgd_ws_, sgd_ws_n_, st);
  }

  // the weight-gradient stream of the ViT layers' backward (nullptr: all on the caller's)
  void set_wgrad_stream(WgradStream* w) { wgs_ = w; }

 private:
  // ---- the forward + backward of one pass ----------------------------------
  int pass(const float* images, const int64_t* tokens, const int64_t* labels, const float* mask, float* loss_row) {
    int rc;
#define FLR_TRY(x) \
  if ((rc = (x)) != FLR_OK) return rc
    const auto& s = s_;
    const int64_t kc = kc_, Rv = B_ * Tv_, Rb = B_ * Tb_, Dv = Dv_, Db = Db_, BNP = B_ * NP_;
    // ================= forward =================
    // ---- ViT (vit_bert_forward, _encoder_pre_ln) ----
    FLR_TRY(launch(patchify_kernel, kc * BNP * Cpp_, images, patches_, kc * B_, s.in_channels, s.image_size,
                   s.patch));
    FLR_TRY(linear(patches_, BNP * Cpp_, Cpp_, BNP, p_pew_, p_peb_, tok_, FLR_ACT_NONE, nullptr, nullptr));
    if (!dry_) FLR_TRY(flr_vit_tokens(tok_, W(p_cls_), W(p_pos_), kc, B_, NP_, Dv, x0_, st_));
    const float* s_cur = x0_;   // the residual stream s
    const float* r = nullptr;   // the pending MLP branch (added inside the next LayerNorm)
    for (size_t i = 0; i < vl_.size(); ++i) {
      const Layer& L = vl_[i];
      LayerAct& a = va_[i];
      if (!r) {
        FLR_TRY(ln_fwd(s_cur, nullptr, L.ln1w, L.ln1b, a.h, nullptr, a.mean1, a.rstd1, Rv, Dv, 1e-6f));
      } else {
        FLR_TRY(ln_fwd(s_cur, r, L.ln1w, L.ln1b, a.h, a.s1, a.mean1, a.rstd1, Rv, Dv, 1e-6f));
        s_cur = a.s1;
      }
      FLR_TRY(linear(a.h, Rv * Dv, Dv, Rv, L.qkvw, L.qkvb, a.qkv, FLR_ACT_NONE, nullptr, nullptr));
      if (!dry_) FLR_TRY(flr_attention_fwd(a.qkv, kc * B_, Tv_, s.vit_heads, 64, a.ctx, a.lse, st_));
      FLR_TRY(linear(a.ctx, Rv * Dv, Dv, Rv, L.projw, L.projb, va_tmp_, FLR_ACT_NONE, nullptr, nullptr));
      FLR_TRY(ln_fwd(s_cur, va_tmp_, L.ln2w, L.ln2b, a.y2, a.s2, a.mean2, a.rstd2, Rv, Dv, 1e-6f));
      s_cur = a.s2;
      FLR_TRY(linear(a.y2, Rv * Dv, Dv, Rv, L.fc1w, L.fc1b, a.hm, FLR_ACT_GELU, nullptr, a.pre));
      FLR_TRY(linear(a.hm, Rv * Mv_, Mv_, Rv, L.fc2w, L.fc2b, va_tmp_, FLR_ACT_NONE, nullptr, nullptr));
      r = va_tmp_;
    }
    FLR_TRY(ln_fwd(s_cur, r, p_nw_, p_nb_, yf_, sf_, meanf_, rstdf_, Rv, Dv, 1e-6f));
    // img = the class-token rows of yf: [kc][B][Dv] at strides (Rv*Dv, Tv*Dv, 1)
    // ---- BERT (_encoder_post_ln) ----
    FLR_TRY(launch(bert_ids_kernel, Rb, type_ids_, pos_ids_, Rb, Tb_));
    if (!dry_)
      FLR_TRY(flr_embedding_fwd(W(p_word_), s.vocab * Db, s.vocab, tokens, Rb, W(p_type_), 2 * Db, 2, type_ids_, 0,
                                W(p_bpos_), s.bert_max_pos * Db, s.bert_max_pos, pos_ids_, 0, kc, Rb, Db, e_, st_));
    FLR_TRY(ln_fwd(e_, nullptr, p_ew_, p_eb_, xe_, nullptr, meane_, rstde_, Rb, Db, 1e-12f));
    const float* x = xe_;
    for (size_t i = 0; i < bl_.size(); ++i) {
      const Layer& L = bl_[i];
      LayerAct& a = ba_[i];
      FLR_TRY(linear(x, Rb * Db, Db, Rb, L.qkvw, L.qkvb, a.qkv, FLR_ACT_NONE, nullptr, nullptr));
      if (!dry_) FLR_TRY(flr_attention_fwd(a.qkv, kc * B_, Tb_, s.bert_heads, 64, a.ctx, a.lse, st_));
      FLR_TRY(linear(a.ctx, Rb * Db, Db, Rb, L.projw, L.projb, ba_tmp_, FLR_ACT_NONE, nullptr, nullptr));
      FLR_TRY(ln_fwd(x, ba_tmp_, L.ln1w, L.ln1b, a.y1, a.s1, a.mean1, a.rstd1, Rb, Db, 1e-12f));
      FLR_TRY(linear(a.y1, Rb * Db, Db, Rb, L.fc1w, L.fc1b, a.hm, FLR_ACT_GELU, nullptr, a.pre));
      FLR_TRY(linear(a.hm, Rb * Fb_, Fb_, Rb, L.fc2w, L.fc2b, ba_tmp_, FLR_ACT_NONE, nullptr, nullptr));
      FLR_TRY(ln_fwd(a.y1, ba_tmp_, L.ln2w, L.ln2b, a.y2, a.s2, a.mean2, a.rstd2, Rb, Db, 1e-12f));
      x = a.y2;
    }
    // pooler: txt = tanh(x[:, 0] Wp^T + bp), x's first-token rows at strides (Rb*Db, Tb*Db, 1)
    FLR_TRY(linear(x, Rb * Db, Tb_ * Db, B_, p_poolw_, p_poolb_, txt_, FLR_ACT_TANH, nullptr, nullptr));
    // ---- fusion head (ClientMLP over the column blocks [img | txt]) ----
    const int64_t Din = Dv + Db;
    FLR_TRY(gemm(yf_, Rv * Dv, Tv_ * Dv, 1, W(p_f1w_), F_ * Din, Din, 1, h1_, B_ * F_, F_, 1, W(p_f1b_), F_, nullptr,
                 FLR_ACT_NONE, nullptr, nullptr, nullptr, B_, F_, Dv));
    FLR_TRY(gemm(txt_, B_ * Db, Db, 1, W(p_f1w_) + Dv, F_ * Din, Din, 1, h1_, B_ * F_, F_, 1, nullptr, 0, h1_,
                 FLR_ACT_RELU, mask, nullptr, nullptr, B_, F_, Db));
    FLR_TRY(linear(h1_, B_ * F_, F_, B_, p_f2w_, p_f2b_, logits_, FLR_ACT_NONE, nullptr, nullptr));
    if (!dry_) {
      FLR_TRY(flr_cross_entropy(logits_, labels, kc, B_, C_, loss_, dlogits_, rows_, st_));
      FLR_TRY(flr_copy_rows(loss_, kc, kc, loss_row, kc, 1, st_));
    }
    // ================= backward =================
    // ---- head (ClientMLP.backward, ReLU + dropout mask) ----
    FLR_TRY(gemm(dlogits_, B_ * C_, C_, 1, W(p_f2w_), C_ * F_, 1, F_, dpre_h_, B_ * F_, F_, 1, nullptr, 0, nullptr,
                 FLR_ACT_DRELU, mask, h1_, nullptr, B_, F_, C_));
    FLR_TRY(dweight(dlogits_, B_ * C_, C_, B_, h1_, B_ * F_, F_, G(p_f2w_), F_, F_));
    FLR_TRY(rowsum(dlogits_, B_ * C_, C_, B_, C_, G(p_f2b_)));
    FLR_TRY(gemm(dpre_h_, B_ * F_, F_, 1, W(p_f1w_), F_ * Din, 1, Din, dimg_, B_ * Dv, Dv, 1, nullptr, 0, nullptr,
                 FLR_ACT_NONE, nullptr, nullptr, nullptr, B_, Dv, F_));
    FLR_TRY(dweight(dpre_h_, B_ * F_, F_, B_, yf_, Rv * Dv, Tv_ * Dv, G(p_f1w_), Din, Dv));
    FLR_TRY(gemm(dpre_h_, B_ * F_, F_, 1, W(p_f1w_) + Dv, F_ * Din, 1, Din, dtxt_, B_ * Db, Db, 1, nullptr, 0,
                 nullptr, FLR_ACT_NONE, nullptr, nullptr, nullptr, B_, Db, F_));
    FLR_TRY(dweight(dpre_h_, B_ * F_, F_, B_, txt_, B_ * Db, Db, G(p_f1w_) + Dv, Din, Db));
    FLR_TRY(rowsum(dpre_h_, B_ * F_, F_, B_, F_, G(p_f1b_)));
    // ---- pooler (ClientLinearAct.backward, tanh) ----
    if (!dry_) FLR_TRY(flr_act_bwd(dtxt_, txt_, nullptr, FLR_ACT_DTANH, dpre_p_, kc * B_ * Db, st_));
    FLR_TRY(dinput(dpre_p_, B_, p_poolw_, Db, dxp_));
    FLR_TRY(dweight(dpre_p_, B_ * Db, Db, B_, x, Rb * Db, Tb_ * Db, G(p_poolw_), Db, Db));
    FLR_TRY(rowsum(dpre_p_, B_ * Db, Db, B_, Db, G(p_poolb_)));
    // the select's backward: zeros but the first-token rows
    float *bdx = bd_[0], *bdy2 = bd_[1], *bdm = bd_[2], *bdsum = bd_[3], *bd1 = bd_[4], *bdc = bd_[5];
    if (!dry_) {
      FLR_TRY(flr_fill(bdx, kc * Rb * Db, 0.f, st_));
      FLR_TRY(flr_copy_rows(dxp_, Db, Db, bdx, Tb_ * Db, kc * B_, st_));
    }
    // ---- BERT layers, last first; bdx = dL/d(layer output) ----
    // With the weight-gradient stream, layer i's weight / bias gradients run on it (as the
    // ViT layers' below): what they read (d(f), dpre, d(attn), dqkv) alternates between two
    // copies, rewritten two layers later after the caller's stream waited on that layer.
    wev_ = 0;
    side_ = wgs_ != nullptr && !dry_ && vl_.size() <= 64 && bl_.size() <= 64 &&
            5 * (vl_.size() + bl_.size()) <= (size_t)WgradStream::NEV;
    hipEvent_t bdone[64];
    int bit = 0;
    for (int i = (int)bl_.size() - 1; i >= 0; --i, ++bit) {
      const Layer& L = bl_[i];
      LayerAct& a = ba_[i];
      const float* xin = i > 0 ? ba_[i - 1].y2 : xe_;
      if (use_side() && bit >= 2 && hipStreamWaitEvent(st_, bdone[(bit - 2) & 63], 0) != hipSuccess)
        return launch_status("train_vit_bert: weight-gradient join");
      const bool odd = use_side() && (bit & 1);
      float* by2 = odd ? bdy2b_ : bdy2;
      float* bp = odd ? bdp2_ : bdp_;
      float* b1 = odd ? bd1b_ : bd1;
      float* bq = odd ? bdq2_ : bdq_;
      FLR_TRY(ln_bwd(bdx, a.s2, L.ln2w, L.ln2b, a.mean2, a.rstd2, nullptr, by2, Rb, Db));  // d(y1) and d(f)
      FLR_TRY(mlp_bwd(by2, Rb, Db, Fb_, L, a.y1, a.pre, a.hm, bp, bdm));
      FLR_TRY(launch(add_kernel, kc * Rb * Db, by2, bdm, bdsum, kc * Rb * Db));  // y1 feeds LN2 and the MLP
      FLR_TRY(ln_bwd(bdsum, a.s1, L.ln1w, L.ln1b, a.mean1, a.rstd1, nullptr, b1, Rb, Db));  // d(x) and d(attn)
      if (use_side()) FLR_TRY(link(st_, wgs_->s));
      FLR_TRY(dinput(b1, Rb, L.projw, Db, bdc));
      FLR_TRY(dweight(b1, Rb * Db, Db, Rb, a.ctx, Rb * Db, Db, G(L.projw), Db, Db));
      FLR_TRY(rowsum(b1, Rb * Db, Db, Rb, Db, G(L.projb)));
      if (!dry_) FLR_TRY(flr_attention_bwd(a.qkv, a.ctx, bdc, a.lse, kc * B_, Tb_, s.bert_heads, 64, bq, st_));
      if (use_side()) FLR_TRY(link(st_, wgs_->s));
      FLR_TRY(dinput(bq, Rb, L.qkvw, Db, bdm));
      FLR_TRY(dweight(bq, Rb * 3 * Db, 3 * Db, Rb, xin, Rb * Db, Db, G(L.qkvw), Db, Db));
      FLR_TRY(rowsum(bq, Rb * 3 * Db, 3 * Db, Rb, 3 * Db, G(L.qkvb)));
      if (use_side()) FLR_TRY(mark(&bdone[bit & 63]));
      FLR_TRY(launch(add_kernel, kc * Rb * Db, b1, bdm, bdx, kc * Rb * Db));  // x feeds LN1 and qkv
    }
    if (use_side())
      for (int j = std::max(0, bit - 2); j < bit; ++j)
        if (hipStreamWaitEvent(st_, bdone[j & 63], 0) != hipSuccess)
          return launch_status("train_vit_bert: weight-gradient join");
    side_ = false;
    FLR_TRY(ln_bwd(bdx, e_, p_ew_, p_eb_, meane_, rstde_, nullptr, bdm, Rb, Db));
    if (!dry_) {
      // one flr_embedding_bwd per table (ClientEmbeddingSum.backward): word, type, position
      FLR_TRY(flr_embedding_bwd(bdm, tokens, Rb, kc, Rb, s.vocab, Db, G(p_word_), s.vocab * Db, 1, ews_, ews_n_,
                                st_));
      FLR_TRY(flr_embedding_bwd(bdm, type_ids_, 0, kc, Rb, 2, Db, G(p_type_), 2 * Db, 1, ews_, ews_n_, st_));
      FLR_TRY(flr_embedding_bwd(bdm, pos_ids_, 0, kc, Rb, s.bert_max_pos, Db, G(p_bpos_), s.bert_max_pos * Db, 1,
                                ews_, ews_n_, st_));
    } else {
      ews_n_ = std::max(ews_n_, flr_embedding_bwd_workspace(KC_, Rb));
    }
    // ---- ViT, last block first ----
    float *vdA = vd_[0], *vdB = vd_[1], *vdx2 = vd_[2], *vdm = vd_[3], *vdc = vd_[4], *vdh = vd_[5];
    if (!dry_) {
      FLR_TRY(flr_fill(vdm, kc * Rv * Dv, 0.f, st_));
      FLR_TRY(flr_copy_rows(dimg_, Dv, Dv, vdm, Tv_ * Dv, kc * B_, st_));
    }
    // the final LayerNorm: its dx is the gradient of both s (x) and the last MLP branch r
    FLR_TRY(ln_bwd(vdm, sf_, p_nw_, p_nb_, meanf_, rstdf_, nullptr, vdA, Rv, Dv));
    // With the weight-gradient stream, layer i's weight / bias gradients run on it beside
    // the data-gradient chain of layers i and i-1: the scratch they read (dL/dr in a ring
    // of three, d(attn), dqkv, the MLP's dpre in two copies) is rewritten only two layers
    // later, after the caller's stream waited on that layer's side events.
    // (wev_ continues from the BERT layers: one event set per pass)
    side_ = wgs_ != nullptr && !dry_ && vl_.size() <= 64 && bl_.size() <= 64 &&
            5 * (vl_.size() + bl_.size()) <= (size_t)WgradStream::NEV;
    float* ring[3] = {vdA, vdB, vdr3_};
    hipEvent_t done[64];
    int it = 0;
    for (int i = (int)vl_.size() - 1; i >= 0; --i, ++it) {
      const Layer& L = vl_[i];
      LayerAct& a = va_[i];
      if (use_side() && it >= 2 && hipStreamWaitEvent(st_, done[(it - 2) & 63], 0) != hipSuccess)
        return launch_status("train_vit_bert: weight-gradient join");
      vdA = use_side() ? ring[it % 3] : vdA;
      vdB = use_side() ? ring[(it + 1) % 3] : vdB;
      float* vx2 = use_side() && (it & 1) ? vdx2b_ : vdx2;
      float* vq = use_side() && (it & 1) ? vdq2_ : vdq_;
      float* vp = use_side() && (it & 1) ? vdp2_ : vdp_;
      // vdA = dL/d(s2_i) = dL/d(r_i): the next LayerNorm's dx
      FLR_TRY(mlp_bwd(vdA, Rv, Dv, Mv_, L, a.y2, a.pre, a.hm, vp, vdm));  // vdm = d(y2)
      FLR_TRY(ln_bwd(vdm, a.s2, L.ln2w, L.ln2b, a.mean2, a.rstd2, vdA, vx2, Rv, Dv));  // d(s_in) and d(attn)
      if (use_side()) FLR_TRY(link(st_, wgs_->s));
      FLR_TRY(dinput(vx2, Rv, L.projw, Dv, vdc));
      FLR_TRY(dweight(vx2, Rv * Dv, Dv, Rv, a.ctx, Rv * Dv, Dv, G(L.projw), Dv, Dv));
      FLR_TRY(rowsum(vx2, Rv * Dv, Dv, Rv, Dv, G(L.projb)));
      if (!dry_) FLR_TRY(flr_attention_bwd(a.qkv, a.ctx, vdc, a.lse, kc * B_, Tv_, s.vit_heads, 64, vq, st_));
      if (use_side()) FLR_TRY(link(st_, wgs_->s));
      FLR_TRY(dinput(vq, Rv, L.qkvw, Dv, vdh));
      FLR_TRY(dweight(vq, Rv * 3 * Dv, 3 * Dv, Rv, a.h, Rv * Dv, Dv, G(L.qkvw), Dv, Dv));
      FLR_TRY(rowsum(vq, Rv * 3 * Dv, 3 * Dv, Rv, 3 * Dv, G(L.qkvb)));
      if (use_side()) FLR_TRY(mark(&done[it & 63]));
      if (i > 0) {
        // LN1 with the residual: ds = vdx2 (s1 feeds LN2 only); dx -> d(s2_{i-1}) = d(r_{i-1})
        FLR_TRY(ln_bwd(vdh, a.s1, L.ln1w, L.ln1b, a.mean1, a.rstd1, vx2, vdB, Rv, Dv));
        std::swap(vdA, vdB);
      } else {
        // block 0: x0 feeds LN1 (no residual) and LN2 (as x): the two paths summed (into
        // vdA, which this layer's side work reads: joined first)
        FLR_TRY(ln_bwd(vdh, x0_, L.ln1w, L.ln1b, a.mean1, a.rstd1, nullptr, vdB, Rv, Dv));
        if (use_side() && hipStreamWaitEvent(st_, done[it & 63], 0) != hipSuccess)
          return launch_status("train_vit_bert: weight-gradient join");
        FLR_TRY(launch(add_kernel, kc * Rv * Dv, vdB, vx2, vdA, kc * Rv * Dv));
      }
    }
    // every side event of the layers joined (the last two were not waited on yet)
    if (use_side())
      for (int j = std::max(0, it - 2); j < it; ++j)
        if (hipStreamWaitEvent(st_, done[j & 63], 0) != hipSuccess)
          return launch_status("train_vit_bert: weight-gradient join");
    side_ = false;
    // ClientViTTokens.backward: dpos / dcls = sums over the batch rows, dtok = the patch rows
    if (!dry_) {
      FLR_TRY(flr_sum_rows(vdA, Rv * Dv, Tv_ * Dv, kc, B_, Tv_ * Dv, G(p_pos_), Tv_ * Dv, st_));
      FLR_TRY(flr_sum_rows(vdA, Rv * Dv, Tv_ * Dv, kc, B_, Dv, G(p_cls_), Dv, st_));
      FLR_TRY(flr_copy_rows(vdA + Dv, Tv_ * Dv, NP_ * Dv, dtok_, NP_ * Dv, kc * B_, st_));
    }
    // patch embedding (ClientLinear.backward; the patches need no gradient)
    FLR_TRY(dweight(dtok_, BNP * Dv, Dv, BNP, patches_, BNP * Cpp_, Cpp_, G(p_pew_), Cpp_, Cpp_));
    FLR_TRY(rowsum(dtok_, BNP * Dv, Dv, BNP, Dv, G(p_peb_)));
#undef FLR_TRY
    return FLR_OK;
  }

  // ClientMLP.backward (GELU, one input block): dy -> dW2, db2, dW1, db1 and dx
  int mlp_bwd(const float* dy, int64_t M, int64_t D, int64_t Fh, const Layer& L, const float* x, const float* pre,
              const float* hm, float* dpre, float* dx) {
    int rc;
    if (use_side() && (rc = link(st_, wgs_->s)) != FLR_OK) return rc;  // dy ready
    if ((rc = gemm(dy, M * D, D, 1, W(L.fc2w), D * Fh, 1, Fh, dpre, M * Fh, Fh, 1, nullptr, 0, nullptr,
                   FLR_ACT_DGELU, nullptr, pre, nullptr, M, Fh, D)) != FLR_OK)
      return rc;
    if ((rc = dweight(dy, M * D, D, M, hm, M * Fh, Fh, G(L.fc2w), Fh, Fh)) != FLR_OK) return rc;
    if ((rc = rowsum(dy, M * D, D, M, D, G(L.fc2b))) != FLR_OK) return rc;
    if (use_side() && (rc = link(st_, wgs_->s)) != FLR_OK) return rc;  // dpre ready
    if ((rc = dinput(dpre, M, L.fc1w, D, dx)) != FLR_OK) return rc;
    if ((rc = dweight(dpre, M * Fh, Fh, M, x, M * D, D, G(L.fc1w), D, D)) != FLR_OK) return rc;
    return rowsum(dpre, M * Fh, Fh, M, Fh, G(L.fc1b));
  }

  // y [kc][M][out] = act(x W^T + b) (ClientLinear / ClientLinearAct forward);
  // x rows at client stride xk, row stride xm
  int linear(const float* x, int64_t xk, int64_t xm, int64_t M, int pw, int pb, float* y, int act, const float* mul,
             float* pre) {
    const Param& w = ps_[pw];
    const int64_t out = w.shape[0], in = w.shape[1];
    return gemm(x, xk, xm, 1, W(pw), w.n, in, 1, y, M * out, out, 1, pb >= 0 ? W(pb) : nullptr, out, nullptr, act,
                mul, nullptr, pre, M, out, in);
  }
  // dx [kc][M][in] = dy W (contiguous dy [kc][M][out])
  int dinput(const float* dy, int64_t M, int pw, int64_t in, float* dx) {
    const Param& w = ps_[pw];
    const int64_t out = w.shape[0];
    return gemm(dy, M * out, out, 1, W(pw), w.n, 1, in, dx, M * in, in, 1, nullptr, 0, nullptr, FLR_ACT_NONE, nullptr,
                nullptr, nullptr, M, in, out);
  }
  // dW [kc][out][in] (row stride ldw) = dy^T x: dy [kc][M][out] (client stride dyk, row stride out),
  // x rows at client stride xk / row stride xm
  int dweight(const float* dy, int64_t dyk, int64_t out, int64_t M, const float* x, int64_t xk, int64_t xm,
              float* dW, int64_t ldw, int64_t in) {
    // the gradient block's client stride: the parameter's numel (out x ldw)
    if (use_side()) return gemm_side(dy, dyk, 1, out, x, xk, 1, xm, dW, out * ldw, ldw, 1, out, in, M);
    return gemm(dy, dyk, 1, out, x, xk, 1, xm, dW, out * ldw, ldw, 1, nullptr, 0, nullptr, FLR_ACT_NONE, nullptr,
                nullptr, nullptr, out, in, M);
  }
  int gemm(const float* A, int64_t ak, int64_t am, int64_t ar, const float* Bm, int64_t bk, int64_t bn, int64_t br,
           float* C, int64_t ck, int64_t cm, int64_t cn, const float* bias, int64_t bias_k, const float* add, int act,
           const float* mul, const float* aux, float* pre, int64_t M, int64_t N, int64_t R) {
    if (dry_) {
      gws_n_ = std::max(gws_n_, flr_bgemm_workspace(KC_, M, N, R));
      return FLR_OK;
    }
    return flr_bgemm_ex(A, ak, am, ar, Bm, bk, bn, br, C, ck, cm, cn, bias, bias_k, add, act, mul, aux, pre, kc_, M,
                        N, R, gws_, gws_n_, st_);
  }
  // the weight-gradient stream's GEMM and row sums (its own workspaces)
  int gemm_side(const float* A, int64_t ak, int64_t am, int64_t ar, const float* Bm, int64_t bk, int64_t bn,
                int64_t br, float* C, int64_t ck, int64_t cm, int64_t cn, int64_t M, int64_t N, int64_t R) {
    return flr_bgemm_ex(A, ak, am, ar, Bm, bk, bn, br, C, ck, cm, cn, nullptr, 0, nullptr, FLR_ACT_NONE, nullptr,
                        nullptr, nullptr, kc_, M, N, R, gws2_, gws_n_, wgs_->s);
  }
  // event e recorded on `from`; `to` waits on it
  int link(hipStream_t from, hipStream_t to) {
    if (wev_ >= WgradStream::NEV) return FLR_ERR_UNSUPPORTED;
    hipEvent_t e = wgs_->ev[wev_++];
    if (hipEventRecord(e, from) != hipSuccess || hipStreamWaitEvent(to, e, 0) != hipSuccess)
      return launch_status("train_vit_bert: weight-gradient stream event");
    return FLR_OK;
  }
  // the layer's side work so far, as an event the caller waits on later
  int mark(hipEvent_t* out) {
    if (wev_ >= WgradStream::NEV) return FLR_ERR_UNSUPPORTED;
    *out = wgs_->ev[wev_++];
    return hipEventRecord(*out, wgs_->s) == hipSuccess ? FLR_OK : launch_status("train_vit_bert: side mark");
  }
  bool use_side() const { return side_ && wgs_ && !dry_; }
  int rowsum(const float* X, int64_t xk, int64_t xm, int64_t M, int64_t N, float* out) {
    if (dry_) {
      rws_n_ = std::max(rws_n_, flr_sum_rows_workspace(KC_, M, N));
      return FLR_OK;
    }
    if (use_side()) return flr_sum_rows_ex(X, xk, xm, kc_, M, N, out, N, rws2_, rws_n_, wgs_->s);
    return flr_sum_rows_ex(X, xk, xm, kc_, M, N, out, N, rws_, rws_n_, st_);
  }
  int ln_fwd(const float* x, const float* res, int pg, int pb, float* y, float* s_out, float* mean, float* rstd,
             int64_t R, int64_t D, float eps) {
    if (dry_) return FLR_OK;
    return flr_layernorm_fwd(x, D, res, D, W(pg), W(pb), y, D, s_out, D, mean, rstd, kc_ * R, D, R, eps, st_);
  }
  int ln_bwd(const float* dy, const float* s, int pg, int pb, const float* mean, const float* rstd,
             const float* dskip, float* dx, int64_t R, int64_t D) {
    if (dry_) {
      lws_n_ = std::max(lws_n_, flr_layernorm_bwd_workspace(KC_, R, D));
      return FLR_OK;
    }
    return flr_layernorm_bwd(dy, D, s, D, W(pg), mean, rstd, dskip, D, dx, D, G(pg), G(pb), kc_, R, D, lws_, lws_n_,
                             st_);
  }
  template <class... KArgs, class... Args>
  int launch(void (*k)(KArgs...), int64_t n, Args... args) {
    if (dry_) return FLR_OK;
    hipLaunchKernelGGL(k, dim3(grid_for(n)), dim3(THREADS), 0, st_, args...);
    return launch_status("train_vit_bert");
  }

  // parameter j of the pass's first client (client stride numel), its gradient block
  float* W(int j) const { return ps_[j].w + c0_ * ps_[j].n; }
  float* G(int j) const { return ps_[j].g; }

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
  Layer add_layer(const std::string& pre, int64_t D, int64_t Fh) {
    Layer L;
    L.ln1w = add_param(pre + "ln1.weight", {D});
    L.ln1b = add_param(pre + "ln1.bias", {D});
    L.qkvw = add_param(pre + "qkv.weight", {3 * D, D});
    L.qkvb = add_param(pre + "qkv.bias", {3 * D});
    L.projw = add_param(pre + "proj.weight", {D, D});
    L.projb = add_param(pre + "proj.bias", {D});
    L.ln2w = add_param(pre + "ln2.weight", {D});
    L.ln2b = add_param(pre + "ln2.bias", {D});
    L.fc1w = add_param(pre + "fc1.weight", {Fh, D});
    L.fc1b = add_param(pre + "fc1.bias", {Fh});
    L.fc2w = add_param(pre + "fc2.weight", {D, Fh});
    L.fc2b = add_param(pre + "fc2.bias", {D});
    return L;
  }
  void stats(LayerAct& a, int64_t rows) {
    a.mean1 = alloc<float>(rows);
    a.rstd1 = alloc<float>(rows);
    a.mean2 = alloc<float>(rows);
    a.rstd2 = alloc<float>(rows);
  }

  flr_vit_bert_spec s_;
  int64_t K_, B_, KC_, steps_;
  char* base_;
  size_t off_ = 0;
  bool dry_ = false;
  int64_t c0_ = 0, kc_ = 0;
  hipStream_t st_ = nullptr;
  std::vector<Param> ps_;
  std::vector<Layer> vl_, bl_;
  std::vector<LayerAct> va_, ba_;
  int64_t Dv_ = 0, Db_ = 0, Mv_ = 0, Fb_ = 0, F_ = 0, C_ = 0, Tb_ = 0, G_ = 0, NP_ = 0, Tv_ = 0, Cpp_ = 0, P_ = 0;
  int p_cls_ = 0, p_pos_ = 0, p_pew_ = 0, p_peb_ = 0, p_nw_ = 0, p_nb_ = 0, p_word_ = 0, p_bpos_ = 0, p_type_ = 0,
      p_ew_ = 0, p_eb_ = 0, p_poolw_ = 0, p_poolb_ = 0, p_f1w_ = 0, p_f1b_ = 0, p_f2w_ = 0, p_f2b_ = 0;
  char *sgd_ws_ = nullptr, *gws_ = nullptr, *rws_ = nullptr, *lws_ = nullptr, *ews_ = nullptr;
  size_t sgd_ws_n_ = 0, gws_n_ = 0, rws_n_ = 0, lws_n_ = 0, ews_n_ = 0;
  float *patches_ = nullptr, *tok_ = nullptr, *x0_ = nullptr, *sf_ = nullptr, *yf_ = nullptr, *meanf_ = nullptr,
        *rstdf_ = nullptr, *va_tmp_ = nullptr;
  int64_t *type_ids_ = nullptr, *pos_ids_ = nullptr;
  float *e_ = nullptr, *xe_ = nullptr, *meane_ = nullptr, *rstde_ = nullptr, *ba_tmp_ = nullptr;
  float *txt_ = nullptr, *h1_ = nullptr, *logits_ = nullptr, *dlogits_ = nullptr, *rows_ = nullptr, *loss_ = nullptr;
  float *dpre_h_ = nullptr, *dimg_ = nullptr, *dtxt_ = nullptr, *dpre_p_ = nullptr, *dxp_ = nullptr;
  float* vd_[6] = {};
  float *vdq_ = nullptr, *vdp_ = nullptr, *dtok_ = nullptr;
  float *vdq2_ = nullptr, *vdp2_ = nullptr, *vdx2b_ = nullptr, *vdr3_ = nullptr;
  char *gws2_ = nullptr, *rws2_ = nullptr;
  WgradStream* wgs_ = nullptr;  // the weight-gradient stream (nullptr: everything on st_)
  bool side_ = false;           // route dweight / rowsum to it (set around the ViT layers)
  int wev_ = 0;                 // events used this pass
  float* bd_[6] = {};
  float *bdq_ = nullptr, *bdp_ = nullptr;
  float *bdq2_ = nullptr, *bdp2_ = nullptr, *bdy2b_ = nullptr, *bd1b_ = nullptr;
};

inline int64_t auto_chunk(int64_t K, int64_t chunk) { return chunk > 0 ? std::min(chunk, K) : std::min<int64_t>(K, 32); }

}  // namespace tv
}  // namespace flr

using namespace flr;

extern "C" int64_t flr_vit_bert_num_params(const flr_vit_bert_spec* spec) {
  if (!spec) return -1;
  tv::Net net(*spec, 1, 1, 1, 1, nullptr);
  if (net.layout() != FLR_OK) return -1;
  return net.P();
}

extern "C" size_t flr_train_vit_bert_workspace(const flr_vit_bert_spec* spec, int64_t K, int64_t B, int64_t steps,
                                               int64_t chunk) {
  if (!spec || K < 1 || B < 1 || steps < 1 || chunk < 0) return 0;
  wgrad_stream(true);  // created here, before any capture of the training call
  tv::Net net(*spec, K, B, tv::auto_chunk(K, chunk), steps, nullptr);
  if (net.layout() != FLR_OK) return 0;
  return align_up(net.bytes(), 256) + align_up((size_t)steps * K * sizeof(float), 256) + 256;
}

extern "C" int flr_train_vit_bert(const flr_vit_bert_spec* spec, const float* global, float* X, int64_t ld,
                                  const float* images, const int64_t* tokens, const int64_t* labels,
                                  const float* dropout_masks, int64_t steps, int64_t K, int64_t B, float lr,
                                  float momentum, float weight_decay, float max_norm, int64_t nneg, float* loss_out,
                                  float* norms_out, unsigned flags, int64_t chunk, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (!spec || !global || !X || !images || !tokens || !labels || !loss_out || steps < 1 || K < 1 || B < 1 ||
      nneg < 0 || chunk < 0)
    return FLR_ERR_ARG;
  if (flags & ~(unsigned)FLR_TC_TRAIN_ORDER) return FLR_ERR_ARG;
  if (!workspace || workspace_bytes < flr_train_vit_bert_workspace(spec, K, B, steps, chunk)) return FLR_ERR_WORKSPACE;
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  const int64_t KC = tv::auto_chunk(K, chunk);
  tv::Net net(*spec, K, B, KC, steps, base);
  int rc = net.layout();
  if (rc != FLR_OK) return rc;
  if (ld < net.P()) return FLR_ERR_ARG;
  float* step_loss = reinterpret_cast<float*>(base + align_up(net.bytes(), 256));
  hipStream_t st = as_stream(stream);
  net.set_wgrad_stream(wgrad_stream(true, st));
  // every client starts from the global model (run_experiments.py:203); the
  // family has no layout change, so training order is the parameters() order
  if ((rc = net.load_global(global, st)) != FLR_OK) return rc;
  const int64_t img = spec->in_channels * spec->image_size * spec->image_size, T = spec->seq_len;
  for (int64_t s = 0; s < steps; ++s)
    for (int64_t c0 = 0; c0 < K; c0 += KC) {
      const int64_t kc = std::min(KC, K - c0), r0 = s * K + c0;
      rc = net.step(images + r0 * B * img, tokens + r0 * B * T, labels + r0 * B,
                    dropout_masks ? dropout_masks + r0 * B * spec->fusion : nullptr, c0, kc, s == 0, s == steps - 1,
                    step_loss + r0, lr, momentum, weight_decay, max_norm, X, ld, nneg, norms_out, st);
      if (rc != FLR_OK) return rc;
    }
  return flr_mean_rows(step_loss, steps, K, loss_out, st);
}
