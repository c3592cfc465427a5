/*
 * gvl.h — C-ABI of libgvl, the MI355X (gfx950) kernel library behind the
 * gpt2-vision-language drop-in modules.
 *
 * The reference (theophile-lt/gpt2-vision-language) is pure Python/PyTorch: its
 * operator boundary is the ATen op set its nn.Modules call.  Each
 * entry point below replaces one or more of those ATen calls; the reference call
 * site it stands in for is cited as file:line into /root/reference.
 *
 * Conventions (all entry points):
 *   - plain device pointers + int64 sizes/strides (in ELEMENTS), no torch types;
 *   - bf16 tensors are raw 16-bit words; fp32 where stated;
 *   - `stream` is a hipStream_t (the caller's torch.cuda.current_stream());
 *   - return 0 on success, -1 on a rejected argument (shape/alignment),
 *     -2 on a HIP launch error; gvl_last_error() returns the thread-local text;
 *   - the library allocates nothing: every buffer and workspace is owned by the
 *     caller (sizes from the *_workspace_size queries); no entry point
 *     synchronises the device, so every call is capturable into a hipGraph.
 */
#ifndef GVL_H_
#define GVL_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GVL_ABI_VERSION 14

/* Dropout seeds: every dropout mask is rng(seed_eff, element index) with
 * seed_eff = seed when seed_ptr is NULL or *seed_ptr == 0, else seed ^ mix64(*seed_ptr).
 * A training step captured into a hipGraph keeps its host seeds frozen; advancing the
 * device-side offset once per replay gives every step fresh masks (forward and backward
 * of one step read the same offset, so they agree). */

typedef void* gvl_stream_t;

const char* gvl_last_error(void);
int gvl_abi_version(void);
/* Measurement hook (bench.py roofline): arm a (start, stop) pair of timing-enabled
 * hipEvent_t for the calling thread; the main kernel of the next gvl_gemm / gvl_attn_fwd /
 * gvl_attn_bwd call on this thread is launched with hipExtLaunchKernelGGL bound to them, so
 * hipEventElapsedTime gives that kernel's execution time as its dispatch records it.  Not
 * for use under hipGraph capture. */
int gvl_set_launch_events(void* start, void* stop);

/* ------------------------------------------------------------------------- */
/* GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16), fp32 accumulate, fused epilogue.
 *   C[m][n] = epi( alpha * sum_k opA[m][k] * opB[k][n] )
 *   opA: a_mn=0 -> A stored [M][K] (row stride lda);  a_mn=1 -> A stored [K][M].
 *   opB: b_mn=0 -> B stored [N][K] (nn.Linear weight); b_mn=1 -> B stored [K][N].
 * Epilogue order: *alpha_ptr, +bias[n], *dgelu(pre_in), {pre_out=v; v=gelu(v)},
 *   (with gate and no act, pre_out receives the un-gated branch),
 *   dropout(p, seed, index m*N+n), *tanh(*gate), +residual, store (bf16 or fp32).
 * Replaces: nn.Linear forward/backward (addmm/mm) at source/gpt2/train_gpt2.py:26-27,
 *   50-58,96-97; gpt2_linear/model.py:125-129,172; gpt2_cross-att/model.py:39-41,81;
 *   gpt2_q_former/model.py:119-130,151 and the gelu/dropout/residual adds around them. */
typedef struct gvl_gemm_desc {
  const void* a;
  const void* b;
  void* c;
  int64_t m, n, k;
  int64_t lda, ldb, ldc;
  int32_t a_mn, b_mn;
  float alpha;
  const float* alpha_ptr; /* optional fp32 device scalar multiplied into alpha */
  const void* bias;       /* optional bf16 [N] */
  int32_t act;            /* 0 none, 1 gelu-tanh, 2 gelu-erf (pre_out <- x);
                             3 gelu-tanh, 4 gelu-erf with pre_out <- gelu'(x) (ABI v4);
                             5 quick-GELU x sigmoid(1.702 x), needs bias, no pre_out, no dact
                             (ABI v14: the frozen CLIP tower's fc1, gvl/clip.py) */
  int32_t dact;           /* 0 none, 1 dgelu-tanh, 2 dgelu-erf (of pre_in = x);
                             3: multiply by pre_in = gelu'(x) as stored by act 3/4 (ABI v4) */
  void* pre_out;          /* optional bf16 [M][ldp]: value before activation */
  const void* pre_in;     /* bf16 [M][ldp]: pre-activation for dact */
  int64_t ldp;
  const void* residual;   /* optional bf16 [M][ldr], may alias c */
  int64_t ldr;
  const void* gate;       /* optional bf16 scalar g: branch *= tanh(g) */
  float drop_p;           /* dropout probability on the branch (0 = off) */
  uint64_t seed;
  int32_t c_fp32;         /* 1: C is fp32 */
  void* workspace;        /* optional fp32 scratch for split-K (few output tiles, long K) */
  int64_t workspace_bytes;
  const uint64_t* seed_ptr; /* optional device step offset re-keying `seed` (see below) */
  /* ABI v5: optional arrival tickets for the in-launch two-way split-K combine (the two
   * K-halves of an output tile meet inside one launch; no separate reduce kernel).  The
   * caller allocates them zero-filled once; every call leaves them zero again.  Needs
   * ticket_count >= 8 * output tiles of the split GEMM; fewer -> the two-kernel path. */
  uint32_t* tickets;
  int64_t ticket_count;
} gvl_gemm_desc;
int gvl_gemm(const gvl_gemm_desc* d, gvl_stream_t stream);
/* count (<= 16) GEMMs of one shape and layout that differ only in a, b, c (and residual,
 * which is null for all or equal to c for all: C += AB) as ONE persistent launch: the
 * weight gradients of the 12 GPT-2 blocks of a micro-step (source/gpt2/train_gpt2.py:471,
 * loss.backward() -> the nn.Linear weight grads of every Block), each of which alone is too
 * few output tiles to fill the chip.  Other epilogues / shapes run one by one. */
int gvl_gemm_batched(const gvl_gemm_desc* d, int32_t count, gvl_stream_t stream);
/* As gvl_gemm_batched for weight gradients (a_mn = b_mn = 1, residual == c) that also add
 * each problem's bias gradient: dbias[i] (bf16 [m]) += row sums of A_i^T over k, i.e. the
 * column sums of dY — the nn.Linear bias grad beside its weight grad, computed from the same
 * operand tiles (no second pass over dY).  Returns -1 when the batch cannot run fused and
 * nothing was launched (the caller then uses gvl_gemm_batched + gvl_colsum_batched); any other
 * non-zero return is a launch failure after the GEMM may have added into C (fatal). */
int gvl_gemm_batched_dbias(const gvl_gemm_desc* d, void* const* dbias, int32_t count,
                           gvl_stream_t stream);
/* ABI v9: weight gradients of DIFFERENT shapes in one launch — the Q-Former bridge's deferred
 * nn.Linear weight grads of one backward (source/gpt2_q_former/model.py:114-168, the
 * out_proj / MLP Linears' grads that loss.backward() produces, each too few output tiles to
 * fill the chip alone): each problem a_mn = b_mn = 1, residual == c (C += dY^T X), the same
 * alpha; dbias[i] (bf16 [m], may be null; the array may be null) += column sums of dY_i.
 * count <= 48 (round 4: also every GPT-2 block's four weight grads of one LM backward flush,
 * train_gpt2.py:55-59,71-74, sizes and strides < 2^30).
 * ABI v11: a problem's alpha_ptr may be set (the tied lm_head's weight grad, scaled by the
 * device scalar dloss / count, train_gpt2.py:469 + the reference's loss scaling): every non-null
 * alpha_ptr of one call must be the same pointer; those problems get alpha * *alpha_ptr, the
 * others alpha.
 * Returns 0 when launched, -1 when the problems do not qualify and nothing was launched. */
int gvl_gemm_grouped(const gvl_gemm_desc* d, void* const* dbias, int32_t count,
                     gvl_stream_t stream);
/* Process-wide GEMM implementation knob (benchmarking / A-B tests; env GVL_GEMM_IMPL):
 * impl 3 (default) = persistent ping-pong 256x256 kernel (split-K for few tiles) where
 * the work items fill the chip, else the 128x128 LDS-DMA ring; 2 = ring / non-persistent
 * ping-pong family; 1 = LDS-DMA v2 (K % 64 == 0); 0 = register-staged kernel always.
 * cfg -1 = pick by shape; otherwise forces a tile config of the family (impl 2: 0 = 256x256,
 * 1 = 256x128, 2 = 128x128, 3 = 256x256/5 slots, 4/5 = ping-pong, 6 = 64x128); impl 3:
 * cfg 3 forces the persistent kernel, 10 the four-wave narrow-output kernels (192x128 /
 * 128x128 tiles, direct-A where K % 384 == 0) where they apply, 11 = default routing without
 * them (and without the AGPR four-wave kernel), 12 (ABI v8, round 4) the AGPR four-wave kernel
 * (gemm_w4x.hip: 256 x 192 / 128 x 192 tiles, K-contiguous A, plain or bias + residual) where
 * it applies; 13 (ABI v10) = cfg 11 with the persistent kernel's in-launch two-way combine
 * enabled for single GEMMs (tests; otherwise only with env GVL_PP3_COMBINE=1, since the
 * callers' tickets are passed to every gvl_gemm by gvl.kernels); other cfg values route as -1.  impl 4 (the removed 64-deep quadrant-phase
 * kernel) is rejected. */
int gvl_gemm_tune(int32_t impl, int32_t cfg);
/* Name of the kernel template instance gvl_gemm would launch for d (profiling: lets a
 * caller attribute event timings to the rocprofv3 kernel-trace rows). */
int gvl_gemm_kernel_name(const gvl_gemm_desc* d, char* buf, int32_t len);
/* ABI v7: name of the kernel instance the calling thread's last gvl_gemm_batched /
 * gvl_gemm_batched_dbias call launched as one batched launch ("" when it ran the problems one
 * by one through gvl_gemm): the bench attributes the batched weight-gradient launches too. */
int gvl_gemm_batched_kernel_name(char* buf, int32_t len);
/* (ABI v8-v9 had gvl_gemm_lib_route: plain N = 768 GEMMs handed to hipBLASLt.  Removed in
 * ABI v10: every GEMM runs on libgvl's own kernels; libgvl links no vendor BLAS.) */

/* ------------------------------------------------------------------------- */
/* LayerNorm over the last dim (eps given; reference uses 1e-5).
 * Replaces nn.LayerNorm at source/gpt2/train_gpt2.py:66,68,94 (ln_1/ln_2/ln_f),
 * gpt2_cross-att/model.py:91 (ln_x), gpt2_q_former/model.py:118-125. */
int gvl_layernorm_fwd(const void* x, int64_t ldx, const void* w, const void* b,
                      void* y, int64_t ldy, float* mean, float* rstd,
                      int64_t rows, int64_t cols, float eps, gvl_stream_t stream);
/* dx (bf16) = LN'(dy); if accumulate_dx, dx += result (residual-stream grad).
 * dw/db (bf16, optional) get column sums; they need workspace
 * gvl_layernorm_bwd_workspace_size(rows, cols) bytes. accumulate_wb adds into dw/db. */
int64_t gvl_layernorm_bwd_workspace_size(int64_t rows, int64_t cols);
int gvl_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx,
                      const void* w, const float* mean, const float* rstd,
                      void* dx, int64_t lddx, int32_t accumulate_dx,
                      void* dw, void* db, int32_t accumulate_wb, void* workspace,
                      int64_t rows, int64_t cols, gvl_stream_t stream);
/* ABI v12: accumulate_wb bit 1 (value 2 | accumulate) defers the dw / db column sums: the
 * per-block partials stay in `workspace` (gvl_layernorm_bwd_blocks(rows) blocks of 2 * cols
 * floats) and dw / db are left untouched; one gvl_layernorm_bwd_finalize_batched launch later
 * reduces up to 64 such workspaces of one width into their dw[i] / db[i] (either may be null),
 * adding into them when accumulate_wb bit 0 is set — the end-of-backward flush of every
 * LayerNorm weight grad of a GPT-2 micro-step (train_gpt2.py:66,68,94) in one launch instead
 * of 25. */
int32_t gvl_layernorm_bwd_blocks(int64_t rows);
int gvl_layernorm_bwd_finalize_batched(const float* const* ws, const int32_t* nblk, int32_t count,
                                       int64_t cols, void* const* dw, void* const* db,
                                       int32_t accumulate_wb, gvl_stream_t stream);
/* dx = res + LayerNorm backward (the residual-stream gradient of a pre-LN block:
 * source/gpt2/train_gpt2.py:72-73, x + attn(ln_1(x)) / x + mlp(ln_2(x))) with the residual
 * read from its own buffer, so the caller needs no copy of it; otherwise as above. */
int gvl_layernorm_bwd_res(const void* dy, int64_t lddy, const void* x, int64_t ldx,
                          const void* w, const float* mean, const float* rstd,
                          const void* res, int64_t ldr, void* dx, int64_t lddx,
                          void* dw, void* db, int32_t accumulate_wb, void* workspace,
                          int64_t rows, int64_t cols, gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Fused attention, head dim 64, bf16 in/out, fp32 online softmax.
 * q/k/v/o element (b,t,h,d) at ptr + b*s_b + t*s_t + h*s_h + d, so the packed
 * c_attn output [B,T,3C] is consumed in place and o is written as [B,T,C]
 * (the transpose(1,2).contiguous() of the reference is fused away).
 * Replaces F.scaled_dot_product_attention at source/gpt2/train_gpt2.py:40 (causal),
 * gpt2_cross-att/model.py:55 (non-causal bridge cross-attention) and the
 * nn.MultiheadAttention core at gpt2_q_former/model.py:135,140 (attention-prob
 * dropout p; need_weights output is discarded by the reference and not produced). */
typedef struct gvl_attn_desc {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse; /* fp32 [B][H][Tq], natural-log row logsumexp of scale*q.k */
  int64_t B, H, Tq, Tk;
  int64_t q_sb, q_st, q_sh;
  int64_t k_sb, k_st, k_sh;
  int64_t v_sb, v_st, v_sh;
  int64_t o_sb, o_st, o_sh;
  int32_t causal;
  float scale;
  float drop_p;
  uint64_t seed;
  const uint64_t* seed_ptr; /* optional device step offset re-keying `seed` */
} gvl_attn_desc;
int gvl_attn_fwd(const gvl_attn_desc* d, gvl_stream_t stream);
/* Backward: dO has the layout of o (do_* strides); dq/dk/dv the layouts of q/k/v
 * (dq_*, dk_*, dv_* strides).  workspace: gvl_attn_bwd_workspace_size bytes. */
typedef struct gvl_attn_bwd_desc {
  const void* dout;
  int64_t do_sb, do_st, do_sh;
  void* dq;
  int64_t dq_sb, dq_st, dq_sh;
  void* dk;
  int64_t dk_sb, dk_st, dk_sh;
  void* dv;
  int64_t dv_sb, dv_st, dv_sh;
  void* workspace;
} gvl_attn_bwd_desc;
int64_t gvl_attn_bwd_workspace_size(const gvl_attn_desc* d);
int gvl_attn_bwd(const gvl_attn_desc* d, const gvl_attn_bwd_desc* g, gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Row-wise cross-entropy over bf16 logits (fp32 math), fused softmax gradient.
 * Logits row for target r: (r / rows_per_group) * group_stride + row_offset + r % rows_per_group
 * (lets the caption loss read logits[:, M:M+T] in place).  targets int64 with
 * ignore_index=-100; optional uint8 mask weights rows (cross-att masked mean).
 * `vocab` need not be a multiple of 8 (GPTConfig()'s 50257): ldl / ldd are multiples of 8
 * >= vocab rounded up to 8, and the pad columns read as -inf and get dlogits 0.  A
 * target outside [0, vocab) (other than -100) gives row_loss NaN, never an out-of-row read.
 * Writes row_loss[r] (fp32), dlogits[r] = softmax - onehot (bf16, unscaled, 0 for
 * ignored rows, row stride ldd) and out[0]=mean loss, out[1]=1/count (count
 * clamped to >=1 when mask_mode, torch 0/0 semantics otherwise).
 * Replaces F.cross_entropy at source/gpt2/train_gpt2.py:124, gpt2_linear/model.py:206-210,
 * gpt2_cross-att/model.py:170-185. */
int gvl_cross_entropy(const void* logits, int64_t ldl, int64_t rows, int64_t vocab,
                      int64_t rows_per_group, int64_t group_stride, int64_t row_offset,
                      const int64_t* targets, const uint8_t* mask, int32_t mask_mode,
                      float* row_loss, void* dlogits, int64_t ldd, float* out,
                      gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Token + position embedding gather: out[row(r)] = wte[idx[r]] + wpe[r % T],
 * row(r) = (r / T) * out_rows_per_seq + out_offset + r % T  (caption models write the
 * text embeddings after the M image tokens).  `vocab` = rows of wte: an id outside
 * [0, vocab) is never dereferenced (it embeds as row 0 / is dropped from the scatter);
 * callers check ids on the host first, as nn.Embedding raises on them (ABI v3).
 * Replaces nn.Embedding x2 + add (+cat) at source/gpt2/train_gpt2.py:114-117,
 * gpt2_linear/model.py:187-200, gpt2_cross-att/model.py:155-158. */
int gvl_embedding_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out,
                      int64_t n_tokens, int64_t T, int64_t C, int64_t vocab,
                      int64_t out_rows_per_seq, int64_t out_offset, gvl_stream_t stream);
/* Backward: fp32 scatter-add into dwte_acc [V][C] and dwpe_acc [T][C] (caller zeroes). */
int gvl_embedding_bwd(const int64_t* idx, const void* dout, float* dwte_acc, float* dwpe_acc,
                      int64_t n_tokens, int64_t T, int64_t C, int64_t vocab,
                      int64_t out_rows_per_seq, int64_t out_offset, gvl_stream_t stream);
/* ABI v6: deterministic embedding backward accumulated IN PLACE into bf16 gradients:
 * dwte[v] += sum of dout[row(r)] over the tokens r with idx[r] == v (summed in fp32 in token
 * order, one bf16 read-modify-write per touched row — no atomics, bit-identical run to run);
 * dwpe[t] += sum over sequences of dout[row(seq, t)].  Either pointer may be NULL.  The tied
 * wte's gradient is the lm_head weight gradient plus this (train_gpt2.py:114-117, :108 tying);
 * both accumulate into one arena gradient.  `keys`: uint32 scratch of
 * gvl_embedding_bwd_workspace(n_tokens) entries.  C % 8 == 0, C <= 1024, vocab < 2^18 - 1,
 * n_tokens % T == 0; ids outside [0, vocab) contribute nothing. */
/* ABI v6: grouped bf16 row copy: for g < G and t < T, dst row (g*dst_rows + dst_off + t) =
 * src row (g*src_rows + src_off + t) (src_rows = 0 broadcasts one block of T rows to every
 * group); with zero_rest the other dst_rows - T rows of each group are zeroed.  Replaces the
 * caption path's torch.cat of image tokens before the text embeddings
 * (gpt2_linear/model.py:191), query_tokens.expand (gpt2_q_former/model.py:160-161) and the
 * zero-filled [B, S, C] gradient around the text-row lm_head gradient (model.py:219-230). */
int gvl_copy_rows(const void* src, int64_t ld_src, int64_t src_rows, int64_t src_off, void* dst,
                  int64_t ld_dst, int64_t dst_rows, int64_t dst_off, int64_t T, int64_t G,
                  int64_t cols, int32_t zero_rest, gvl_stream_t stream);
int64_t gvl_embedding_bwd_workspace(int64_t n_tokens);
int gvl_embedding_bwd_det(const int64_t* idx, const void* dout, void* dwte, void* dwpe,
                          int64_t n_tokens, int64_t T, int64_t C, int64_t vocab,
                          int64_t out_rows_per_seq, int64_t out_offset, uint32_t* keys,
                          int64_t keys_count, gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* CLIP token pooling: [CLS] + adaptive_avg_pool2d(side x side -> 4 x 8) + L2 normalise
 * (eps 1e-12).  in: [B][1+side*side][D] (fp32 or bf16), out: [B][33][D] (fp32 or bf16).
 * Replaces pool_clip_197_to_33_avg_with_cls, gpt2_linear/model.py:240-254. */
int gvl_pool_clip(const void* in, int32_t in_fp32, void* out, int32_t out_fp32,
                  int64_t B, int64_t L, int64_t D, gvl_stream_t stream);
/* As gvl_pool_clip with the L2 normalisation optional (ABI v3): the pixel-input path pools
 * CLIP's layer-normed hidden states BEFORE the (linear, bias-free) visual projection — the
 * average commutes with it — so the projection runs on 33 tokens instead of 257, then
 * normalises with gvl_l2_normalize_rows (F.normalize(dim=-1, eps=1e-12), D <= 1024). */
int gvl_pool_clip_ex(const void* in, int32_t in_fp32, void* out, int32_t out_fp32, int64_t B,
                     int64_t L, int64_t D, int32_t normalize, gvl_stream_t stream);
int gvl_l2_normalize_rows(const void* in, void* out, int32_t fp32, int64_t rows, int64_t D,
                          gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Optimizer path over flat bf16 arenas (params / grads / exp_avg / exp_avg_sq).
 * gvl_grad_norm: out[0] = ||g||_2 (fp32), out[1] = clip coefficient
 *   min(1, max_norm / (norm + 1e-6)) — torch.nn.utils.clip_grad_norm_ at
 *   source/gpt2/train_gpt2.py:472.  workspace: gvl_grad_norm_workspace_size(n).
 * gvl_adamw: decoupled weight decay on elements [0, n_decay), none after; grads are
 *   multiplied by *grad_scale (the clip coefficient) on the fly; bias corrections use
 *   `step` (1-based) — torch.optim.AdamW(fused=True) at train_gpt2.py:140-143, :476. */
int64_t gvl_grad_norm_workspace_size(int64_t n);
int gvl_grad_norm(const void* g, int64_t n, float max_norm, void* workspace, float* out,
                  gvl_stream_t stream);
int gvl_adamw(void* p, const void* g, void* m, void* v, int64_t n, int64_t n_decay,
              float lr, float beta1, float beta2, float eps, float weight_decay,
              int64_t step, const float* grad_scale, gvl_stream_t stream);
/* As gvl_adamw with lr and the 1-based step read on the device from hyper[0], hyper[1]
 * (fp32): a step captured into a hipGraph stays correct across replays when the caller
 * advances `hyper` (param_groups[i]['lr'] written before each step, train_gpt2.py:474-476). */
int gvl_adamw_dev(void* p, const void* g, void* m, void* v, int64_t n, int64_t n_decay,
                  const float* hyper, float beta1, float beta2, float eps, float weight_decay,
                  const float* grad_scale, gvl_stream_t stream);

/* Mixed-precision form (gvl.optim.AdamW default): fp32 master weights p_master and fp32
 * moments m/v are updated; the bf16 compute copy p the model reads is written from the
 * new master (28 B/param).  Same math and device-side {lr, step} as gvl_adamw_dev.  Keeps
 * sub-ulp updates (LayerNorm gains ~1.0: bf16 ulp 2^-7 >> lr) that a bf16-only step
 * rounds away, so training follows the reference's fp32 path (ABI v3). */
int gvl_adamw_master_dev(void* p, float* p_master, const void* g, float* m, float* v, int64_t n,
                         int64_t n_decay, const float* hyper, float beta1, float beta2, float eps,
                         float weight_decay, const float* grad_scale, gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Incremental decoding (ABI v3).  gvl_attn_decode: one new query per sequence attends all Tk
 * cached keys (non-causal over the cache = causal for the newest position); q element
 * (b, h, d) at q + b*q_sb + h*64 + d, key t at k + b*k_sb + t*k_st + h*64 (same for v),
 * output o + b*o_sb + h*64.  Tk <= 4096.  Replaces the full-sequence recompute of the
 * reference's decode loops (train_gpt2.py:440-449, gpt2_linear/data.py:111-127) with a KV cache.
 * gvl_sample: per row, softmax(logits / temperature), keep the top_k largest (0 = all), then
 * the reference's top-p set (sorted cumulative probability before the token <= top_p, 1 =
 * all; gpt2_linear/data.py:117-122), and draw with the caller's uniform u[row] in [0, 1) by
 * inverse CDF in token-index order.  V <= 65536; out int64 [rows]. */
int gvl_attn_decode(const void* q, int64_t q_sb, const void* k, int64_t k_sb, int64_t k_st,
                    const void* v, int64_t v_sb, int64_t v_st, void* o, int64_t o_sb, int64_t B,
                    int64_t H, int64_t Tk, float scale, gvl_stream_t stream);
int gvl_sample(const void* logits, int64_t ld, int32_t logits_fp32, int64_t rows, int64_t V,
               float temperature, int32_t top_k, float top_p, const float* u, int64_t* out,
               gvl_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Small fused elementwise helpers on the hot path. */
/* Column sums of a bf16 [rows][cols] matrix (row stride ld) -> bf16 out[cols]
 * (bias gradients); accumulate adds into out. workspace: gvl_colsum_workspace_size. */
int64_t gvl_colsum_workspace_size(int64_t rows, int64_t cols);
int gvl_colsum(const void* x, int64_t rows, int64_t cols, int64_t ld, void* out,
               int32_t accumulate, void* workspace, gvl_stream_t stream);
/* count (<= 16) column sums of one shape in one launch pair: out[i] (+)= colsum(x[i]) — the
 * deferred bias gradients of the 12 GPT-2 blocks (train_gpt2.py:471, nn.Linear bias grads).
 * workspace: gvl_colsum_batched_workspace_size(count, rows, cols) bytes. */
int64_t gvl_colsum_batched_workspace_size(int32_t count, int64_t rows, int64_t cols);
int gvl_colsum_batched(const void* const* x, void* const* out, int32_t count, int64_t rows,
                       int64_t cols, int64_t ld, int32_t accumulate, void* workspace,
                       gvl_stream_t stream);
/* out[r][c] = in[r][c] * keep(seed, r*cols+c) / (1-p) — dropout backward, with the
 * same counter-based mask the GEMM epilogue applies. */
int gvl_dropout_mask_apply(const void* in, int64_t ld_in, void* out, int64_t ld_out,
                           int64_t rows, int64_t cols, float p, uint64_t seed,
                           const uint64_t* seed_ptr, gvl_stream_t stream);
/* out[i] = tanh(*gate) * in[i] and gate_grad (fp32 scalar, accumulated) +=
 * (1 - tanh^2) * sum_i in[i] * y[i] — backward of x + tanh(g) * y
 * (gpt2_cross-att/model.py:101). */
int gvl_gate_bwd(const void* dx, const void* y, const void* gate, void* dy, float* gate_grad,
                 int64_t n, void* workspace, gvl_stream_t stream);
int64_t gvl_gate_bwd_workspace_size(int64_t n);
/* ABI v13: as gvl_gate_bwd, the gate gradient added into the bf16 scalar gate_grad (the gate
 * parameter's own .grad): gate_grad = bf16(gate_grad + bf16(dgate)), the roundings of
 * autograd's AccumulateGrad on a bf16 parameter — no fp32 scalar, zero-fill or conversion. */
int gvl_gate_bwd_acc_bf16(const void* dx, const void* y, const void* gate, void* dy,
                          void* gate_grad, int64_t n, void* workspace, gvl_stream_t stream);
/* fp32 -> bf16 conversion with optional accumulate into the bf16 destination. */
int gvl_f32_to_bf16(const float* in, void* out, int64_t n, int32_t accumulate,
                    gvl_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GVL_H_ */
