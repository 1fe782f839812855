/*
 * rp_api.h — C ABI of librepurpose_amd.so, the MI355X (gfx950) HIP implementation of the
 * Repurpose tri-modal temporal-localisation hot path.
 *
 * Every entry point takes raw device pointers, sizes, leading dimensions and a hipStream_t
 * (passed as void*), enqueues asynchronously on that stream, never allocates or frees caller
 * memory, and returns 0 (RP_OK) or an RP_ERR_* code; rp_last_error() returns the message
 * (thread-local).  No torch types cross this boundary.
 *
 * Which reference interface each family replaces (paths relative to the reference repo):
 *   rp_concat_rows        torch.cat of the three modalities      models/MMCTransformer.py:118
 *   rp_gemm               nn.Linear fwd/dgrad/wgrad              models/MMCTransformer.py:32,121,63-93;
 *                         and MHA in_proj/out_proj, linear1/2 of the 16 nn.TransformerEncoderLayer
 *                         (constructed at models/MMCTransformer.py:41-55)
 *   rp_gemm_ln_fwd/bwd    Linear + residual + LayerNorm seams of the pre-LN encoder layers
 *                         models/MMCTransformer.py:41-55 (out_proj/linear2 -> norm2/norm1 and back)
 *   rp_layernorm_fwd/bwd  nn.LayerNorm (+ PE add, ReLU, dropout)  models/MMCTransformer.py:35,124,127,
 *                         58,141,65,72,84; encoder-layer norm1/norm2
 *   rp_attn_fwd/bwd       nn.MultiheadAttention -> SDPA (key padding mask, dropout 0.1)
 *                         models/MMCTransformer.py:132-138
 *   rp_focal_*            sigmoid_focal_loss + mask + sum        models/losses.py:4-53,
 *                         models/MMCTransformer.py:159-179
 *   rp_rowdot_*           final Linear(256->1 / 256->2) of cls/reg heads models/MMCTransformer.py:71-93
 *   rp_colsum             bias / LayerNorm-affine gradient reductions (autograd of the above)
 *   rp_adam_step(_dev)    torch.optim.Adam(lr, weight_decay) step  main.py:190-191,369
 *   rp_infer_select       inference_single_video                 models/MMCTransformer.py:181-229
 *   rp_softnms            soft_nms_intervals_cpu                 models/softnms.py:3-38
 *   rp_mha_fwd/bwd        models/transformer.py:37-81 MultiHeadAttention core (self / cross)
 *   rp_tiou_hits          calculate_tiou (batched)               utils/metrics.py:82-111
 *   rp_pad_rows           collate_fn / preprocessing padding     dataset/RepurposeClip.py:449-533
 *   rp_diou_fwd/bwd       ctr_diou_loss_1d                       models/losses.py:56-116
 *   (gradient all-reduce over RCCL is issued by the host layer through torch.distributed,
 *    replacing utils/distributed.py:396-433 DDP; no collective lives in this library)
 */
#ifndef RP_API_H
#define RP_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Element dropout used by the GEMM and LayerNorm epilogues, dropout(v, p, seed, idx):
 *   keep(seed, idx): w0 = rp_hash(seed, idx >> 3); w1..w3 = x ^ c after successive MWC64X steps
 *   (t = 4294883355*x + c; x = lo32(t); c = hi32(t)) from x = w0, c = w0 >> 1; element idx reads
 *   the 16 bits ((idx & 1) ? high : low) of
 *   w((idx & 7) >> 1) as int16 and is kept iff they are >= round(p*65536) - 32768;
 *   kept values are scaled by 1/(1-p).  rp_hash: repurpose_amd/csrc/rp_common.h. */
enum { RP_OK = 0, RP_ERR_ARG = 1, RP_ERR_LAUNCH = 2 };
enum { RP_F32 = 0, RP_BF16 = 1, RP_F16 = 2, RP_F64 = 3, RP_I64 = 4 };  /* F16/F64/I64: rp_pad_rows sources */

int rp_version(void);
/* Copies the last error message of the calling thread into buf (NUL-terminated). */
int rp_last_error(char* buf, size_t n);

/* K1: out[r, :] = [v[r, 0:dv] | a[r, 0:da] | t[r, 0:dt]] (inputs fp32, contiguous rows),
 * out row stride dv+da+dt, out dtype RP_F32 or RP_BF16.  dv/da/dt may be 0. */
int rp_concat_rows(const float* v, int dv, const float* a, int da, const float* t, int dt,
                   int64_t rows, void* out, int out_dtype, void* stream);

/* dst[i] = bf16(src[i]) (round to nearest even) */
int rp_cast_f32_to_bf16(const float* src, void* dst, int64_t n, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* GEMM: C[m, n] = epilogue( alpha * sum_k A(m, k) * B(n, k) )
 *   A(m, k) = A[m*lda + k] if a_kmajor else A[k*lda + m]
 *   B(n, k) = B[n*ldb + k] if b_kmajor else B[k*ldb + n]
 * A and B share `dtype` (RP_F32: exact-f32 MFMA parity mode; RP_BF16: bf16 MFMA, fp32 acc).
 * Requirements: the contiguous dimension of A, B and C is a multiple of 8 elements, leading
 * dimensions multiples of 8, base pointers 16-byte aligned (bias, residual and gate too; ldg a
 * multiple of 8, ldr of 4).
 * Epilogue order: v = alpha*acc (+ bias[n]); v *= col_scale if n < col_scale_n; relu;
 *   dropout(p, seed, index m*N+n);
 *   gate: v *= gate_scale * (gate[m, n] > 0);  residual: v += residual[m, n];
 *   accumulate (fp32 C only): C[m, n] += v, else C[m, n] = v. */
typedef struct rp_gemm_epilogue {
  const float* bias;
  int relu;
  float dropout_p;
  uint32_t dropout_seed;
  const float* residual;
  int64_t ldr;
  const void* gate;
  int gate_dtype;
  int64_t ldg;
  float gate_scale;
  int accumulate;
  int64_t col_scale_n; /* multiple of 8; 0 = off.  The Q columns of the QKV projection use it to emit
                          Q * scale * log2(e) for the attention kernels (RP_ATTN_Q_PRESCALED) */
  float col_scale;
  const uint32_t* seed_base; /* optional device word: dropout draws with rp_hash(*seed_base, dropout_seed)
                                (see "Graph-replayable dropout" below); NULL: dropout_seed as is */
} rp_gemm_epilogue;

int rp_gemm(int dtype, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, int a_kmajor,
            const void* B, int64_t ldb, int b_kmajor, void* C, int64_t ldc, int c_dtype, float alpha,
            const rp_gemm_epilogue* ep, void* stream);

/* The attention output's gradient with the attention backward's delta pre-pass fused into its
 * epilogue (bf16): dO = dY W (the self_attn.out_proj dgrad of models/MMCTransformer.py:41-55 under
 * loss.backward(); dY [M, ldy] k-major, W [K, ldw] the out_proj weight, dO [M, ldo] bf16 written) and,
 * per row m = b*T + t and head h, delta = sum_d dO[m][64h + d] * (out + out_lo)[m][64h + d] into
 * delta_ws planes 0..2 exactly as rp_attn_bwd_delta writes them (bitwise: the stored bf16 dO, the
 * same summation order), so rp_mha_bwd / rp_attn_bwd_given_delta can skip the pre-pass.
 * M = B*T and H*64 multiples of 128, K a multiple of 64. */
int rp_gemm_attn_dout_delta(const void* dY, int64_t ldy, const void* W, int64_t ldw, int64_t M, int64_t K, void* dO,
                            int64_t ldo, const void* out, const void* out_lo, int64_t ld_out, const float* lse, int B,
                            int T, int H, float dropout_p, float* delta_ws, void* stream);

/* Weight gradient of a Linear layer: dW[m, n] (+)= sum_k dY[k, m] * X[k, n] and (if db)
 * db[m] (+)= sum_k dY[k, m] — the token dimension K is split over workgroups (deterministic
 * split-K: fp32 partial slabs in `workspace`, reduced in a fixed order); the bias gradient is
 * accumulated from the dY tiles the GEMM already stages (no separate pass over dY).
 * dY [K, ldy] and X [K, ldx] share `dtype`; dW is fp32 [M, N] contiguous.
 * workspace: at least rp_gemm_wgrad_workspace(M, N, K) bytes, 16-byte aligned. */
int64_t rp_gemm_wgrad_workspace(int64_t M, int64_t N, int64_t K);
int rp_gemm_wgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dY, int64_t ldy, const void* X,
                  int64_t ldx, float* dW, float* db, int accumulate, void* workspace, int64_t ws_bytes,
                  void* stream);

/* Grouped weight gradients (bf16 operands): for every item, dW (+)= dY^T X and, if db, db (+)= colsum
 * dY over the SAME token count K (a multiple of 64), each output tile reduced over the
 * whole K range in one workgroup — no split-K slabs, no workspace, deterministic.  Replaces the
 * per-layer weight-gradient launches of the encoder's backward (autograd of the nn.Linear layers of
 * models/MMCTransformer.py:41-55 under loss.backward(), main.py:365) when they are deferred to the
 * end of the backward.  At most 64 items per call (256 x 256 output tiles);
 * dY [K, ldy], X [K, ldx] bf16, dW fp32 [M, N]. */
typedef struct {
  const void* dY;
  const void* X;
  float* dW;
  float* db;
  int64_t M, N, ldy, ldx;
} rp_wgrad_item;
int rp_gemm_wgrad_grouped(int64_t K, const rp_wgrad_item* items, int n_items, int accumulate, void* stream);

/* GEMM + LayerNorm over whole 512-wide rows (bf16 operands, fp32 accumulate), one launch per
 * pre-LN encoder-layer seam (models/MMCTransformer.py:41-55, d_model = 512):
 *   rp_gemm_ln_fwd:  x_out = dropout(A W^T + bias) + residual          (rp_gemm with that epilogue)
 *                    h_out = LayerNorm(x_out; gamma, beta, eps), mean/rstd saved (rp_layernorm_fwd)
 *     A [M, lda] bf16 (k-major), W [512, ldw >= K] bf16 (the nn.Linear weight); x_out fp32, h_out bf16.
 *     Replaces x1 = x + drop1(out_proj(.)) followed by norm2(x1), and x2 = x1 + drop2(linear2(.))
 *     followed by the next layer's norm1 (or encoder_norm).
 *   rp_gemm_ln_bwd:  dh = A W (A = dY [M, lda] bf16, W [K, ldw >= 512] bf16: the dgrad of a Linear
 *                    whose weight is [K][512]), then rp_layernorm_bwd's row computation on dh
 *                    (x, mean, rstd, gamma, dres -> dx fp32, dx_lp bf16 with dropout(lp_dropout_p,
 *                    lp_seed), gamma / beta partials per 32-row block as rp_layernorm_bwd writes them).
 *     dh itself is never written.  Replaces linear1 / in_proj dgrad followed by norm2 / norm1 backward.
 * Without an exchange workspace (xchg below) results are bitwise those of the unfused calls (same MFMA
 * k order, same epilogue and LayerNorm arithmetic).  M % 64 == 0, K % 64 == 0; one workgroup per 64 rows. */
typedef struct rp_gemm_ln_args {
  const void* A;
  int64_t lda;
  const void* W;
  int64_t ldw;
  /* forward */
  const float* bias;
  float dropout_p;
  uint32_t dropout_seed;
  const uint32_t* seed_base; /* optional, as rp_gemm_epilogue.seed_base (dropout_seed and lp_seed) */
  const float* residual;
  int64_t ldr;
  float* x_out;
  int64_t ldx_out;
  const float* gamma;
  const float* beta;
  float eps;
  void* h_out;
  int64_t ldh;
  float* mean; /* fwd: written; bwd: read */
  float* rstd;
  /* backward */
  const float* x;
  int64_t ldx;
  const float* dres; /* optional */
  int64_t lddres;
  float* dx;
  int64_t lddx;
  void* dx_lp; /* optional */
  int64_t lddx_lp;
  float lp_dropout_p;
  uint32_t lp_seed;
  float* dgamma_part; /* optional: [M/32][ld_part] */
  float* dbeta_part;
  int64_t ld_part;
  /* optional: exchange workspace (rp_gemm_ln_xchg_bytes(M) bytes, 256-byte aligned, zero-filled before
   * its first use; every launch leaves it zeroed, so one workspace serves the launches of a stream).
   * With it the seam runs on 128 x 128, 64 x 128 or 32 x 128 GEMM tiles (the tallest whose grid gives
   * every CU two workgroups), whose four column tiles per row block exchange the per-row LayerNorm
   * statistics through it; x_out is then
   * still bitwise the unfused GEMM's, h_out / mean / rstd / dx / dx_lp / the partials agree with the
   * unfused LayerNorm to fp32 rounding of the row sums.  Null: the 64-row full-row kernels above.
   * Launches sharing one workspace must be ordered (one stream, or event-ordered).
   * Progress: a seam is issued as launches of at most the co-resident capacity (CUs x workgroups per CU
   * from the occupancy query, at most 2) whole row blocks each, so every partner of a waiting workgroup
   * is resident, or becomes resident once other streams' kernels retire.  A partner wait is bounded
   * (10 s); one that gives up sets a process-wide fault word: from then on rp_gemm_ln_fwd / bwd and
   * rp_gemm_ln_status return RP_ERR_LAUNCH (the outputs of that launch are invalid and its workspace is
   * inconsistent) until rp_gemm_ln_reset re-zeroes the workspace. */
  void* xchg;
} rp_gemm_ln_args;
int rp_gemm_ln_fwd(int64_t M, int64_t K, const rp_gemm_ln_args* a, void* stream);
int rp_gemm_ln_bwd(int64_t M, int64_t K, const rp_gemm_ln_args* a, void* stream);
int64_t rp_gemm_ln_xchg_bytes(int64_t M);
/* RP_OK, or RP_ERR_LAUNCH when an exchange wait gave up since the last reset (no synchronisation: a
 * launch is seen once it has run). */
int rp_gemm_ln_status(void);
/* After a give-up: synchronise `stream`, zero the workspace (rp_gemm_ln_xchg_bytes(M) bytes; xchg may be
 * NULL) and clear the fault word. */
int rp_gemm_ln_reset(void* xchg, int64_t M, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* LayerNorm over the last dim D (<= 4096, multiple of 4), one row per wavefront.
 * y = ((x - mean) * rstd) * gamma + beta;  y += pe[(row % pe_period) * D + c] if pe;
 * y = relu(y) if relu;  y = dropout(y, p, seed, index row*D+c) if dropout_p > 0.
 * Writes y to out_f32 and/or out_lp (dtype out_lp_dtype); saves mean/rstd if non-NULL. */
typedef struct rp_ln_fwd_args {
  const void* x;
  int x_dtype;
  int64_t ldx;
  const float* gamma;
  const float* beta;
  float eps;
  const float* pe;
  int64_t pe_period;
  int relu;
  float dropout_p;
  uint32_t dropout_seed;
  float* out_f32;
  int64_t ld_out_f32;
  void* out_lp;
  int out_lp_dtype;
  int64_t ld_out_lp;
  float* mean;
  float* rstd;
  const uint32_t* seed_base; /* optional, as rp_gemm_epilogue.seed_base */
} rp_ln_fwd_args;

int rp_layernorm_fwd(int64_t rows, int64_t D, const rp_ln_fwd_args* a, void* stream);

/* LayerNorm backward.  dy is the gradient w.r.t. the forward output after relu/dropout.
 *   g = dy;  if dropout_p > 0: g *= keep(seed, row*D+c) / (1-p);  if y: g *= (y > 0)  (relu)
 *   dx = rstd * (g*gamma - mean(g*gamma) - xhat * mean(g*gamma*xhat));  dx += dres
 *   dx_f32 (if non-NULL) = dx;  dx_lp (if non-NULL) = dx * keep(dx_lp_seed)/(1-dx_lp_dropout_p)
 *   dgamma_part[blk, c] = sum over the block's rows of g*xhat;  dbeta_part[blk, c] = sum g
 * Partials have rp_layernorm_bwd_blocks(rows) rows of row stride ld_part (0 = D); reduce them with
 * rp_colsum (dgamma_part = P, dbeta_part = P + D, ld_part = 2D reduces both in one launch). */
typedef struct rp_ln_bwd_args {
  const void* dy;
  int dy_dtype;
  int64_t lddy;
  const void* x;
  int x_dtype;
  int64_t ldx;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const void* y;
  int y_dtype;
  int64_t ldy;
  float dropout_p;
  uint32_t dropout_seed;
  const float* dres;
  int64_t lddres;
  float* dx_f32;
  int64_t lddx;
  void* dx_lp;
  int dx_lp_dtype;
  int64_t lddx_lp;
  float dx_lp_dropout_p;
  uint32_t dx_lp_seed;
  float* dgamma_part;
  float* dbeta_part;
  int64_t ld_part;
  const uint32_t* seed_base; /* optional, as rp_gemm_epilogue.seed_base (both dropout_seed and dx_lp_seed) */
} rp_ln_bwd_args;

int64_t rp_layernorm_bwd_blocks(int64_t rows);
int rp_layernorm_bwd(int64_t rows, int64_t D, const rp_ln_bwd_args* a, void* stream);

/* out[c] (+)= sum_r w[r] * X[r*ldx + c]  (w NULL -> 1).  X dtype RP_F32 / RP_BF16.
 * workspace: rp_colsum_workspace(rows, cols) floats.  Deterministic (fixed reduction order). */
int64_t rp_colsum_workspace(int64_t rows, int64_t cols);
int rp_colsum(const void* X, int dtype, int64_t rows, int64_t cols, int64_t ldx, const float* w,
              float* out, int accumulate, float* workspace, void* stream);

/* Many fp32 column sums in one launch (no weights): out_k[c] (+)= sum_r X_k[r*ldx_k + c] with the
 * same fixed summation order as rp_colsum's single pass (so the results are bitwise those of
 * per-item rp_colsum calls with rows <= 2048).  Used to reduce every LayerNorm's gamma / beta
 * partials of a backward together (the LayerNorm affine gradients of models/MMCTransformer.py
 * under loss.backward()).  At most 64 items per call. */
typedef struct {
  const float* X;
  float* out;
  int64_t rows, cols, ldx;
  int accumulate;
} rp_colsum_item;
int rp_colsum_batched(const rp_colsum_item* items, int n_items, void* stream);

/* Sums of squares of many fp32 vectors in one launch: *out_k = sum_i x_k[i]^2, accumulated in fp64
 * in a fixed order.  Replaces the per-tensor `.grad.norm().item()` host syncs of the trainer's
 * gradient-norm logging (main.py:345-367); repurpose_amd.gradnorm.grad_norms copies every result
 * to the host at once.  At most 64 items per call. */
typedef struct {
  const float* x;
  int64_t n;
  double* out;
} rp_sumsq_item;
int rp_sumsq_batched(const rp_sumsq_item* items, int n_items, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Flag or-ed into the dtype argument of every rp_attn_* / rp_mha_* entry point: the q operand
 * already holds Q * scale * log2(e), rounded to the operand dtype (rp_gemm's col_scale epilogue
 * on the Q columns of the QKV projection).  The kernels then skip their own prescale, and the
 * backward's recomputed scores are the forward's bit for bit in bf16 too.  dq is still the gradient
 * w.r.t. the unscaled Q (the producer's pre-scale output), so it chains into the producer's
 * backward unchanged.  Without the flag the kernels compute the same bf16(Q * scale * log2 e)
 * themselves (the forward and dQ kernels in registers, the dK/dV kernel as it stages Q tiles). */
enum { RP_ATTN_Q_PRESCALED = 0x100 };
/* 0x200 (RP_ATTN_NO_SPLIT of rounds 1-4, removed with the split kernels' switch) is still accepted in the
 * dtype argument and ignored. */

/* Multi-head self attention, flash-style (no T x T materialisation).
 * qkv: [B*T, 3*H*dk] rows = (q heads | k heads | v heads), dk == 64.
 * key_valid: [B, T] uint8 (0 -> key masked with -inf, torch key_padding_mask semantics).
 * out: [B*T, H*dk];  lse: [B, H, T] fp32 (natural-log sum-exp of scaled scores; bf16 with dropout
 * sums the bf16-rounded probabilities the P.V product uses, on the matrix core).
 * out_lo (bf16, optional): bf16(O - bf16(O)), the rounding residual of out, for the backward's
 * delta = rowsum(dout * O) (pass the same pointer to the backward; NULL: delta from out alone).
 * Dropout on the attention probabilities with probability p: for query q and group g one
 * multiply-with-carry stream (MWC64X) x = rp_hash(rp_hash(seed, b*H+h), q*4 + g),
 * c = rp_hash(x, 0x6A09E667) >> 1 is stepped (t = 4294883355*x + c; x = lo32(t); c = hi32(t)) eight
 * times per 64-key tile, tiles in order, each step giving the word x ^ c; in tile t word j (1..8th of the tile)
 * holds the keys 64t + 16*(j>>1) + 4g + 2*(j&1) + {0: low 16 bits, 1: high 16 bits}; a key is kept iff its 16 bits
 * read as int16 are >= round(p*65536) - 32768 (rp_hash: repurpose_amd/csrc/rp_common.h).
 * The forward writes the keep bits to `dropmask` (uint16 [B*H][ceil(T/64)][4][roundup(T,128)],
 * bit (kt*4 + r) of word (bh, tile, g, q) = keep(q, 64*tile + 16*kt + 4*g + r);
 * rp_attn_dropmask_elems() words), the backward reads them back.  dropmask may be NULL when
 * p == 0. */
int64_t rp_attn_dropmask_elems(int B, int T, int H);

/* General multi-head attention (self or cross): q rows [B*Tq] with stride ldq, k / v rows [B*Tk]
 * with strides ldk / ldv (head h = columns h*dk .. h*dk+dk-1 of a row, any row stride that is a
 * multiple of 8 elements), key_valid [B, Tk] (0 -> the key is masked with -inf for every query:
 * torch key_padding_mask semantics; models/transformer.py's masked_fill(-1e9) is identical unless
 * a sequence has no valid key at all).  out [B*Tq, ldo]; lse [B, H, Tq] fp32.  Backward: dout
 * [B*Tq, lddo]; dq [B*Tq, lddq], dk / dv [B*Tk, lddk / lddv] are fully overwritten; delta_ws
 * [3, B, H, Tq] fp32 (plane 0 = delta; see rp_attn_bwd).  Dropout keep bits (forward -> backward) as for rp_attn_fwd with T -> (Tq, Tk):
 * rp_mha_dropmask_elems(B, Tq, Tk, H) uint16 words [B*H][ceil(Tk/64)][4][roundup(Tq,128)].
 * Replaces models/transformer.py:37-81 MultiHeadAttention's score/softmax/PV core (self attention
 * of EncoderLayer :84-102, cross attention of CrossAttentionEncoderLayer :105-130 and
 * CrossSelfEncoderLayer :133-176). */
typedef struct rp_mha_args {
  const void* q;
  int64_t ldq;
  const void* k;
  int64_t ldk;
  const void* v;
  int64_t ldv;
  const uint8_t* key_valid;
  int B, Tq, Tk, H, head_dim;
  float scale;
  float dropout_p;
  uint32_t seed;
  void* out;
  int64_t ldo;
  float* lse;
  uint16_t* dropmask;
  const void* dout;
  int64_t lddo;
  void* dq;
  int64_t lddq;
  void* dk;
  int64_t lddk;
  void* dv;
  int64_t lddv;
  float* delta_ws;
  void* out_lo;            /* bf16 only, optional: the forward also writes bf16(O - bf16(O)) here [B*Tq, ldo];
                              the backward then forms delta = rowsum(dout * O) from the unrounded O */
  int empty_rows_uniform;  /* a sequence with no valid key attends uniformly to ALL its keys (output =
                              mean of V, dq = dk = 0): models/transformer.py's masked_fill(-1e9) semantics.
                              0 = torch key_padding_mask semantics (-inf: such rows are NaN) */
  const uint32_t* seed_base; /* optional, as rp_gemm_epilogue.seed_base (forward dropout stream seed) */
} rp_mha_args;

/* General attention core (fp32) for head dims the flash kernels do not serve (d_k > 64) and masks
 * that differ between queries or heads — models/transformer.py:52-81 exactly: scores = scale * Q K^T,
 * scores[mask == 0] = -1e9, P = softmax(scores), out = P V; backward with no gradient through masked
 * scores.  q / k / v rows as rp_mha_args (fp32, head h at columns h*head_dim ..); mask (optional)
 * uint8 addressed mask[b*mask_sb + h*mask_sh + q*mask_sq + k*mask_sk] (element strides, 0 on a
 * broadcast dimension).  probs: [B, H, Tq, Tk] fp32 workspace the forward fills and the backward reads;
 * dscores: [B, H, Tq, Tk] fp32 backward workspace; dq / dk / dv fully overwritten. */
typedef struct rp_mha_general_args {
  const float* q;
  int64_t ldq;
  const float* k;
  int64_t ldk;
  const float* v;
  int64_t ldv;
  int B, Tq, Tk, H, head_dim;
  float scale;
  const uint8_t* mask;
  int64_t mask_sb, mask_sh, mask_sq, mask_sk;
  float* probs;
  float* out;
  int64_t ldo;
  const float* dout;
  int64_t lddo;
  float* dscores;
  float* dq;
  int64_t lddq;
  float* dk;
  int64_t lddk;
  float* dv;
  int64_t lddv;
} rp_mha_general_args;
int rp_mha_general_fwd(const rp_mha_general_args* args, void* stream);
int rp_mha_general_bwd(const rp_mha_general_args* args, void* stream);

int64_t rp_mha_dropmask_elems(int B, int Tq, int Tk, int H);
int rp_mha_fwd(int dtype, const rp_mha_args* args, void* stream);
/* phases: 1 = delta pre-pass, 2 = dK/dV, 4 = dQ.  1 and 4 together fuse the delta pre-pass into the
 * dQ kernel, which then runs before dK/dV (7 = all: fused dQ + delta, then dK/dV). */
int rp_mha_bwd(int dtype, const rp_mha_args* args, int phases, void* stream);
int rp_attn_fwd(int dtype, const void* qkv, const uint8_t* key_valid, int B, int T, int H, int dk,
                float scale, float dropout_p, uint32_t seed, const uint32_t* seed_base, void* out, void* out_lo,
                float* lse, uint16_t* dropmask, void* stream);
/* Backward; dqkv: [B*T, 3*H*dk] (fully overwritten); delta_ws: [3, B, H, T] fp32 workspace (plane 0:
 * delta = rowsum(dout * O); planes 1, 2: the dK/dV kernel's row constants -delta/(1/(1-p)) and
 * -lse*log2(e) + log2(1/(1-p)), written by whichever call formed delta).
 * = rp_attn_bwd_dq_delta (dQ columns of dqkv, one workgroup per 128-query block, which also writes
 * delta = rowsum(dout * out) to delta_ws), then rp_attn_bwd_dkdv (dK, dV columns, one workgroup per
 * 128-key block, reading delta).  The phases are also exported separately (per-kernel timing);
 * rp_attn_bwd_delta + rp_attn_bwd_dq is the unfused equivalent of rp_attn_bwd_dq_delta.
 * bf16 with RP_ATTN_Q_PRESCALED where both grids have at least one 128-row block per compute unit
 * (B*H*ceil(T/128) >= 256 on 256 CUs: the metric shape, configs 2 and 4): rp_attn_bwd and rp_mha_bwd
 * with phases 7 instead run rp_attn_bwd_delta's pass and ONE launch whose workgroups take either role
 * (dK/dV blocks, then dQ blocks): same results up to the rounding of delta's sum.
 * rp_attn_bwd_uses_roles tells whether rp_attn_bwd takes that form for a shape (1) or the two kernels
 * (0), so a caller timing the phases separately (bench.py's roofline) can time the launch the step
 * really runs. */
int rp_attn_bwd_uses_roles(int dtype, int B, int T, int H, int dk);
int rp_attn_bwd(int dtype, const void* qkv, const void* out, const void* out_lo, const void* dout,
                const float* lse, const uint8_t* key_valid, int B, int T, int H, int dk, float scale,
                float dropout_p, const uint16_t* dropmask, void* dqkv, float* delta_ws, void* stream);
/* rp_attn_bwd without the delta pre-pass: delta_ws already holds its three planes (rp_attn_bwd_delta or
 * rp_gemm_attn_dout_delta); the two-role launch, or the dQ kernel reading the planes then dK/dV. */
int rp_attn_bwd_given_delta(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                            const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                            const uint16_t* dropmask, void* dqkv, void* stream);
int rp_attn_bwd_delta(int dtype, const void* out, const void* out_lo, const void* dout, const float* lse, int B,
                      int T, int H, int dk, float dropout_p, float* delta_ws, void* stream);
int rp_attn_bwd_dkdv(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                     const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                     const uint16_t* dropmask, void* dqkv, void* stream);
int rp_attn_bwd_dq_delta(int dtype, const void* qkv, const void* out, const void* out_lo, const void* dout,
                         const float* lse, float* delta_ws, const uint8_t* key_valid, int B, int T, int H, int dk,
                         float scale, float dropout_p, const uint16_t* dropmask, void* dqkv, void* stream);
int rp_attn_bwd_dq(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                   const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                   const uint16_t* dropmask, void* dqkv, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Focal loss (alpha, gamma) on n frames.  mask may be NULL (all ones).
 * fwd_sum: *loss = sum_i mask_i * focal(x_i, t_i)   (single deterministic reduction)
 * elementwise: out_i = focal(x_i, t_i)
 * bwd: dx_i = (*grad_out) * mask_i * d focal / d x_i  (grad_out: device scalar, or per-element
 *      array when grad_per_elem != 0) */
int rp_focal_fwd_sum(const float* x, const float* t, const uint8_t* mask, int64_t n, float alpha,
                     float gamma, float* loss, void* stream);
/* The same sum over many workgroups (the training step's form): per-chunk partials into ws (at least
 * rp_focal_ws_elems(n) floats), then one wave sums them in index order — deterministic for a given n, a
 * different summation order from rp_focal_fwd_sum's single workgroup. */
int64_t rp_focal_ws_elems(int64_t n);
int rp_focal_fwd_sum_ws(const float* x, const float* t, const uint8_t* mask, int64_t n, float alpha,
                        float gamma, float* ws, int64_t ws_elems, float* loss, void* stream);
int rp_focal_elementwise(const float* x, const float* t, int64_t n, float alpha, float gamma,
                         float* out, void* stream);
int rp_focal_bwd(const float* x, const float* t, const uint8_t* mask, int64_t n, float alpha,
                 float gamma, const float* grad_out, int grad_per_elem, float* dx, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Small-N linear (N <= 4): out[r, j] = act(sum_k X[r, k] * W[j, k] + b[j]).
 * bwd_dx: dX[r, k] = (sum_j dout[r, j] * W[j, k]) * gate_scale * (G[r, k] > 0 if G) */
int rp_rowdot_fwd(int x_dtype, const void* X, int64_t ldx, int64_t rows, int K, const float* W,
                  const float* b, int nout, int relu, float* out, int64_t ldo, void* stream);
int rp_rowdot_bwd_dx(const float* dout, int64_t ldd, int64_t rows, int K, const float* W, int nout,
                     const void* G, int g_dtype, int64_t ldg, float gate_scale, void* dX,
                     int dx_dtype, int64_t lddx, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* torch.optim.Adam (coupled L2 weight decay) over a flat fp32 buffer; step is 1-based.
 * p_lp (optional): refreshed bf16 copy of the updated parameters. */
int rp_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, int step, void* p_lp, void* stream);
/* The same update with its coefficients read from device memory when the kernel runs (a captured
 * HIP graph replays one launch with the host's per-step values): coef_dev[6] = the output of
 * rp_adam_coefficients {lr/(1-beta1^step), beta1, beta2, eps, weight_decay, sqrt(1-beta2^step)},
 * computed on the host exactly as rp_adam_step computes them (bitwise identical updates). */
int rp_adam_coefficients(float lr, float beta1, float beta2, float eps, float weight_decay, int step,
                         float* coef);
int rp_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* coef_dev,
                     void* p_lp, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Graph-replayable dropout streams (the captured training step, repurpose_amd/graph.py).
 * Every launch that draws dropout (rp_gemm epilogue, rp_layernorm_fwd/bwd, rp_attn_fwd / rp_mha_fwd)
 * takes an optional device word `seed_base` in its own arguments: when it is non-NULL the kernel
 * draws with the seed rp_hash(*seed_base, seed) — *seed_base read when the kernel RUNS — instead of
 * `seed`, so one captured launch gives a fresh stream per replay once the host rewrites the word.
 * The pointer travels per call: the library keeps no process-wide dropout state (two models, or an
 * eager step beside a captured one, never share a stream).  4-byte aligned. */

/* ---------------------------------------------------------------------------------------- */
/* Inference.  rp_infer_select: per video b (one workgroup), prob = sigmoid(logit)*mask,
 * candidates prob > thresh, stable sort (prob desc, index asc), first min(topk, n),
 * left = idx - off0, right = idx + off1, keep dur_min < right-left < dur_max.
 * Outputs: count[b]; idx/score/seg rows [b, 0:count[b]] (capacity topk per video).  T <= 8192. */
int rp_infer_select(const float* logits, const uint8_t* mask, const float* offsets, int B, int T,
                    float thresh, int topk, float dur_min, float dur_max, int* count,
                    int64_t* idx, float* score, float* seg, void* stream);
/* Soft-NMS with the exact semantics of soft_nms_intervals_cpu (one workgroup per video,
 * n = count[b] <= cap candidates, any cap).  keep[b, 0:keep_count[b]] = positions into the candidate
 * list.  final_scores (optional): the decayed, permuted score array the reference leaves behind.
 * The Gaussian decay uses numpy's float32 exp algorithm bit for bit (reference softnms.py:35).
 * Candidates live in LDS up to cap = 6144; above that the kernel keeps them in `workspace`
 * (rp_softnms_workspace(B, cap) bytes, 0 below the LDS limit: workspace may then be NULL). */
int64_t rp_softnms_workspace(int B, int cap);
int rp_softnms(const float* scores, const float* segs, const int* count, int B, int cap,
               float sigma, float thresh, const int* max_seg, int* keep, int* keep_count,
               float* final_scores, void* workspace, int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Batch collation on the device (dataset/RepurposeClip.py:449-533 preprocessing): the rows of B
 * ragged sequences, concatenated in src ([sum len_b, D], dtype RP_F16 / RP_F32 / RP_F64 / RP_I64),
 * row_offsets[B+1] their prefix sums; dst fp32 [B, T, D] = padded batch (pad where t >= len_b),
 * converted like torch's copy (fp64 -> fp32 round to nearest even). */
int rp_pad_rows(const void* src, int src_dtype, const int64_t* row_offsets, int B, int T, int D, float pad, float* dst,
                void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Evaluation metric (utils/metrics.py:82-111 calculate_tiou, batched): pred [V][P][2] fp32 segments
 * (start, end), pred_count[V] valid rows; ref [V][R][2] fp64 reference segments, ref_count[V];
 * thresholds[n_thr] (1..32).  hits[V][n_thr] = number of predictions whose best IoU over the
 * video's references (0 when it has none) is >= the threshold; IoU in double exactly as the
 * reference's Python floats.  precision = hits / pred_count (0 if pred_count == 0). */
int rp_tiou_hits(const float* pred, const int* pred_count, int P, const double* ref, const int* ref_count, int R,
                 const double* thresholds, int n_thr, int V, int* hits, void* stream);

/* 1-D distance-IoU loss (models/losses.py:56-116 ctr_diou_loss_1d) on n (left, right) offset pairs.
 * reduction 0: out[n] per element; 1: *out = mean; 2: *out = sum (single deterministic pass).
 * Backward: dpred / dgt (either may be NULL) = grad_scale * grad_out (per element if per_elem, else
 * the device scalar grad_out[0]) * d loss / d offsets (torch's tie / clamp subgradients). */
int rp_diou_fwd(const float* pred, const float* gt, int64_t n, float eps, int reduction, float* out, void* stream);
int rp_diou_bwd(const float* pred, const float* gt, int64_t n, float eps, const float* grad_out, int per_elem,
                float grad_scale, float* dpred, float* dgt, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Test hooks (not used by the product path).
 * rp_debug_gemm_ln_partial: the exchange launch of rp_gemm_ln_fwd (fwd != 0) / bwd with only its first
 *   `tiles` workgroups and a give-up bound of timeout_s: a row block whose partner is never launched must
 *   set the fault word (rp_gemm_ln_status), not hang or return silently wrong statistics.
 * rp_debug_occupy: `blocks` 256-thread workgroups with 64 KiB of LDS each that hold their CU slots for
 *   `us` microseconds (a seam launched beside another stream's long kernel).
 * rp_debug_set_lnx_rows: force the exchange tile height (32, 64 or 128 rows; 0 = automatic) process-wide. */
int rp_debug_gemm_ln_partial(int fwd, int64_t M, int64_t K, const rp_gemm_ln_args* a, int64_t tiles, double timeout_s,
                             void* stream);
int rp_debug_occupy(int blocks, int us, void* stream);
int rp_debug_set_lnx_rows(int rows);

#ifdef __cplusplus
}
#endif
#endif /* RP_API_H */
