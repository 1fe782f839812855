// Host-side error paths of the C ABI (include/rp_api.h), built with AddressSanitizer and
// UndefinedBehaviorSanitizer on the host code (`make asan`; SURVEY.md §5 "sanitizers on the CPU
// build").  Every call below must be rejected (RP_ERR_ARG + a message) or be a no-op before any
// device work is enqueued, so this runs on a machine without a GPU.  Exit status 0 = all passed.
#include <stdio.h>
#include <string.h>

#include "rp_api.h"

static int g_fail = 0, g_n = 0;

static void expect(const char* what, int rc, int want, const char* needle = nullptr) {
  ++g_n;
  char msg[512];
  rp_last_error(msg, sizeof msg);
  bool ok = rc == want;
  if (ok && want == RP_ERR_ARG) ok = msg[0] != 0 && (!needle || strstr(msg, needle));
  if (!ok) {
    ++g_fail;
    fprintf(stderr, "FAIL %-40s rc=%d want=%d msg='%s' needle='%s'\n", what, rc, want, msg, needle ? needle : "");
  }
}
#define BAD(call, needle) expect(#call, (call), RP_ERR_ARG, needle)
#define NOOP(call) expect(#call, (call), RP_OK)

int main() {
  // fake, never dereferenced device addresses (validation only looks at values / alignment)
  void* P = (void*)(uintptr_t)0x100000;
  float* F = (float*)P;
  void* MIS = (void*)(uintptr_t)0x100004;  // 4-byte aligned, not 16

  if (rp_version() != 1) { fprintf(stderr, "rp_version\n"); return 1; }
  // rp_last_error: truncation to small buffers, n = 0 must not write
  BAD(rp_cast_f32_to_bf16(F, P, -1, nullptr), "negative n");
  char small[4] = {'x', 'x', 'x', 'x'};
  rp_last_error(small, 0);
  if (small[0] != 'x') { ++g_fail; fprintf(stderr, "FAIL rp_last_error(n=0) wrote\n"); }
  rp_last_error(small, 1);
  if (small[0] != 0) { ++g_fail; fprintf(stderr, "FAIL rp_last_error(n=1)\n"); }
  rp_last_error(small, sizeof small);
  if (small[3] != 0) { ++g_fail; fprintf(stderr, "FAIL rp_last_error truncation\n"); }

  // concat / cast
  BAD(rp_concat_rows(F, -4, F, 0, F, 0, 8, P, RP_BF16, nullptr), "negative");
  BAD(rp_concat_rows(F, 6, F, 0, F, 0, 8, P, RP_BF16, nullptr), "multiples of 4");
  BAD(rp_concat_rows(nullptr, 4, nullptr, 0, nullptr, 0, 8, P, RP_BF16, nullptr), "null");
  BAD(rp_concat_rows(F, 4, F, 4, F, 4, 8, MIS, RP_BF16, nullptr), nullptr);
  BAD(rp_concat_rows(F, 4, F, 4, F, 4, 1ll << 40, P, RP_BF16, nullptr), "too many rows");
  NOOP(rp_cast_f32_to_bf16(nullptr, nullptr, 0, nullptr));
  BAD(rp_cast_f32_to_bf16(nullptr, P, 16, nullptr), "null");

  // GEMM family
  BAD(rp_gemm(RP_F32, 8, 8, 7, P, 8, 1, P, 8, 1, P, 8, RP_F32, 1.f, nullptr, nullptr), "K=7");
  BAD(rp_gemm(RP_F32, -1, 8, 8, P, 8, 1, P, 8, 1, P, 8, RP_F32, 1.f, nullptr, nullptr), nullptr);
  BAD(rp_gemm(RP_BF16, 16, 16, 16, MIS, 16, 1, P, 16, 1, P, 16, RP_F32, 1.f, nullptr, nullptr), nullptr);
  BAD(rp_gemm(7, 16, 16, 16, P, 16, 1, P, 16, 1, P, 16, RP_F32, 1.f, nullptr, nullptr), nullptr);
  NOOP(rp_gemm(RP_BF16, 0, 16, 16, nullptr, 16, 1, nullptr, 16, 1, nullptr, 16, RP_BF16, 1.f, nullptr, nullptr));
  rp_gemm_epilogue ep;
  memset(&ep, 0, sizeof ep);
  ep.dropout_p = 1.5f;
  BAD(rp_gemm(RP_BF16, 16, 16, 16, P, 16, 1, P, 16, 1, P, 16, RP_F32, 1.f, &ep, nullptr), "dropout_p");
  if (rp_gemm_wgrad_workspace(2048, 512, 16384) < 2048ll * 512 * 4) { ++g_fail; fprintf(stderr, "FAIL ws\n"); }
  BAD(rp_gemm_wgrad(RP_BF16, 512, 512, 1024, P, 512, P, 512, F, nullptr, 0, P, 16, nullptr), nullptr);
  rp_wgrad_item wi;
  memset(&wi, 0, sizeof wi);
  BAD(rp_gemm_wgrad_grouped(100, &wi, 1, 0, nullptr), nullptr);
  BAD(rp_gemm_wgrad_grouped(128, &wi, 65, 0, nullptr), nullptr);
  BAD(rp_gemm_wgrad_grouped(128, nullptr, 3, 0, nullptr), nullptr);

  // LayerNorm
  rp_ln_fwd_args lf;
  memset(&lf, 0, sizeof lf);
  BAD(rp_layernorm_fwd(4, 512, &lf, nullptr), "null");
  BAD(rp_layernorm_fwd(4, 512, nullptr, nullptr), "null");
  lf.x = P; lf.gamma = F; lf.beta = F; lf.x_dtype = RP_F32; lf.ldx = 512;
  BAD(rp_layernorm_fwd(4, 300, &lf, nullptr), "D=300");
  lf.x_dtype = 9;
  BAD(rp_layernorm_fwd(4, 512, &lf, nullptr), "dtype");
  lf.x_dtype = RP_F32; lf.pe = F; lf.pe_period = 0;
  BAD(rp_layernorm_fwd(4, 512, &lf, nullptr), "pe_period");
  lf.pe = nullptr; lf.dropout_p = 1.0f;
  BAD(rp_layernorm_fwd(4, 512, &lf, nullptr), "dropout_p");
  rp_ln_bwd_args lb;
  memset(&lb, 0, sizeof lb);
  BAD(rp_layernorm_bwd(4, 512, &lb, nullptr), "null");
  BAD(rp_layernorm_bwd(4, 512, nullptr, nullptr), "null");
  lb.dy = P; lb.x = P; lb.mean = F; lb.rstd = F; lb.gamma = F; lb.dx_lp_dropout_p = -0.5f;
  BAD(rp_layernorm_bwd(4, 512, &lb, nullptr), "dropout_p");
  if (rp_layernorm_bwd_blocks(16384) != 512) { ++g_fail; fprintf(stderr, "FAIL ln blocks\n"); }

  // column sums / sums of squares
  BAD(rp_colsum(P, RP_F32, -1, 8, 8, nullptr, F, 0, F, nullptr), "negative");
  BAD(rp_colsum(P, RP_F32, 8, 8, 8, nullptr, nullptr, 0, F, nullptr), "null");
  NOOP(rp_colsum(nullptr, RP_F32, 8, 0, 8, nullptr, nullptr, 0, nullptr, nullptr));
  rp_colsum_item ci;
  memset(&ci, 0, sizeof ci);
  BAD(rp_colsum_batched(&ci, 65, nullptr), "items");
  BAD(rp_colsum_batched(nullptr, 2, nullptr), "null");
  BAD(rp_colsum_batched(&ci, 1, nullptr), nullptr);
  NOOP(rp_colsum_batched(nullptr, 0, nullptr));
  rp_sumsq_item si;
  memset(&si, 0, sizeof si);
  BAD(rp_sumsq_batched(&si, 1000, nullptr), "items");
  BAD(rp_sumsq_batched(&si, 1, nullptr), "item 0");
  si.x = (const float*)(uintptr_t)0x100002; si.n = 4; si.out = (double*)P;
  BAD(rp_sumsq_batched(&si, 1, nullptr), "aligned");
  NOOP(rp_sumsq_batched(nullptr, 0, nullptr));

  // attention
  BAD(rp_attn_fwd(RP_BF16, nullptr, nullptr, 1, 1, 1, 32, 1.f, 0.f, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                  nullptr), "head dim");
  BAD(rp_attn_fwd(RP_BF16, P, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 0.1f, 0, nullptr, P, nullptr, F, nullptr,
                  nullptr), "dropmask");
  BAD(rp_attn_fwd(RP_BF16, P, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 1.0f, 0, nullptr, P, nullptr, F, nullptr,
                  nullptr), "dropout_p");
  BAD(rp_attn_fwd(RP_BF16, MIS, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 0.f, 0, nullptr, P, nullptr, F, nullptr,
                  nullptr), "alignment");
  BAD(rp_attn_fwd(RP_BF16 | RP_ATTN_Q_PRESCALED, P, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 0.1f, 0,
                  (const uint32_t*)(uintptr_t)0x100002, P, nullptr, F, (uint16_t*)P, nullptr), "seed_base");
  BAD(rp_attn_bwd(RP_BF16, P, P, nullptr, nullptr, F, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 0.f, nullptr, P, F,
                  nullptr), "dout");
  BAD(rp_attn_bwd_dkdv(RP_BF16, P, P, F, nullptr, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 0.f, nullptr, P, nullptr),
      "delta");
  BAD(rp_attn_bwd_dq(RP_F32, P, P, F, F, (const uint8_t*)P, 2, 64, 8, 48, 0.125f, 0.f, nullptr, P, nullptr),
      "head dim");
  BAD(rp_attn_bwd_dq_delta(RP_F32, P, nullptr, nullptr, P, F, F, (const uint8_t*)P, 2, 64, 8, 64, 0.125f, 0.f,
                           nullptr, P, nullptr), nullptr);
  BAD(rp_attn_bwd_delta(RP_BF16, nullptr, nullptr, P, F, 2, 64, 8, 64, 0.f, F, nullptr), nullptr);
  if (rp_attn_dropmask_elems(2, 100, 8) != 2ll * 8 * 2 * 4 * 128 || rp_attn_dropmask_elems(1, 129, 1) != 3ll * 4 * 256) { ++g_fail; fprintf(stderr, "FAIL dm elems\n"); }
  if (rp_mha_dropmask_elems(0, 100, 100, 8) != 0) { ++g_fail; fprintf(stderr, "FAIL dm elems 0\n"); }
  rp_mha_args ma;
  memset(&ma, 0, sizeof ma);
  BAD(rp_mha_fwd(RP_BF16, nullptr, nullptr), "null");
  BAD(rp_mha_fwd(RP_BF16, &ma, nullptr), "head dim");
  ma.head_dim = 64; ma.H = 8; ma.B = 1; ma.Tq = 4; ma.Tk = 4; ma.q = ma.k = ma.v = P;
  ma.ldq = ma.ldk = ma.ldv = 100;  // not a multiple of 8
  BAD(rp_mha_fwd(RP_BF16, &ma, nullptr), "leading dims");
  ma.ldq = ma.ldk = ma.ldv = 512;
  BAD(rp_mha_bwd(RP_BF16, &ma, 0, nullptr), "phases");
  BAD(rp_mha_bwd(RP_BF16, &ma, 8, nullptr), "phases");
  BAD(rp_mha_fwd(RP_BF16, &ma, nullptr), "null pointer");

  // GEMM + LayerNorm seams, general attention core
  rp_gemm_ln_args gl;
  memset(&gl, 0, sizeof gl);
  BAD(rp_gemm_ln_fwd(100, 512, &gl, nullptr), "multiple of 64");
  BAD(rp_gemm_ln_fwd(128, 512, nullptr, nullptr), "null");
  BAD(rp_gemm_ln_fwd(128, 512, &gl, nullptr), "null operand");
  gl.A = P; gl.lda = 512; gl.W = P; gl.ldw = 512; gl.gamma = F; gl.mean = F; gl.rstd = F; gl.dropout_p = 2.f;
  BAD(rp_gemm_ln_fwd(128, 512, &gl, nullptr), "dropout_p");
  gl.dropout_p = 0.f;
  BAD(rp_gemm_ln_fwd(128, 512, &gl, nullptr), "null operand");
  BAD(rp_gemm_ln_bwd(128, 512, &gl, nullptr), "null x");
  gl.x = F; gl.ldx = 512; gl.dx = F; gl.lddx = 512; gl.lp_dropout_p = -1.f;
  BAD(rp_gemm_ln_bwd(128, 512, &gl, nullptr), "lp_dropout_p");
  rp_mha_general_args mg;
  memset(&mg, 0, sizeof mg);
  BAD(rp_mha_general_fwd(nullptr, nullptr), "null");
  BAD(rp_mha_general_fwd(&mg, nullptr), "bad shape");
  mg.B = 1; mg.Tq = 4; mg.Tk = 4; mg.H = 2; mg.head_dim = 96; mg.q = mg.k = mg.v = F; mg.probs = F;
  mg.ldq = mg.ldk = mg.ldv = 100;
  BAD(rp_mha_general_fwd(&mg, nullptr), "leading dims");
  mg.ldq = mg.ldk = mg.ldv = 192;
  BAD(rp_mha_general_fwd(&mg, nullptr), "bad out");
  BAD(rp_mha_general_bwd(&mg, nullptr), "dout");

  // losses / heads
  BAD(rp_focal_fwd_sum(F, F, nullptr, -1, 0.7f, 2.f, F, nullptr), nullptr);
  BAD(rp_focal_fwd_sum(nullptr, nullptr, nullptr, 4, 0.7f, 2.f, F, nullptr), "null");
  NOOP(rp_focal_elementwise(nullptr, nullptr, 0, 0.7f, 2.f, nullptr, nullptr));
  BAD(rp_focal_elementwise(F, nullptr, 4, 0.7f, 2.f, F, nullptr), "null");
  BAD(rp_focal_bwd(F, F, nullptr, 4, 0.7f, 2.f, nullptr, 0, F, nullptr), "null");
  BAD(rp_rowdot_fwd(RP_F32, P, 256, 16, 256, F, F, 5, 0, F, 5, nullptr), "nout");
  BAD(rp_rowdot_fwd(RP_F32, P, 256, 16, 0, F, F, 1, 0, F, 1, nullptr), "size");
  BAD(rp_rowdot_bwd_dx(F, 2, 16, 256, F, 0, nullptr, RP_F32, 0, 1.f, P, RP_F32, 256, nullptr), "nout");
  BAD(rp_diou_fwd(F, F, 4, 1e-8f, 3, F, nullptr), "bad");
  BAD(rp_diou_fwd(F, nullptr, 4, 1e-8f, 0, F, nullptr), "null");
  BAD(rp_diou_bwd(F, F, 4, 1e-8f, F, 0, 1.f, nullptr, nullptr, nullptr), "null");
  NOOP(rp_diou_bwd(nullptr, nullptr, 0, 1e-8f, nullptr, 0, 1.f, nullptr, nullptr, nullptr));

  // optimizer (rp_adam_coefficients is host arithmetic: check values too)
  float coef[6];
  BAD(rp_adam_coefficients(1e-3f, 0.9f, 0.999f, 1e-8f, 1e-4f, 0, coef), "step");
  BAD(rp_adam_coefficients(1e-3f, 0.9f, 0.999f, 1e-8f, 1e-4f, 1, nullptr), "null");
  NOOP(rp_adam_coefficients(1e-3f, 0.9f, 0.999f, 1e-8f, 1e-4f, 1, coef));
  if (!(coef[0] > 0.0099f && coef[0] < 0.0101f && coef[1] == 0.9f && coef[2] == 0.999f)) {
    ++g_fail;
    fprintf(stderr, "FAIL adam coefficients %g %g %g\n", coef[0], coef[1], coef[2]);
  }
  NOOP(rp_adam_coefficients(1e-3f, 0.9f, 0.999f, 1e-8f, 1e-4f, 2000000000, coef));  // huge step: no overflow UB
  BAD(rp_adam_step(F, F, F, F, 16, 1e-3f, 0.9f, 0.999f, 1e-8f, 0.f, 0, nullptr, nullptr), "step");
  BAD(rp_adam_step(nullptr, F, F, F, 16, 1e-3f, 0.9f, 0.999f, 1e-8f, 0.f, 1, nullptr, nullptr), "null");
  BAD(rp_adam_step_dev(F, F, F, F, 16, nullptr, nullptr, nullptr), "coef");

  // inference / collation / metrics
  BAD(rp_infer_select(F, (const uint8_t*)P, F, 1, 9000, 0.5f, 1000, 10.f, 90.f, (int*)P, (int64_t*)P, F, F, nullptr),
      "exceeds");
  BAD(rp_infer_select(F, (const uint8_t*)P, F, -1, 10, 0.5f, 1000, 10.f, 90.f, (int*)P, (int64_t*)P, F, F, nullptr),
      "bad shape");
  BAD(rp_infer_select(F, (const uint8_t*)P, F, 2, 10, 0.5f, 1000, 10.f, 90.f, nullptr, (int64_t*)P, F, F, nullptr),
      "null count");
  NOOP(rp_infer_select(nullptr, nullptr, nullptr, 0, 10, 0.5f, 1000, 10.f, 90.f, nullptr, nullptr, nullptr, nullptr,
                       nullptr));
  if (rp_softnms_workspace(2, 1000) != 0 || rp_softnms_workspace(2, 7000) != 2ll * 5 * 7000 * 4) {
    ++g_fail;
    fprintf(stderr, "FAIL softnms ws\n");
  }
  BAD(rp_softnms(F, F, (const int*)P, 1, 7000, 0.5f, 0.01f, (const int*)P, (int*)P, (int*)P, nullptr, nullptr, 0,
                 nullptr), "workspace");
  BAD(rp_softnms(F, F, nullptr, 1, 100, 0.5f, 0.01f, (const int*)P, (int*)P, (int*)P, nullptr, nullptr, 0, nullptr),
      "null");
  BAD(rp_pad_rows(P, RP_F32, nullptr, 2, 10, 4, 0.f, F, nullptr), "null");
  BAD(rp_pad_rows(P, RP_F32, (const int64_t*)P, 2, 10, 0, 0.f, F, nullptr), "shape");
  NOOP(rp_pad_rows(nullptr, RP_F32, nullptr, 0, 10, 4, 0.f, nullptr, nullptr));
  BAD(rp_tiou_hits(F, (const int*)P, 4, (const double*)P, (const int*)P, 4, (const double*)P, 0, 2, (int*)P, nullptr),
      "thresholds");
  BAD(rp_tiou_hits(F, nullptr, 4, (const double*)P, (const int*)P, 4, (const double*)P, 3, 2, (int*)P, nullptr),
      "null");

  printf("%d checks, %d failed\n", g_n, g_fail);
  return g_fail ? 1 : 0;
}
