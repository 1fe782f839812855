// General multi-head attention core for the models/transformer.py drop-ins (reference
// MultiHeadAttention, models/transformer.py:52-81): any head dim d_k and any mask broadcastable to
// the scores [B, H, Tq, Tk] with the reference's semantics
//     scores = (Q K^T) * scale;  scores[mask == 0] = -1e9  (masked_fill, :69-71);  P = softmax(scores);
//     out = P V
// and its exact backward (masked_fill passes no gradient to the masked scores).  The flash kernels of
// rp_attention.hip serve d_k <= 64 with per-key masks; this path serves what they cannot: head dims
// above 64 and masks that differ between queries (causal, per-head, the [B, Tk] mask the reference
// broadcasts as [1, B, 1, Tk]).  The probabilities are materialised ([B, H, Tq, Tk] fp32 workspace,
// saved for the backward), one wavefront per score row, fp32 FMAs — a correctness path for the
// secondary modules, not the hot path.
#include "rp_common.h"

namespace {

constexpr int GW = 4;  // waves per workgroup (one score row each)

struct GenDev {
  const float* q; int64_t ldq; const float* k; int64_t ldk; const float* v; int64_t ldv;
  int B, Tq, Tk, H, dk; float scale;
  const uint8_t* mask; int64_t msb, msh, msq, msk;
  float* P;
  float* out; int64_t ldo;
  const float* dout; int64_t lddo;
  float* dS;
  float* dq; int64_t lddq; float* dkp; int64_t lddk; float* dv; int64_t lddv;
};

__device__ __forceinline__ bool kept(const GenDev& a, int b, int h, int q, int kk) {
  return !a.mask || a.mask[b * a.msb + h * a.msh + q * a.msq + kk * a.msk] != 0;
}

// one wave per (b, h, q): scores -> masked -> softmax -> P row; then out row = P V
__global__ __launch_bounds__(64 * GW) void gen_fwd_kernel(GenDev a) {
  const int lane = threadIdx.x & 63;
  const int64_t rowid = (int64_t)blockIdx.x * GW + (threadIdx.x >> 6);
  if (rowid >= (int64_t)a.B * a.H * a.Tq) return;
  const int q = (int)(rowid % a.Tq), bh = (int)(rowid / a.Tq), b = bh / a.H, h = bh % a.H;
  const float* qr = a.q + ((int64_t)b * a.Tq + q) * a.ldq + (int64_t)h * a.dk;
  float* pr = a.P + rowid * a.Tk;
  float mx = -INFINITY;
  for (int kk = lane; kk < a.Tk; kk += 64) {
    const float* kr = a.k + ((int64_t)b * a.Tk + kk) * a.ldk + (int64_t)h * a.dk;
    float s = 0.f;
    for (int d = 0; d < a.dk; ++d) s = fmaf(qr[d], kr[d], s);
    s = kept(a, b, h, q, kk) ? s * a.scale : -1e9f;
    pr[kk] = s;
    mx = fmaxf(mx, s);
  }
  mx = rp_wave_max(mx);
  float sum = 0.f;
  for (int kk = lane; kk < a.Tk; kk += 64) {
    const float e = expf(pr[kk] - mx);
    pr[kk] = e;
    sum += e;
  }
  const float inv = 1.f / rp_wave_sum(sum);
  for (int kk = lane; kk < a.Tk; kk += 64) pr[kk] *= inv;
  __threadfence_block();  // this wave's P row is re-read below by every lane
  float* orow = a.out + ((int64_t)b * a.Tq + q) * a.ldo + (int64_t)h * a.dk;
  for (int d = lane; d < a.dk; d += 64) {
    float o = 0.f;
    for (int kk = 0; kk < a.Tk; ++kk) o = fmaf(pr[kk], a.v[((int64_t)b * a.Tk + kk) * a.ldv + (int64_t)h * a.dk + d], o);
    orow[d] = o;
  }
}

// one wave per (b, h, q): dP = dO V^T, delta = sum_k P dP, dS = mask ? P (dP - delta) : 0 (row of the
// dS workspace), then dq row = scale * dS K
__global__ __launch_bounds__(64 * GW) void gen_bwd_q_kernel(GenDev a) {
  const int lane = threadIdx.x & 63;
  const int64_t rowid = (int64_t)blockIdx.x * GW + (threadIdx.x >> 6);
  if (rowid >= (int64_t)a.B * a.H * a.Tq) return;
  const int q = (int)(rowid % a.Tq), bh = (int)(rowid / a.Tq), b = bh / a.H, h = bh % a.H;
  const float* dor = a.dout + ((int64_t)b * a.Tq + q) * a.lddo + (int64_t)h * a.dk;
  const float* pr = a.P + rowid * a.Tk;
  float* sr = a.dS + rowid * a.Tk;
  float dl = 0.f;
  for (int kk = lane; kk < a.Tk; kk += 64) {
    const float* vr = a.v + ((int64_t)b * a.Tk + kk) * a.ldv + (int64_t)h * a.dk;
    float dp = 0.f;
    for (int d = 0; d < a.dk; ++d) dp = fmaf(dor[d], vr[d], dp);
    sr[kk] = dp;
    dl = fmaf(pr[kk], dp, dl);
  }
  dl = rp_wave_sum(dl);
  for (int kk = lane; kk < a.Tk; kk += 64) sr[kk] = kept(a, b, h, q, kk) ? pr[kk] * (sr[kk] - dl) : 0.f;
  __threadfence_block();
  float* dqr = a.dq + ((int64_t)b * a.Tq + q) * a.lddq + (int64_t)h * a.dk;
  for (int d = lane; d < a.dk; d += 64) {
    float s = 0.f;
    for (int kk = 0; kk < a.Tk; ++kk) s = fmaf(sr[kk], a.k[((int64_t)b * a.Tk + kk) * a.ldk + (int64_t)h * a.dk + d], s);
    dqr[d] = s * a.scale;
  }
}

// one wave per (b, h, key): dk row = scale * dS^T Q, dv row = P^T dO (columns of the workspaces)
__global__ __launch_bounds__(64 * GW) void gen_bwd_kv_kernel(GenDev a) {
  const int lane = threadIdx.x & 63;
  const int64_t rowid = (int64_t)blockIdx.x * GW + (threadIdx.x >> 6);
  if (rowid >= (int64_t)a.B * a.H * a.Tk) return;
  const int kk = (int)(rowid % a.Tk), bh = (int)(rowid / a.Tk), b = bh / a.H, h = bh % a.H;
  const float* pc = a.P + (int64_t)bh * a.Tq * a.Tk + kk;
  const float* sc = a.dS + (int64_t)bh * a.Tq * a.Tk + kk;
  float* dkr = a.dkp + ((int64_t)b * a.Tk + kk) * a.lddk + (int64_t)h * a.dk;
  float* dvr = a.dv + ((int64_t)b * a.Tk + kk) * a.lddv + (int64_t)h * a.dk;
  for (int d = lane; d < a.dk; d += 64) {
    float sk = 0.f, sv = 0.f;
    for (int q = 0; q < a.Tq; ++q) {
      const int64_t r = (int64_t)b * a.Tq + q;
      sk = fmaf(sc[(int64_t)q * a.Tk], a.q[r * a.ldq + (int64_t)h * a.dk + d], sk);
      sv = fmaf(pc[(int64_t)q * a.Tk], a.dout[r * a.lddo + (int64_t)h * a.dk + d], sv);
    }
    dkr[d] = sk * a.scale;
    dvr[d] = sv;
  }
}

int gen_dev(const char* fn, const rp_mha_general_args* p, bool bwd, GenDev& a) {
  RP_REQUIRE(p, "%s: null args", fn);
  RP_REQUIRE(p->B >= 0 && p->Tq >= 0 && p->Tk > 0 && p->H > 0 && p->head_dim > 0, "%s: bad shape", fn);
  const int64_t w = (int64_t)p->H * p->head_dim;
  RP_REQUIRE(p->q && p->k && p->v && p->probs, "%s: null q / k / v / probs", fn);
  RP_REQUIRE(p->ldq >= w && p->ldk >= w && p->ldv >= w, "%s: leading dims below H * head_dim", fn);
  a = GenDev{};
  a.q = p->q; a.ldq = p->ldq; a.k = p->k; a.ldk = p->ldk; a.v = p->v; a.ldv = p->ldv;
  a.B = p->B; a.Tq = p->Tq; a.Tk = p->Tk; a.H = p->H; a.dk = p->head_dim; a.scale = p->scale;
  a.mask = p->mask; a.msb = p->mask_sb; a.msh = p->mask_sh; a.msq = p->mask_sq; a.msk = p->mask_sk;
  a.P = p->probs;
  a.out = p->out; a.ldo = p->ldo;
  if (!bwd) {
    RP_REQUIRE(p->out && p->ldo >= w, "%s: bad out / ldo", fn);
  } else {
    RP_REQUIRE(p->dout && p->lddo >= w && p->dscores, "%s: bad dout / dscores", fn);
    RP_REQUIRE(p->dq && p->dk && p->dv && p->lddq >= w && p->lddk >= w && p->lddv >= w, "%s: bad dq / dk / dv", fn);
    a.dout = p->dout; a.lddo = p->lddo; a.dS = p->dscores;
    a.dq = p->dq; a.lddq = p->lddq; a.dkp = p->dk; a.lddk = p->lddk; a.dv = p->dv; a.lddv = p->lddv;
  }
  return RP_OK;
}

}  // namespace

extern "C" int rp_mha_general_fwd(const rp_mha_general_args* p, void* stream) {
  GenDev a;
  const int rc = gen_dev("rp_mha_general_fwd", p, false, a);
  if (rc) return rc;
  const int64_t rows = (int64_t)a.B * a.H * a.Tq;
  if (rows == 0) return RP_OK;
  hipLaunchKernelGGL(gen_fwd_kernel, dim3((unsigned)((rows + GW - 1) / GW)), dim3(64 * GW), 0, (hipStream_t)stream, a);
  return rp_check_launch("rp_mha_general_fwd");
}

extern "C" int rp_mha_general_bwd(const rp_mha_general_args* p, void* stream) {
  GenDev a;
  const int rc = gen_dev("rp_mha_general_bwd", p, true, a);
  if (rc) return rc;
  const int64_t rq = (int64_t)a.B * a.H * a.Tq, rk = (int64_t)a.B * a.H * a.Tk;
  hipStream_t s = (hipStream_t)stream;
  if (rq > 0) hipLaunchKernelGGL(gen_bwd_q_kernel, dim3((unsigned)((rq + GW - 1) / GW)), dim3(64 * GW), 0, s, a);
  // no queries (Tq = 0): the key-side kernel still runs and writes dK = dV = 0 (sums over no queries),
  // as the reference's autograd gives; the caller's dk / dv are never left unwritten
  if (rk > 0) hipLaunchKernelGGL(gen_bwd_kv_kernel, dim3((unsigned)((rk + GW - 1) / GW)), dim3(64 * GW), 0, s, a);
  return rp_check_launch("rp_mha_general_bwd");
}
