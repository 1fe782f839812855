// Evaluation metric and the regression loss of the Repurpose path.
//
//  * rp_tiou_hits: models utils/metrics.py:82-111 calculate_tiou for a batch of videos — for every
//    predicted segment the best IoU over the video's reference segments (max(..., default=0)), then
//    per threshold the number of predictions with best >= threshold.  IoU arithmetic in double,
//    as Python floats do: start_max = max(s1, s2), end_min = min(e1, e2), inter = max(0, end_min -
//    start_max), union = (e1 - s1) + (e2 - s2) - inter, iou = union != 0 ? inter / union : 0.
//    One workgroup per video; integer counts (exact, order independent).
//  * rp_diou_*: models/losses.py:56-116 ctr_diou_loss_1d (1-D distance IoU on (left, right) offsets)
//    forward (elementwise or deterministic sum) and backward for both operands, with torch's
//    subgradient conventions: min / max ties split the gradient in halves, clamp(min = eps) passes
//    the gradient where the input is >= eps.
#include "rp_common.h"

namespace {

constexpr int TIOU_NT = 256;

__global__ __launch_bounds__(TIOU_NT) void tiou_hits_kernel(const float* __restrict__ pred, const int* __restrict__ npred,
                                                            int P, const double* __restrict__ ref,
                                                            const int* __restrict__ nref, int R,
                                                            const double* __restrict__ thr, int nthr,
                                                            int* __restrict__ hits) {
  const int v = blockIdx.x;
  const int np = npred[v] < P ? npred[v] : P;
  const int nr = nref[v] < R ? nref[v] : R;
  const float* pv = pred + (int64_t)v * P * 2;
  const double* rv = ref + (int64_t)v * R * 2;
  __shared__ int cnt[32];
  if (threadIdx.x < 32) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < np; p += TIOU_NT) {
    const double s1 = pv[2 * p], e1 = pv[2 * p + 1];
    double best = 0.0;
    for (int r = 0; r < nr; ++r) {
      const double s2 = rv[2 * r], e2 = rv[2 * r + 1];
      const double smax = s1 > s2 ? s1 : s2;
      const double emin = e1 < e2 ? e1 : e2;
      const double inter = emin - smax > 0.0 ? emin - smax : 0.0;
      const double uni = (e1 - s1) + (e2 - s2) - inter;
      const double iou = uni != 0.0 ? inter / uni : 0.0;
      best = (r == 0 || iou > best) ? iou : best;  // max over a non-empty list; 0 when there is none
    }
    for (int j = 0; j < nthr && j < 32; ++j)
      if (best >= thr[j]) atomicAdd(&cnt[j], 1);
  }
  __syncthreads();
  if (threadIdx.x < nthr && threadIdx.x < 32) hits[(int64_t)v * nthr + threadIdx.x] = cnt[threadIdx.x];
}

// ---------------------------------------------------------------- DIoU ---------------------------
struct Diou {
  float loss, dlp, drp, dlg, drg;
};

// d min(a, b) / da with torch's tie rule
__device__ __forceinline__ float dmin_a(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float dmax_a(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }

__device__ __forceinline__ Diou diou_eval(float lp, float rp, float lg, float rg, float eps, bool grad) {
  const float lk = fminf(lp, lg), rk = fminf(rp, rg);
  const float inter = rk + lk;
  const float uni = (lp + rp) + (lg + rg) - inter;
  const float uc = fmaxf(uni, eps);
  const float iou = inter / uc;
  const float lc = fmaxf(lp, lg), rc = fmaxf(rp, rg);
  const float len = lc + rc;
  const float lenc = fmaxf(len, eps);
  const float rho = 0.5f * (rp - lp - rg + lg);
  const float q = rho / lenc;
  Diou d;
  d.loss = 1.f - iou + q * q;
  d.dlp = d.drp = d.dlg = d.drg = 0.f;
  if (grad) {
    const float um = uni >= eps ? 1.f : 0.f, cm = len >= eps ? 1.f : 0.f;
    // loss = 1 - I/Uc + (rho/Cc)^2 ;  dI, dU = d(sum) - dI, dC, drho per operand
    const float dI[4] = {dmin_a(lp, lg), dmin_a(rp, rg), dmin_a(lg, lp), dmin_a(rg, rp)};
    const float dC[4] = {dmax_a(lp, lg), dmax_a(rp, rg), dmax_a(lg, lp), dmax_a(rg, rp)};
    const float dr[4] = {-0.5f, 0.5f, 0.5f, -0.5f};
    float out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float dU = (1.f - dI[j]) * um;
      const float diou = (dI[j] * uc - inter * dU) / (uc * uc);
      const float dq = (dr[j] * lenc - rho * dC[j] * cm) / (lenc * lenc);
      out[j] = -diou + 2.f * q * dq;
    }
    d.dlp = out[0];
    d.drp = out[1];
    d.dlg = out[2];
    d.drg = out[3];
  }
  return d;
}

__global__ void diou_elem_kernel(const float* __restrict__ pr, const float* __restrict__ gt, int64_t n, float eps,
                                 float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = diou_eval(pr[2 * i], pr[2 * i + 1], gt[2 * i], gt[2 * i + 1], eps, false).loss;
}

__global__ __launch_bounds__(1024) void diou_sum_kernel(const float* __restrict__ pr, const float* __restrict__ gt,
                                                        int64_t n, float eps, float scale, float* __restrict__ out) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x)
    s += diou_eval(pr[2 * i], pr[2 * i + 1], gt[2 * i], gt[2 * i + 1], eps, false).loss;
  s = rp_wave_sum(s);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
    *out = tot * scale;
  }
}

__global__ void diou_bwd_kernel(const float* __restrict__ pr, const float* __restrict__ gt, int64_t n, float eps,
                                const float* __restrict__ gout, int per_elem, float gscale, float* __restrict__ dpr,
                                float* __restrict__ dgt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float g = (per_elem ? gout[i] : gout[0]) * gscale;
    const Diou d = diou_eval(pr[2 * i], pr[2 * i + 1], gt[2 * i], gt[2 * i + 1], eps, true);
    if (dpr) {
      dpr[2 * i] = g * d.dlp;
      dpr[2 * i + 1] = g * d.drp;
    }
    if (dgt) {
      dgt[2 * i] = g * d.dlg;
      dgt[2 * i + 1] = g * d.drg;
    }
  }
}

unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" int rp_tiou_hits(const float* pred, const int* pred_count, int P, const double* ref, const int* ref_count,
                            int R, const double* thresholds, int n_thr, int V, int* hits, void* stream) {
  RP_REQUIRE(V >= 0 && P >= 0 && R >= 0, "rp_tiou_hits: bad sizes");
  RP_REQUIRE(n_thr >= 1 && n_thr <= 32, "rp_tiou_hits: 1..32 thresholds");
  if (V == 0) return RP_OK;
  RP_REQUIRE(pred_count && ref_count && thresholds && hits, "rp_tiou_hits: null pointer");
  RP_REQUIRE((P == 0 || pred) && (R == 0 || ref), "rp_tiou_hits: null segments");
  hipLaunchKernelGGL(tiou_hits_kernel, dim3((unsigned)V), dim3(TIOU_NT), 0, (hipStream_t)stream, pred, pred_count, P,
                     ref, ref_count, R, thresholds, n_thr, hits);
  return rp_check_launch("rp_tiou_hits");
}

extern "C" int rp_diou_fwd(const float* pred, const float* gt, int64_t n, float eps, int reduction, float* out,
                           void* stream) {
  RP_REQUIRE(n >= 0 && reduction >= 0 && reduction <= 2, "rp_diou_fwd: bad arguments");
  RP_REQUIRE(out && (n == 0 || (pred && gt)), "rp_diou_fwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (reduction == 0) {
    if (n == 0) return RP_OK;
    hipLaunchKernelGGL(diou_elem_kernel, dim3(grid_for(n)), dim3(256), 0, s, pred, gt, n, eps, out);
  } else {
    const float scale = reduction == 1 ? (n > 0 ? 1.f / (float)n : 0.f) : 1.f;
    hipLaunchKernelGGL(diou_sum_kernel, dim3(1), dim3(1024), 0, s, pred, gt, n, eps, scale, out);
  }
  return rp_check_launch("rp_diou_fwd");
}

extern "C" int rp_diou_bwd(const float* pred, const float* gt, int64_t n, float eps, const float* grad_out,
                           int per_elem, float grad_scale, float* dpred, float* dgt, void* stream) {
  RP_REQUIRE(n >= 0, "rp_diou_bwd: bad n");
  if (n == 0) return RP_OK;
  RP_REQUIRE(pred && gt && grad_out && (dpred || dgt), "rp_diou_bwd: null pointer");
  hipLaunchKernelGGL(diou_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, pred, gt, n, eps, grad_out,
                     per_elem, grad_scale, dpred, dgt);
  return rp_check_launch("rp_diou_bwd");
}
