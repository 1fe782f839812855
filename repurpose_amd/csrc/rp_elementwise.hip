// HBM-bound helpers of the hot path:
//   rp_concat_rows      K1, modality concat (+ bf16 cast)      models/MMCTransformer.py:118
//   rp_cast_f32_to_bf16 master-weight -> bf16 operand copy
//   rp_colsum           bias / LayerNorm affine gradients (deterministic two-pass column sum)
//   rp_focal_*          sigmoid_focal_loss (alpha .7, gamma 2) + mask + sum and its gradient
//                       models/losses.py:4-53, models/MMCTransformer.py:159-179
//   rp_rowdot_*         the N<=4 head outputs (cls_head[7], reg_head[7]+ReLU) :71-93
//   rp_adam_step        torch.optim.Adam with coupled weight decay over one flat buffer
#include <math.h>

#include "rp_common.h"

namespace {

// ---------------------------------------------------------------- concat / cast ------------
template <typename TO>
__global__ void concat_kernel(const float* __restrict__ v, int dv, const float* __restrict__ a, int da,
                              const float* __restrict__ t, int dt, int64_t rows, TO* __restrict__ out) {
  // one workgroup per row (no index division); 16-byte loads, one vector store per 4 elements
  const int D = dv + da + dt;
  const int64_t r = blockIdx.x;
  TO* orow = out + r * D;
  // CU loads per thread issued together before any store (a load-convert-store loop keeps one load in
  // flight per wave: latency-bound at ~3.6 TB/s for the step's 16384 x 2944 rows)
  constexpr int CU = 4;
  for (int c0 = threadIdx.x * 4; c0 < D; c0 += CU * blockDim.x * 4) {
    float4 q[CU];
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const int c = c0 + u * blockDim.x * 4;
      if (c >= D) break;
      // the features are read once: non-temporal (the output stays cached for the projection GEMM)
      if (c < dv)
        q[u] = rp_ld16f(v + r * dv + c, 2);
      else if (c < dv + da)
        q[u] = rp_ld16f(a + r * da + (c - dv), 2);
      else
        q[u] = rp_ld16f(t + r * dt + (c - dv - da), 2);
    }
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const int c = c0 + u * blockDim.x * 4;
      if (c >= D) break;
      if constexpr (std::is_same<TO, float>::value) {
        *reinterpret_cast<float4*>(orow + c) = q[u];
      } else {
        *reinterpret_cast<bf16x4*>(orow + c) = bf16x4{(bf16)q[u].x, (bf16)q[u].y, (bf16)q[u].z, (bf16)q[u].w};
      }
    }
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ s, bf16* __restrict__ d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = (bf16)s[i];
}

inline unsigned grid_for(int64_t n, int bs) {
  int64_t g = (n + bs - 1) / bs;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---------------------------------------------------------------- colsum -------------------
constexpr int CS_ROWS = 64;
constexpr int CS_THREADS = 256;

template <typename T>
__global__ void colsum_pass1(const T* __restrict__ X, int64_t rows, int64_t cols, int64_t ldx,
                             const float* __restrict__ w, float* __restrict__ ws) {
  const int64_t c = (int64_t)blockIdx.y * CS_THREADS + threadIdx.x;
  if (c >= cols) return;
  const int64_t r0 = (int64_t)blockIdx.x * CS_ROWS;
  const int n = (int)(rows - r0 < CS_ROWS ? rows - r0 : CS_ROWS);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = 0;
  if (n == CS_ROWS) {
    // a whole block: every row's load issued before the first add (one memory round trip instead of
    // one per eight rows), the sums in the loop's order below (bitwise the same)
    float x[CS_ROWS], wr[CS_ROWS];
#pragma unroll
    for (int u = 0; u < CS_ROWS; ++u) {
      x[u] = rp_ld(X + (r0 + u) * ldx + c);
      wr[u] = w ? w[r0 + u] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < CS_ROWS; ++u) s[u & 7] += w ? wr[u] * x[u] : x[u];
    r = n;
  }
  for (; r + 8 <= n; r += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float x = rp_ld(X + (r0 + r + u) * ldx + c);
      s[u] += w ? w[r0 + r + u] * x : x;
    }
  }
  for (; r < n; ++r) {
    const float x = rp_ld(X + (r0 + r) * ldx + c);
    s[0] += w ? w[r0 + r] * x : x;
  }
  ws[(int64_t)blockIdx.x * cols + c] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// single pass for short inputs (rows <= CS1_MAX_ROWS): a block owns 64 columns (16 float4 chunks)
// and 64 row groups; each thread sums its rows in order, the groups are added in order through LDS
constexpr int CS1_MAX_ROWS = 2048;
template <typename T>
__device__ __forceinline__ void colsum_block(const T* __restrict__ X, int64_t rows, int64_t cols, int64_t ldx,
                                             const float* __restrict__ w, float* __restrict__ out, int accumulate,
                                             int64_t cblk) {
  const int ch = threadIdx.x & 15, rg = threadIdx.x >> 4;  // 16 column chunks x 64 row groups
  const int64_t c = cblk * 64 + ch * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < cols) {
    const bool vec = std::is_same<T, float>::value && c + 3 < cols && (ldx & 3) == 0;
    // rows rg, rg + 64, ... in order, eight loads in flight per step
    for (int64_t r0 = rg; r0 < rows; r0 += 64 * 8) {
      float4 v[8];
      float wr[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t r = r0 + 64 * u;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        wr[u] = 0.f;
        if (r < rows) {
          const T* p = X + r * ldx + c;
          wr[u] = w ? w[r] : 1.f;
          if (vec) {
            v[u] = *reinterpret_cast<const float4*>(p);
          } else {
            v[u].x = rp_ld(p);
            v[u].y = c + 1 < cols ? rp_ld(p + 1) : 0.f;
            v[u].z = c + 2 < cols ? rp_ld(p + 2) : 0.f;
            v[u].w = c + 3 < cols ? rp_ld(p + 3) : 0.f;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s.x += wr[u] * v[u].x; s.y += wr[u] * v[u].y; s.z += wr[u] * v[u].z; s.w += wr[u] * v[u].w;
      }
    }
  }
  __shared__ float4 red[64][16];
  red[rg][ch] = s;
  __syncthreads();
  // fixed-shape tree over the 64 row groups (deterministic)
#pragma unroll
  for (int h = 32; h >= 1; h >>= 1) {
    if (rg < h) {
      const float4 q = red[rg + h][ch];
      float4 t = red[rg][ch];
      t.x += q.x; t.y += q.y; t.z += q.z; t.w += q.w;
      red[rg][ch] = t;
    }
    __syncthreads();
  }
  if (rg == 0 && c < cols) {
    const float4 t = red[0][ch];
    // explicit stores: a dynamically indexed local array would live in scratch
    out[c] = accumulate ? out[c] + t.x : t.x;
    if (c + 1 < cols) out[c + 1] = accumulate ? out[c + 1] + t.y : t.y;
    if (c + 2 < cols) out[c + 2] = accumulate ? out[c + 2] + t.z : t.z;
    if (c + 3 < cols) out[c + 3] = accumulate ? out[c + 3] + t.w : t.w;
  }
}

template <typename T>
__global__ __launch_bounds__(1024) void colsum_onepass(const T* __restrict__ X, int64_t rows, int64_t cols,
                                                       int64_t ldx, const float* __restrict__ w,
                                                       float* __restrict__ out, int accumulate) {
  colsum_block<T>(X, rows, cols, ldx, w, out, accumulate, blockIdx.x);
}

// many fp32 column sums in one launch (the LayerNorm gamma / beta partials of a whole backward):
// item k owns blocks [start[k], start[k+1]), one 64-column slice each, same sums as colsum_onepass
constexpr int CSB_MAX = 64;
struct CsItem {
  const float* X;
  float* out;
  int rows, cols, ldx, accumulate;
};
struct CsBatch {
  int n;
  int start[CSB_MAX + 1];
  CsItem it[CSB_MAX];
};

__global__ __launch_bounds__(1024) void colsum_batched_kernel(const CsBatch bt) {
  const int blk = blockIdx.x;
  int k = 0;
  while (k + 1 < bt.n && blk >= bt.start[k + 1]) ++k;
  const CsItem c = bt.it[k];
  colsum_block<float>(c.X, c.rows, c.cols, c.ldx, nullptr, c.out, c.accumulate, blk - bt.start[k]);
}

__global__ void colsum_pass2(const float* __restrict__ ws, int64_t nrb, int64_t cols, float* __restrict__ out,
                             int accumulate) {
  const int64_t c = (int64_t)blockIdx.x * CS_THREADS + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int64_t b = 0; b < nrb; ++b) s += ws[b * cols + c];
  out[c] = accumulate ? out[c] + s : s;
}

// ---------------------------------------------------------------- focal loss ---------------
struct Focal {
  float loss, grad;
};

__device__ __forceinline__ Focal focal_eval(float x, float t, float alpha, float gamma, bool need_grad) {
  const float p = 1.f / (1.f + expf(-x));
  const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float omp = 1.f - pt;
  const float mod = (gamma == 2.f) ? omp * omp : powf(omp, gamma);
  const float at = alpha >= 0.f ? alpha * t + (1.f - alpha) * (1.f - t) : 1.f;
  Focal f;
  f.loss = at * ce * mod;
  f.grad = 0.f;
  if (need_grad) {
    const float dmod = (gamma == 2.f) ? 2.f * omp : gamma * powf(omp, gamma - 1.f);
    const float dpt = p * (1.f - p) * (2.f * t - 1.f);
    f.grad = at * ((p - t) * mod - ce * dmod * dpt);
  }
  return f;
}

__global__ __launch_bounds__(1024) void focal_sum_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                         const uint8_t* __restrict__ mask, int64_t n, float alpha,
                                                         float gamma, float* __restrict__ loss) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (mask && !mask[i]) continue;
    s += focal_eval(x[i], t[i], alpha, gamma, false).loss;
  }
  s = rp_wave_sum(s);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
    *loss = tot;
  }
}

// Multi-workgroup form (rp_focal_fwd_sum_ws): workgroup b sums elements [b chunk, (b + 1) chunk) in the
// order of focal_sum_kernel's loop (thread-strided, wave sums, the waves in order) into ws[b]; one wave
// then sums the partials in index order.  Deterministic for a given n (the chunking depends on n only).
constexpr int FOCAL_WG = 256;
constexpr int64_t FOCAL_CHUNK = 512;  // two elements per thread: 32 workgroups for 16,384 frames
__global__ __launch_bounds__(FOCAL_WG) void focal_part_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                              const uint8_t* __restrict__ mask, int64_t n, float alpha,
                                                              float gamma, float* __restrict__ ws) {
  const int64_t lo = (int64_t)blockIdx.x * FOCAL_CHUNK;
  const int64_t hi = lo + FOCAL_CHUNK < n ? lo + FOCAL_CHUNK : n;
  float s = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += FOCAL_WG) {
    if (mask && !mask[i]) continue;
    s += focal_eval(x[i], t[i], alpha, gamma, false).loss;
  }
  s = rp_wave_sum(s);
  __shared__ float red[FOCAL_WG / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < FOCAL_WG / 64; ++w) tot += red[w];
    ws[blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(64) void focal_final_kernel(const float* __restrict__ ws, int64_t parts,
                                                         float* __restrict__ loss) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < parts; i += 64) s += ws[i];
  s = rp_wave_sum(s);
  if (threadIdx.x == 0) *loss = s;
}

__global__ void focal_elem_kernel(const float* __restrict__ x, const float* __restrict__ t, int64_t n, float alpha,
                                  float gamma, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = focal_eval(x[i], t[i], alpha, gamma, false).loss;
}

__global__ void focal_bwd_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                 const uint8_t* __restrict__ mask, int64_t n, float alpha, float gamma,
                                 const float* __restrict__ gout, int per_elem, float* __restrict__ dx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float g = per_elem ? gout[i] : gout[0];
    if (mask && !mask[i]) g = 0.f;
    dx[i] = g == 0.f ? 0.f : g * focal_eval(x[i], t[i], alpha, gamma, true).grad;
  }
}

// ---------------------------------------------------------------- rowdot (N <= 4) ----------
template <typename T>
__global__ __launch_bounds__(256) void rowdot_fwd_kernel(const T* __restrict__ X, int64_t ldx, int64_t rows, int K,
                                                         const float* __restrict__ W, const float* __restrict__ b,
                                                         int nout, int relu, float* __restrict__ out, int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k = lane; k < K; k += 64) {
    const float xv = rp_ld(X + r * ldx + k);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < nout) acc[j] += xv * W[(int64_t)j * K + k];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j >= nout) break;
    float s = rp_wave_sum(acc[j]) + (b ? b[j] : 0.f);
    if (relu) s = fmaxf(s, 0.f);
    if (lane == 0) out[r * ldo + j] = s;
  }
}

// bf16 rows with 16-byte chunks (K % 8 == 0, X and ldx 16-byte aligned): eight lanes per row, each a
// bf16x8 chunk per 64-column step, the row's partials summed over its eight lanes (quad perms +
// half-mirror); 32 rows per workgroup.  The heads' [M, 256] projections: one wave per row spent its time
// on 2-byte loads and a 64-lane reduction per row.
__global__ __launch_bounds__(256) void rowdot_fwd8_kernel(const bf16* __restrict__ X, int64_t ldx, int64_t rows, int K,
                                                          const float* __restrict__ W, const float* __restrict__ b,
                                                          int nout, int relu, float* __restrict__ out, int64_t ldo) {
  const int l8 = threadIdx.x & 7;
  const int64_t r = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  const bool live = r < rows;  // every lane runs the reductions (DPP)
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    const bf16* xr = X + r * ldx;
    for (int k = l8 * 8; k < K; k += 64) {
      const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xr + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nout) break;
        const float4 w0 = *reinterpret_cast<const float4*>(W + (int64_t)j * K + k);
        const float4 w1 = *reinterpret_cast<const float4*>(W + (int64_t)j * K + k + 4);
        acc[j] += (((float)xv[0] * w0.x + (float)xv[1] * w0.y) + ((float)xv[2] * w0.z + (float)xv[3] * w0.w)) +
                  (((float)xv[4] * w1.x + (float)xv[5] * w1.y) + ((float)xv[6] * w1.z + (float)xv[7] * w1.w));
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j >= nout) break;
    float s = rp_sum8(acc[j]) + (b ? b[j] : 0.f);
    if (relu) s = fmaxf(s, 0.f);
    if (live && l8 == 0) out[r * ldo + j] = s;
  }
}

template <typename TG, typename TX>
__global__ void rowdot_bwd_kernel(const float* __restrict__ dout, int64_t ldd, int64_t rows, int K,
                                  const float* __restrict__ W, int nout, const TG* __restrict__ G, int64_t ldg,
                                  float gate_scale, TX* __restrict__ dX, int64_t lddx) {
  const int64_t n = rows * (int64_t)K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / K;
    const int k = (int)(i % K);
    float s = 0.f;
    for (int j = 0; j < nout; ++j) s += dout[r * ldd + j] * W[(int64_t)j * K + k];
    if (G) s = rp_ld(G + r * ldg + k) > 0.f ? s * gate_scale : 0.f;
    rp_st(dX + r * lddx + k, s);
  }
}

// ---------------------------------------------------------------- Adam ---------------------
// coef = {lr / bc1, beta1, beta2, eps, weight_decay, sqrt(bc2)} (rp_adam_coefficients)
__device__ __forceinline__ void adam_elem(float& pi, float gi, float& mi, float& vi, const float (&c)[6]) {
  if (c[4] != 0.f) gi = gi + c[4] * pi;
  mi = mi + (1.f - c[1]) * (gi - mi);
  vi = vi * c[2] + (1.f - c[2]) * gi * gi;
  const float denom = sqrtf(vi) / c[5] + c[3];
  pi = pi - c[0] * (mi / denom);
}

// one element per thread-iteration (measured on MI355X: 243-246 us per step for 52.6 M parameters,
// against 258-269 us for a float4 variant).  DEV: the coefficients are read from device memory when
// the kernel runs (graph replay), else taken from the arguments.
template <bool DEV>
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, const float* __restrict__ coef_dev, float c0, float c1,
                            float c2, float c3, float c4, float c5, bf16* __restrict__ plp) {
  float c[6];
  if (DEV) {
#pragma unroll
    for (int i = 0; i < 6; ++i) c[i] = coef_dev[i];
  } else {
    c[0] = c0; c[1] = c1; c[2] = c2; c[3] = c3; c[4] = c4; c[5] = c5;
  }
  // the fp32 master, the moments and the gradient are touched once per step: non-temporal (the bf16
  // operand copy, read by the next forward's GEMMs, is stored plainly)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pi = __builtin_nontemporal_load(p + i), mi = __builtin_nontemporal_load(m + i),
          vi = __builtin_nontemporal_load(v + i);
    adam_elem(pi, __builtin_nontemporal_load(g + i), mi, vi, c);
    __builtin_nontemporal_store(pi, p + i);
    __builtin_nontemporal_store(mi, m + i);
    __builtin_nontemporal_store(vi, v + i);
    if (plp) plp[i] = (bf16)pi;
  }
}

}  // namespace

// ---------------------------------------------------------------- ragged -> padded batch -----------
// dst[b][t][d] = t < len_b ? (float)src[(offs[b] + t) * D + d] : pad   (len_b = offs[b+1] - offs[b])
// torch's copy conversion: fp16 -> fp32 exact, fp64 -> fp32 round-to-nearest-even, int64 -> fp32.
template <typename S>
__device__ __forceinline__ float to_f32(S v) { return (float)v; }

template <typename S>
__global__ void pad_rows_kernel(const S* __restrict__ src, const int64_t* __restrict__ offs, int B, int T, int D,
                                float pad, float* __restrict__ dst) {
  const int64_t n = (int64_t)B * T * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bt = i / D;
    const int d = (int)(i - bt * D);
    const int b = (int)(bt / T), t = (int)(bt - (int64_t)b * T);
    const int64_t o = offs[b], len = offs[b + 1] - o;
    dst[i] = t < len ? to_f32(src[(o + t) * D + d]) : pad;
  }
}

extern "C" int rp_concat_rows(const float* v, int dv, const float* a, int da, const float* t, int dt, int64_t rows,
                              void* out, int out_dtype, void* stream) {
  RP_REQUIRE(dv >= 0 && da >= 0 && dt >= 0 && rows >= 0, "rp_concat_rows: negative size");
  RP_REQUIRE(dv % 4 == 0 && da % 4 == 0 && dt % 4 == 0, "rp_concat_rows: widths must be multiples of 4");
  RP_REQUIRE(rows < (1ll << 31), "rp_concat_rows: too many rows");
  RP_REQUIRE((dv == 0 || v) && (da == 0 || a) && (dt == 0 || t) && out, "rp_concat_rows: null pointer");
  RP_REQUIRE(rp_aligned16(out) && rp_aligned16(v) && rp_aligned16(a) && rp_aligned16(t),
             "rp_concat_rows: 16-byte aligned buffers required");
  const int64_t n4 = rows * (int64_t)((dv + da + dt) / 4);
  if (n4 == 0) return RP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (out_dtype == RP_BF16)
    hipLaunchKernelGGL(concat_kernel<bf16>, dim3((unsigned)rows), dim3(256), 0, s, v, dv, a, da, t, dt, rows, (bf16*)out);
  else if (out_dtype == RP_F32)
    hipLaunchKernelGGL(concat_kernel<float>, dim3((unsigned)rows), dim3(256), 0, s, v, dv, a, da, t, dt, rows, (float*)out);
  else {
    rp_set_error("rp_concat_rows: bad dtype");
    return RP_ERR_ARG;
  }
  return rp_check_launch("rp_concat_rows");
}

extern "C" int rp_cast_f32_to_bf16(const float* src, void* dst, int64_t n, void* stream) {
  RP_REQUIRE(n >= 0, "rp_cast_f32_to_bf16: negative n");
  if (n == 0) return RP_OK;
  RP_REQUIRE(src && dst, "rp_cast_f32_to_bf16: null");
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, src, (bf16*)dst, n);
  return rp_check_launch("rp_cast_f32_to_bf16");
}

extern "C" int rp_colsum_batched(const rp_colsum_item* items, int n_items, void* stream) {
  RP_REQUIRE(n_items >= 0 && n_items <= CSB_MAX, "rp_colsum_batched: 0..%d items per launch", CSB_MAX);
  if (n_items == 0) return RP_OK;
  RP_REQUIRE(items, "rp_colsum_batched: null items");
  CsBatch bt{};
  bt.n = n_items;
  int64_t blocks = 0;
  for (int i = 0; i < n_items; ++i) {
    const rp_colsum_item& c = items[i];
    RP_REQUIRE(c.rows >= 0 && c.cols > 0 && c.ldx >= c.cols && c.rows <= INT32_MAX && c.ldx <= INT32_MAX &&
                   c.cols <= INT32_MAX,
               "rp_colsum_batched: item %d: bad shape", i);
    RP_REQUIRE(c.out && (c.rows == 0 || c.X), "rp_colsum_batched: item %d: null pointer", i);
    bt.start[i] = (int)blocks;
    bt.it[i] = CsItem{c.X, c.out, (int)c.rows, (int)c.cols, (int)c.ldx, c.accumulate};
    blocks += (c.cols + 63) / 64;
  }
  RP_REQUIRE(blocks < (1 << 30), "rp_colsum_batched: too many blocks");
  bt.start[n_items] = (int)blocks;
  hipLaunchKernelGGL(colsum_batched_kernel, dim3((unsigned)blocks), dim3(1024), 0, (hipStream_t)stream, bt);
  return rp_check_launch("rp_colsum_batched");
}

extern "C" int64_t rp_colsum_workspace(int64_t rows, int64_t cols) {
  return ((rows + CS_ROWS - 1) / CS_ROWS) * cols;
}

extern "C" int rp_colsum(const void* X, int dtype, int64_t rows, int64_t cols, int64_t ldx, const float* w, float* out,
                         int accumulate, float* workspace, void* stream) {
  RP_REQUIRE(rows >= 0 && cols >= 0, "rp_colsum: negative size");
  if (cols == 0) return RP_OK;
  RP_REQUIRE(out && workspace, "rp_colsum: null output/workspace");
  hipStream_t s = (hipStream_t)stream;
  if (rows > 0 && rows <= CS1_MAX_ROWS) {
    RP_REQUIRE(X, "rp_colsum: null X");
    const dim3 g((unsigned)((cols + 63) / 64));
    if (dtype == RP_BF16)
      hipLaunchKernelGGL(colsum_onepass<bf16>, g, dim3(1024), 0, s, (const bf16*)X, rows, cols, ldx, w, out, accumulate);
    else
      hipLaunchKernelGGL(colsum_onepass<float>, g, dim3(1024), 0, s, (const float*)X, rows, cols, ldx, w, out,
                         accumulate);
    return rp_check_launch("rp_colsum");
  }
  const int64_t nrb = (rows + CS_ROWS - 1) / CS_ROWS;
  if (nrb > 0) {
    RP_REQUIRE(X, "rp_colsum: null X");
    dim3 g1((unsigned)nrb, (unsigned)((cols + CS_THREADS - 1) / CS_THREADS));
    if (dtype == RP_BF16)
      hipLaunchKernelGGL(colsum_pass1<bf16>, g1, dim3(CS_THREADS), 0, s, (const bf16*)X, rows, cols, ldx, w, workspace);
    else
      hipLaunchKernelGGL(colsum_pass1<float>, g1, dim3(CS_THREADS), 0, s, (const float*)X, rows, cols, ldx, w, workspace);
  }
  // second pass over the nrb partial rows with the single-pass kernel (nrb <= CS1_MAX_ROWS for any
  // rows < CS1_MAX_ROWS * CS_ROWS; beyond that the serial pass)
  if (nrb <= CS1_MAX_ROWS)
    hipLaunchKernelGGL(colsum_onepass<float>, dim3((unsigned)((cols + 63) / 64)), dim3(1024), 0, s, workspace, nrb, cols,
                       cols, (const float*)nullptr, out, accumulate);
  else
    hipLaunchKernelGGL(colsum_pass2, dim3((unsigned)((cols + CS_THREADS - 1) / CS_THREADS)), dim3(CS_THREADS), 0, s,
                       workspace, nrb, cols, out, accumulate);
  return rp_check_launch("rp_colsum");
}

extern "C" int64_t rp_focal_ws_elems(int64_t n) { return n > 0 ? (n + FOCAL_CHUNK - 1) / FOCAL_CHUNK : 1; }

extern "C" int rp_focal_fwd_sum_ws(const float* x, const float* t, const uint8_t* mask, int64_t n, float alpha,
                                   float gamma, float* ws, int64_t ws_elems, float* loss, void* stream) {
  RP_REQUIRE(n >= 0 && loss, "rp_focal_fwd_sum_ws: bad args");
  RP_REQUIRE(n == 0 || (x && t), "rp_focal_fwd_sum_ws: null input");
  const int64_t parts = rp_focal_ws_elems(n);
  RP_REQUIRE(ws && ws_elems >= parts, "rp_focal_fwd_sum_ws: workspace of %lld floats needed", (long long)parts);
  RP_REQUIRE(parts < (1 << 30), "rp_focal_fwd_sum_ws: n too large");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    hipLaunchKernelGGL(focal_final_kernel, dim3(1), dim3(64), 0, s, ws, (int64_t)0, loss);
    return rp_check_launch("rp_focal_fwd_sum_ws");
  }
  hipLaunchKernelGGL(focal_part_kernel, dim3((unsigned)parts), dim3(FOCAL_WG), 0, s, x, t, mask, n, alpha, gamma, ws);
  hipLaunchKernelGGL(focal_final_kernel, dim3(1), dim3(64), 0, s, ws, parts, loss);
  return rp_check_launch("rp_focal_fwd_sum_ws");
}

extern "C" int rp_focal_fwd_sum(const float* x, const float* t, const uint8_t* mask, int64_t n, float alpha, float gamma,
                                float* loss, void* stream) {
  RP_REQUIRE(n >= 0 && loss, "rp_focal_fwd_sum: bad args");
  RP_REQUIRE(n == 0 || (x && t), "rp_focal_fwd_sum: null input");
  hipLaunchKernelGGL(focal_sum_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, t, mask, n, alpha, gamma, loss);
  return rp_check_launch("rp_focal_fwd_sum");
}

extern "C" int rp_focal_elementwise(const float* x, const float* t, int64_t n, float alpha, float gamma, float* out,
                                    void* stream) {
  RP_REQUIRE(n >= 0, "rp_focal_elementwise: negative n");
  if (n == 0) return RP_OK;
  RP_REQUIRE(x && t && out, "rp_focal_elementwise: null");
  hipLaunchKernelGGL(focal_elem_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, t, n, alpha, gamma, out);
  return rp_check_launch("rp_focal_elementwise");
}

extern "C" int rp_focal_bwd(const float* x, const float* t, const uint8_t* mask, int64_t n, float alpha, float gamma,
                            const float* grad_out, int grad_per_elem, float* dx, void* stream) {
  RP_REQUIRE(n >= 0, "rp_focal_bwd: negative n");
  if (n == 0) return RP_OK;
  RP_REQUIRE(x && t && grad_out && dx, "rp_focal_bwd: null");
  hipLaunchKernelGGL(focal_bwd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, t, mask, n, alpha,
                     gamma, grad_out, grad_per_elem, dx);
  return rp_check_launch("rp_focal_bwd");
}

extern "C" int rp_rowdot_fwd(int x_dtype, const void* X, int64_t ldx, int64_t rows, int K, const float* W, const float* b,
                             int nout, int relu, float* out, int64_t ldo, void* stream) {
  RP_REQUIRE(nout >= 1 && nout <= 4, "rp_rowdot_fwd: nout must be 1..4");
  RP_REQUIRE(rows >= 0 && K > 0, "rp_rowdot_fwd: bad size");
  if (rows == 0) return RP_OK;
  RP_REQUIRE(X && W && out, "rp_rowdot_fwd: null");
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == RP_BF16 && K % 8 == 0 && ldx % 8 == 0 && rp_aligned16(X) && rp_aligned16(W))
    hipLaunchKernelGGL(rowdot_fwd8_kernel, dim3((unsigned)((rows + 31) / 32)), dim3(256), 0, s, (const bf16*)X, ldx,
                       rows, K, W, b, nout, relu, out, ldo);
  else if (x_dtype == RP_BF16)
    hipLaunchKernelGGL(rowdot_fwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)X, ldx, rows, K, W, b, nout, relu, out, ldo);
  else
    hipLaunchKernelGGL(rowdot_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)X, ldx, rows, K, W, b, nout, relu, out, ldo);
  return rp_check_launch("rp_rowdot_fwd");
}

extern "C" int rp_rowdot_bwd_dx(const float* dout, int64_t ldd, int64_t rows, int K, const float* W, int nout, const void* G,
                                int g_dtype, int64_t ldg, float gate_scale, void* dX, int dx_dtype, int64_t lddx,
                                void* stream) {
  RP_REQUIRE(nout >= 1 && nout <= 4, "rp_rowdot_bwd_dx: nout must be 1..4");
  if (rows <= 0) return RP_OK;
  RP_REQUIRE(dout && W && dX, "rp_rowdot_bwd_dx: null");
  const int64_t n = rows * (int64_t)K;
  dim3 grid(grid_for(n, 256));
  hipStream_t s = (hipStream_t)stream;
#define RP_RD_LAUNCH(TG, TX) \
  hipLaunchKernelGGL((rowdot_bwd_kernel<TG, TX>), grid, dim3(256), 0, s, dout, ldd, rows, K, W, nout, (const TG*)G, ldg, gate_scale, (TX*)dX, lddx)
  if (g_dtype == RP_BF16) {
    if (dx_dtype == RP_BF16) RP_RD_LAUNCH(bf16, bf16); else RP_RD_LAUNCH(bf16, float);
  } else {
    if (dx_dtype == RP_BF16) RP_RD_LAUNCH(float, bf16); else RP_RD_LAUNCH(float, float);
  }
#undef RP_RD_LAUNCH
  return rp_check_launch("rp_rowdot_bwd_dx");
}

extern "C" int rp_adam_coefficients(float lr, float beta1, float beta2, float eps, float weight_decay, int step,
                                    float* coef) {
  RP_REQUIRE(step >= 1 && coef, "rp_adam_coefficients: bad step / null output");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  coef[0] = (float)(lr / bc1);
  coef[1] = beta1;
  coef[2] = beta2;
  coef[3] = eps;
  coef[4] = weight_decay;
  coef[5] = (float)sqrt(bc2);
  return RP_OK;
}

static int adam_launch(float* p, const float* g, float* m, float* v, int64_t n, const float* coef_dev,
                       const float* c, void* p_lp, void* stream) {
  if (n == 0) return RP_OK;
  RP_REQUIRE(p && g && m && v, "rp_adam_step: null");
  const dim3 grid(grid_for(n, 256));
  if (coef_dev)
    hipLaunchKernelGGL(adam_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, coef_dev, 0.f, 0.f,
                       0.f, 0.f, 0.f, 0.f, (bf16*)p_lp);
  else
    hipLaunchKernelGGL(adam_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, nullptr, c[0], c[1],
                       c[2], c[3], c[4], c[5], (bf16*)p_lp);
  return rp_check_launch("rp_adam_step");
}

extern "C" int rp_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                            float eps, float weight_decay, int step, void* p_lp, void* stream) {
  RP_REQUIRE(n >= 0 && step >= 1, "rp_adam_step: bad n/step");
  float c[6];
  rp_adam_coefficients(lr, beta1, beta2, eps, weight_decay, step, c);
  return adam_launch(p, g, m, v, n, nullptr, c, p_lp, stream);
}

extern "C" int rp_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* coef_dev,
                                void* p_lp, void* stream) {
  RP_REQUIRE(n >= 0 && coef_dev, "rp_adam_step_dev: bad n / null coef");
  return adam_launch(p, g, m, v, n, coef_dev, nullptr, p_lp, stream);
}

extern "C" int rp_pad_rows(const void* src, int src_dtype, const int64_t* row_offsets, int B, int T, int D, float pad,
                           float* dst, void* stream) {
  RP_REQUIRE(B >= 0 && T >= 0 && D > 0, "rp_pad_rows: bad shape");
  if (B == 0 || T == 0) return RP_OK;
  RP_REQUIRE(row_offsets && dst, "rp_pad_rows: null pointer");
  const int64_t n = (int64_t)B * T * D;
  int64_t g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  hipStream_t s = (hipStream_t)stream;
  switch (src_dtype) {
    case RP_F32: hipLaunchKernelGGL(pad_rows_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, (const float*)src, row_offsets, B, T, D, pad, dst); break;
    case RP_F16: hipLaunchKernelGGL(pad_rows_kernel<_Float16>, dim3((unsigned)g), dim3(256), 0, s, (const _Float16*)src, row_offsets, B, T, D, pad, dst); break;
    case RP_F64: hipLaunchKernelGGL(pad_rows_kernel<double>, dim3((unsigned)g), dim3(256), 0, s, (const double*)src, row_offsets, B, T, D, pad, dst); break;
    case RP_I64: hipLaunchKernelGGL(pad_rows_kernel<int64_t>, dim3((unsigned)g), dim3(256), 0, s, (const int64_t*)src, row_offsets, B, T, D, pad, dst); break;
    default: rp_set_error("rp_pad_rows: bad src dtype %d", src_dtype); return RP_ERR_ARG;
  }
  return rp_check_launch("rp_pad_rows");
}
