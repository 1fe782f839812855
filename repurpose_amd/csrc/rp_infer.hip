// Inference post-processing on the GPU, one workgroup per video:
//   rp_infer_select  = inference_single_video   (reference models/MMCTransformer.py:181-229)
//   rp_softnms       = soft_nms_intervals_cpu   (reference models/softnms.py:3-38)
// Both are latency-bound (T <= 8192 frames, <= 1000 candidates per video); all per-video state
// lives in LDS and a batch of videos runs as one launch instead of a Python loop with a
// device->host copy per video (reference :248-273).
//
// Soft-NMS reproduces every reference quirk bit-for-bit in float32:
// positional (stale) lengths, pre-swap selection score, first-index argmax, break before decay,
// IEEE-rounded arithmetic and numpy's own float32 exp (np_expf below).
#include <math.h>

#include "rp_common.h"

namespace {

constexpr int SEL_THREADS = 1024;
constexpr int SEL_MAXT = 8192;

// ---------------------------------------------------------------- block scan helpers -------
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
  // 1024 threads, 16 waves
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  if (w == 0) {
    int s = lane < (int)(blockDim.x >> 6) ? sh[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < 16) sh[16 + lane] = s;  // inclusive wave totals
  }
  __syncthreads();
  const int base = w > 0 ? sh[16 + w - 1] : 0;
  total = sh[16 + (int)(blockDim.x >> 6) - 1];
  __syncthreads();
  return base + x - v;
}

__global__ __launch_bounds__(SEL_THREADS) void select_kernel(const float* __restrict__ logits,
                                                             const uint8_t* __restrict__ mask,
                                                             const float* __restrict__ offsets, int T_, float thresh,
                                                             int topk, float dmin, float dmax, int* __restrict__ count,
                                                             int64_t* __restrict__ idx_out, float* __restrict__ score_out,
                                                             float* __restrict__ seg_out) {
  __shared__ unsigned long long key[SEL_MAXT];
  __shared__ int sh[32];
  const int b = blockIdx.x;
  int npad = 1;
  while (npad < T_) npad <<= 1;
  // composite key: prob bits (prob >= 0 -> monotone) high, ~index low -> descending sort gives
  // (prob desc, index asc), i.e. a stable descending order
  for (int t = threadIdx.x; t < npad; t += blockDim.x) {
    unsigned long long k = 0ull;
    if (t < T_) {
      const float x = logits[(int64_t)b * T_ + t];
      const float p = (1.f / (1.f + expf(-x))) * (mask[(int64_t)b * T_ + t] ? 1.f : 0.f);
      if (p > thresh) k = ((unsigned long long)__float_as_uint(p) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)t);
    }
    key[t] = k;
  }
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= npad; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < npad; t += blockDim.x) {
        const int partner = t ^ stride;
        if (partner > t) {
          const bool desc = (t & size) == 0;
          unsigned long long a = key[t], c = key[partner];
          if (desc ? (a < c) : (a > c)) {
            key[t] = c;
            key[partner] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // candidates are the non-zero keys (all at the front); keep the first min(topk, n)
  int ncand_part = 0;
  for (int t = threadIdx.x; t < npad; t += blockDim.x) ncand_part += key[t] != 0ull;
  int ncand = 0;
  (void)block_excl_scan(ncand_part, sh, ncand);
  const int kk = ncand < topk ? ncand : topk;
  // position p (< kk, <= topk <= 1024 handled by thread p in chunks)
  int written = 0;
  for (int p0 = 0; p0 < kk; p0 += blockDim.x) {
    const int p = p0 + threadIdx.x;
    int ok = 0;
    float left = 0.f, right = 0.f, prob = 0.f;
    int64_t frame = 0;
    if (p < kk) {
      const unsigned long long k = key[p];
      frame = (int64_t)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull));
      prob = __uint_as_float((uint32_t)(k >> 32));
      const float fi = (float)frame;
      const float o0 = offsets[((int64_t)b * T_ + frame) * 2 + 0];
      const float o1 = offsets[((int64_t)b * T_ + frame) * 2 + 1];
      left = fi - o0;
      right = fi + o1;
      const float dur = right - left;
      ok = (dur > dmin) && (dur < dmax);
    }
    int tot = 0;
    const int pos = written + block_excl_scan(ok, sh, tot);
    if (ok) {
      const int64_t o = (int64_t)b * topk + pos;
      idx_out[o] = frame;
      score_out[o] = prob;
      seg_out[o * 2 + 0] = left;
      seg_out[o * 2 + 1] = right;
    }
    written += tot;
  }
  if (threadIdx.x == 0) count[b] = written;
}

// ---------------------------------------------------------------- Soft-NMS -----------------
constexpr int NMS_THREADS = 1024;
constexpr int NMS_LDS_CAP = 6144;  // candidates held in LDS (5 floats each, 120 KiB); beyond: workspace

// numpy's float32 exp, the SIMD routine np.exp runs on AVX2 / AVX512F hosts (what the reference's
// `np.exp(-(r*r)/sigma)` executes, models/softnms.py:35): Cody-Waite reduction by round(x*log2 e)
// with a two-constant ln 2, a [5/2] rational minimax polynomial evaluated with FMAs, one IEEE
// division and a 2^k scale.  It is not correctly rounded (about 10 % of the float32 inputs in
// [-2, 0] land one ulp away from the correctly rounded exp); this restatement matches numpy 2.2
// bit for bit on every float32 of [-2, 0] (checked exhaustively on a host: tests/golden/np_exp_check.py).
__device__ __forceinline__ float np_expf(float x) {
  if (x != x) return x;
  if (x > 88.72283935546875f) return INFINITY;
  if (x < -103.97208404541015625f) return 0.f;
  const float q = rintf(__fmul_rn(x, 1.442695040888963407359924681001892137f));
  float y = fmaf(q, -6.93145752e-1f, x);
  y = fmaf(q, -1.42860677e-6f, y);
  float num = fmaf(5.082762527590693718096e-04f, y, 6.757896990527504603057e-03f);
  num = fmaf(num, y, 5.114512081637298353406e-02f);
  num = fmaf(num, y, 2.473615434895520810817e-01f);
  num = fmaf(num, y, 7.257664613233124478488e-01f);
  num = fmaf(num, y, 9.999999999980870924916e-01f);
  float den = fmaf(2.159509375685829852307e-02f, y, -2.742335390411667452936e-01f);
  den = fmaf(den, y, 1.0f);
  return ldexpf(__fdiv_rn(num, den), (int)q);
}

// One workgroup per video; per-candidate state (score, begin, end, original index, positional length)
// in LDS for n <= NMS_LDS_CAP, else in a global workspace slice of the video (GLOBAL): the workgroup
// barriers order those accesses the same way (workgroup-scope fences, one CU).
template <bool GLOBAL>
__global__ __launch_bounds__(NMS_THREADS) void softnms_kernel(const float* __restrict__ scores,
                                                              const float* __restrict__ segs,
                                                              const int* __restrict__ count, int cap, float sigma,
                                                              float thresh, const int* __restrict__ max_seg,
                                                              int* __restrict__ keep, int* __restrict__ keep_count,
                                                              float* __restrict__ final_scores, float* __restrict__ ws) {
  extern __shared__ float dyn[];
  __shared__ float wv[16];
  __shared__ int wi[16];
  __shared__ int sh[32];
  __shared__ int bj;
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int n = count[b];
  const int ms = max_seg[b];
  const int limit = ms < n ? ms : n;
  float* base = GLOBAL ? ws + (int64_t)b * 5 * cap : dyn;
  const int st = GLOBAL ? cap : n;
  float* s = base;
  float* beg = base + st;
  float* en = base + 2 * st;
  float* org = base + 3 * st;
  float* len = base + 4 * st;
  for (int e = t; e < n; e += NMS_THREADS) {
    s[e] = scores[(int64_t)b * cap + e];
    beg[e] = segs[((int64_t)b * cap + e) * 2 + 0];
    en[e] = segs[((int64_t)b * cap + e) * 2 + 1];
    org[e] = (float)e;
    len[e] = en[e] - beg[e];  // positional, never swapped (reference softnms.py:13)
  }
  __threadfence_block();
  __syncthreads();
  int picked = 0;
  for (int i = 0; i < n; ++i) {
    const float ts = s[i];  // pre-swap score (:18)
    if (i != n - 1) {
      // first-index argmax over s[i+1 : n]: each thread scans its elements in increasing order
      // (strict > keeps the first), then the wave / workgroup reductions break ties by index
      float v = -INFINITY;
      int vi = 0x7fffffff;
      for (int e = t; e < n; e += NMS_THREADS) {
        if (e <= i) continue;
        const float x = s[e];
        if (vi == 0x7fffffff || x > v) {
          v = x;
          vi = e;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(vi, o, 64);
        if (oi != 0x7fffffff && (vi == 0x7fffffff || ov > v || (ov == v && oi < vi))) {
          v = ov;
          vi = oi;
        }
      }
      if (lane == 0) {
        wv[w] = v;
        wi[w] = vi;
      }
      __syncthreads();
      if (t == 0) {
        float bv = wv[0];
        int bi = wi[0];
        for (int k = 1; k < NMS_THREADS / 64; ++k)
          if (wi[k] != 0x7fffffff && (bi == 0x7fffffff || wv[k] > bv || (wv[k] == bv && wi[k] < bi))) {
            bv = wv[k];
            bi = wi[k];
          }
        bj = (ts < bv) ? bi : -1;  // np.amax / np.argmax; a NaN never compares greater
        if (bj >= 0) {
          // swap rows i <-> j (begin, end, original index) and scores (:23-25)
          float x;
          x = beg[i]; beg[i] = beg[bj]; beg[bj] = x;
          x = en[i]; en[i] = en[bj]; en[bj] = x;
          x = org[i]; org[i] = org[bj]; org[bj] = x;
          x = s[i]; s[i] = s[bj]; s[bj] = x;
        }
      }
      __threadfence_block();
      __syncthreads();
    }
    if (ts > thresh) {
      ++picked;
      if (picked >= limit) break;  // before the decay (:26-29)
    }
    const float bi = beg[i], ei = en[i], li = len[i];
    for (int e = t; e < n; e += NMS_THREADS) {
      if (e <= i) continue;
      const float ov = fmaxf(__fsub_rn(fminf(ei, en[e]), fmaxf(bi, beg[e])), 0.f);
      const float tl = __fsub_rn(__fadd_rn(li, len[e]), ov);
      const float r = __fdiv_rn(ov, tl);
      const float ex = __fdiv_rn(-__fmul_rn(r, r), sigma);
      s[e] = __fmul_rn(np_expf(ex), s[e]);
    }
    __threadfence_block();
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  // keep = rows[s > thresh][:limit, 2], in row order, 1024 rows per pass
  int written = 0;
  for (int e0 = 0; e0 < n && written < limit; e0 += NMS_THREADS) {
    const int e = e0 + t;
    const int ok = (e < n) && (s[e] > thresh);
    int tot = 0;
    const int pos = written + block_excl_scan(ok, sh, tot);
    if (ok && pos < limit) keep[(int64_t)b * cap + pos] = (int)org[e];
    written += tot;
  }
  if (t == 0) keep_count[b] = written < limit ? written : limit;
  if (final_scores)
    for (int e = t; e < n; e += NMS_THREADS) final_scores[(int64_t)b * cap + e] = s[e];
}

}  // namespace

extern "C" int rp_infer_select(const float* logits, const uint8_t* mask, const float* offsets, int B, int T, float thresh,
                               int topk, float dur_min, float dur_max, int* count, int64_t* idx, float* score, float* seg,
                               void* stream) {
  RP_REQUIRE(B >= 0 && T >= 0 && topk >= 0, "rp_infer_select: bad shape");
  RP_REQUIRE(T <= SEL_MAXT, "rp_infer_select: T=%d exceeds %d", T, SEL_MAXT);
  if (B == 0) return RP_OK;
  RP_REQUIRE(count, "rp_infer_select: null count");
  RP_REQUIRE(T == 0 || (logits && mask && offsets), "rp_infer_select: null input");
  RP_REQUIRE(topk == 0 || (idx && score && seg), "rp_infer_select: null output");
  hipLaunchKernelGGL(select_kernel, dim3(B), dim3(SEL_THREADS), 0, (hipStream_t)stream, logits, mask, offsets, T, thresh,
                     topk, dur_min, dur_max, count, idx, score, seg);
  return rp_check_launch("rp_infer_select");
}

extern "C" int64_t rp_softnms_workspace(int B, int cap) {
  return cap > NMS_LDS_CAP && B > 0 ? (int64_t)B * 5 * cap * (int64_t)sizeof(float) : 0;
}

extern "C" int rp_softnms(const float* scores, const float* segs, const int* count, int B, int cap, float sigma,
                          float thresh, const int* max_seg, int* keep, int* keep_count, float* final_scores,
                          void* workspace, int64_t ws_bytes, void* stream) {
  RP_REQUIRE(B >= 0 && cap >= 0, "rp_softnms: bad shape");
  if (B == 0) return RP_OK;
  RP_REQUIRE(count && max_seg && keep_count, "rp_softnms: null pointer");
  RP_REQUIRE(cap == 0 || (scores && segs && keep), "rp_softnms: null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (cap <= NMS_LDS_CAP) {
    const size_t lds = (size_t)5 * (cap > 0 ? cap : 1) * sizeof(float);
    if (lds > 65536) {  // above 64 KiB of dynamic LDS (up to 120 KiB of the CU's 160): opt the kernel in
      // the attribute is per device: set it on every such launch (cheap), not once per process, so a
      // later launch on another device is opted in as well
      const hipError_t opt = hipFuncSetAttribute((const void*)softnms_kernel<false>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)(5 * NMS_LDS_CAP * sizeof(float)));
      RP_REQUIRE(opt == hipSuccess, "rp_softnms: cannot enable %zu bytes of dynamic LDS: %s", lds,
                 hipGetErrorString(opt));
    }
    hipLaunchKernelGGL(softnms_kernel<false>, dim3(B), dim3(NMS_THREADS), lds, st, scores, segs, count, cap, sigma,
                       thresh, max_seg, keep, keep_count, final_scores, (float*)nullptr);
  } else {
    RP_REQUIRE(workspace && ws_bytes >= rp_softnms_workspace(B, cap),
               "rp_softnms: cap %d > %d needs rp_softnms_workspace(B, cap) bytes of workspace", cap, NMS_LDS_CAP);
    hipLaunchKernelGGL(softnms_kernel<true>, dim3(B), dim3(NMS_THREADS), 0, st, scores, segs, count, cap, sigma, thresh,
                       max_seg, keep, keep_count, final_scores, (float*)workspace);
  }
  return rp_check_launch("rp_softnms");
}
