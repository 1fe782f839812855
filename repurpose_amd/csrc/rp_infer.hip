// Inference post-processing on the GPU, one workgroup per video:
//   rp_infer_select  = inference_single_video   (reference models/MMCTransformer.py:181-229)
//   rp_softnms       = soft_nms_intervals_cpu   (reference models/softnms.py:3-38)
// Both are latency-bound (T <= 8192 frames, <= 1000 candidates per video); all per-video state
// lives in LDS and a batch of videos runs as one launch instead of a Python loop with a
// device->host copy per video (reference :248-273).
//
// Soft-NMS reproduces every reference quirk bit-for-bit in float32:
// positional (stale) lengths, pre-swap selection score, first-index argmax, break before decay,
// IEEE-rounded division and a correctly rounded exp (computed in double, rounded once).
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

__global__ __launch_bounds__(NMS_THREADS) void softnms_kernel(const float* __restrict__ scores,
                                                              const float* __restrict__ segs,
                                                              const int* __restrict__ count, int cap, float sigma,
                                                              float thresh, const int* __restrict__ max_seg,
                                                              int* __restrict__ keep, int* __restrict__ keep_count,
                                                              float* __restrict__ final_scores) {
  __shared__ float s[NMS_THREADS], beg[NMS_THREADS], en[NMS_THREADS], org[NMS_THREADS], len[NMS_THREADS];
  __shared__ float wv[16];
  __shared__ int wi[16];
  __shared__ int sh[32];
  __shared__ int bj;
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int n = count[b];
  const int ms = max_seg[b];
  const int limit = ms < n ? ms : n;
  if (t < n) {
    s[t] = scores[(int64_t)b * cap + t];
    beg[t] = segs[((int64_t)b * cap + t) * 2 + 0];
    en[t] = segs[((int64_t)b * cap + t) * 2 + 1];
    org[t] = (float)t;
    len[t] = en[t] - beg[t];  // positional, never swapped (reference softnms.py:13)
  }
  __syncthreads();
  int picked = 0;
  for (int i = 0; i < n; ++i) {
    const float ts = s[i];  // pre-swap score (:18)
    if (i != n - 1) {
      // first-index argmax over s[i+1 : n]
      float v = -INFINITY;
      int vi = 0x7fffffff;
      if (t > i && t < n) {
        v = s[t];
        vi = t;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(vi, o, 64);
        if (ov > v || (ov == v && oi < vi)) {
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
          if (wv[k] > bv || (wv[k] == bv && wi[k] < bi)) {
            bv = wv[k];
            bi = wi[k];
          }
        bj = (ts < bv) ? bi : -1;
        if (bj >= 0) {
          // swap rows i <-> j (begin, end, original index) and scores (:23-25)
          float x;
          x = beg[i]; beg[i] = beg[bj]; beg[bj] = x;
          x = en[i]; en[i] = en[bj]; en[bj] = x;
          x = org[i]; org[i] = org[bj]; org[bj] = x;
          x = s[i]; s[i] = s[bj]; s[bj] = x;
        }
      }
      __syncthreads();
    }
    if (ts > thresh) {
      ++picked;
      if (picked >= limit) break;  // before the decay (:26-29)
    }
    if (t > i && t < n) {
      const float ov = fmaxf(fminf(en[i], en[t]) - fmaxf(beg[i], beg[t]), 0.f);
      const float tl = (len[i] + len[t]) - ov;
      const float r = __fdiv_rn(ov, tl);
      const float e = __fdiv_rn(-(r * r), sigma);
      const float wgt = (float)exp((double)e);
      s[t] = __fmul_rn(wgt, s[t]);
    }
    __syncthreads();
  }
  __syncthreads();
  // keep = rows[s > thresh][:limit, 2]
  const int ok = (t < n) && (s[t] > thresh);
  int tot = 0;
  const int pos = block_excl_scan(ok, sh, tot);
  if (ok && pos < limit) keep[(int64_t)b * cap + pos] = (int)org[t];
  if (t == 0) keep_count[b] = tot < limit ? tot : limit;
  if (final_scores && t < n) final_scores[(int64_t)b * cap + t] = s[t];
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

extern "C" int rp_softnms(const float* scores, const float* segs, const int* count, int B, int cap, float sigma,
                          float thresh, const int* max_seg, int* keep, int* keep_count, float* final_scores,
                          void* stream) {
  RP_REQUIRE(B >= 0 && cap >= 0 && cap <= NMS_THREADS, "rp_softnms: cap must be <= %d", NMS_THREADS);
  if (B == 0) return RP_OK;
  RP_REQUIRE(count && max_seg && keep_count, "rp_softnms: null pointer");
  RP_REQUIRE(cap == 0 || (scores && segs && keep), "rp_softnms: null pointer");
  hipLaunchKernelGGL(softnms_kernel, dim3(B), dim3(NMS_THREADS), 0, (hipStream_t)stream, scores, segs, count, cap, sigma,
                     thresh, max_seg, keep, keep_count, final_scores);
  return rp_check_launch("rp_softnms");
}
