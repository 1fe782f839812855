// Issue cost of candidate dropout-stream generators on gfx950 (tuning aid for the attention
// forward, whose tile loop is VALU-issue bound): xorshift32 (the shipping stream, 6 VALU per 32-bit
// word) vs multiply-with-carry (one v_mad_u64_u32 per word).  Every lane runs 8 independent
// streams; 8 waves per CU over all CUs; the XOR of all words goes to one store per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(512) void xs(uint32_t* out, int iters) {
  uint32_t st[8];
  for (int j = 0; j < 8; ++j) st[j] = 0x9E3779B9u * (threadIdx.x + 1 + j * 977u) + blockIdx.x;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t x = st[j];
      x ^= x << 13;
      x ^= x >> 17;
      x ^= x << 5;
      st[j] = x;
      acc += x;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ __launch_bounds__(512) void mwc(uint32_t* out, int iters) {
  uint64_t st[8];
  for (int j = 0; j < 8; ++j) st[j] = (uint64_t)(0x9E3779B9u * (threadIdx.x + 1 + j * 977u) + blockIdx.x) | (1ull << 40);
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)4294957665u * (uint32_t)st[j] + (st[j] >> 32);
      st[j] = t;
      acc += (uint32_t)t;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = ncu, threads = 512, iters = 4096;
  uint32_t* d;
  hipMalloc(&d, (size_t)blocks * threads * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL(xs, dim3(blocks), dim3(threads), 0, 0, d, iters);
      else hipLaunchKernelGGL(mwc, dim3(blocks), dim3(threads), 0, 0, d, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double words = (double)blocks * threads * iters * 8;
      // per SIMD: two waves of this CU's 8; cycles at an assumed 2.1 GHz
      const double wave_words_per_simd = words / 64 / (ncu * 4);
      printf("%s: %.3f ms, %.2f ns per word per SIMD-wave-instruction, ~%.1f cycles/word @2.1GHz\n",
             v == 0 ? "xorshift32" : "mwc(mad_u64_u32)", ms, ms * 1e6 / wave_words_per_simd,
             ms * 1e-3 * 2.1e9 / wave_words_per_simd);
    }
  }
  hipFree(d);
  return 0;
}
