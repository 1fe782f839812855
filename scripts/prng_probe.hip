// Probe of gfx950's v_prng_b32 (__builtin_amdgcn_prng_b32): prints the outputs for chosen inputs so
// the function can be characterised on the host (tuning aid for the attention dropout stream).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const unsigned* in, unsigned* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_prng_b32(in[i]);
}
int main() {
  const int n = 4096;
  unsigned h[n], o[n];
  for (int i = 0; i < 64; ++i) h[i] = i < 32 ? (1u << i) : (unsigned)(i - 32);
  unsigned x = 0x12345678u;
  for (int i = 64; i < n; ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; h[i] = x; }
  unsigned *din, *dout;
  hipMalloc(&din, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(din, h, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, din, dout, n);
  hipMemcpy(o, dout, n * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("%08x %08x\n", h[i], o[i]);
  return 0;
}
