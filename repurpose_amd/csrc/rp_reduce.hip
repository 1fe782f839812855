// rp_reduce — batched sums of squares for the trainer's gradient-norm logging (reference
// main.py:345-367: every 10 iterations, rank 0 takes `.grad.norm().item()` of each nn.Linear weight
// and bias and of every parameter for the total — one host sync per tensor).  Here every tensor's
// sum of squares is one workgroup of one launch (64 tensors per launch), accumulated in fp64 in a
// fixed order (deterministic), written to a device array the caller copies to the host once.
#include "rp_common.h"

namespace {

constexpr int SSQ_MAX = 64;
constexpr int SSQ_NT = 1024;

struct SsqBatch {
  rp_sumsq_item it[SSQ_MAX];
};

__global__ __launch_bounds__(SSQ_NT) void sumsq_batched_kernel(const SsqBatch b) {
  const rp_sumsq_item t = b.it[blockIdx.x];
  const float* __restrict__ x = t.x;
  const int64_t n = t.n;
  const int tid = threadIdx.x;
  double s = 0.0;
  // 16-byte chunks from the first aligned element, scalar head / tail
  const int64_t head = (int64_t)((16 - ((uintptr_t)x & 15)) & 15) / 4;
  const int64_t h = head < n ? head : n;
  for (int64_t i = tid; i < h; i += SSQ_NT) s = fma((double)x[i], (double)x[i], s);
  const int64_t nv = (n - h) / 4;
  const float4* __restrict__ xv = reinterpret_cast<const float4*>(x + h);
  for (int64_t i = tid; i < nv; i += SSQ_NT) {
    const float4 v = xv[i];
    s = fma((double)v.x, (double)v.x, s);
    s = fma((double)v.y, (double)v.y, s);
    s = fma((double)v.z, (double)v.z, s);
    s = fma((double)v.w, (double)v.w, s);
  }
  for (int64_t i = h + nv * 4 + tid; i < n; i += SSQ_NT) s = fma((double)x[i], (double)x[i], s);
  // wave tree, then the 16 wave sums in order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ double ws[SSQ_NT / 64];
  if ((tid & 63) == 0) ws[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < SSQ_NT / 64; ++w) r += ws[w];
    *t.out = r;
  }
}

}  // namespace

extern "C" int rp_sumsq_batched(const rp_sumsq_item* items, int n_items, void* stream) {
  RP_REQUIRE(n_items >= 0 && n_items <= SSQ_MAX, "rp_sumsq_batched: 0..%d items per call, got %d", SSQ_MAX, n_items);
  RP_REQUIRE(n_items == 0 || items, "rp_sumsq_batched: null item array");
  if (n_items == 0) return RP_OK;
  SsqBatch b;
  for (int i = 0; i < n_items; ++i) {
    RP_REQUIRE(items[i].n >= 0 && items[i].out && (items[i].n == 0 || items[i].x), "rp_sumsq_batched: item %d", i);
    RP_REQUIRE(((uintptr_t)items[i].x & 3) == 0, "rp_sumsq_batched: item %d not 4-byte aligned", i);
    b.it[i] = items[i];
  }
  hipLaunchKernelGGL(sumsq_batched_kernel, dim3(n_items), dim3(SSQ_NT), 0, (hipStream_t)stream, b);
  return rp_check_launch("rp_sumsq_batched");
}
