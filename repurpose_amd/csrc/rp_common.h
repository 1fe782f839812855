// Shared device/host helpers for the Repurpose MI355X (gfx950) kernels.
//
// Conventions used by every kernel in this directory
//   * element types: RP_F32 (float) and RP_BF16 (__bf16 storage, fp32 math)
//   * one wavefront = 64 lanes; MFMA 16x16x32 bf16 / 16x16x4 f32 (exact-f32 parity mode)
//   * every launcher is enqueued on the caller's hipStream_t and never synchronises
//   * dropout masks are regenerated from a counter hash (seed, stream index), never stored
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

#include "../../include/rp_api.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

#define RP_WAVE 64

// ----------------------------------------------------------------------------------------------
// host-side error plumbing (rp_last_error)
// ----------------------------------------------------------------------------------------------
void rp_set_error(const char* fmt, ...);
int rp_check_launch(const char* what);

#define RP_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      rp_set_error(__VA_ARGS__);              \
      return RP_ERR_ARG;                      \
    }                                         \
  } while (0)

static inline bool rp_aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

// ----------------------------------------------------------------------------------------------
// dropout hash: lowbias32-style finaliser over (seed, index).  keep <=> (h & 0xffff) >= thresh16
// thresh16 = round(p * 65536); kept values are scaled by 1/(1-p).
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rp_hash(uint32_t seed, uint32_t idx) {
  uint32_t h = idx * 0x9E3779B1u + seed;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

typedef short i16x2 __attribute__((ext_vector_type(2)));

// multiply-with-carry step (MWC64X): state x | c << 32 -> lo / hi of A x + c; output word x ^ c
constexpr uint32_t RP_MWC_A = 4294883355u;
__device__ __forceinline__ uint32_t rp_mwc_next(uint64_t& st) {
  st = (uint64_t)RP_MWC_A * (uint32_t)st + (st >> 32);
  return (uint32_t)st ^ (uint32_t)(st >> 32);
}

// Element dropout (GEMM / LayerNorm epilogues), per aligned group of 8 elements (index idx ->
// group idx >> 3, slot e = idx & 7): w0 = rp_hash(seed, group), then w1..w3 from the MWC64X
// stream seeded x = w0, c = w0 >> 1; slot e reads the 16-bit half (e & 1) of w(e >> 1) as int16
// and is kept iff it is >= thresh16 - 32768 (probability 1 - p to 2^-16).  Returns the 8 keep bits
// (bit e).  One hash + 3 one-multiply MWC steps per 8 elements (rounds 1-3: 3 xorshift32 steps,
// six shift / xor ops each); the keep test is a saturating packed 16-bit subtract + arithmetic
// shift per pair (no 32-bit multiply per element).
__device__ __forceinline__ uint32_t rp_keep8(uint32_t seed, uint32_t group, uint32_t thresh16) {
  uint32_t w = rp_hash(seed, group);
  uint64_t st = (uint64_t)w | ((uint64_t)(w >> 1) << 32);
  const short ts = (short)((int)thresh16 - 32768);
  const i16x2 t2 = {ts, ts};
  uint32_t acc = 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j) w = rp_mwc_next(st);
    const i16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(i16x2, w), t2);  // < 0: dropped
    const uint32_t m = __builtin_bit_cast(uint32_t, (i16x2)(d >> (short)15));
    acc |= ~m & ((1u << (2 * j)) | (1u << (16 + 2 * j + 1)));
  }
  return (acc & 0xFFFFu) | (acc >> 16);
}

// keep bits of VPT consecutive elements starting at idx0 (idx0 % VPT == 0, VPT a power of two)
template <int VPT>
__device__ __forceinline__ uint32_t rp_keep_bits(uint32_t seed, uint32_t idx0, uint32_t thresh16) {
  if constexpr (VPT >= 8) {
    uint32_t b = 0u;
#pragma unroll
    for (int g = 0; g < VPT / 8; ++g) b |= rp_keep8(seed, (idx0 >> 3) + g, thresh16) << (8 * g);
    return b;
  } else {
    return (rp_keep8(seed, idx0 >> 3, thresh16) >> (idx0 & 7)) & ((1u << VPT) - 1u);
  }
}

// Graph-replayable dropout streams: a launch's optional seed_base argument (per call, never process
// state) goes into its kernel arguments and the kernels draw with rp_hash(*base, seed), the base word
// read on the device when the kernel runs (a captured HIP graph replays with whatever the host last
// wrote there); with no base the seed argument is used as is.
__device__ __forceinline__ uint32_t rp_seed_eff(const uint32_t* base, uint32_t seed) {
  return base ? rp_hash(*base, seed) : seed;
}

static inline uint32_t rp_dropout_thresh(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 65536.0 + 0.5;
  if (t > 65536.0) t = 65536.0;
  return (uint32_t)t;
}

// ----------------------------------------------------------------------------------------------
// element load/store helpers (fp32 math everywhere)
// ----------------------------------------------------------------------------------------------
// 2^x as the bare v_exp_f32 (no denormal-range fix-up: results below 2^-126 flush to 0, which
// softmax weights tolerate; exp2f() adds ~6 VALU per call for that fix-up)
__device__ __forceinline__ float rp_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float rp_ld(const float* p) { return *p; }
__device__ __forceinline__ float rp_ld(const bf16* p) { return (float)(*p); }
__device__ __forceinline__ void rp_st(float* p, float v) { *p = v; }
__device__ __forceinline__ void rp_st(bf16* p, float v) { *p = (bf16)v; }

template <typename T>
struct rp_vec16;  // 16-byte vector of T
template <>
struct rp_vec16<float> {
  typedef float4 type;
  static constexpr int n = 4;
};
template <>
struct rp_vec16<bf16> {
  typedef uint4 type;
  static constexpr int n = 8;
};

// wave-wide reductions (64 lanes)
__device__ __forceinline__ float rp_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float rp_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over the 8 lanes of the lane's aligned group, on the VALU: DPP quad_perm [1,0,3,2], [2,3,0,1],
// then row_half_mirror.  Lane 8k gets bitwise the value of the __shfl_xor 1 / 2 / 4 tree (the same
// pairs, fp addition commuting), without its three LDS round trips (ds_bpermute).
template <int CTRL>
__device__ __forceinline__ float rp_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// rp_keep_bits<4> of a lane's 4-element chunks in two rows (element indices ia, ib), where the lane pair
// l, l ^ 1 holds the two halves of each aligned 8-element group (even lane: elements 0-3): each lane draws
// ONE group (the even lane row a's, the odd lane row b's) and takes the other from its partner, so the
// pair makes two rp_keep8 draws instead of four.  Bitwise rp_keep_bits<4>.
__device__ __forceinline__ void rp_keep4_pair(uint32_t seed, uint32_t ia, uint32_t ib, uint32_t thresh16, bool odd,
                                              uint32_t& ka, uint32_t& kb) {
  const uint32_t mine = rp_keep8(seed, (odd ? ib : ia) >> 3, thresh16);
  const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0xB1, 0xF, 0xF, false);  // l ^ 1
  const int sh = odd ? 4 : 0;
  ka = ((odd ? other : mine) >> sh) & 0xFu;
  kb = ((odd ? mine : other) >> sh) & 0xFu;
}

__device__ __forceinline__ float rp_sum8(float s) {
  s += rp_dpp<0xB1>(s);
  s += rp_dpp<0x4E>(s);
  return s + rp_dpp<0x141>(s);
}

// XCD-aware bijective workgroup remap (MI355X: 8 XCDs, blocks dealt round-robin).
// Consecutive logical tiles end up on one XCD so they share its L2.
__device__ __forceinline__ int rp_xcd_remap(int bid, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx;
  int x = bid % nx, i = bid / nx;
  int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + i;
}

// One LDS-DMA wave instruction (global_load_lds_dwordx4): lane l's 16 bytes at g land at LDS byte
// address lds + 16 l.  Inline asm on purpose: the compiler does not track it, so it inserts no
// conservative vmcnt(0) before the LDS reads of a pipelined loop (its alias analysis cannot tell
// that they read another ring slot) — the caller orders every DMA before its readers with a counted
// s_waitcnt vmcnt + barrier.  m0 is saved and restored around it.
__device__ __forceinline__ void rp_dma16(const void* g, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, off\n\t"
      "s_nop 0\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "v"(g)
      : "memory");
}

// A 16-byte output store under a cache policy: 0 plain (the line stays dirty in the XCD's L2 and is
// written back at the kernel-end release), 1 sc1 (write-through: the bytes go on to HBM while the
// epilogue runs), 2 nt (streaming).  The asm store ends in s_nop 1 so its data registers are read
// before the next instruction can overwrite them.
typedef uint32_t rp_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void rp_st16(void* p, uint4 v, int pol) {
  const rp_u32x4 w = {v.x, v.y, v.z, v.w};
  if (pol == 1)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  else if (pol == 2)
    __builtin_nontemporal_store(w, reinterpret_cast<rp_u32x4*>(p));
  else
    *reinterpret_cast<rp_u32x4*>(p) = w;
}
__device__ __forceinline__ void rp_st16(void* p, float4 v, int pol) {
  rp_st16(p, make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)), pol);
}

// A 16-byte fp32 load under a cache policy: 2 nt (streaming: the line is not kept), else plain
typedef float rp_f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 rp_ld16f(const float* p, int pol) {
  if (pol == 2) {
    const rp_f32x4v w = __builtin_nontemporal_load(reinterpret_cast<const rp_f32x4v*>(p));
    return make_float4(w.x, w.y, w.z, w.w);
  }
  return *reinterpret_cast<const float4*>(p);
}

__device__ __forceinline__ uint32_t rp_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
