// Flash-style multi-head self attention for the 16 encoder layers (reference: the stock
// nn.MultiheadAttention -> F.scaled_dot_product_attention path of the nn.TransformerEncoderLayer
// built at models/MMCTransformer.py:41-55, key padding mask from :132; dropout 0.1 on P in train).
//
// Layout: qkv [B*T, 3*H*64] (q heads | k heads | v heads, the in_proj output order), out
// [B*T, H*64], lse [B, H, T].  The T x T score matrix is never materialised.
//
// MI355X design
//  * "key on the MFMA row" (swapped) products: the forward computes S^T = K Q^T so that the score
//    accumulator, packed to bf16, IS the B operand of O^T += V^T P^T (no LDS round trip for P);
//    V^T fragments come from the row-major V tile through the gfx950 transposed LDS read
//    ds_read_b64_tr_b16.  The k order inside an MFMA is permuted consistently on both operands.
//  * backward = two kernels without atomics: dK/dV per 128-key block (S, dP computed with the
//    query on the MFMA row so P^T / dS^T feed dV, dK directly) and dQ per 128-query block
//    (S^T, dP^T so dS feeds dQ directly).  Deterministic, no fp32 atomics.
//  * online softmax in the exp2 domain; the row max is reduced over the 4 lanes sharing a query
//    with two __shfl_xor per tile, the row sum stays per lane until the epilogue; the O rescale is
//    skipped when no row max grew (wave-uniform test); mask bias only on tiles with masked keys.
//  * dropout (p = 0.1 in training): the forward draws the keep bits ONCE (one 32-bit hash per key
//    pair, 16-bit threshold -> p exact to 1e-5) and stores them as a bit mask, 2 bytes per
//    (query, 16 keys) — 1/16 of the bf16 P matrix; both backward kernels read the bits instead of
//    re-hashing (the hash is the dominant VALU cost of a dk = 64 attention).
//  * bf16: v_mfma_f32_16x16x32_bf16; fp32 parity mode: exact v_mfma_f32_16x16x4_f32 with the
//    same data flow (k-slot g <-> key 4g+r).
#include <math.h>

#include "rp_common.h"

namespace {

constexpr int HD = 64;   // head dim (dk) — the Repurpose config (512 / 8 heads)
constexpr int NW = 4;    // waves per workgroup
constexpr int NT = NW * 64;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float RESCALE_LOG2 = 8.f;  // forward: deferred-rescale threshold (log2 units)


template <typename T>
struct AttnCfg {
  // bf16 tiles: 128-byte rows, XOR-swizzled (see lds_off); fp32 parity tiles: 16-byte row padding
  static constexpr int ROWB = std::is_same<T, bf16>::value ? HD * 2 : HD * 4 + 16;
  static constexpr int CPR = HD * (int)sizeof(T) / 16;  // 16-byte chunks per row
};

// Byte offset of (row, byte-in-row) in an LDS tile.  bf16: the 16-byte chunk index is XORed with
// lds_swz(row) = ((row >> 1) & 3) << 1, i.e. the 32-byte pair index with (row >> 1) & 3, which makes
// both 16x16x32 access patterns conflict-free: ds_read_b128 row fragments (16 lanes = 16 rows x 2
// adjacent chunks cover all 16 bank quads) and ds_read_b64_tr_b16 column fragments (8 consecutive
// rows x one 32-byte pair cover all 8 bank octets).  (Adding the chunk-parity bit (row >> 3) & 1,
// which spreads a 32x32x16 row fragment over all 16 quads, made these 16x16 kernels 6-9 % slower,
// +0.27 ms per step: measured and reverted, round 3.)
__device__ __forceinline__ int lds_swz(int row) { return ((row >> 1) & 3) << 1; }
template <typename T>
__device__ __forceinline__ int lds_off(int row, int byte) {
  if constexpr (std::is_same<T, bf16>::value)
    return row * 128 + (byte ^ (lds_swz(row) << 4));
  else
    return row * AttnCfg<T>::ROWB + byte;
}

// keep-bit mask layout (the forward's register layout, so the forward and dQ kernels move one
// 16-bit word per lane and key tile): [B*H][KT = ceil(T/64)][4 lane groups g][ldm = roundup(T,128)]
// (a row covers every query of the last 128-query block, so block-wide stores and DMA pieces of a
// row never reach the next one)
// uint16; bit (kt*4 + r) of word (bh, tile, g, q) = keep(q, key = 64*tile + 16*kt + 4*g + r)
__host__ __device__ inline int64_t mask_ld(int T) { return ((int64_t)T + 127) / 128 * 128; }
__host__ __device__ inline int mask_kt(int T) { return (T + 63) / 64; }

// ----- problem description (device side of rp_mha_args) ------------------------------------------
// q [B*Tq rows, ldq], k / v [B*Tk rows, ldk / ldv]: head h at columns h*64..h*64+63 of each row;
// out / dout [B*Tq rows, ldo / lddo]; dq [B*Tq, lddq], dk / dv [B*Tk, lddk / lddv];
// lse / delta [B, H, Tq] fp32; key_valid [B, Tk]; dropout keep bits over (Tq, Tk) (see mask_ld).
struct MhaDev {
  const void* q; const void* k; const void* v;
  int64_t ldq, ldk, ldv;
  const uint8_t* kvalid;
  int B, Tq, Tk, H;
  float scale;
  uint32_t drop_thresh; float drop_scale; uint32_t seed;
  const uint32_t* seed_base;  // graph-replayable dropout base word (the launch's seed_base argument), or null
  void* out; int64_t ldo;
  void* out_lo;  // bf16: O - bf16(O) rounded to bf16 (same layout as out), or null
  float* lse;
  uint16_t* dmask;
  const void* dout; int64_t lddo;
  float* delta;
  void* dq; int64_t lddq; void* dk; int64_t lddk; void* dv; int64_t lddv;
  int qpre;  // RP_ATTN_Q_PRESCALED: q holds Q * scale * log2(e) (see include/rp_api.h)
  int empty_uniform;  // a sequence with no valid key attends uniformly to all keys (masked_fill(-1e9))
  uint64_t mwc_jump;  // split forward: A^(8 n) * 2^64 mod M, n = the key tiles of one part (mwc_jump)
};

// MWC64X skip-ahead.  The state S = c * 2^32 + x steps as S' = A * S mod M, M = A * 2^32 - 1, so n
// steps are one multiplication by A^n mod M.  mwc_mulmod(s, p) = s * p * 2^-64 mod M by two reduction
// steps of the form Y * 2^-32 = (Y >> 32) + (Y mod 2^32) * A (mod M, as A * 2^32 = 1); the host folds
// the 2^64 into the multiplier (mwc_jump).  s, p < M.
constexpr uint64_t RP_MWC_M = ((uint64_t)RP_MWC_A << 32) - 1u;
__host__ __device__ inline uint64_t mwc_mulmod(uint64_t s, uint64_t p) {
  const uint64_t lo = s * p;
#ifdef __HIP_DEVICE_COMPILE__
  const uint64_t hi = __umul64hi(s, p);
#else
  const uint64_t hi = (uint64_t)(((unsigned __int128)s * p) >> 64);
#endif
  // Y1 = X * 2^-32 = (hi:lo >> 32) + (lo mod 2^32) * A  (< 2^96 + 2^64: y1h never wraps, hi < 2^64 - 2^33)
  const uint64_t t = (uint64_t)(uint32_t)lo * RP_MWC_A;
  const uint64_t mid = (hi << 32) | (lo >> 32);
  const uint64_t y1l = mid + t;
  const uint64_t y1h = (hi >> 32) + (y1l < t ? 1u : 0u);
  // Z = Y1 * 2^-32 = (Y1 >> 32) + (Y1 mod 2^32) * A  (< 2^65)
  const uint64_t u = (uint64_t)(uint32_t)y1l * RP_MWC_A;
  const uint64_t v = (y1h << 32) | (y1l >> 32);
  uint64_t r = v + u;
  if (r < u) {  // Z >= 2^64: Z - M = r + (2^64 - M), once more if that still wraps
    const uint64_t k64 = 0u - RP_MWC_M;
    const uint64_t r2 = r + k64;
    r = r2 < r ? r2 + k64 : r2;
  }
  return r >= RP_MWC_M ? r - RP_MWC_M : r;
}
// host: A^(8 n) * 2^64 mod M (the multiplier that advances a stream by n 64-key tiles, 8 steps each)
static inline uint64_t mwc_jump(int n) {
  const unsigned __int128 m = RP_MWC_M;
  unsigned __int128 r = ((unsigned __int128)1 << 64) % m, b = RP_MWC_A;
  for (uint64_t e = 8u * (uint64_t)n; e; e >>= 1) {
    if (e & 1u) r = r * b % m;
    b = b * b % m;
  }
  return (uint64_t)r;
}

// empty_uniform: does sequence b have no valid key at all?  (whole workgroup; uniform result)
__device__ __forceinline__ bool seq_has_no_key(const MhaDev& a, int b, int tid) {
  if (!a.empty_uniform) return false;
  int any = 0;
  for (int k = tid; k < a.Tk; k += NT) any |= a.kvalid[(int64_t)b * a.Tk + k];
  return __syncthreads_or(any) == 0;
}

// ----- global [rows][64] (row stride ld elements) <-> LDS [rows][ROWB] staging ------------------
template <typename T, int ROWS>
struct Stage {
  static constexpr int PER = ROWS * AttnCfg<T>::CPR / NT;
  uint4 r[PER];
  __device__ __forceinline__ void load(const T* __restrict__ base, int64_t ld, int row0, int nrows, int tid) {
    if (row0 + ROWS <= nrows) {  // whole tile in range (uniform): no per-row predication
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int id = tid + NT * i;
        const int row = id / AttnCfg<T>::CPR, c = id % AttnCfg<T>::CPR;
        r[i] = *reinterpret_cast<const uint4*>(base + (int64_t)(row0 + row) * ld + c * (16 / (int)sizeof(T)));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int id = tid + NT * i;
      int row = id / AttnCfg<T>::CPR, c = id % AttnCfg<T>::CPR;
      if (row0 + row < nrows)
        r[i] = *reinterpret_cast<const uint4*>(base + (int64_t)(row0 + row) * ld + c * (16 / (int)sizeof(T)));
      else
        r[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int id = tid + NT * i;
      int row = id / AttnCfg<T>::CPR, c = id % AttnCfg<T>::CPR;
      *reinterpret_cast<uint4*>(lds + lds_off<T>(row, c * 16)) = r[i];
    }
  }
  __device__ __forceinline__ void store_zero(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int id = tid + NT * i;
      int row = id / AttnCfg<T>::CPR, c = id % AttnCfg<T>::CPR;
      *reinterpret_cast<uint4*>(lds + lds_off<T>(row, c * 16)) = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  // bf16 only: store bf16(x * c) — the same rounding as the forward's prescale of Q
  __device__ __forceinline__ void store_scaled(char* lds, int tid, float c) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int id = tid + NT * i;
      int row = id / AttnCfg<T>::CPR, cc = id % AttnCfg<T>::CPR;
      bf16x8 v = __builtin_bit_cast(bf16x8, r[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] * c);
      *reinterpret_cast<uint4*>(lds + lds_off<T>(row, cc * 16)) = __builtin_bit_cast(uint4, v);
    }
  }
};

// ----- fragment helpers -------------------------------------------------------------------------
// bf16 row fragment: lane holds X[r0 + (l&15)][k0 + 8*(l>>4) + j]   (MFMA 16x16x32 A/B operand)
__device__ __forceinline__ bf16x8 row_frag_lds(const char* lds, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + lds_off<bf16>(r0 + (lane & 15), (k0 + 8 * (lane >> 4)) * 2));
}
__device__ __forceinline__ bf16x8 row_frag_gmem(const bf16* base, int64_t ld, int r0, int nrows, int k0, int lane) {
  int r = r0 + (lane & 15);
  if (r >= nrows) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
    return z;
  }
  return *reinterpret_cast<const bf16x8*>(base + (int64_t)r * ld + k0 + 8 * (lane >> 4));
}
// bf16 "column" fragment through ds_read_b64_tr_b16: lane (g = l>>4, i = l&15) receives
//   X[R + 4g + {0..3}][c0 + i]  and  X[R + 16 + 4g + {0..3}][c0 + i]     (8 values)
// i.e. the k-slot order (g, j) <-> row R + (j<4 ? 4g+j : 16+4g+j-4) used by the accumulators.
__device__ __forceinline__ bf16x8 col_frag_lds(const char* lds, int R, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const char* p0 = lds + lds_off<bf16>(R + 4 * g + q, (c0 + 4 * p) * 2);  // R % 16 == 0
  const char* p1 = p0 + 16 * AttnCfg<bf16>::ROWB;                          // same swizzle 16 rows on
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// pack accumulator registers {a[0..3], b[0..3]} -> bf16x8 (k-slot order above)
__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}
__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_f32(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// f32 scalar LDS read X[r][c]
__device__ __forceinline__ float ldsf(const char* lds, int r, int c) {
  return *reinterpret_cast<const float*>(lds + r * AttnCfg<float>::ROWB + c * 4);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// max / sum over the 4 lanes l, l^16, l^32, l^48 (one query of an S^T accumulator) with the gfx950
// row-swap permutes (VALU, no LDS round trip like ds_bpermute)
__device__ __forceinline__ float quad_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float quad_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Attention dropout stream (include/rp_api.h, rp_attn_fwd): for query q and lane group g one
// multiply-with-carry stream (MWC64X: x' = lo(A x + c), c' = hi(A x + c), A = 4294883355, output
// word x' ^ c') runs over the whole key range, seeded x = rp_hash(seed_bh, q*4 + g), c =
// rp_hash(x, 0x6A09E667) >> 1; eight steps per 64-key tile, in tile order; in tile `tile` word j
// covers keys 64*tile + 16*(j>>1) + 4*g + r with r = 2*(j&1) + {0: low half, 1: high half}; a key is
// kept iff its half, read as a signed 16-bit integer, is >= round(p*65536) - 32768 (probability
// 1 - p, exact to 2^-16).  One step is one v_mad_u64_u32 (+ the carry move and the output xor):
// ~11 issue cycles per word against ~26 for the xorshift32 stream of rounds 1-3, in a tile loop
// that is VALU-issue bound (scripts/rng_cost_probe.hip).  Outputs dm[j] (0xFFFF in each dropped
// half: the AND-NOT mask of the packed bf16 P pair) and returns the 16 keep bits, bit (kt*4 + r).
__device__ __forceinline__ uint64_t mwc_seed(uint32_t x) {
  return (uint64_t)x | ((uint64_t)(rp_hash(x, 0x6A09E667u) >> 1) << 32);
}
__device__ __forceinline__ uint32_t drop_masks(uint64_t& st, uint32_t thr, uint32_t dm[8]) {
  const short ts = (short)((int)thr - 32768);
  const i16x2 t2 = {ts, ts};
  uint32_t acc = 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t wd = rp_mwc_next(st);
    const i16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(i16x2, wd), t2);  // < 0 <=> dropped
    const uint32_t m = __builtin_bit_cast(uint32_t, (i16x2)(d >> (short)15));
    dm[j] = m;
    // keep bit of the low half -> bit 4*(j>>1) + 2*(j&1); high half -> 16 + that + 1 (folded below)
    const int b = 4 * (j >> 1) + 2 * (j & 1);
    acc |= ~m & ((1u << b) | (1u << (16 + b + 1)));
  }
  return (acc & 0xFFFFu) | (acc >> 16);
}

// Dropout select in the backward kernels: m ? a : b per bit for an all-ones / all-zero lane mask m
// (the stored keep bit sign-extended by v_bfe_i32) as ONE gfx950 v_bitop3_b32 (truth table 0xCA =
// S0 ? S1 : S2).  Written as C the compiler turns it into compare + cndmask (with the bit test
// 3 VALU per element), or into and/xor/or once the mask is opaque.
__device__ __forceinline__ uint32_t keep_mask(uint32_t w, int off) {
  return (uint32_t)__builtin_amdgcn_sbfe((int)w, off, 1);
}
__device__ __forceinline__ float bfi_select(uint32_t m, float a, float b) {
  return __uint_as_float(__builtin_amdgcn_bitop3_b32(m, __float_as_uint(a), __float_as_uint(b), 0xCA));
}

// =================================================================================================
// forward
// =================================================================================================
constexpr int FW_QB = NW * 32;  // queries per workgroup (dQ kernel; the forward's QT = 2 block)
constexpr int FW_KT = 64;       // keys per tile

// QT query tiles of 16 per wave: QT = 2 (128 queries per workgroup) by default; QT = 1 (64 per
// workgroup) doubles the waves of a small problem (B*H*T/128 below two workgroups per CU)
template <typename T, bool DROP, int QT>
__global__ __launch_bounds__(NT, (std::is_same<T, bf16>::value && !DROP) ? 3 : 2) void attn_fwd_kernel(MhaDev a) {
  constexpr int QB = NW * 16 * QT;  // queries per workgroup
  using C = AttnCfg<T>;
  constexpr int TILE = FW_KT * C::ROWB;
  constexpr int BUF = 2 * TILE + FW_KT * 4 + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const uint8_t* __restrict__ kvalid = a.kvalid;
  const float scale = a.scale;
  const uint32_t drop_thresh = a.drop_thresh;
  const float drop_scale = a.drop_scale;
  float* __restrict__ lse = a.lse;
  const int nqb = (Tq + QB - 1) / QB;
  const int L = rp_xcd_remap(blockIdx.x, nqb * B * H);
  const int bh = L / nqb, qb = L % nqb;
  const int b = bh / H, h = bh % H;
  const int64_t ldq = a.ldq, ldk = a.ldk, ldv = a.ldv;
  const T* Qg = (const T*)a.q + (int64_t)b * Tq * ldq + h * HD;
  const T* Kg = (const T*)a.k + (int64_t)b * Tk * ldk + h * HD;
  const T* Vg = (const T*)a.v + (int64_t)b * Tk * ldv + h * HD;
  const int q0 = qb * QB + w * 16 * QT;  // this wave's first query
  const uint32_t seed_bh = rp_hash(rp_seed_eff(a.seed_base, a.seed), (uint32_t)bh);
  const float c = scale * LOG2E;
  const int KT = mask_kt(Tk);
  const int64_t ldm = mask_ld(Tq);
  uint16_t* mrow = a.dmask ? a.dmask + (int64_t)bh * KT * 4 * ldm : nullptr;
  // no valid key + empty_uniform: every key counts and every score is 0 (Q taken as 0), so the
  // output is the mean of V — softmax of a row masked_fill'ed to a constant
  const bool novalid = seq_has_no_key(a, b, tid);

  // Q^T operand (B operand of S^T = K Q^T): lane holds Q[q0 + qt*16 + i][dk slots]
  constexpr bool BF = std::is_same<T, bf16>::value;
  bf16x8 qf[QT][2];
  float qs[QT][16];
  if constexpr (BF) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int s = 0; s < 2; ++s) qf[qt][s] = row_frag_gmem((const bf16*)Qg, ldq, q0 + qt * 16, Tq, s * 32, lane);
  } else {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      int q = q0 + qt * 16 + i;
#pragma unroll
      for (int s = 0; s < 16; ++s) qs[qt][s] = q < Tq ? (float)Qg[(int64_t)q * ldq + 4 * s + g] : 0.f;
    }
  }

  if (novalid) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if constexpr (BF) {
        qf[qt][0] = qf[qt][1] = bf16x8{};
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) qs[qt][s2] = 0.f;
      }
    }
  }
  // Q enters S^T = K Q^T prescaled by c = scale*log2(e) (log2-domain scores; already done by the
  // producer when a.qpre), and the S^T accumulators start at -m, the running reference max:
  // P = exp2(acc) needs no per-score op unless the reference moves on this tile.
#pragma unroll
  for (int qt = 0; qt < QT && !a.qpre; ++qt) {
    if constexpr (BF) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qt][s2][j] = (bf16)((float)qf[qt][s2][j] * c);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) qs[qt][s2] *= c;
    }
  }

  f32x4 o[QT][4];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = zero4();
  // m: reference max (log2 units) once set (mset); 0 before, when O and l are still zero
  float m[QT], lp[QT];
  bool mset[QT];
  float gthr[QT];  // grow bound of the lane-local test: -inf until the reference is set, then RESCALE_LOG2
  // dropout stream state of this lane's queries (carried across the key tiles)
  uint64_t dst[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    m[qt] = 0.f;
    lp[qt] = 0.f;
    mset[qt] = false;
    gthr[qt] = -INFINITY;
    dst[qt] = 0u;
  }
  if constexpr (DROP) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) dst[qt] = mwc_seed(rp_hash(seed_bh, (uint32_t)(q0 + qt * 16 + i) * 4u + (uint32_t)g));
  }

  Stage<T, FW_KT> sk, sv;
  const int nkt = (Tk + FW_KT - 1) / FW_KT;
  // key-valid flags of a tile: loaded with the K/V prefetch (wave 0, one byte per lane), staged as
  // an additive bias + a "no masked key" flag at the LDS write
  auto load_valid = [&](int k0) -> bool {
    const int k = k0 + lane;
    return w == 0 && k < Tk && (novalid || kvalid[(int64_t)b * Tk + k]);
  };
  auto stage_mask = [&](char* buf, bool ok) {
    float* kb = reinterpret_cast<float*>(buf + 2 * TILE);
    if (w == 0) {
      kb[lane] = ok ? 0.f : -INFINITY;
      const unsigned long long bal = __ballot(ok);
      if (lane == 0) *reinterpret_cast<int*>(buf + 2 * TILE + FW_KT * 4) = bal == ~0ull;
    }
  };
  sk.load(Kg, ldk, 0, Tk, tid);
  sv.load(Vg, ldv, 0, Tk, tid);
  bool kvn = load_valid(0);
  sk.store(lds, tid);
  sv.store(lds + TILE, tid);
  stage_mask(lds, kvn);
  __syncthreads();

  for (int kt_i = 0; kt_i < nkt; ++kt_i) {
    char* cur = lds + (kt_i & 1) * BUF;
    char* nxt = lds + ((kt_i + 1) & 1) * BUF;
    const bool more = kt_i + 1 < nkt;
    const int k0 = kt_i * FW_KT;
    if (more) {
      sk.load(Kg, ldk, k0 + FW_KT, Tk, tid);
      sv.load(Vg, ldv, k0 + FW_KT, Tk, tid);
      kvn = load_valid(k0 + FW_KT);
    }
    const char* Kl = cur;
    const char* Vl = cur + TILE;
    const float* kbias = reinterpret_cast<const float*>(cur + 2 * TILE);
    const bool full = *reinterpret_cast<const int*>(cur + 2 * TILE + FW_KT * 4) != 0;

    // ---- S^T[key][q] = K (cQ)^T - m ----
    f32x4 s[4][QT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[kt][qt] = f32x4{-m[qt], -m[qt], -m[qt], -m[qt]};
    if constexpr (BF) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          bf16x8 kf = row_frag_lds(Kl, kt * 16, ss * 32, lane);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) s[kt][qt] = mfma_bf16(kf, qf[qt][ss], s[kt][qt]);
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 16; ++ss) {
          float kf = ldsf(Kl, kt * 16 + i, 4 * ss + g);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) s[kt][qt] = mfma_f32(kf, qs[qt][ss], s[kt][qt]);
        }
    }
    // ---- mask (only tiles with masked keys) + column max, relative to the reference ----
    // Deferred rescale: the reference m only moves when the tile max exceeds it by more than
    // RESCALE_LOG2 (P <= 2^8 meanwhile, exact in fp32/bf16 range), or on the first finite max;
    // l and O share the reference, so out = O / l is unchanged and the lse uses the same m.
    float rel[QT];
    uint64_t grow = 0;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if (!full) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[kt][qt][r] += kbias[kt * 16 + 4 * g + r];
      }
      float mx = s[0][qt][0];  // chain -> v_max3
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
      // the lane-local test decides the wave-uniform branch exactly as the quad maximum would (the
      // quad maximum exceeds a bound iff one of its lanes does); the cross-lane reduction runs
      // only inside the branch, on the tiles that move the reference
      rel[qt] = mx;
      grow |= __ballot(mx > gthr[qt]);  // no NaN anywhere
    }
    if (grow != 0) {  // wave-uniform branch: move the reference of the growing lanes
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        rel[qt] = quad_max(rel[qt]);
        const bool gq = mset[qt] ? rel[qt] > RESCALE_LOG2 : rel[qt] > -INFINITY;
        const float alpha = gq ? (mset[qt] ? rp_exp2(-rel[qt]) : 0.f) : 1.f;
        const float sub = gq ? rel[qt] : 0.f;
        lp[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        m[qt] += sub;
        mset[qt] = mset[qt] || gq;
        gthr[qt] = mset[qt] ? RESCALE_LOG2 : -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) s[kt][qt] -= sub;
      }
    }
    // ---- P = exp2(acc); per-lane partial row sums (before dropout), tree order ----
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float t4[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kt][qt][r] = rp_exp2(s[kt][qt][r]);
        t4[kt] = (s[kt][qt][0] + s[kt][qt][1]) + (s[kt][qt][2] + s[kt][qt][3]);
      }
      lp[qt] += (t4[0] + t4[1]) + (t4[2] + t4[3]);
    }
    // ---- dropout: 8 drop masks per (query, tile) from one MWC stream; keep bits stored ----
    uint32_t dm[QT][8];
    if constexpr (DROP) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const int q = q0 + qt * 16 + i;
        const uint32_t word = drop_masks(dst[qt], drop_thresh, dm[qt]);
        if (q < Tq) mrow[((int64_t)kt_i * 4 + g) * ldm + q] = (uint16_t)word;
      }
    }
    // ---- O^T[dk][q] += V^T P^T ----
    if constexpr (BF) {
      bf16x8 pf[QT][2];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          pf[qt][ks] = pack8(s[2 * ks][qt], s[2 * ks + 1][qt]);
          if constexpr (DROP) {
            uint4 u = __builtin_bit_cast(uint4, pf[qt][ks]);
            u.x &= ~dm[qt][4 * ks + 0];
            u.y &= ~dm[qt][4 * ks + 1];
            u.z &= ~dm[qt][4 * ks + 2];
            u.w &= ~dm[qt][4 * ks + 3];
            pf[qt][ks] = __builtin_bit_cast(bf16x8, u);
          }
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          bf16x8 vf = col_frag_lds(Vl, ks * 32, dt * 16, lane);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) o[qt][dt] = mfma_bf16(vf, pf[qt][ks], o[qt][dt]);
        }
    } else {
      if constexpr (DROP) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              s[kt][qt][r] = ((dm[qt][2 * kt + (r >> 1)] >> (16 * (r & 1))) & 1u) ? 0.f : s[kt][qt][r];
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            float vf = ldsf(Vl, kt * 16 + 4 * g + r, dt * 16 + i);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) o[qt][dt] = mfma_f32(vf, s[kt][qt][r], o[qt][dt]);
          }
    }
    if (more) {
      sk.store(nxt, tid);
      sv.store(nxt + TILE, tid);
      stage_mask(nxt, kvn);
    }
    __syncthreads();
  }

  // ---- epilogue: O[q][dk] = O^T / l ; lse ----
  const int64_t ldo = a.ldo;
  T* __restrict__ out = (T*)a.out;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const float l = quad_sum(lp[qt]);
    const int q = q0 + qt * 16 + i;
    if (q >= Tq) continue;
    const float inv = drop_scale / l;
    T* orow = out + ((int64_t)b * Tq + q) * ldo + h * HD;
    if constexpr (BF) {  // the lane's 4 consecutive dims of a 16-dim tile -> one 8-byte store
      bf16* lorow = a.out_lo ? (bf16*)a.out_lo + ((int64_t)b * Tq + q) * ldo + h * HD : nullptr;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 v, vl;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = o[qt][dt][r] * inv;
          v[r] = (bf16)x;
          vl[r] = (bf16)(x - (float)v[r]);  // the rounding residual: rowsum(dO * O) to ~2^-17
        }
        *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = v;
        if (lorow) *reinterpret_cast<bf16x4*>(lorow + dt * 16 + 4 * g) = vl;
      }
    } else {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) rp_st(orow + dt * 16 + 4 * g + r, o[qt][dt][r] * inv);
    }
    if (g == 0) lse[(int64_t)bh * Tq + q] = m[qt] * 0.6931471805599453f + logf(l);  // m: log2 units
  }
}

// =================================================================================================
// backward pre-pass: delta[bh][q] = sum_d dO[q][d] * O[q][d]
// =================================================================================================
// one wave per DELTA_RPW query rows, 8 lanes per head; bf16 (D = 512): every load of the wave's rows
// is issued before the first use, so a wave keeps 3 x DELTA_RPW x 1 KB in flight and the grid's
// 4,096 waves (metric shape) are all resident at once — one HBM round trip instead of two rounds of
// one-row waves (14.5 us -> see DESIGN.md §8 round 5)
constexpr int DELTA_RPW = 4;
__device__ __forceinline__ void delta_store(const MhaDev& a, int64_t row, int e, float s) {
  const int b = (int)(row / a.Tq), t = (int)(row % a.Tq);
  const int64_t at = ((int64_t)b * a.H + e / HD) * a.Tq + t, plane = (int64_t)a.B * a.H * a.Tq;
  a.delta[at] = s;
  // the dK/dV kernel's row constants (plane 1, 2): -delta/ds and -lse*log2(e) + log2(ds)
  a.delta[plane + at] = -s / a.drop_scale;
  if (a.lse) a.delta[2 * plane + at] = -(a.lse[at] * LOG2E - log2f(a.drop_scale));
}
template <typename T>
__global__ void attn_delta_kernel(MhaDev a) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = (int64_t)a.B * a.Tq;
  const int D = a.H * HD;
  if constexpr (std::is_same<T, bf16>::value) {
    if (D == 8 * 64) {  // the metric shape's d_model = 512: lane = 8 columns of one head, 4 rows per wave
      const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * DELTA_RPW;
      const int e = lane * 8;
      bf16x8 ov[DELTA_RPW], dv[DELTA_RPW], lv[DELTA_RPW];
#pragma unroll
      for (int r = 0; r < DELTA_RPW; ++r) {
        const int64_t row = row0 + r < rows ? row0 + r : rows - 1;
        ov[r] = *reinterpret_cast<const bf16x8*>((const bf16*)a.out + row * a.ldo + e);
        dv[r] = *reinterpret_cast<const bf16x8*>((const bf16*)a.dout + row * a.lddo + e);
        if (a.out_lo) lv[r] = *reinterpret_cast<const bf16x8*>((const bf16*)a.out_lo + row * a.ldo + e);
      }
#pragma unroll
      for (int r = 0; r < DELTA_RPW; ++r) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += ((float)ov[r][j] + (a.out_lo ? (float)lv[r][j] : 0.f)) * (float)dv[r][j];
        s = rp_sum8(s);
        if ((lane & 7) == 0 && row0 + r < rows) delta_store(a, row0 + r, e, s);
      }
      return;
    }
  }
  // general: one wave per (b, t) query row
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* o = (const T*)a.out + row * a.ldo;
  const T* ol = a.out_lo ? (const T*)a.out_lo + row * a.ldo : nullptr;
  const T* d = (const T*)a.dout + row * a.lddo;
  for (int e = lane * 8; e < D; e += 512) {
    float s = 0.f;
    if constexpr (std::is_same<T, bf16>::value) {  // one 16-byte load per operand (ld % 8 == 0)
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(o + e);
      const bf16x8 dv = *reinterpret_cast<const bf16x8*>(d + e);
      bf16x8 lv;
      if (ol) lv = *reinterpret_cast<const bf16x8*>(ol + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += ((float)ov[j] + (ol ? (float)lv[j] : 0.f)) * (float)dv[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (rp_ld(o + e + j) + (ol ? rp_ld(ol + e + j) : 0.f)) * rp_ld(d + e + j);
    }
    s = rp_sum8(s);
    if ((lane & 7) == 0) delta_store(a, row, e, s);
  }
}
template <typename T>
dim3 delta_grid(const MhaDev& a) {
  const int64_t rows = (int64_t)a.B * a.Tq;
  const int64_t rpb = (std::is_same<T, bf16>::value && a.H * HD == 512) ? 4 * DELTA_RPW : 4;
  return dim3((unsigned)((rows + rpb - 1) / rpb));
}

// =================================================================================================
// backward: dK, dV per 128-key block (4 waves x 32 keys; 64 / 16 for small problems), sweep over
// 64-query tiles
// =================================================================================================
constexpr int KV_KB = NW * 32;  // keys per workgroup at KTW = 2
constexpr int KV_QT = 64;

// KTW key tiles of 16 per wave: 2 (128 keys per workgroup) by default, 1 (64) for small problems
template <typename T, bool DROP, int KTW>
__global__ __launch_bounds__(NT, 2) void attn_bwd_kv_kernel(MhaDev a) {
  constexpr int KB = NW * 16 * KTW;  // keys per workgroup
  using C = AttnCfg<T>;
  constexpr bool BF = std::is_same<T, bf16>::value;
  constexpr int TILE = KV_QT * C::ROWB;
  constexpr int MASKB = (KB / 64) * 4 * KV_QT * 2;    // KB/64 key tiles x 4 groups x 64 queries, u16
  constexpr int BUF = 2 * TILE + 2 * KV_QT * 4 + MASKB;  // Q, dO, lse*log2e, delta, keep bits
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const uint8_t* __restrict__ kvalid = a.kvalid;
  const float scale = a.scale, drop_scale = a.drop_scale;
  const uint16_t* __restrict__ dmask = a.dmask;
  const int nkb = (Tk + KB - 1) / KB;
  const int L = rp_xcd_remap(blockIdx.x, nkb * B * H);
  const int bh = L / nkb, kb = L % nkb;
  const int b = bh / H, h = bh % H;
  const int64_t ldq = a.ldq, ldk = a.ldk, ldv = a.ldv, lddo = a.lddo;
  const T* Qg = (const T*)a.q + (int64_t)b * Tq * ldq + h * HD;
  const T* Kg = (const T*)a.k + (int64_t)b * Tk * ldk + h * HD;
  const T* Vg = (const T*)a.v + (int64_t)b * Tk * ldv + h * HD;
  const T* dOg = (const T*)a.dout + (int64_t)b * Tq * lddo + h * HD;
  const float* lse_bh = a.lse + (int64_t)bh * Tq;
  const float* del_bh = a.delta + (int64_t)bh * Tq;
  const int kw0 = kb * KB + w * 16 * KTW;
  const float c = scale * LOG2E;
  const float kc = a.qpre ? 1.f : c;  // fp32 path: K prescale
  // no valid key + empty_uniform: uniform P (Q staged as 0), dK = dS^T 0 = 0, dV = mean of dO
  const bool novalid = seq_has_no_key(a, b, tid);
  const bool scale_q = BF && !a.qpre;  // bf16 path: Q prescale at LDS staging
  const float dk_scale = (BF || a.qpre) ? 1.f / LOG2E : scale;  // dS^T Q' -> dK
  const float inv_ds = DROP ? 1.f / drop_scale : 1.f;
  const int KT = mask_kt(Tk);
  const int64_t ldm = mask_ld(Tq);

  // K, V as B operands of S = Q K^T and dP = dO V^T: lane holds X[kw0 + kt*16 + i][dk slots]
  bf16x8 kf[KTW][2], vf[KTW][2];
  float ks_[KTW][16], vs_[KTW][16];
  if constexpr (BF) {
#pragma unroll
    for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        kf[kt][s] = row_frag_gmem((const bf16*)Kg, ldk, kw0 + kt * 16, Tk, s * 32, lane);
        vf[kt][s] = row_frag_gmem((const bf16*)Vg, ldv, kw0 + kt * 16, Tk, s * 32, lane);
      }
  } else {
#pragma unroll
    for (int kt = 0; kt < KTW; ++kt) {
      const int k = kw0 + kt * 16 + i;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        ks_[kt][s] = k < Tk ? (float)Kg[(int64_t)k * ldk + 4 * s + g] * kc : 0.f;
        vs_[kt][s] = k < Tk ? (float)Vg[(int64_t)k * ldv + 4 * s + g] : 0.f;
      }
    }
  }
  // S = Q' K^T must reproduce the forward's log2-domain scores bit for bit, so that the recomputed
  // P is the forward's P.  bf16: Q' = bf16(Q * c) exactly as the forward rounds it — either the
  // producer wrote it (a.qpre) or the Q tiles are scaled as they are staged into LDS — and K stays
  // as is; dK = dS^T Q' / log2(e).  fp32 (no rounding to speak of): K * c in registers unless a.qpre.

  f32x4 dk[KTW][4], dv[KTW][4];
#pragma unroll
  for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kt][dt] = dv[kt][dt] = zero4();

  Stage<T, KV_QT> sq, sdo;
  uint4 mreg = make_uint4(0u, 0u, 0u, 0u);
  // keep-bit words of this workgroup's KB/64 key tiles x 4 groups x 64 queries: thread
  // t < (KB/64)*32 moves 16 bytes (row = tile*4 + g, 8 queries)
  constexpr int MT = (KB / 64) * 32;
  auto load_mask = [&](int qs0) {
    if (DROP && tid < MT) {
      const int r = tid >> 3, cch = tid & 7;
      const int tile = kb * (KB / 64) + (r >> 2);
      if (tile < KT)
        mreg = *reinterpret_cast<const uint4*>(dmask + (((int64_t)bh * KT + tile) * 4 + (r & 3)) * ldm + qs0 + cch * 8);
      else
        mreg = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  // per-query lse / delta of a tile: loaded with the Q/dO prefetch (wave 0), staged at the LDS write
  float lse_r = 0.f, del_r = 0.f;
  auto load_rows = [&](int qs0) {
    if (tid < KV_QT) {
      const int q = qs0 + tid;
      // the S accumulators' start, -lse*log2(e) (-inf -> P = 0 for padded rows); with dropout the
      // 1/(1-p) scale rides in the exponent
      lse_r = q < Tq ? -(lse_bh[q] * LOG2E - (DROP ? log2f(drop_scale) : 0.f)) : -INFINITY;
      del_r = q < Tq ? -del_bh[q] * inv_ds : 0.f;     // -delta/ds: the dP accumulators' start
    }
  };
  auto stage_rows = [&](char* buf) {
    float* lb = reinterpret_cast<float*>(buf + 2 * TILE);
    if (tid < KV_QT) {
      lb[tid] = lse_r;
      lb[KV_QT + tid] = del_r;
    }
    if (DROP && tid < MT) *reinterpret_cast<uint4*>(buf + 2 * TILE + 2 * KV_QT * 4 + tid * 16) = mreg;
  };
  const int nqt = (Tq + KV_QT - 1) / KV_QT;
  auto store_q = [&](char* buf) {
    if (novalid) {
      sq.store_zero(buf, tid);
      return;
    }
    if constexpr (BF) {
      if (scale_q) {
        sq.store_scaled(buf, tid, c);
        return;
      }
    }
    sq.store(buf, tid);
  };
  sq.load(Qg, ldq, 0, Tq, tid);
  sdo.load(dOg, lddo, 0, Tq, tid);
  load_mask(0);
  load_rows(0);
  store_q(lds);
  sdo.store(lds + TILE, tid);
  stage_rows(lds);
  __syncthreads();

  for (int it = 0; it < nqt; ++it) {
    char* cur = lds + (it & 1) * BUF;
    char* nxt = lds + ((it + 1) & 1) * BUF;
    const bool more = it + 1 < nqt;
    const int qs0 = it * KV_QT;
    if (more) {
      sq.load(Qg, ldq, qs0 + KV_QT, Tq, tid);
      sdo.load(dOg, lddo, qs0 + KV_QT, Tq, tid);
      load_mask(qs0 + KV_QT);
      load_rows(qs0 + KV_QT);
    }
    const char* Ql = cur;
    const char* dOl = cur + TILE;
    const float* lrow = reinterpret_cast<const float*>(cur + 2 * TILE);
    const float* drow = lrow + KV_QT;
    const uint16_t* mw = reinterpret_cast<const uint16_t*>(cur + 2 * TILE + 2 * KV_QT * 4);

    // two 32-query halves per staged 64-query tile (keeps the S / dP accumulators at 32 regs)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      // S[q][key], dP[q][key]: C-layout row q = (2hf+qq)*16 + 4g + r, col key = kt*16 + i
      // dP starts at -delta/ds (row constant as the initial accumulator): dS = p*ds*acc
      f32x4 s[2][KTW], dp[2][KTW], ndq[2], nl[2];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        ndq[qq] = *reinterpret_cast<const f32x4*>(drow + (2 * hf + qq) * 16 + 4 * g);
        nl[qq] = *reinterpret_cast<const f32x4*>(lrow + (2 * hf + qq) * 16 + 4 * g);
      }
      if constexpr (BF) {
        // the row constants enter as the first MFMA's C operand (no register copies)
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            bf16x8 qa = row_frag_lds(Ql, (2 * hf + qq) * 16, ss * 32, lane);
            bf16x8 da = row_frag_lds(dOl, (2 * hf + qq) * 16, ss * 32, lane);
#pragma unroll
            for (int kt = 0; kt < KTW; ++kt) {
              s[qq][kt] = mfma_bf16(qa, kf[kt][ss], ss == 0 ? nl[qq] : s[qq][kt]);
              dp[qq][kt] = mfma_bf16(da, vf[kt][ss], ss == 0 ? ndq[qq] : dp[qq][kt]);
            }
          }
      } else {
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int kt = 0; kt < KTW; ++kt) {
            s[qq][kt] = nl[qq];
            dp[qq][kt] = ndq[qq];
          }
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int ss = 0; ss < 16; ++ss) {
            float qa = ldsf(Ql, (2 * hf + qq) * 16 + i, 4 * ss + g);
            float da = ldsf(dOl, (2 * hf + qq) * 16 + i, 4 * ss + g);
#pragma unroll
            for (int kt = 0; kt < KTW; ++kt) {
              s[qq][kt] = mfma_f32(qa, ks_[kt][ss], s[qq][kt]);
              dp[qq][kt] = mfma_f32(da, vs_[kt][ss], dp[qq][kt]);
            }
          }
      }
      // P (dropped, for dV) -> s ; dS (for dK) -> dp.  Masked keys are not masked here: their P / dS
      // only reach their own dK / dV rows, which the epilogue writes as zeros.
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int qrow = (2 * hf + qq) * 16 + 4 * g;
#pragma unroll
        for (int kt = 0; kt < KTW; ++kt) {
          // this lane's key: ko = key % 64 -> word row (tile half, group (ko%16)/4), bit (ko/16)*4 + ko%4
          const int kw = w * 16 * KTW + kt * 16 + i;
          const int ko = kw & 63;
          const int mrow_l = (kw >> 6) * 4 + ((ko & 15) >> 2);
          const int bit = (ko >> 4) * 4 + (ko & 3);
          uint2 bits = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
          if constexpr (DROP) bits = *reinterpret_cast<const uint2*>(mw + mrow_l * KV_QT + qrow);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = rp_exp2(s[qq][kt][r]);  // with dropout: p * ds
            if constexpr (DROP) {  // dS = p*(keep*ds*dP - delta) = p*ds*(keep ? acc : -delta/ds)
              const uint32_t km = keep_mask(r < 2 ? bits.x : bits.y, bit + 16 * (r & 1));
              s[qq][kt][r] = bfi_select(km, p, 0.f);
              dp[qq][kt][r] = p * bfi_select(km, dp[qq][kt][r], ndq[qq][r]);
            } else {
              s[qq][kt][r] = p;
              dp[qq][kt][r] = p * dp[qq][kt][r];
            }
          }
        }
      }
      // dV[key][dk] += P_d^T dO ; dK[key][dk] += dS^T Q     (key on the row, k = query slots)
      if constexpr (BF) {
        bf16x8 pa[KTW], sa[KTW];
#pragma unroll
        for (int kt = 0; kt < KTW; ++kt) {
          pa[kt] = pack8(s[0][kt], s[1][kt]);
          sa[kt] = pack8(dp[0][kt], dp[1][kt]);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const bf16x8 dob = col_frag_lds(dOl, hf * 32, dt * 16, lane);
          const bf16x8 qb = col_frag_lds(Ql, hf * 32, dt * 16, lane);
#pragma unroll
          for (int kt = 0; kt < KTW; ++kt) {
            dv[kt][dt] = mfma_bf16(pa[kt], dob, dv[kt][dt]);
            dk[kt][dt] = mfma_bf16(sa[kt], qb, dk[kt][dt]);
          }
        }
      } else {
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
              const float dob = ldsf(dOl, (2 * hf + qq) * 16 + 4 * g + r, dt * 16 + i);
              const float qb = ldsf(Ql, (2 * hf + qq) * 16 + 4 * g + r, dt * 16 + i);
#pragma unroll
              for (int kt = 0; kt < KTW; ++kt) {
                dv[kt][dt] = mfma_f32(s[qq][kt][r], dob, dv[kt][dt]);
                dk[kt][dt] = mfma_f32(dp[qq][kt][r], qb, dk[kt][dt]);
              }
            }
      }
    }
    if (more) {
      store_q(nxt);
      sdo.store(nxt + TILE, tid);
      stage_rows(nxt);
    }
    __syncthreads();
  }
  // store: dk[kt][dt][r] = dK[key = kw0 + kt*16 + 4g + r][dk = dt*16 + i]; masked keys -> 0
  T* dK = (T*)a.dk + (int64_t)b * Tk * a.lddk + h * HD;
  T* dV = (T*)a.dv + (int64_t)b * Tk * a.lddv + h * HD;
#pragma unroll
  for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kw0 + kt * 16 + 4 * g + r;
      if (key >= Tk) continue;
      const bool ok = novalid || kvalid[(int64_t)b * Tk + key] != 0;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        rp_st(dK + (int64_t)key * a.lddk + dt * 16 + i, ok ? dk[kt][dt][r] * dk_scale : 0.f);
        rp_st(dV + (int64_t)key * a.lddv + dt * 16 + i, ok ? dv[kt][dt][r] : 0.f);
      }
    }
}

// =================================================================================================
// backward: dK, dV — bf16, LDS-DMA staged variant (the default for bf16; RP_ATTN_DMA=0 selects the
// register-staged kernel above).  Same math and register layouts as attn_bwd_kv_kernel; what changes
// is how the query tiles reach LDS:
//  * global_load_lds (LDS-DMA) writes the Q / dO tiles straight into the XOR-swizzled images (the
//    swizzle goes on the per-lane source address), the raw lse / delta rows and the keep-bit words:
//    no staging registers, no ds_write, no per-tile VALU for the copies;
//  * a three-buffer ring with the DMA two tiles ahead (a tile's loads have a whole tile of compute
//    plus a barrier to land), one barrier per tile: it both publishes tile it and frees the buffer
//    the DMA of tile it + 2 overwrites;
//  * rows past Tq repeat the last row (clamped source rows, no zero fill); their probabilities are
//    forced to 0 through the S accumulators' start (-inf), so they contribute nothing.
// =================================================================================================
typedef __attribute__((address_space(3))) void lds_void_t;


// One LDS-DMA wave instruction: lane l's 16 bytes at g land at LDS byte address lds + 16 l.  Issued as
// inline asm on purpose: the compiler then does not track it, so it inserts no conservative
// vmcnt(0) before the LDS reads of a step (its alias tracking cannot tell that those read another
// ring slot, and across the loop back-edge it loses the count) — the kernels' explicit counted
// vmcnt + barrier order every DMA before its readers.  m0 is saved and restored around it.
__device__ __forceinline__ void dma16(const void* g, uint32_t lds) {
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

// the same for 4 bytes per lane (lane l -> lds + 4 l)
__device__ __forceinline__ void dma4(const void* g, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %2, off\n\t"
      "s_nop 0\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "v"(g)
      : "memory");
}

// DMA source of the S start of query rows past Tq: -inf, so P = 0 on those rows
__device__ const float kPadStart[1] = {-INFINITY};

__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// rows [row0, row0 + 64) of a [rows][64] bf16 operand (row stride ld) -> the swizzled 8 KB image of
// lds_off<bf16>: eight 1 KB pieces (8 rows each), two per wave; lane l of a piece lands at physical
// 16-byte chunk l & 7 of row l >> 3, which holds logical chunk (l & 7) ^ lds_swz(row)
__device__ __forceinline__ void dma_rows64(const bf16* __restrict__ base, int64_t ld, int row0, int nrows, char* tile,
                                           int w, int lane) {
  const uint32_t t = lds_addr(tile);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int I = w * 2 + j;
    const int r = I * 8 + (lane >> 3);
    const int c = (lane & 7) ^ lds_swz(r);
    int rr = row0 + r;
    rr = rr < nrows ? rr : nrows - 1;
    dma16(base + (int64_t)rr * ld + c * 8, t + I * 1024);
  }
}

// Buffer-descriptor form of the LDS-DMA pieces (the tile loops' steady state).  A lane's source
// address inside a tile is fixed for the whole sweep (its row of the 8-row piece, its swizzled chunk),
// so it is computed ONCE as a 32-bit voffset; a tile then costs one scalar offset (row0 * row bytes)
// and one buffer_load ... lds per piece.  The global_load_lds form recomputed a clamped 64-bit address
// per piece every tile (two v_mul_lo_u32 + v_mad_u64_u32 + 64-bit adds per piece: ~30 VALU + ~30 SALU
// per tile and wave of the dK/dV kernel).  Partial tiles (row0 + 64 > nrows) keep the clamped path.
typedef int rp_srd __attribute__((ext_vector_type(4)));
__device__ __forceinline__ rp_srd make_srd(const void* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  rp_srd s;
  s[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  s[1] = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xFFFFu);  // stride 0
  s[2] = -1;          // num_records: no range check — callers only load inside the operand
  s[3] = 0x00020000;  // raw buffer, 32-bit data format (cdna_hip_programming.md T8 recipe)
  return s;
}
// lane l's 16 (4) bytes at srd.base + voff + soff land at LDS byte lds + 16 l (4 l); untracked by the
// compiler like dma16 (the kernels' counted vmcnt orders it)
__device__ __forceinline__ void dma16b(const rp_srd& srd, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_nop 0\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "v"(voff), "s"(srd), "s"(soff)
      : "memory");
}

// A tile's four row pieces (two operands x two 1 KB pieces, each operand one descriptor and one scalar
// offset) in one asm block: m0 saved / restored once around the group instead of per piece (the
// per-piece form spent 5 scalar instructions per piece: ~30 % of the loop's SALU)
__device__ __forceinline__ void dma16b_x4(const rp_srd& s0, uint32_t v00, uint32_t v01, uint32_t o0, const rp_srd& s1,
                                          uint32_t v10, uint32_t v11, uint32_t o1, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %5, %9, %11 offen lds\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %6, %9, %11 offen lds\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %7, %10, %12 offen lds\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %8, %10, %12 offen lds\n\t"
      "s_nop 0\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "s"(lds + 1024u), "s"(lds + 8192u), "s"(lds + 9216u), "v"(v00), "v"(v01), "v"(v10), "v"(v11),
        "s"(s0), "s"(s1), "s"(o0), "s"(o1)
      : "memory");
}

// rows [row0, row0 + 64) of a [rows][64] bf16 operand -> the swizzled 8 KB image (two 1 KB pieces per
// wave, as dma_rows64), descriptor form for full tiles: piece j of wave w is
// dma16b(srd, vo_j, row0 * rowbytes, image + (2w + j) * 1 KB)
struct Rows64 {
  const bf16* base;
  int64_t ld;
  rp_srd srd;
  uint32_t vo0, vo1, rowbytes;
  bool fast;  // every full tile's byte offsets fit 32 bits
  __device__ __forceinline__ void init(const bf16* b, int64_t ld_, int nrows, int w, int lane) {
    base = b;
    ld = ld_;
    srd = make_srd(b);
    const int r0 = (w * 2) * 8 + (lane >> 3), r1 = r0 + 8;
    const int c0 = (lane & 7) ^ lds_swz(r0), c1 = (lane & 7) ^ lds_swz(r1);
    vo0 = (uint32_t)((r0 * ld_ + c0 * 8) * 2);
    vo1 = (uint32_t)((r1 * ld_ + c1 * 8) * 2);
    rowbytes = (uint32_t)(ld_ * 2);
    fast = ((int64_t)nrows + 64) * ld_ * 2 < ((int64_t)1 << 31);
  }
};

// raw workgroup barrier: no release / acquire fence, so the compiler adds no vmcnt(0) for the LDS-DMA
// loads still in flight (the explicit counted vmcnt before it is what makes a tile's DMA visible);
// the empty asm statements keep the compiler from moving memory operations across it
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one ring slot of the dK/dV kernel: Q and dO images of a query tile plus four 1 KB side regions
constexpr int KV_DMA_BUF = 2 * KV_QT * AttnCfg<bf16>::ROWB + 4 * 1024;

// SPL = 2 (grids that fill the CUs only once: config 4, B = 1, T = 4096): eight waves, waves 4-7 run
// the same key block over the second half of the query tiles on a ring of their own, and the two
// halves' dK / dV partials are added through LDS at the end (dK = own + partner on half 0, which stores
// dK; dV likewise on half 1) — two waves per SIMD where one 4-wave workgroup per CU had one
template <bool DROP, int KTW, bool PIPE, int SPL = 1>
__device__ __forceinline__ void attn_bwd_kv_dma_body(const MhaDev& a, const int blk, char* lds) {
  constexpr int KB = NW * 16 * KTW;  // keys per workgroup
  using C = AttnCfg<bf16>;
  constexpr int TILE = KV_QT * C::ROWB;
  // keep bits: KB/64 key tiles x 4 groups x 64 queries, u16 — one full 1 KB DMA piece (at KB = 64 the
  // second half holds a copy of the first)
  // slot: Q, dO images, then four 1 KB regions — raw lse row, raw delta row, keep bits, scratch — one
  // per wave's fifth DMA piece (wave 0, and wave 3 without dropout, load a dummy row into the scratch
  // region, so every wave issues five DMA instructions per tile and one counted wait serves all)
  constexpr int XR = 1024;
  constexpr int BUF = 2 * TILE + 4 * XR;
  constexpr int NBUF = 3;
  // three separate arrays rather than one indexed ring: every LDS address of a step is then a per-lane
  // base plus an immediate offset
  static_assert(BUF == KV_DMA_BUF, "KV_DMA_BUF out of date");
  char* const ring0 = lds;  // the caller's LDS: three slots at 1 KB-aligned constant offsets
  char* const ring1 = lds + SPL * BUF;
  char* const ring2 = lds + 2 * SPL * BUF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wq & (NW - 1);                // wave within its query half
  const int hv = SPL == 1 ? 0 : wq / NW;      // query half (SPL = 2)
  const int hoff = hv * BUF;                  // the half's ring region
  const int g = lane >> 4, i = lane & 15;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const uint8_t* __restrict__ kvalid = a.kvalid;
  const float drop_scale = a.drop_scale;
  const uint16_t* __restrict__ dmask = a.dmask;
  const int nkb = (Tk + KB - 1) / KB;
  const int L = rp_xcd_remap(blk, nkb * B * H);
  const int bh = L / nkb, kb = L % nkb;
  const int b = bh / H, h = bh % H;
  const int64_t ldq = a.ldq, ldk = a.ldk, ldv = a.ldv, lddo = a.lddo;
  const bf16* Qg = (const bf16*)a.q + (int64_t)b * Tq * ldq + h * HD;
  const bf16* Kg = (const bf16*)a.k + (int64_t)b * Tk * ldk + h * HD;
  const bf16* Vg = (const bf16*)a.v + (int64_t)b * Tk * ldv + h * HD;
  const bf16* dOg = (const bf16*)a.dout + (int64_t)b * Tq * lddo + h * HD;
  // the delta workspace's row constants (written by whichever kernel formed delta): the S accumulators
  // start at -lse*log2(e) + log2(ds) (plane 2), the dP accumulators at -delta/ds (plane 1)
  const int64_t plane = (int64_t)B * H * Tq;
  const float* nls_bh = a.delta + 2 * plane + (int64_t)bh * Tq;
  const float* ndl_bh = a.delta + plane + (int64_t)bh * Tq;
  const int kw0 = kb * KB + w * 16 * KTW;
  const int KT = mask_kt(Tk);
  const int64_t ldm = mask_ld(Tq);
  // the kernel-side Q prescale (no RP_ATTN_Q_PRESCALED) and empty_uniform have no DMA form: the
  // launcher sends those calls to the register-staged kernel

  // K, V as B operands of S = Q' K^T and dP = dO V^T: lane holds X[kw0 + kt*16 + i][dk slots]
  bf16x8 kf[KTW][2], vf[KTW][2];
#pragma unroll
  for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      kf[kt][s] = row_frag_gmem(Kg, ldk, kw0 + kt * 16, Tk, s * 32, lane);
      vf[kt][s] = row_frag_gmem(Vg, ldv, kw0 + kt * 16, Tk, s * 32, lane);
    }
  // consume K / V here, before the loop: otherwise the compiler places the wait for these loads at
  // their first use inside the loop body, where it runs every ring cycle as a full vmcnt(0)
#pragma unroll
  for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
    for (int s = 0; s < 2; ++s) asm volatile("" ::"v"(kf[kt][s]), "v"(vf[kt][s]));

  f32x4 dk[KTW][4], dv[KTW][4];
#pragma unroll
  for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kt][dt] = dv[kt][dt] = zero4();

  auto ring = [&](auto bi) -> char* {
    constexpr int BI = decltype(bi)::value;
    return (BI == 0 ? ring0 : (BI == 1 ? ring1 : ring2)) + hoff;
  };
  // query tiles: this half's nqt tiles start at tile qt0; both halves run nsteps ring steps (the half
  // with one tile fewer idles through the last one: every wave passes every barrier)
  const int nqt_all = (Tq + KV_QT - 1) / KV_QT;
  const int nh0 = SPL == 1 ? nqt_all : (nqt_all + 1) / 2;
  const int qt0 = hv * nh0;
  const int nqt = SPL == 1 ? nqt_all : (hv == 0 ? nh0 : nqt_all - nh0);
  const int nsteps = nh0;
  // LDS-DMA of query tile it into ring slot BI: Q and dO (two 1 KB pieces each per wave), the S start
  // (wave 1; -inf past Tq) and dP start (wave 2) rows and the keep-bit words (wave 3, with dropout):
  // D = 4 DMA instructions per wave, 5 for waves 1, 2 and (with dropout) 3
  Rows64 rq, rdo;
  rq.init(Qg, ldq, Tq, w, lane);
  rdo.init(dOg, lddo, Tq, w, lane);
  // the wave's fifth piece: wave 1 the lse row constants, wave 2 the delta ones (lanes 0..15 cover the
  // tile's 64 floats, the other lanes repeat them), wave 3 the keep bits, the rest a dummy delta row
  const bool xmask = DROP && w == 3;
  const uint16_t* mslab = DROP ? dmask + (int64_t)bh * KT * 4 * ldm : dmask;
  const rp_srd srd_x = make_srd(xmask ? (const void*)mslab : (const void*)(w == 1 ? nls_bh : ndl_bh));
  uint32_t vo_x = (uint32_t)(lane & 15) * 16u;
  const uint32_t bpr_x = xmask ? 2u : 4u;  // source bytes per query row
  const uint32_t xo = (uint32_t)(2 * TILE + XR * (w == 1 ? 0 : (w == 2 ? 1 : (xmask ? 2 : 3))));
  // keep-bit region: LDS row r (= tile half * 4 + lane group) holds 64 queries' words; its 16-byte chunks
  // are XOR-swizzled by mswz(r) = (r >> 1) & 1 so that the readers' rows r and r + 2 (128 bytes x 2 =
  // the same banks) land 16 bytes apart: the dropout path's ds_read_b64 of the bits is conflict-free
  // (it was 2-way: 6.3 M conflict cycles per launch at p = 0.1, 0 at p = 0)
  if (xmask) {
    const int r = (lane >> 3) & ((KB / 64) * 4 - 1), cch = (lane & 7) ^ ((lane >> 4) & 1);
    int tile = kb * (KB / 64) + (r >> 2);
    tile = tile < KT ? tile : KT - 1;  // keys past Tk: their dK / dV rows are written as zeros
    // KB = 64: lanes 32..63 repeat lanes 0..31's words into the unused second half of the region
    vo_x = (uint32_t)((((int64_t)tile * 4 + (r & 3)) * ldm + cch * 8) * 2);
  }
  const bool xfast = (int64_t)KT * 4 * ldm * 2 < ((int64_t)1 << 31) && rq.fast && rdo.fast;
  const uint32_t slot_lds[3] = {lds_addr(ring0) + (uint32_t)hoff, lds_addr(ring1) + (uint32_t)hoff,
                                 lds_addr(ring2) + (uint32_t)hoff};
  auto issue = [&](int it, auto bi) {
    constexpr int BI = decltype(bi)::value;
    char* buf = ring(bi);
    const int qs0 = (qt0 + it) * KV_QT;
    if (xfast && qs0 + KV_QT <= Tq) {
      const uint32_t t = slot_lds[BI];
      const uint32_t pq = t + (uint32_t)(w * 2) * 1024u;
      static_assert(TILE == 8192, "dma16b_x4 places the second operand 8 KB on");
      dma16b_x4(rq.srd, rq.vo0, rq.vo1, (uint32_t)qs0 * rq.rowbytes, rdo.srd, rdo.vo0, rdo.vo1,
                (uint32_t)qs0 * rdo.rowbytes, pq);
      dma16b(srd_x, vo_x, (uint32_t)qs0 * bpr_x, t + xo);
    } else {  // partial tile: clamped rows, -inf S start past Tq
      dma_rows64(Qg, ldq, qs0, Tq, buf, w, lane);
      dma_rows64(dOg, lddo, qs0, Tq, buf + TILE, w, lane);
      const int q = qs0 + lane;
      if (xmask) {
        const int r = (lane >> 3) & ((KB / 64) * 4 - 1), cch = (lane & 7) ^ ((lane >> 4) & 1);
        int tile = kb * (KB / 64) + (r >> 2);
        tile = tile < KT ? tile : KT - 1;
        dma16(dmask + (((int64_t)bh * KT + tile) * 4 + (r & 3)) * ldm + qs0 + cch * 8, lds_addr(buf + xo));
      } else if (w == 1) {
        dma4(q < Tq ? nls_bh + q : kPadStart, lds_addr(buf + xo));
      } else {
        dma4(ndl_bh + (q < Tq ? q : Tq - 1), lds_addr(buf + xo));
      }
    }
  };
  // step it waits for DMA(it); issued after it by then: DMA(it + 1) (5 instructions, if it exists)
  auto wait_tile = [&](bool next) {
    if (!next)
      wait_vm<0>();
    else
      wait_vm<5>();
  };

  if (nqt > 0) issue(0, std::integral_constant<int, 0>());
  if (nqt > 1) issue(1, std::integral_constant<int, 1>());
  auto step = [&](auto bi, int it) {
    constexpr int BI = decltype(bi)::value;
    wait_tile(it + 1 < nqt);
    raw_barrier();
    if (SPL > 1 && it >= nqt) return;
    if (it + 2 < nqt) issue(it + 2, std::integral_constant<int, (BI + 2) % NBUF>());
    const char* cur = ring(bi);
    const char* Ql = cur;
    const char* dOl = cur + TILE;
    const float* lrow = reinterpret_cast<const float*>(cur + 2 * TILE);
    const float* drow = reinterpret_cast<const float*>(cur + 2 * TILE + XR);
    const uint16_t* mw = reinterpret_cast<const uint16_t*>(cur + 2 * TILE + 2 * XR);

    // one half = 32 queries: S / dP products (16 MFMAs), the probability / dS VALU, then the dV / dK
    // products (16 MFMAs) that consume both 16-query rows of the half
    auto sdp = [&](int hf, f32x4 (&s)[2][KTW], f32x4 (&dp)[2][KTW], f32x4 (&ndq)[2]) {
      f32x4 nl[2];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int r0 = (2 * hf + qq) * 16 + 4 * g;
        nl[qq] = *reinterpret_cast<const f32x4*>(lrow + r0);
        ndq[qq] = *reinterpret_cast<const f32x4*>(drow + r0);
      }
#pragma unroll
      for (int qq = 0; qq < 2; ++qq)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          bf16x8 qa = row_frag_lds(Ql, (2 * hf + qq) * 16, ss * 32, lane);
          bf16x8 da = row_frag_lds(dOl, (2 * hf + qq) * 16, ss * 32, lane);
#pragma unroll
          for (int kt = 0; kt < KTW; ++kt) {
            s[qq][kt] = mfma_bf16(qa, kf[kt][ss], ss == 0 ? nl[qq] : s[qq][kt]);
            dp[qq][kt] = mfma_bf16(da, vf[kt][ss], ss == 0 ? ndq[qq] : dp[qq][kt]);
          }
        }
    };
    auto prob = [&](int hf, f32x4 (&s)[2][KTW], f32x4 (&dp)[2][KTW], const f32x4 (&ndq)[2], bf16x8 (&pa)[KTW],
                    bf16x8 (&sa)[KTW]) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int qrow = (2 * hf + qq) * 16 + 4 * g;
#pragma unroll
        for (int kt = 0; kt < KTW; ++kt) {
          // this lane's key: ko = key % 64 -> word row (tile half, group (ko%16)/4), bit (ko/16)*4 + ko%4
          const int kw = w * 16 * KTW + kt * 16 + i;
          const int ko = kw & 63;
          const int mrow_l = (kw >> 6) * 4 + ((ko & 15) >> 2);
          const int bit = (ko >> 4) * 4 + (ko & 3);
          uint2 bits = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
          if constexpr (DROP)
            bits = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(mw) + mrow_l * (KV_QT * 2) +
                                                   ((((qrow >> 3) ^ ((mrow_l >> 1) & 1)) << 4) | ((qrow & 7) << 1)));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pr = rp_exp2(s[qq][kt][r]);  // with dropout: p * ds
            if constexpr (DROP) {
              const uint32_t km = keep_mask(r < 2 ? bits.x : bits.y, bit + 16 * (r & 1));
              s[qq][kt][r] = bfi_select(km, pr, 0.f);
              dp[qq][kt][r] = pr * bfi_select(km, dp[qq][kt][r], ndq[qq][r]);
            } else {
              s[qq][kt][r] = pr;
              dp[qq][kt][r] = pr * dp[qq][kt][r];
            }
          }
        }
      }
#pragma unroll
      for (int kt = 0; kt < KTW; ++kt) {
        pa[kt] = pack8(s[0][kt], s[1][kt]);
        sa[kt] = pack8(dp[0][kt], dp[1][kt]);
      }
    };
    auto dvdk = [&](int hf, const bf16x8 (&pa)[KTW], const bf16x8 (&sa)[KTW]) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 dob = col_frag_lds(dOl, hf * 32, dt * 16, lane);
        const bf16x8 qb = col_frag_lds(Ql, hf * 32, dt * 16, lane);
#pragma unroll
        for (int kt = 0; kt < KTW; ++kt) {
          dv[kt][dt] = mfma_bf16(pa[kt], dob, dv[kt][dt]);
          dk[kt][dt] = mfma_bf16(sa[kt], qb, dk[kt][dt]);
        }
      }
    };
    if constexpr (PIPE) {
      // both halves' S / dP products are issued before the first half's VALU, so the VALU of half 0
      // runs beside the MFMAs of half 1 and the VALU of half 1 beside the dV / dK MFMAs of half 0
      f32x4 s0[2][KTW], dp0[2][KTW], nd0[2], s1[2][KTW], dp1[2][KTW], nd1[2];
      bf16x8 pa0[KTW], sa0[KTW], pa1[KTW], sa1[KTW];
      sdp(0, s0, dp0, nd0);
      sdp(1, s1, dp1, nd1);
      prob(0, s0, dp0, nd0, pa0, sa0);
      dvdk(0, pa0, sa0);
      prob(1, s1, dp1, nd1, pa1, sa1);
      dvdk(1, pa1, sa1);
    } else {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        f32x4 s[2][KTW], dp[2][KTW], ndq[2];
        bf16x8 pa[KTW], sa[KTW];
        sdp(hf, s, dp, ndq);
        prob(hf, s, dp, ndq, pa, sa);
        dvdk(hf, pa, sa);
      }
    }
  };
  for (int it = 0; it < nsteps; it += NBUF) {
    step(std::integral_constant<int, 0>(), it);
    if (it + 1 < nsteps) step(std::integral_constant<int, 1>(), it + 1);
    if (it + 2 < nsteps) step(std::integral_constant<int, 2>(), it + 2);
  }
  if constexpr (SPL > 1) {
    // every DMA has landed (each half's last step waited vmcnt(0)); after this barrier no wave reads a
    // ring again.  Half 1 hands its dK partial over in ring0, half 0 its dV partial in ring1 (lane-major
    // rows of 64 floats: conflict-free), and each half adds the other's (a + b: the same sum on
    // either side)
    static_assert(NW * 64 * 4 * KTW * 16 <= SPL * BUF, "a partial fits one ring array");
    raw_barrier();
    float* xo_ = reinterpret_cast<float*>(hv == 1 ? ring0 : ring1) + w * (KTW * 16 * 64) + lane;
#pragma unroll
    for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) xo_[((kt * 4 + dt) * 4 + r) * 64] = hv == 1 ? dk[kt][dt][r] : dv[kt][dt][r];
    __syncthreads();
    const float* xi = reinterpret_cast<const float*>(hv == 0 ? ring0 : ring1) + w * (KTW * 16 * 64) + lane;
#pragma unroll
    for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = xi[((kt * 4 + dt) * 4 + r) * 64];
          if (hv == 0)
            dk[kt][dt][r] += o;
          else
            dv[kt][dt][r] += o;
        }
  }
  // store: dk[kt][dt][r] = dK[key = kw0 + kt*16 + 4g + r][dk = dt*16 + i]; masked keys -> 0;
  // dK = dS^T Q' / log2(e).  SPL = 2: half 0 stores dK, half 1 dV
  const bool st_k = SPL == 1 || hv == 0, st_v = SPL == 1 || hv == 1;
  bf16* dK = (bf16*)a.dk + (int64_t)b * Tk * a.lddk + h * HD;
  bf16* dV = (bf16*)a.dv + (int64_t)b * Tk * a.lddv + h * HD;
#pragma unroll
  for (int kt = 0; kt < KTW; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kw0 + kt * 16 + 4 * g + r;
      if (key >= Tk) continue;
      const bool ok = kvalid[(int64_t)b * Tk + key] != 0;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        if (st_k) rp_st(dK + (int64_t)key * a.lddk + dt * 16 + i, ok ? dk[kt][dt][r] * (1.f / LOG2E) : 0.f);
        if (st_v) rp_st(dV + (int64_t)key * a.lddv + dt * 16 + i, ok ? dv[kt][dt][r] : 0.f);
      }
    }
}

template <bool DROP, int KTW, bool PIPE, int SPL = 1>
__global__ __launch_bounds__(NT * SPL, 2 / SPL) void attn_bwd_kv_dma_kernel(MhaDev a) {
  __shared__ __attribute__((aligned(1024))) char lds[3 * SPL * KV_DMA_BUF];
  attn_bwd_kv_dma_body<DROP, KTW, PIPE, SPL>(a, blockIdx.x, lds);
}

// =================================================================================================
// backward: dQ per 128-query block (4 waves x 32 queries), sweep over 64-key tiles
// =================================================================================================
// DELTA: the kernel also forms delta = rowsum(dO * O) of its queries (the lane's 16 dims of dO are
// already in registers; the 4 lanes of a query combine by quad_sum) and writes it for the dK/dV
// kernel, which then runs second — no separate delta pre-pass over dO and O.
template <typename T, bool DROP, bool DELTA, int QT>
__global__ __launch_bounds__(NT, 2) void attn_bwd_q_kernel(MhaDev a) {
  constexpr int QB = NW * 16 * QT;  // queries per workgroup (QT query tiles of 16 per wave)
  using C = AttnCfg<T>;
  constexpr bool BF = std::is_same<T, bf16>::value;
  constexpr int TILE = FW_KT * C::ROWB;
  constexpr int BUF = 2 * TILE + FW_KT * 4 + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const uint8_t* __restrict__ kvalid = a.kvalid;
  const float scale = a.scale, drop_scale = a.drop_scale;
  const float* __restrict__ lse = a.lse;
  const float* __restrict__ delta = a.delta;
  const int nqb = (Tq + QB - 1) / QB;
  const int L = rp_xcd_remap(blockIdx.x, nqb * B * H);
  const int bh = L / nqb, qb = L % nqb;
  const int b = bh / H, h = bh % H;
  const int64_t ldq = a.ldq, ldk = a.ldk, ldv = a.ldv, lddo = a.lddo;
  const T* Qg = (const T*)a.q + (int64_t)b * Tq * ldq + h * HD;
  const T* Kg = (const T*)a.k + (int64_t)b * Tk * ldk + h * HD;
  const T* Vg = (const T*)a.v + (int64_t)b * Tk * ldv + h * HD;
  const T* dOg = (const T*)a.dout + (int64_t)b * Tq * lddo + h * HD;
  const int q0 = qb * QB + w * 16 * QT;
  const float c = scale * LOG2E;
  const int KT = mask_kt(Tk);
  const int64_t ldm = mask_ld(Tq);
  const uint16_t* mrow = a.dmask ? a.dmask + (int64_t)bh * KT * 4 * ldm : nullptr;

  bf16x8 qf[QT][2], df[QT][2];
  float qs[QT][16], dsv[QT][16];
  float lq[QT], dq[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = q0 + qt * 16 + i;
    // with dropout the 1/(1-p) scale rides in the exponent: exp2(S*c - lq) = p * ds
    lq[qt] = q < Tq ? lse[(int64_t)bh * Tq + q] * LOG2E - (DROP ? log2f(drop_scale) : 0.f) : INFINITY;
    if constexpr (!DELTA)
      dq[qt] = q < Tq ? -delta[(int64_t)bh * Tq + q] * (DROP ? 1.f / drop_scale : 1.f) : 0.f;  // -delta/ds
    float part = 0.f;  // DELTA: this lane's share of rowsum(dO * O)
    if constexpr (BF) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        qf[qt][s] = row_frag_gmem((const bf16*)Qg, ldq, q0 + qt * 16, Tq, s * 32, lane);
        df[qt][s] = row_frag_gmem((const bf16*)dOg, lddo, q0 + qt * 16, Tq, s * 32, lane);
        if constexpr (DELTA) {
          const bf16x8 of = row_frag_gmem((const bf16*)a.out + (int64_t)b * Tq * a.ldo + h * HD, a.ldo,
                                          q0 + qt * 16, Tq, s * 32, lane);
          if (a.out_lo) {  // O = hi + lo: delta from the unrounded output (exact rowsum(dO * O))
            const bf16x8 ol = row_frag_gmem((const bf16*)a.out_lo + (int64_t)b * Tq * a.ldo + h * HD, a.ldo,
                                            q0 + qt * 16, Tq, s * 32, lane);
#pragma unroll
            for (int j = 0; j < 8; ++j) part += (float)df[qt][s][j] * ((float)of[j] + (float)ol[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) part += (float)df[qt][s][j] * (float)of[j];
          }
        }
      }
    } else {
      const T* Og = (const T*)a.out + (int64_t)b * Tq * a.ldo + h * HD;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        qs[qt][s] = q < Tq ? (float)Qg[(int64_t)q * ldq + 4 * s + g] : 0.f;
        dsv[qt][s] = q < Tq ? (float)dOg[(int64_t)q * lddo + 4 * s + g] : 0.f;
        if constexpr (DELTA) part += dsv[qt][s] * (q < Tq ? (float)Og[(int64_t)q * a.ldo + 4 * s + g] : 0.f);
      }
    }
    if constexpr (DELTA) {
      const float dl = quad_sum(part);
      dq[qt] = q < Tq ? -dl * (DROP ? 1.f / drop_scale : 1.f) : 0.f;
      if (g == 0 && q < Tq) {  // delta and the dK/dV kernel's row constants (planes 1, 2)
        const int64_t plane = (int64_t)B * H * Tq;
        a.delta[(int64_t)bh * Tq + q] = dl;
        a.delta[plane + (int64_t)bh * Tq + q] = dq[qt];
        a.delta[2 * plane + (int64_t)bh * Tq + q] = -lq[qt];
      }
    }
  }
  // no valid key + empty_uniform: the scores were constants (masked_fill), so dQ = 0 (delta above
  // is still written: the dK/dV kernel reads it)
  if (seq_has_no_key(a, b, tid)) {
    T* dQz = (T*)a.dq + (int64_t)b * Tq * a.lddq + h * HD;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + qt * 16 + 4 * g + r;
        if (q >= Tq) continue;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) rp_st(dQz + (int64_t)q * a.lddq + dt * 16 + i, 0.f);
      }
    return;
  }

  // Q enters S^T = K Q^T prescaled by c = scale*log2(e) (Q feeds no other product here), so with
  // S^T starting at -lse*log2(e) (+ the key bias) the probability is exp2 of the accumulator
  float nlq[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    nlq[qt] = -lq[qt];
    if (a.qpre) continue;  // the producer already wrote Q * c
    if constexpr (BF) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qt][s2][j] = (bf16)((float)qf[qt][s2][j] * c);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) qs[qt][s2] *= c;
    }
  }

  f32x4 dqa[QT][4];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dqa[qt][dt] = zero4();

  Stage<T, FW_KT> sk, sv;
  auto load_valid = [&](int k0) -> bool {
    const int k = k0 + lane;
    return w == 0 && k < Tk && kvalid[(int64_t)b * Tk + k];
  };
  auto stage_mask = [&](char* buf, bool ok) {
    float* kbm = reinterpret_cast<float*>(buf + 2 * TILE);
    if (w == 0) {
      kbm[lane] = ok ? 0.f : -INFINITY;  // key bias, added to the S^T accumulators' start
      const unsigned long long bal = __ballot(ok);
      if (lane == 0) *reinterpret_cast<int*>(buf + 2 * TILE + FW_KT * 4) = bal == ~0ull;  // no masked key
    }
  };
  const int nkt = (Tk + FW_KT - 1) / FW_KT;
  sk.load(Kg, ldk, 0, Tk, tid);
  sv.load(Vg, ldv, 0, Tk, tid);
  bool kvn = load_valid(0);
  sk.store(lds, tid);
  sv.store(lds + TILE, tid);
  stage_mask(lds, kvn);
  __syncthreads();

  for (int it = 0; it < nkt; ++it) {
    char* cur = lds + (it & 1) * BUF;
    char* nxt = lds + ((it + 1) & 1) * BUF;
    const bool more = it + 1 < nkt;
    const int k0 = it * FW_KT;
    // keep-bit word of this lane's queries for the tile (same register layout as the forward)
    uint32_t kwd[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) kwd[qt] = 0u;
    if constexpr (DROP) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const int q = q0 + qt * 16 + i;
        kwd[qt] = q < Tq ? (uint32_t)mrow[((int64_t)it * 4 + g) * ldm + q] : 0u;
      }
    }
    if (more) {
      sk.load(Kg, ldk, k0 + FW_KT, Tk, tid);
      sv.load(Vg, ldv, k0 + FW_KT, Tk, tid);
      kvn = load_valid(k0 + FW_KT);
    }
    const char* Kl = cur;
    const char* Vl = cur + TILE;
    const float* kbias = reinterpret_cast<const float*>(cur + 2 * TILE);

    // S^T[key][q] = K Q^T, dP^T[key][q] = V dO^T : row key = kt*16 + 4g + r, col q = qt*16 + i.
    // Row / column constants as the initial accumulators: S^T starts at -lse*log2(e) plus the key
    // bias (0 / -inf: masked keys give P = 0 with no select; added only on tiles with a masked
    // key), dP^T at -delta/ds.
    const bool full = *reinterpret_cast<const int*>(cur + 2 * TILE + FW_KT * 4) != 0;
    f32x4 s[4][QT], dp[4][QT];
    if constexpr (BF) {
      // the constants enter as the first MFMA's C operand (no per-tile register copies); the key
      // bias is added after the chain (0 + x == x, -inf + x == -inf: same values as adding it first)
      f32x4 s0[QT], d0[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        s0[qt] = f32x4{nlq[qt], nlq[qt], nlq[qt], nlq[qt]};
        d0[qt] = f32x4{dq[qt], dq[qt], dq[qt], dq[qt]};
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          bf16x8 ka = row_frag_lds(Kl, kt * 16, ss * 32, lane);
          bf16x8 va = row_frag_lds(Vl, kt * 16, ss * 32, lane);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            s[kt][qt] = mfma_bf16(ka, qf[qt][ss], ss == 0 ? s0[qt] : s[kt][qt]);
            dp[kt][qt] = mfma_bf16(va, df[qt][ss], ss == 0 ? d0[qt] : dp[kt][qt]);
          }
        }
      if (!full) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const f32x4 kb4 = *reinterpret_cast<const f32x4*>(kbias + kt * 16 + 4 * g);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) s[kt][qt] += kb4;
        }
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          s[kt][qt] = f32x4{nlq[qt], nlq[qt], nlq[qt], nlq[qt]};
          dp[kt][qt] = f32x4{dq[qt], dq[qt], dq[qt], dq[qt]};
        }
      }
      if (!full) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const f32x4 kb4 = *reinterpret_cast<const f32x4*>(kbias + kt * 16 + 4 * g);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) s[kt][qt] += kb4;
        }
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 16; ++ss) {
          float ka = ldsf(Kl, kt * 16 + i, 4 * ss + g);
          float va = ldsf(Vl, kt * 16 + i, 4 * ss + g);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            s[kt][qt] = mfma_f32(ka, qs[qt][ss], s[kt][qt]);
            dp[kt][qt] = mfma_f32(va, dsv[qt][ss], dp[kt][qt]);
          }
        }
    }
    // dS^T = P^T (keep*ds*dP^T - delta) = P^T*ds*(keep ? acc : -delta/ds)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = rp_exp2(s[kt][qt][r]);  // with dropout: p * ds
          if constexpr (DROP) {
            const uint32_t km = keep_mask(kwd[qt], 4 * kt + r);
            s[kt][qt][r] = p * bfi_select(km, dp[kt][qt][r], dq[qt]);
          } else {
            s[kt][qt][r] = p * dp[kt][qt][r];
          }
        }
    }
    // dQ[q][dk] += dS K : A = dS (q on row = lane i, key slots), B = K columns (tr read)
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 sa[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) sa[qt] = pack8(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          bf16x8 kb = col_frag_lds(Kl, ks * 32, dt * 16, lane);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) dqa[qt][dt] = mfma_bf16(sa[qt], kb, dqa[qt][dt]);
        }
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const float kb = ldsf(Kl, kt * 16 + 4 * g + r, dt * 16 + i);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) dqa[qt][dt] = mfma_f32(s[kt][qt][r], kb, dqa[qt][dt]);
          }
    }
    if (more) {
      sk.store(nxt, tid);
      sv.store(nxt + TILE, tid);
      stage_mask(nxt, kvn);
    }
    __syncthreads();
  }
  // store: dqa[qt][dt][r] = dQ[q = q0 + qt*16 + 4g + r][dk = dt*16 + i]
  T* dQ = (T*)a.dq + (int64_t)b * Tq * a.lddq + h * HD;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + qt * 16 + 4 * g + r;
      if (q >= Tq) continue;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) rp_st(dQ + (int64_t)q * a.lddq + dt * 16 + i, dqa[qt][dt][r] * scale);
    }
}

// =================================================================================================
// backward: dQ (+ the fused delta) — bf16, LDS-DMA staged variant (the default for bf16 with
// 128-query blocks and Tk <= QD_TKMAX; RP_ATTN_DMA=0 selects the register-staged kernel above).
// Same math and register layouts as attn_bwd_q_kernel<bf16, DROP, true, 2>; what changes is how
// the key tiles reach LDS:
//  * K and V tiles and this block's keep-bit words of a key tile arrive by LDS-DMA (the swizzled
//    images of dma_rows64; the words as one 1 KB piece) in a three-slot ring two tiles ahead, one
//    barrier per tile — the register-staged kernel has one tile of compute to hide the K / V loads
//    and loads its keep-bit word from global memory inside the tile;
//  * the sequence's key-valid bytes are staged in LDS once, with a per-tile "no masked key" flag;
//    rows past Tk (clamped DMA sources) are invalid keys there, so they get P = 0.
// =================================================================================================
constexpr int QD_TKMAX = 8192;
// one ring slot of the dQ kernel (a 64-key K and V image plus 1 KB of keep bits) and its whole LDS
constexpr int QD_DMA_BUF = 2 * FW_KT * AttnCfg<bf16>::ROWB + 1024;
constexpr int QD_DMA_LDS(int spl) { return 3 * spl * QD_DMA_BUF + QD_TKMAX + QD_TKMAX / FW_KT * 4; }

// SPL = 2 (grids that fill the CUs once but not twice): eight waves, waves 4-7 the same 128 queries over
// the second half of the key tiles on a ring of their own; both halves form the prologue's row
// constants (half 0 writes delta), the dQ partials are added through LDS (half 0 stores query rows
// qt = 0, half 1 qt = 1; own + partner on either side)
// FD = false: delta was formed by attn_delta_kernel beforehand (the dQ kernel then runs beside the
// dK/dV kernel instead of before it); the row constants -delta/ds are read from its plane 1 and no O
// rows are loaded
template <bool DROP, int SPL = 1, bool FD = true>
__device__ __forceinline__ void attn_bwd_q_dma_body(const MhaDev& a, const int blk, char* lds) {
  constexpr int QT = 2, QB = NW * 16 * QT;  // 128 queries per workgroup
  using C = AttnCfg<bf16>;
  constexpr int TILE = FW_KT * C::ROWB;  // one 64-key K or V image (8 KB)
  constexpr int MASKB = 1024;            // keep bits of the tile: 4 lane groups x 128 queries x u16
  constexpr int BUF = 2 * TILE + MASKB;
  constexpr int NBUF = 3;
  constexpr int NTS = NT * SPL;
  static_assert(BUF == QD_DMA_BUF, "QD_DMA_BUF out of date");
  char* const ring0 = lds;  // the caller's LDS: three slots, then the key-valid bytes and tile flags
  char* const ring1 = lds + SPL * BUF;
  char* const ring2 = lds + 2 * SPL * BUF;
  uint8_t* const kvl = reinterpret_cast<uint8_t*>(lds + 3 * SPL * BUF);
  int* const kfull = reinterpret_cast<int*>(lds + 3 * SPL * BUF + QD_TKMAX);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wq & (NW - 1);            // wave within its key half
  const int hv = SPL == 1 ? 0 : wq / NW;  // key half (SPL = 2)
  const int hoff = hv * BUF;
  const int g = lane >> 4, i = lane & 15;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const float scale = a.scale, drop_scale = a.drop_scale;
  const float* __restrict__ lse = a.lse;
  const int nqb = (Tq + QB - 1) / QB;
  const int L = rp_xcd_remap(blk, nqb * B * H);
  const int bh = L / nqb, qb = L % nqb;
  const int b = bh / H, h = bh % H;
  const int64_t ldq = a.ldq, ldk = a.ldk, ldv = a.ldv, lddo = a.lddo;
  const bf16* Qg = (const bf16*)a.q + (int64_t)b * Tq * ldq + h * HD;
  const bf16* Kg = (const bf16*)a.k + (int64_t)b * Tk * ldk + h * HD;
  const bf16* Vg = (const bf16*)a.v + (int64_t)b * Tk * ldv + h * HD;
  const bf16* dOg = (const bf16*)a.dout + (int64_t)b * Tq * lddo + h * HD;
  const int q0 = qb * QB + w * 16 * QT;
  const float c = scale * LOG2E;
  const int KT = mask_kt(Tk);
  const int64_t ldm = mask_ld(Tq);
  const uint16_t* mrow = a.dmask ? a.dmask + (int64_t)bh * KT * 4 * ldm : nullptr;

  // ---- prologue: Q, dO fragments, lse, delta (= rowsum(dO * O), written for the dK/dV kernel) ----
  bf16x8 qf[QT][2], df[QT][2];
  float lq[QT], dq[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = q0 + qt * 16 + i;
    lq[qt] = q < Tq ? lse[(int64_t)bh * Tq + q] * LOG2E - (DROP ? log2f(drop_scale) : 0.f) : INFINITY;
    float part = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      qf[qt][s2] = row_frag_gmem(Qg, ldq, q0 + qt * 16, Tq, s2 * 32, lane);
      df[qt][s2] = row_frag_gmem(dOg, lddo, q0 + qt * 16, Tq, s2 * 32, lane);
      if constexpr (!FD) continue;
      const bf16x8 of = row_frag_gmem((const bf16*)a.out + (int64_t)b * Tq * a.ldo + h * HD, a.ldo, q0 + qt * 16, Tq,
                                      s2 * 32, lane);
      if (a.out_lo) {  // O = hi + lo: delta from the unrounded output (exact rowsum(dO * O))
        const bf16x8 ol = row_frag_gmem((const bf16*)a.out_lo + (int64_t)b * Tq * a.ldo + h * HD, a.ldo,
                                        q0 + qt * 16, Tq, s2 * 32, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)df[qt][s2][j] * ((float)of[j] + (float)ol[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)df[qt][s2][j] * (float)of[j];
      }
    }
    const int64_t plane = (int64_t)B * H * Tq;
    if constexpr (!FD) {
      dq[qt] = q < Tq ? a.delta[plane + (int64_t)bh * Tq + q] : 0.f;  // -delta/ds, precomputed
      continue;
    }
    const float dl = quad_sum(part);
    dq[qt] = q < Tq ? -dl * (DROP ? 1.f / drop_scale : 1.f) : 0.f;
    if (g == 0 && q < Tq && hv == 0) {  // delta and the dK/dV kernel's row constants (planes 1, 2)
      a.delta[(int64_t)bh * Tq + q] = dl;
      a.delta[plane + (int64_t)bh * Tq + q] = dq[qt];
      a.delta[2 * plane + (int64_t)bh * Tq + q] = -lq[qt];
    }
  }
  if (seq_has_no_key(a, b, tid)) {  // empty_uniform: dQ = 0 (delta above is still written)
    bf16* dQz = (bf16*)a.dq + (int64_t)b * Tq * a.lddq + h * HD;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + qt * 16 + 4 * g + r;
        if (q >= Tq) continue;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dQz[(int64_t)q * a.lddq + dt * 16 + i] = (bf16)0.f;
      }
    return;
  }
  float nlq[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    nlq[qt] = -lq[qt];
    if (!a.qpre) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qt][s2][j] = (bf16)((float)qf[qt][s2][j] * c);
    }
  }
  // key-valid bytes of the sequence (0 past Tk) and per-tile "no masked key" flags, staged once
  const int nkt = (Tk + FW_KT - 1) / FW_KT;
  for (int k = tid; k < nkt * FW_KT; k += NTS) kvl[k] = k < Tk ? (a.kvalid[(int64_t)b * Tk + k] != 0) : 0;
  __syncthreads();
  for (int t = tid; t < nkt; t += NTS) {
    int ok = 1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t v = reinterpret_cast<const uint32_t*>(kvl)[t * 16 + j];
      ok &= ((v - 0x01010101u) & ~v & 0x80808080u) == 0u;  // no zero byte
    }
    kfull[t] = ok;
  }
  // consume Q / dO here, before the loop: otherwise their wait lands at the first use inside the
  // loop as a full vmcnt(0) on every ring cycle
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) asm volatile("" ::"v"(qf[qt][s2]), "v"(df[qt][s2]));
  __syncthreads();

  f32x4 dqa[QT][4];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dqa[qt][dt] = zero4();

  auto ring = [&](auto bi) -> char* {
    constexpr int BI = decltype(bi)::value;
    return (BI == 0 ? ring0 : (BI == 1 ? ring1 : ring2)) + hoff;
  };
  // key tiles: this half's nkh tiles start at tile kt0; both halves run nsteps ring steps (the half
  // with one tile fewer idles through the last one: every wave passes every barrier)
  const int nh0 = SPL == 1 ? nkt : (nkt + 1) / 2;
  const int kt0 = hv * nh0;
  const int nkh = SPL == 1 ? nkt : (hv == 0 ? nh0 : nkt - nh0);
  // LDS-DMA of key tile it into slot BI: K and V (two 1 KB pieces each per wave) and, with dropout,
  // wave 1 the 4 x 128 keep-bit words of this query block (columns past ldm clamped: their queries
  // are past Tq and never read)
  Rows64 rk, rv;
  rk.init(Kg, ldk, Tk, w, lane);
  rv.init(Vg, ldv, Tk, w, lane);
  // keep bits (wave 1): lane (g, c) reads words [tile][g][this block's 128 queries], column chunk
  // c ^ 2g into LDS chunk c: row g's 32-byte chunks are XOR-swizzled by g, so the tile loop's 16-bit
  // reads (lanes of groups g and g ^ 1 share an LDS lane group; rows are 256 B = 0 mod 32 banks apart)
  // hit different bank octets — conflict-free (the unswizzled rows were 2-way conflicted at p > 0).
  // ldm is a multiple of 128, so the block's 128 columns are always inside the row.
  const rp_srd srd_m = make_srd(mrow);
  const int64_t mcol = (int64_t)qb * QB + ((lane & 15) ^ (2 * (lane >> 4))) * 8;
  const uint32_t vo_m = (uint32_t)((((int64_t)(lane >> 4)) * ldm + mcol) * 2);
  const bool xfast = (int64_t)KT * 4 * ldm * 2 < ((int64_t)1 << 31) && rk.fast && rv.fast;
  const uint32_t slot_lds[3] = {lds_addr(ring0) + (uint32_t)hoff, lds_addr(ring1) + (uint32_t)hoff,
                                 lds_addr(ring2) + (uint32_t)hoff};
  auto issue = [&](int itl, auto bi) {
    constexpr int BI = decltype(bi)::value;
    char* buf = ring(bi);
    const int it = kt0 + itl;
    const int k0 = it * FW_KT;
    if (xfast && k0 + FW_KT <= Tk) {
      const uint32_t t = slot_lds[BI];
      const uint32_t pk = t + (uint32_t)(w * 2) * 1024u;
      static_assert(TILE == 8192, "dma16b_x4 places the second operand 8 KB on");
      dma16b_x4(rk.srd, rk.vo0, rk.vo1, (uint32_t)k0 * rk.rowbytes, rv.srd, rv.vo0, rv.vo1,
                (uint32_t)k0 * rv.rowbytes, pk);
      if (DROP && w == 1) dma16b(srd_m, vo_m, (uint32_t)it * 8u * (uint32_t)ldm, t + 2 * TILE);
    } else {
      dma_rows64(Kg, ldk, k0, Tk, buf, w, lane);
      dma_rows64(Vg, ldv, k0, Tk, buf + TILE, w, lane);
      if (DROP && w == 1) dma16(mrow + ((int64_t)it * 4 + (lane >> 4)) * ldm + mcol, lds_addr(buf + 2 * TILE));
    }
  };
  auto wait_tile = [&](bool next) {
    if (!next)
      wait_vm<0>();
    else if (DROP && w == 1)
      wait_vm<5>();
    else
      wait_vm<4>();
  };
  if (nkh > 0) issue(0, std::integral_constant<int, 0>());
  if (nkh > 1) issue(1, std::integral_constant<int, 1>());

  auto step = [&](auto bi, int itl) {
    constexpr int BI = decltype(bi)::value;
    wait_tile(itl + 1 < nkh);
    raw_barrier();
    if (SPL > 1 && itl >= nkh) return;
    if (itl + 2 < nkh) issue(itl + 2, std::integral_constant<int, (BI + 2) % NBUF>());
    const int it = kt0 + itl;
    const char* Kl = ring(bi);
    const char* Vl = Kl + TILE;
    uint32_t kwd[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      kwd[qt] = 0u;
      if constexpr (DROP)  // this lane's query word, in its 32-byte chunk (w * QT + qt) ^ g of row g
        kwd[qt] = reinterpret_cast<const uint16_t*>(Kl + 2 * TILE)[g * QB + (((w * QT + qt) ^ g) << 4) + i];
    }
    const bool full = kfull[it] != 0;
    f32x4 s[4][QT], dp[4][QT];
    {
      f32x4 s0[QT], d0[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        s0[qt] = f32x4{nlq[qt], nlq[qt], nlq[qt], nlq[qt]};
        d0[qt] = f32x4{dq[qt], dq[qt], dq[qt], dq[qt]};
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const bf16x8 ka = row_frag_lds(Kl, kt * 16, ss * 32, lane);
          const bf16x8 va = row_frag_lds(Vl, kt * 16, ss * 32, lane);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            s[kt][qt] = mfma_bf16(ka, qf[qt][ss], ss == 0 ? s0[qt] : s[kt][qt]);
            dp[kt][qt] = mfma_bf16(va, df[qt][ss], ss == 0 ? d0[qt] : dp[kt][qt]);
          }
        }
    }
    if (!full) {  // key bias 0 / -inf from the staged valid bytes of keys kt*16 + 4g + r
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const uint32_t vb = *reinterpret_cast<const uint32_t*>(kvl + it * FW_KT + kt * 16 + 4 * g);
        f32x4 kb4;
#pragma unroll
        for (int r = 0; r < 4; ++r) kb4[r] = ((vb >> (8 * r)) & 0xFFu) ? 0.f : -INFINITY;
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[kt][qt] += kb4;
      }
    }
    // dS^T = P^T (keep*ds*dP^T - delta) = P^T*ds*(keep ? acc : -delta/ds)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = rp_exp2(s[kt][qt][r]);
          if constexpr (DROP) {
            const uint32_t km = keep_mask(kwd[qt], 4 * kt + r);
            s[kt][qt][r] = p * bfi_select(km, dp[kt][qt][r], dq[qt]);
          } else {
            s[kt][qt][r] = p * dp[kt][qt][r];
          }
        }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 sa[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) sa[qt] = pack8(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 kb = col_frag_lds(Kl, ks * 32, dt * 16, lane);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) dqa[qt][dt] = mfma_bf16(sa[qt], kb, dqa[qt][dt]);
      }
    }
  };
  const int nsteps = SPL == 1 ? nkt : nh0;
  for (int it = 0; it < nsteps; it += NBUF) {
    step(std::integral_constant<int, 0>(), it);
    if (it + 1 < nsteps) step(std::integral_constant<int, 1>(), it + 1);
    if (it + 2 < nsteps) step(std::integral_constant<int, 2>(), it + 2);
  }
  if constexpr (SPL > 1) {
    // every DMA has landed (each half's last step waited vmcnt(0)); after this barrier no wave reads a
    // ring again.  Half 1 hands over its qt = 0 partial in ring0, half 0 its qt = 1 partial in ring1
    // (lane-major rows of 64 floats)
    static_assert(NW * 64 * 16 * 4 <= SPL * BUF, "a partial fits one ring array");
    raw_barrier();
    float* xo_ = reinterpret_cast<float*>(hv == 1 ? ring0 : ring1) + w * (16 * 64) + lane;
    const int qo = hv == 1 ? 0 : 1;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) xo_[(dt * 4 + r) * 64] = dqa[qo][dt][r];
    __syncthreads();
    const float* xi = reinterpret_cast<const float*>(hv == 0 ? ring0 : ring1) + w * (16 * 64) + lane;
    const int qm = hv;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dqa[qm][dt][r] += xi[(dt * 4 + r) * 64];
  }
  // store: dqa[qt][dt][r] = dQ[q = q0 + qt*16 + 4g + r][dk = dt*16 + i]  (SPL = 2: half hv rows qt = hv)
  bf16* dQ = (bf16*)a.dq + (int64_t)b * Tq * a.lddq + h * HD;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + qt * 16 + 4 * g + r;
      if (q >= Tq || (SPL > 1 && qt != hv)) continue;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dQ[(int64_t)q * a.lddq + dt * 16 + i] = (bf16)(dqa[qt][dt][r] * scale);
    }
}

template <bool DROP, int SPL = 1, bool FD = true>
__global__ __launch_bounds__(NT * SPL, 2 / SPL) void attn_bwd_q_dma_kernel(MhaDev a) {
  __shared__ __attribute__((aligned(1024))) char lds[QD_DMA_LDS(SPL)];
  attn_bwd_q_dma_body<DROP, SPL, FD>(a, blockIdx.x, lds);
}

// dK/dV and dQ as ONE launch of two workgroup roles, delta formed beforehand (attn_delta_kernel):
// blocks [0, nkv) run the dK/dV body (128-key blocks), the rest the dQ body reading the precomputed row
// constants (128-query blocks), on one LDS region sized for the larger.  For grids that fill the CUs
// once but not twice (config 4, B = 1, T = 4096: 256 blocks each), where the two kernels would each run
// as eight-wave split workgroups one per CU: here 512 four-wave workgroups two per CU, the dQ blocks
// beside the dK/dV ones, with no partial merge and no cross-stream wait (RP_ATTN_BWD_OVERLAP: 42-68 us).
constexpr int ROLES_LDS = 3 * KV_DMA_BUF > QD_DMA_LDS(1) ? 3 * KV_DMA_BUF : QD_DMA_LDS(1);
template <bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_bwd_roles_kernel(MhaDev a, int nkv) {
  __shared__ __attribute__((aligned(1024))) char lds[ROLES_LDS];
  const int blk = blockIdx.x;
  if (blk < nkv)
    attn_bwd_kv_dma_body<DROP, 2, true, 1>(a, blk, lds);
  else
    attn_bwd_q_dma_body<DROP, 1, false>(a, blk - nkv, lds);
}

// =================================================================================================
// forward — bf16, LDS-DMA staged variant (the default for bf16 with 128-query blocks and
// Tk <= FD_TKMAX; RP_ATTN_DMA_F=0 selects the register-staged kernel).  Same math, register layouts
// and outputs as attn_fwd_kernel<bf16, DROP, 2>; the K / V tiles arrive by LDS-DMA in a three-slot
// ring two tiles ahead (one barrier per tile) instead of registers one tile ahead, and the key-valid
// bytes of the sequence are staged in LDS once with a per-tile "no masked key" flag.  The keep-bit
// words are stored for every query of the block (the rows of the mask are padded to 128 queries), so
// each step issues a fixed number of memory instructions and the counted waits below stay exact
// (VMEM instructions of a wave complete in issue order).
// =================================================================================================
constexpr int FD_TKMAX = 4096;

// SPL = 2 (grids that fill the CUs once but not twice): eight waves, waves 4-7 the same 128 queries over
// the second half of the key tiles on a ring of their own, their dropout streams advanced to that half
// by mwc_mulmod (the keep bits are the unsplit kernel's); the two halves' (max, row sum, O) are merged
// through LDS — half 0 finishes query rows qt = 0, half 1 qt = 1, both from (half 0, half 1) in that order
// SPL = 3: twelve waves, the key tiles in three parts (three waves per SIMD, the unsplit kernel's
// residency, on one block) for grids of at most one block per CU; parts 1 and 2 hand their whole
// state to part 0, which merges in part order and stores
template <bool DROP, int SPL = 1>
__global__ __launch_bounds__(NT * SPL, SPL == 1 ? 3 : 1) void attn_fwd_dma_kernel(MhaDev a) {
  static_assert(SPL >= 1 && SPL <= 3, "one, two or three key parts");
  constexpr int QT = 2, QB = NW * 16 * QT;  // 128 queries per workgroup
  using C = AttnCfg<bf16>;
  constexpr int TILE = FW_KT * C::ROWB;  // 8 KB
  constexpr int BUF = 2 * TILE;
  constexpr int NBUF = 3;
  constexpr int NTS = NT * SPL;
  __shared__ __attribute__((aligned(1024))) char ring0[SPL * BUF];
  __shared__ __attribute__((aligned(1024))) char ring1[SPL * BUF];
  __shared__ __attribute__((aligned(1024))) char ring2[SPL * BUF];
  __shared__ __attribute__((aligned(16))) uint8_t kvl[FD_TKMAX];
  __shared__ int kfull[FD_TKMAX / FW_KT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wq & (NW - 1);            // wave within its key half
  const int hv = SPL == 1 ? 0 : wq / NW;  // key part (SPL > 1)
  const int hoff = hv * BUF;
  const int g = lane >> 4, i = lane & 15;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const uint32_t drop_thresh = a.drop_thresh;
  const float drop_scale = a.drop_scale;
  const float scale = a.scale;
  float* __restrict__ lse = a.lse;
  const int nqb = (Tq + QB - 1) / QB;
  const int L = rp_xcd_remap(blockIdx.x, nqb * B * H);
  const int bh = L / nqb, qb = L % nqb;
  const int b = bh / H, h = bh % H;
  const int64_t ldq = a.ldq, ldk = a.ldk, ldv = a.ldv;
  const bf16* Qg = (const bf16*)a.q + (int64_t)b * Tq * ldq + h * HD;
  const bf16* Kg = (const bf16*)a.k + (int64_t)b * Tk * ldk + h * HD;
  const bf16* Vg = (const bf16*)a.v + (int64_t)b * Tk * ldv + h * HD;
  const int q0 = qb * QB + w * 16 * QT;
  const uint32_t seed_bh = rp_hash(rp_seed_eff(a.seed_base, a.seed), (uint32_t)bh);
  const float c = scale * LOG2E;
  const int KT = mask_kt(Tk);
  const int64_t ldm = mask_ld(Tq);
  uint16_t* mrow = a.dmask ? a.dmask + (int64_t)bh * KT * 4 * ldm : nullptr;
  const bool novalid = seq_has_no_key(a, b, tid);

  bf16x8 qf[QT][2];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) qf[qt][s2] = row_frag_gmem(Qg, ldq, q0 + qt * 16, Tq, s2 * 32, lane);
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    if (novalid) qf[qt][0] = qf[qt][1] = bf16x8{};
    if (!a.qpre) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qt][s2][j] = (bf16)((float)qf[qt][s2][j] * c);
    }
  }
  // key-valid bytes (every key < Tk when the sequence has none: masked_fill semantics) and flags
  const int nkt = (Tk + FW_KT - 1) / FW_KT;
  for (int k = tid; k < nkt * FW_KT; k += NTS)
    kvl[k] = k < Tk ? (novalid || a.kvalid[(int64_t)b * Tk + k] != 0) : 0;
  __syncthreads();
  for (int t = tid; t < nkt; t += NTS) {
    int ok = 1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t v = reinterpret_cast<const uint32_t*>(kvl)[t * 16 + j];
      ok &= ((v - 0x01010101u) & ~v & 0x80808080u) == 0u;  // no zero byte
    }
    kfull[t] = ok;
  }
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) asm volatile("" ::"v"(qf[qt][s2]));
  __syncthreads();

  f32x4 o[QT][4];
  // row sums of P (before dropout).  With dropout (the keep-bit stream makes the tile loop VALU
  // bound) on the matrix core: ls[qt] = ones . P^T over the bf16 P the P.V product uses, every row of
  // the 16 x 16 result holding the sum of query column i (fwd p = 0.1 148.6 -> 142.2 us); without,
  // per-lane fp32 partial sums lp in tree order (the MFMA form measured 109.9 -> 114.3 us there)
  f32x4 ls[QT];
  float lp[QT];
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  float m[QT];
  bool mset[QT];
  float gthr[QT];  // the grow bound of the lane-local test: -inf until the reference is set, then RESCALE_LOG2
  uint64_t dst[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = zero4();
    m[qt] = 0.f;
    ls[qt] = zero4();
    lp[qt] = 0.f;
    mset[qt] = false;
    gthr[qt] = -INFINITY;
    dst[qt] = DROP ? mwc_seed(rp_hash(seed_bh, (uint32_t)(q0 + qt * 16 + i) * 4u + (uint32_t)g)) : 0u;
    if (DROP && SPL > 1)  // to key tile kt0 = hv * nh0
      for (int pj = 0; pj < hv; ++pj) dst[qt] = mwc_mulmod(dst[qt], a.mwc_jump);
  }
  // key tiles: this half's nkh tiles start at tile kt0; both halves run nsteps ring steps (the half
  // with one tile fewer idles through the last one: every wave passes every barrier)
  const int nh0 = SPL == 1 ? nkt : (nkt + SPL - 1) / SPL;
  const int kt0 = hv * nh0;
  const int nkh = SPL == 1 ? nkt : (nkt - kt0 < nh0 ? (nkt - kt0 > 0 ? nkt - kt0 : 0) : nh0);

  auto ring = [&](auto bi) -> char* {
    constexpr int BI = decltype(bi)::value;
    return (BI == 0 ? ring0 : (BI == 1 ? ring1 : ring2)) + hoff;
  };
  Rows64 rk, rv;
  rk.init(Kg, ldk, Tk, w, lane);
  rv.init(Vg, ldv, Tk, w, lane);
  const bool xfast = rk.fast && rv.fast;
  const uint32_t slot_lds[3] = {lds_addr(ring0) + (uint32_t)hoff, lds_addr(ring1) + (uint32_t)hoff,
                                 lds_addr(ring2) + (uint32_t)hoff};
  auto issue = [&](int itl, auto bi) {  // K and V of key tile kt0 + itl: two 1 KB pieces each per wave
    constexpr int BI = decltype(bi)::value;
    const int k0 = (kt0 + itl) * FW_KT;
    if (xfast && k0 + FW_KT <= Tk) {
      const uint32_t pk = slot_lds[BI] + (uint32_t)(w * 2) * 1024u;
      static_assert(TILE == 8192, "dma16b_x4 places the second operand 8 KB on");
      dma16b_x4(rk.srd, rk.vo0, rk.vo1, (uint32_t)k0 * rk.rowbytes, rv.srd, rv.vo0, rv.vo1,
                (uint32_t)k0 * rv.rowbytes, pk);
    } else {
      char* buf = ring(bi);
      dma_rows64(Kg, ldk, k0, Tk, buf, w, lane);
      dma_rows64(Vg, ldv, k0, Tk, buf + TILE, w, lane);
    }
  };
  // step it waits for DMA(it).  Issued after it, in order: (it >= 2) the 2 keep-bit stores of step
  // it - 2, DMA(it + 1) (4), the 2 stores of step it - 1 (it >= 1).
  auto wait_tile = [&](int it) {
    if (it + 1 >= nkh)
      wait_vm<0>();
    else if (!DROP || it == 0)
      wait_vm<4>();
    else if (it == 1)
      wait_vm<6>();
    else
      wait_vm<8>();
  };
  if (nkh > 0) issue(0, std::integral_constant<int, 0>());
  if (nkh > 1) issue(1, std::integral_constant<int, 1>());

  auto step = [&](auto bi, int itl) {
    constexpr int BI = decltype(bi)::value;
    wait_tile(itl);
    raw_barrier();
    if (SPL > 1 && itl >= nkh) return;
    if (itl + 2 < nkh) issue(itl + 2, std::integral_constant<int, (BI + 2) % NBUF>());
    const int kt_i = kt0 + itl;
    const char* Kl = ring(bi);
    const char* Vl = Kl + TILE;
    const bool full = kfull[kt_i] != 0;
    // ---- S^T[key][q] = K (cQ)^T - m ----
    f32x4 s[4][QT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[kt][qt] = f32x4{-m[qt], -m[qt], -m[qt], -m[qt]};
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 kf = row_frag_lds(Kl, kt * 16, ss * 32, lane);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[kt][qt] = mfma_bf16(kf, qf[qt][ss], s[kt][qt]);
      }
    if (!full) {  // key bias 0 / -inf of keys kt*16 + 4g + r
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const uint32_t vb = *reinterpret_cast<const uint32_t*>(kvl + kt_i * FW_KT + kt * 16 + 4 * g);
        f32x4 kb4;
#pragma unroll
        for (int r = 0; r < 4; ++r) kb4[r] = ((vb >> (8 * r)) & 0xFFu) ? 0.f : -INFINITY;
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[kt][qt] += kb4;
      }
    }
    // ---- column max relative to the reference; deferred rescale (see attn_fwd_kernel) ----
    float rel[QT];
    uint64_t grow = 0;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float mx = s[0][qt][0];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
      rel[qt] = mx;  // lane-local test, quad maximum inside the branch (see attn_fwd_kernel)
      grow |= __ballot(mx > gthr[qt]);  // one compare into a lane mask per query tile
    }
    if (grow != 0) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        rel[qt] = quad_max(rel[qt]);
        const bool gq = mset[qt] ? rel[qt] > RESCALE_LOG2 : rel[qt] > -INFINITY;
        const float alpha = gq ? (mset[qt] ? rp_exp2(-rel[qt]) : 0.f) : 1.f;
        const float sub = gq ? rel[qt] : 0.f;
        if constexpr (DROP)
          ls[qt] *= alpha;
        else
          lp[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        m[qt] += sub;
        mset[qt] = mset[qt] || gq;
        gthr[qt] = mset[qt] ? RESCALE_LOG2 : -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) s[kt][qt] -= sub;
      }
    }
    // ---- P = exp2(acc) (+ the VALU row sums without dropout) ----
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float t4[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kt][qt][r] = rp_exp2(s[kt][qt][r]);
        t4[kt] = (s[kt][qt][0] + s[kt][qt][1]) + (s[kt][qt][2] + s[kt][qt][3]);
      }
      if constexpr (!DROP) lp[qt] += (t4[0] + t4[1]) + (t4[2] + t4[3]);
    }
    // ---- dropout masks; keep bits stored for every query of the block (padded rows) ----
    uint32_t dm[QT][8];
    if constexpr (DROP) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const uint32_t word = drop_masks(dst[qt], drop_thresh, dm[qt]);
        mrow[((int64_t)kt_i * 4 + g) * ldm + q0 + qt * 16 + i] = (uint16_t)word;
      }
    }
    // ---- O^T[dk][q] += V^T P^T ----
    bf16x8 pf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        pf[qt][ks] = pack8(s[2 * ks][qt], s[2 * ks + 1][qt]);
        if constexpr (DROP) ls[qt] = mfma_bf16(ones, pf[qt][ks], ls[qt]);  // before dropout
        if constexpr (DROP) {
          uint4 u = __builtin_bit_cast(uint4, pf[qt][ks]);
          u.x &= ~dm[qt][4 * ks + 0];
          u.y &= ~dm[qt][4 * ks + 1];
          u.z &= ~dm[qt][4 * ks + 2];
          u.w &= ~dm[qt][4 * ks + 3];
          pf[qt][ks] = __builtin_bit_cast(bf16x8, u);
        }
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 vf = col_frag_lds(Vl, ks * 32, dt * 16, lane);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[qt][dt] = mfma_bf16(vf, pf[qt][ks], o[qt][dt]);
      }
  };
  const int nsteps = SPL == 1 ? nkt : nh0;
  for (int it = 0; it < nsteps; it += NBUF) {
    step(std::integral_constant<int, 0>(), it);
    if (it + 1 < nsteps) step(std::integral_constant<int, 1>(), it + 1);
    if (it + 2 < nsteps) step(std::integral_constant<int, 2>(), it + 2);
  }
  // the final row sum of query column i for each query tile (every lane of the column holds it)
  float lsum[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) lsum[qt] = DROP ? ls[qt][0] : quad_sum(lp[qt]);
  if constexpr (SPL == 2) {
    // every DMA and keep-bit store has landed (each half's last step waited vmcnt(0)); after this
    // barrier no wave reads a ring again.  Half 1 hands over its qt = 0 state in ring0, half 0 its
    // qt = 1 state in ring1: per lane 16 O values, then m, l, mset (lane-major rows of 64 floats)
    static_assert(NW * 19 * 64 * 4 <= SPL * BUF, "a half's exchange fits one ring array");
    raw_barrier();
    const int qo = hv == 1 ? 0 : 1;
    float* xo_ = reinterpret_cast<float*>(hv == 1 ? ring0 : ring1) + w * (19 * 64) + lane;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) xo_[(dt * 4 + r) * 64] = o[qo][dt][r];
    xo_[16 * 64] = m[qo];
    xo_[17 * 64] = lsum[qo];
    xo_[18 * 64] = mset[qo] ? 1.f : 0.f;
    __syncthreads();
    const int qm = hv;  // the query tile this half finishes
    const float* xi = reinterpret_cast<const float*>(hv == 0 ? ring0 : ring1) + w * (19 * 64) + lane;
    const float pm = xi[16 * 64], pl = xi[17 * 64];
    const bool pset = xi[18 * 64] != 0.f;
    // (m, l, O) of half 0 and half 1 in that order on both sides: the same arithmetic either way
    const float m0 = hv == 0 ? m[qm] : pm, m1 = hv == 0 ? pm : m[qm];
    const float l0 = hv == 0 ? lsum[qm] : pl, l1 = hv == 0 ? pl : lsum[qm];
    const bool s0 = hv == 0 ? mset[qm] : pset, s1 = hv == 0 ? pset : mset[qm];
    const float mm = s0 && s1 ? fmaxf(m0, m1) : (s1 ? m1 : m0);
    const float a0 = s0 ? rp_exp2(m0 - mm) : 0.f, a1 = s1 ? rp_exp2(m1 - mm) : 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float po = xi[(dt * 4 + r) * 64];
        const float o0 = hv == 0 ? o[qm][dt][r] : po, o1 = hv == 0 ? po : o[qm][dt][r];
        o[qm][dt][r] = a0 * o0 + a1 * o1;
      }
    lsum[qm] = a0 * l0 + a1 * l1;
    m[qm] = mm;
  } else if constexpr (SPL > 2) {
    // parts 1 .. SPL-1 write their (O, m, l, mset) of both query tiles (O: 32 floats per lane in ring0 /
    // ring1, the rest: 6 per lane in ring2, lane-major rows of 64 floats); part 0 merges in part order
    static_assert(SPL == 3 && NW * 32 * 64 * 4 <= SPL * BUF && 2 * NW * 6 * 64 * 4 <= SPL * BUF, "exchange fits");
    raw_barrier();
    if (hv > 0) {
      float* xo_ = reinterpret_cast<float*>(hv == 1 ? ring0 : ring1) + w * (32 * 64) + lane;
      float* xs_ = reinterpret_cast<float*>(ring2) + ((hv - 1) * NW + w) * (6 * 64) + lane;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) xo_[((qt * 4 + dt) * 4 + r) * 64] = o[qt][dt][r];
        xs_[(qt * 3 + 0) * 64] = m[qt];
        xs_[(qt * 3 + 1) * 64] = lsum[qt];
        xs_[(qt * 3 + 2) * 64] = mset[qt] ? 1.f : 0.f;
      }
    }
    __syncthreads();
    if (hv > 0) return;  // every barrier of the block is behind: part 0 stores
#pragma unroll
    for (int pp = 1; pp < SPL; ++pp) {
      const float* xi = reinterpret_cast<const float*>(pp == 1 ? ring0 : ring1) + w * (32 * 64) + lane;
      const float* xs = reinterpret_cast<const float*>(ring2) + ((pp - 1) * NW + w) * (6 * 64) + lane;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const float pm = xs[(qt * 3 + 0) * 64], pl = xs[(qt * 3 + 1) * 64];
        const bool pset = xs[(qt * 3 + 2) * 64] != 0.f;
        const float mm = mset[qt] && pset ? fmaxf(m[qt], pm) : (pset ? pm : m[qt]);
        const float a0 = mset[qt] ? rp_exp2(m[qt] - mm) : 0.f, a1 = pset ? rp_exp2(pm - mm) : 0.f;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[qt][dt][r] = a0 * o[qt][dt][r] + a1 * xi[((qt * 4 + dt) * 4 + r) * 64];
        lsum[qt] = a0 * lsum[qt] + a1 * pl;
        m[qt] = mm;
        mset[qt] = mset[qt] || pset;
      }
    }
  }

  // ---- epilogue: O[q][dk] = O^T / l ; lse ----
  const int64_t ldo = a.ldo;
  bf16* __restrict__ out = (bf16*)a.out;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const float l = lsum[qt];
    const int q = q0 + qt * 16 + i;
    if (q >= Tq || (SPL == 2 && qt != hv)) continue;
    const float inv = drop_scale / l;
    bf16* orow = out + ((int64_t)b * Tq + q) * ldo + h * HD;
    bf16* lorow = a.out_lo ? (bf16*)a.out_lo + ((int64_t)b * Tq + q) * ldo + h * HD : nullptr;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 v, vl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = o[qt][dt][r] * inv;
        v[r] = (bf16)x;
        vl[r] = (bf16)(x - (float)v[r]);
      }
      *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = v;
      if (lorow) *reinterpret_cast<bf16x4*>(lorow + dt * 16 + 4 * g) = vl;
    }
    if (g == 0) lse[(int64_t)bh * Tq + q] = m[qt] * 0.6931471805599453f + logf(l);
  }
}

// compute units of the current device (cached per device); every "fills the CUs once / twice" rule
// below is in units of this count (256 on a whole MI355X)
static int64_t attn_cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// 128-row blocks (the LDS-DMA kernels) from one workgroup per CU up; 64-row blocks below.  At one per
// CU the 128-row LDS-DMA kernel still beats the 64-row register-staged one at twice the workgroups
// (config 4, B = 1, T = 4096: fwd 85 vs 96 us; dQ 78 vs 101; step 9.59 -> 9.06 ms)
static bool attn_small(int64_t big_grid) { return big_grid < attn_cu_count(); }

// Split workgroups (SPL = 2: eight waves, the reduced sequence range in two halves, partials merged in
// LDS) for grids of 128-row blocks that fill the CUs once but not twice (config 4: B = 1, T = 4096 is
// 256 blocks): two waves per SIMD instead of one.  RP_ATTN_SPLIT=0 never, =1 whenever the range has
// two tiles (tests), unset: CUs <= grid < 1.5 CUs.  Read per launch (tests flip it).
static bool attn_split(int64_t grid, int tiles) {
  if (tiles < 2) return false;
  const char* e = getenv("RP_ATTN_SPLIT");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  const int64_t cus = attn_cu_count();
  return grid >= cus && grid < cus + cus / 2;
}

template <typename T>
int launch_mha_fwd(const MhaDev& a, hipStream_t s) {
  const int64_t big = (int64_t)((a.Tq + FW_QB - 1) / FW_QB) * a.B * a.H;
  const bool small = attn_small(big);
  const int qb = small ? NW * 16 : FW_QB;
  const int nqb = (a.Tq + qb - 1) / qb;
  const dim3 grid((unsigned)(nqb * a.B * a.H));
  if (small) {
    if (a.drop_thresh)
      hipLaunchKernelGGL((attn_fwd_kernel<T, true, 1>), grid, dim3(NT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<T, false, 1>), grid, dim3(NT), 0, s, a);
  } else if (std::is_same<T, bf16>::value && a.Tk <= FD_TKMAX) {
    const int nkt = (a.Tk + FW_KT - 1) / FW_KT;
    // grids of at most one block per CU (config 4: 256) on the three-part split kernel (three waves
    // per SIMD, the unsplit kernel's residency); RP_ATTN_SPLIT=3 forces it.  Measured and dropped: the
    // metric grid's last partial round (1,024 = 768 + 256 blocks) as a second launch on it: fwd 143 ->
    // 154 us — the single launch already starts tail blocks as first-round blocks retire
    const char* se = getenv("RP_ATTN_SPLIT");
    const bool force3 = se && se[0] == '3';
    const bool autos = !se || (se[0] != '0' && se[0] != '1' && !force3);  // unset / empty / other: auto
    const bool split3 = nkt >= 3 && (force3 || (autos && (int64_t)grid.x <= attn_cu_count()));
    if (split3) {
      MhaDev as = a;
      as.mwc_jump = mwc_jump((nkt + 2) / 3);
      if (a.drop_thresh)
        hipLaunchKernelGGL((attn_fwd_dma_kernel<true, 3>), grid, dim3(3 * NT), 0, s, as);
      else
        hipLaunchKernelGGL((attn_fwd_dma_kernel<false, 3>), grid, dim3(3 * NT), 0, s, as);
    } else if (attn_split((int64_t)grid.x, nkt)) {
      MhaDev as = a;
      as.mwc_jump = mwc_jump((nkt + 1) / 2);
      if (a.drop_thresh)
        hipLaunchKernelGGL((attn_fwd_dma_kernel<true, 2>), grid, dim3(2 * NT), 0, s, as);
      else
        hipLaunchKernelGGL((attn_fwd_dma_kernel<false, 2>), grid, dim3(2 * NT), 0, s, as);
    } else if (a.drop_thresh) {
      hipLaunchKernelGGL((attn_fwd_dma_kernel<true>), grid, dim3(NT), 0, s, a);
    } else {
      hipLaunchKernelGGL((attn_fwd_dma_kernel<false>), grid, dim3(NT), 0, s, a);
    }
  } else {
    if (a.drop_thresh)
      hipLaunchKernelGGL((attn_fwd_kernel<T, true, 2>), grid, dim3(NT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<T, false, 2>), grid, dim3(NT), 0, s, a);
  }
  return rp_check_launch("rp_mha_fwd");
}

// phases: bit 0 = delta pre-pass, bit 1 = dK/dV kernel, bit 2 = dQ kernel.  With bits 0 and 2 both
// set the delta pre-pass is fused into the dQ kernel, which then runs first (dK/dV reads its delta).
template <typename T, int QT>
void launch_bwd_q(bool delta, const MhaDev& a, hipStream_t s) {
  const dim3 grid((unsigned)((a.Tq + NW * 16 * QT - 1) / (NW * 16 * QT) * a.B * a.H));
  if (delta) {
    if (a.drop_thresh)
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, true, true, QT>), grid, dim3(NT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, false, true, QT>), grid, dim3(NT), 0, s, a);
  } else {
    if (a.drop_thresh)
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, true, false, QT>), grid, dim3(NT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, false, false, QT>), grid, dim3(NT), 0, s, a);
  }
}

// the two-role backward (attn_bwd_roles_kernel): bf16 with the producer's Q prescale on the LDS-DMA
// kernels and 128-row blocks on both sides (both grids at least one workgroup per CU).  Config 4 (each
// grid fills the CUs once: 2 x 256 four-wave blocks side by side instead of two launches of eight-wave
// split blocks): step 7.48 -> 7.31 ms; the metric shape (2 x 1,024 blocks, one launch instead of two:
// no drain / fill between the kernels, the roles' different lengths interleaved): 15.39 / 15.42 / 15.44
// -> 15.33 / 15.26 / 15.27 ms (three interleaved pairs, round 5).  RP_ATTN_ROLES=0 keeps the two
// kernels (read per launch)
static bool attn_roles(const MhaDev& a) {
  const char* e = getenv("RP_ATTN_ROLES");
  if (e && e[0] == '0') return false;
  if (!a.qpre || a.empty_uniform || a.Tk > QD_TKMAX) return false;
  const int64_t gkv = (int64_t)((a.Tk + KV_KB - 1) / KV_KB) * a.B * a.H;
  const int64_t gq = (int64_t)((a.Tq + FW_QB - 1) / FW_QB) * a.B * a.H;
  return !attn_small(gkv) && !attn_small(gq);
}

template <typename T>
int launch_mha_bwd(int phases, const MhaDev& a, hipStream_t s) {
  const int64_t rows = (int64_t)a.B * a.Tq;
  const int nkb = (a.Tk + KV_KB - 1) / KV_KB;
  if (std::is_same<T, bf16>::value && (phases & 6) == 6 && attn_roles(a)) {
    if (phases & 1)
      hipLaunchKernelGGL(attn_delta_kernel<T>, delta_grid<T>(a), dim3(256), 0, s, a);
    const int nkv = nkb * a.B * a.H;
    const dim3 grid((unsigned)(nkv + (a.Tq + FW_QB - 1) / FW_QB * a.B * a.H));
    if (a.drop_thresh)
      hipLaunchKernelGGL(attn_bwd_roles_kernel<true>, grid, dim3(NT), 0, s, a, nkv);
    else
      hipLaunchKernelGGL(attn_bwd_roles_kernel<false>, grid, dim3(NT), 0, s, a, nkv);
    return rp_check_launch("rp_mha_bwd");
  }
  // dQ: 128-query blocks unless that leaves fewer than one workgroup per CU (then 64, as the forward)
  const dim3 gq((unsigned)((a.Tq + FW_QB - 1) / FW_QB * a.B * a.H));
  const bool small = attn_small((int64_t)gq.x);
  const bool dma_q = !small && std::is_same<T, bf16>::value && a.Tk <= QD_TKMAX;
  const bool fused = (phases & 5) == 5;
  if (fused) {
    if (dma_q) {
      // bf16, 128-query blocks: the LDS-DMA staged dQ kernel with the delta pre-pass fused in
      if (attn_split((int64_t)gq.x, (a.Tk + FW_KT - 1) / FW_KT)) {
        if (a.drop_thresh)
          hipLaunchKernelGGL((attn_bwd_q_dma_kernel<true, 2>), gq, dim3(2 * NT), 0, s, a);
        else
          hipLaunchKernelGGL((attn_bwd_q_dma_kernel<false, 2>), gq, dim3(2 * NT), 0, s, a);
      } else if (a.drop_thresh) {
        hipLaunchKernelGGL((attn_bwd_q_dma_kernel<true>), gq, dim3(NT), 0, s, a);
      } else {
        hipLaunchKernelGGL((attn_bwd_q_dma_kernel<false>), gq, dim3(NT), 0, s, a);
      }
    } else if (small) {
      launch_bwd_q<T, 1>(true, a, s);
    } else {
      launch_bwd_q<T, 2>(true, a, s);
    }
  } else if (phases & 1) {
    hipLaunchKernelGGL(attn_delta_kernel<T>, delta_grid<T>(a), dim3(256), 0, s, a);
  }
  if (phases & 2) {
    // 128-key blocks unless that leaves fewer than one workgroup per CU: then 64
    const bool small_kv = attn_small((int64_t)nkb * a.B * a.H);
    const dim3 grid(small_kv ? (unsigned)((a.Tk + NW * 16 - 1) / (NW * 16) * a.B * a.H) : (unsigned)(nkb * a.B * a.H));
    // bf16 with the producer's Q prescale: the LDS-DMA staged kernel
    if (std::is_same<T, bf16>::value && a.qpre && !a.empty_uniform) {
      if (small_kv) {
        if (a.drop_thresh)
          hipLaunchKernelGGL((attn_bwd_kv_dma_kernel<true, 1, true>), grid, dim3(NT), 0, s, a);
        else
          hipLaunchKernelGGL((attn_bwd_kv_dma_kernel<false, 1, true>), grid, dim3(NT), 0, s, a);
      } else if (attn_split((int64_t)nkb * a.B * a.H, (a.Tq + KV_QT - 1) / KV_QT)) {
        if (a.drop_thresh)
          hipLaunchKernelGGL((attn_bwd_kv_dma_kernel<true, 2, false, 2>), grid, dim3(2 * NT), 0, s, a);
        else
          hipLaunchKernelGGL((attn_bwd_kv_dma_kernel<false, 2, false, 2>), grid, dim3(2 * NT), 0, s, a);
      } else if (a.drop_thresh) {
        hipLaunchKernelGGL((attn_bwd_kv_dma_kernel<true, 2, true>), grid, dim3(NT), 0, s, a);
      } else {
        hipLaunchKernelGGL((attn_bwd_kv_dma_kernel<false, 2, true>), grid, dim3(NT), 0, s, a);
      }
    } else if (small_kv) {
      if (a.drop_thresh)
        hipLaunchKernelGGL((attn_bwd_kv_kernel<T, true, 1>), grid, dim3(NT), 0, s, a);
      else
        hipLaunchKernelGGL((attn_bwd_kv_kernel<T, false, 1>), grid, dim3(NT), 0, s, a);
    } else {
      if (a.drop_thresh)
        hipLaunchKernelGGL((attn_bwd_kv_kernel<T, true, 2>), grid, dim3(NT), 0, s, a);
      else
        hipLaunchKernelGGL((attn_bwd_kv_kernel<T, false, 2>), grid, dim3(NT), 0, s, a);
    }
  }
  if ((phases & 4) && !fused) {
    if (dma_q) {
      // bf16, 128-query blocks, delta formed beforehand: the LDS-DMA dQ kernel reading it
      if (attn_split((int64_t)gq.x, (a.Tk + FW_KT - 1) / FW_KT)) {
        if (a.drop_thresh)
          hipLaunchKernelGGL((attn_bwd_q_dma_kernel<true, 2, false>), gq, dim3(2 * NT), 0, s, a);
        else
          hipLaunchKernelGGL((attn_bwd_q_dma_kernel<false, 2, false>), gq, dim3(2 * NT), 0, s, a);
      } else if (a.drop_thresh) {
        hipLaunchKernelGGL((attn_bwd_q_dma_kernel<true, 1, false>), gq, dim3(NT), 0, s, a);
      } else {
        hipLaunchKernelGGL((attn_bwd_q_dma_kernel<false, 1, false>), gq, dim3(NT), 0, s, a);
      }
    } else if (small)
      launch_bwd_q<T, 1>(false, a, s);
    else
      launch_bwd_q<T, 2>(false, a, s);
  }
  return rp_check_launch("rp_mha_bwd");
}
int launch_mha_bwd_dtype(int dtype, int phases, const MhaDev& a, hipStream_t s) {
  return dtype == RP_BF16 ? launch_mha_bwd<bf16>(phases, a, s) : launch_mha_bwd<float>(phases, a, s);
}

// host validation of rp_mha_args -> MhaDev; phases 0 = forward
int make_dev(const char* fn, int dtype, int qpre, const rp_mha_args* p, int phases, MhaDev& a) {
  RP_REQUIRE(p, "%s: null args", fn);
  RP_REQUIRE(dtype == RP_BF16 || dtype == RP_F32, "%s: bad dtype %d", fn, dtype);
  RP_REQUIRE(p->head_dim == HD, "%s: head dim %d unsupported (64)", fn, p->head_dim);
  RP_REQUIRE(p->B >= 0 && p->Tq >= 0 && p->Tk >= 0 && p->H > 0, "%s: bad shape", fn);
  RP_REQUIRE(p->dropout_p >= 0.f && p->dropout_p < 1.f, "%s: dropout_p out of range", fn);
  RP_REQUIRE((int64_t)p->Tq * p->Tk < (int64_t)UINT32_MAX, "%s: Tq*Tk too large", fn);
  const int64_t w = (int64_t)p->H * HD;
  RP_REQUIRE(p->ldq >= w && p->ldk >= w && p->ldv >= w && p->ldq % 8 == 0 && p->ldk % 8 == 0 && p->ldv % 8 == 0,
             "%s: q/k/v leading dims must be >= H*dk and multiples of 8", fn);
  RP_REQUIRE(p->q && p->k && p->v && p->key_valid && p->lse, "%s: null pointer", fn);
  RP_REQUIRE(rp_aligned16(p->q) && rp_aligned16(p->k) && rp_aligned16(p->v), "%s: 16-byte alignment required", fn);
  const uint32_t thr = rp_dropout_thresh(p->dropout_p);
  RP_REQUIRE(thr == 0 || (p->dropmask && rp_aligned16(p->dropmask)), "%s: dropout needs the dropmask buffer", fn);
  a = MhaDev{};
  a.q = p->q; a.k = p->k; a.v = p->v; a.ldq = p->ldq; a.ldk = p->ldk; a.ldv = p->ldv;
  a.kvalid = p->key_valid; a.B = p->B; a.Tq = p->Tq; a.Tk = p->Tk; a.H = p->H; a.scale = p->scale;
  a.drop_thresh = thr; a.drop_scale = p->dropout_p > 0.f ? 1.f / (1.f - p->dropout_p) : 1.f; a.seed = p->seed;
  a.seed_base = thr ? p->seed_base : nullptr;
  RP_REQUIRE(!a.seed_base || ((uintptr_t)a.seed_base & 3u) == 0, "%s: misaligned seed_base", fn);
  a.out = p->out; a.ldo = p->ldo; a.lse = p->lse; a.dmask = thr ? p->dropmask : nullptr;
  a.out_lo = dtype == RP_BF16 ? p->out_lo : nullptr;
  a.empty_uniform = p->empty_rows_uniform != 0;
  RP_REQUIRE(!a.out_lo || rp_aligned16(a.out_lo), "%s: out_lo must be 16-byte aligned", fn);
  a.dout = p->dout; a.lddo = p->lddo; a.delta = p->delta_ws;
  a.dq = p->dq; a.lddq = p->lddq; a.dk = p->dk; a.lddk = p->lddk; a.dv = p->dv; a.lddv = p->lddv;
  a.qpre = qpre;
  if (phases == 0 || (phases & 1)) {
    RP_REQUIRE(p->out && p->ldo >= w && p->ldo % 8 == 0 && rp_aligned16(p->out), "%s: bad out / ldo", fn);
  }
  if (phases) {
    RP_REQUIRE(p->dout && p->lddo >= w && p->lddo % 8 == 0 && rp_aligned16(p->dout), "%s: bad dout / lddo", fn);
    RP_REQUIRE(p->delta_ws, "%s: null delta workspace", fn);
  }
  if (phases & 2) {
    RP_REQUIRE(p->dk && p->dv && p->lddk >= w && p->lddv >= w && rp_aligned16(p->dk) && rp_aligned16(p->dv),
               "%s: bad dk / dv", fn);
  }
  if (phases & 4) RP_REQUIRE(p->dq && p->lddq >= w && rp_aligned16(p->dq), "%s: bad dq", fn);
  return RP_OK;
}

// the attention entry points take RP_ATTN_Q_PRESCALED or-ed into their dtype argument
inline int attn_qpre(int dtype) { return (dtype & RP_ATTN_Q_PRESCALED) ? 1 : 0; }
// 0x200 (the removed RP_ATTN_NO_SPLIT of rounds 1-4) is accepted as a no-op, so older callers keep working
inline int attn_dtype(int dtype) { return dtype & ~(RP_ATTN_Q_PRESCALED | 0x200); }

int mha_fwd_entry(int flagged, const rp_mha_args* p, void* stream) {
  const int dtype = attn_dtype(flagged);
  MhaDev a;
  const int rc = make_dev("rp_mha_fwd", dtype, attn_qpre(flagged), p, 0, a);
  if (rc) return rc;
  if (a.B == 0 || a.Tq == 0) return RP_OK;
  RP_REQUIRE(a.Tk > 0, "rp_mha_fwd: no keys");
  hipStream_t s = (hipStream_t)stream;
  return dtype == RP_BF16 ? launch_mha_fwd<bf16>(a, s) : launch_mha_fwd<float>(a, s);
}

int mha_bwd_entry(int flagged, const rp_mha_args* p, int phases, void* stream) {
  RP_REQUIRE(phases >= 1 && phases <= 7, "rp_mha_bwd: phases must be in 1..7");
  const int dtype = attn_dtype(flagged);
  MhaDev a;
  const int rc = make_dev("rp_mha_bwd", dtype, attn_qpre(flagged), p, phases, a);
  if (rc) return rc;
  if (a.B == 0 || a.Tq == 0 || a.Tk == 0) return RP_OK;
  hipStream_t s = (hipStream_t)stream;
  return dtype == RP_BF16 ? launch_mha_bwd<bf16>(phases, a, s) : launch_mha_bwd<float>(phases, a, s);
}

// packed self-attention (qkv [B*T, 3*H*dk]) -> general description
rp_mha_args packed(const void* qkv, const uint8_t* kv, int B, int T, int H, int dk, float scale, float p, uint32_t seed,
                   const uint32_t* seed_base, const void* out, const void* out_lo, float* lse, const uint16_t* dmask, const void* dout, void* dqkv,
                   float* delta) {
  rp_mha_args a{};
  const int64_t ld = 3LL * H * dk, lo = (int64_t)H * dk;
  a.q = qkv; a.k = qkv; a.v = qkv; a.ldq = a.ldk = a.ldv = ld;
  a.key_valid = kv; a.B = B; a.Tq = T; a.Tk = T; a.H = H; a.head_dim = dk; a.scale = scale; a.dropout_p = p; a.seed = seed;
  a.seed_base = seed_base;
  a.out = const_cast<void*>(out); a.ldo = lo; a.lse = lse; a.dropmask = const_cast<uint16_t*>(dmask);
  a.out_lo = const_cast<void*>(out_lo);
  a.dout = dout; a.lddo = lo; a.delta_ws = delta;
  a.dq = dqkv; a.dk = dqkv; a.dv = dqkv; a.lddq = a.lddk = a.lddv = ld;
  return a;
}
// byte offsets of the K and V column blocks of a packed row
void packed_offsets(rp_mha_args& a, int dtype) {
  const int64_t es = dtype == RP_BF16 ? 2 : 4;
  const int64_t off = (int64_t)a.H * a.head_dim * es;
  a.k = (const char*)a.q + off;
  a.v = (const char*)a.q + 2 * off;
  if (a.dq) {
    a.dk = (char*)a.dq + off;
    a.dv = (char*)a.dq + 2 * off;
  }
}

}  // namespace

extern "C" int64_t rp_attn_dropmask_elems(int B, int T, int H) { return rp_mha_dropmask_elems(B, T, T, H); }

extern "C" int64_t rp_mha_dropmask_elems(int B, int Tq, int Tk, int H) {
  if (B <= 0 || Tq <= 0 || Tk <= 0 || H <= 0) return 0;
  return (int64_t)B * H * mask_kt(Tk) * 4 * mask_ld(Tq);
}

extern "C" int rp_mha_fwd(int dtype, const rp_mha_args* args, void* stream) { return mha_fwd_entry(dtype, args, stream); }

extern "C" int rp_mha_bwd(int dtype, const rp_mha_args* args, int phases, void* stream) {
  return mha_bwd_entry(dtype, args, phases, stream);
}

extern "C" int rp_attn_fwd(int dtype, const void* qkv, const uint8_t* key_valid, int B, int T, int H, int dk, float scale,
                           float dropout_p, uint32_t seed, const uint32_t* seed_base, void* out, void* out_lo,
                           float* lse, uint16_t* dropmask, void* stream) {
  RP_REQUIRE(dk == HD, "rp_attn_fwd: head dim %d unsupported (64)", dk);
  RP_REQUIRE(qkv, "rp_attn_fwd: null qkv");
  rp_mha_args a = packed(qkv, key_valid, B, T, H, dk, scale, dropout_p, seed, seed_base, out, out_lo, lse, dropmask, nullptr,
                         nullptr, nullptr);
  packed_offsets(a, attn_dtype(dtype));
  return mha_fwd_entry(dtype, &a, stream);
}

static int attn_bwd_packed(int phases, int dtype, const void* qkv, const void* out, const void* out_lo, const void* dout,
                           const float* lse, const uint8_t* key_valid, int B, int T, int H, int dk, float scale,
                           float dropout_p, const uint16_t* dropmask, void* dqkv, float* delta_ws, void* stream) {
  RP_REQUIRE(dk == HD, "rp_attn_bwd: head dim %d unsupported (64)", dk);
  RP_REQUIRE(qkv && dqkv, "rp_attn_bwd: null qkv / dqkv");
  rp_mha_args a = packed(qkv, key_valid, B, T, H, dk, scale, dropout_p, 0, nullptr, out, out_lo, const_cast<float*>(lse),
                         dropmask, dout, dqkv, delta_ws);
  packed_offsets(a, attn_dtype(dtype));
  return mha_bwd_entry(dtype, &a, phases, stream);
}

extern "C" int rp_attn_bwd_uses_roles(int dtype, int B, int T, int H, int dk) {
  if (attn_dtype(dtype) != RP_BF16 || dk != HD || B <= 0 || T <= 0 || H <= 0) return 0;
  MhaDev a{};
  a.B = B; a.Tq = T; a.Tk = T; a.H = H; a.qpre = attn_qpre(dtype);
  return attn_roles(a) ? 1 : 0;
}

extern "C" int rp_attn_bwd(int dtype, const void* qkv, const void* out, const void* out_lo, const void* dout,
                           const float* lse, const uint8_t* key_valid, int B, int T, int H, int dk, float scale,
                           float dropout_p, const uint16_t* dropmask, void* dqkv, float* delta_ws, void* stream) {
  return attn_bwd_packed(7, dtype, qkv, out, out_lo, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask,
                         dqkv, delta_ws, stream);
}

extern "C" int rp_attn_bwd_given_delta(int dtype, const void* qkv, const void* dout, const float* lse,
                                       const float* delta_ws, const uint8_t* key_valid, int B, int T, int H, int dk,
                                       float scale, float dropout_p, const uint16_t* dropmask, void* dqkv,
                                       void* stream) {
  return attn_bwd_packed(6, dtype, qkv, nullptr, nullptr, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask,
                         dqkv, const_cast<float*>(delta_ws), stream);
}

extern "C" int rp_attn_bwd_delta(int dtype, const void* out, const void* out_lo, const void* dout, const float* lse,
                                 int B, int T, int H, int dk, float dropout_p, float* delta_ws, void* stream) {
  RP_REQUIRE(dk == HD, "rp_attn_bwd_delta: head dim %d unsupported (64)", dk);
  RP_REQUIRE(B >= 0 && T >= 0 && H > 0, "rp_attn_bwd_delta: bad shape");
  if (B == 0 || T == 0) return RP_OK;
  RP_REQUIRE(out && dout && delta_ws, "rp_attn_bwd_delta: null pointer");
  dtype = attn_dtype(dtype);
  RP_REQUIRE(dtype == RP_BF16 || dtype == RP_F32, "rp_attn_bwd_delta: bad dtype");
  MhaDev a{};
  a.B = B; a.Tq = T; a.Tk = T; a.H = H; a.out = const_cast<void*>(out); a.ldo = (int64_t)H * HD; a.dout = dout;
  a.out_lo = dtype == RP_BF16 ? const_cast<void*>(out_lo) : nullptr;
  a.lddo = (int64_t)H * HD; a.delta = delta_ws;
  a.lse = const_cast<float*>(lse);
  a.drop_scale = dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f;
  return launch_mha_bwd_dtype(dtype, 1, a, (hipStream_t)stream);
}

extern "C" int rp_attn_bwd_dkdv(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                                const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                                const uint16_t* dropmask, void* dqkv, void* stream) {
  return attn_bwd_packed(2, dtype, qkv, nullptr, nullptr, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask,
                         dqkv, const_cast<float*>(delta_ws), stream);
}

extern "C" int rp_attn_bwd_dq_delta(int dtype, const void* qkv, const void* out, const void* out_lo, const void* dout,
                                    const float* lse, float* delta_ws, const uint8_t* key_valid, int B, int T, int H, int dk,
                                    float scale, float dropout_p, const uint16_t* dropmask, void* dqkv, void* stream) {
  RP_REQUIRE(out, "rp_attn_bwd_dq_delta: null out");
  return attn_bwd_packed(5, dtype, qkv, out, out_lo, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask,
                         dqkv, delta_ws, stream);
}

extern "C" int rp_attn_bwd_dq(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                              const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                              const uint16_t* dropmask, void* dqkv, void* stream) {
  return attn_bwd_packed(4, dtype, qkv, nullptr, nullptr, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask,
                         dqkv, const_cast<float*>(delta_ws), stream);
}
