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

// Byte offset of (row, byte-in-row) in an LDS tile.  bf16: the 32-byte pair of 16-byte chunks is
// XORed with (row >> 1) & 3, which makes both access patterns conflict-free: ds_read_b128 row
// fragments (16 lanes = 16 rows x 2 adjacent chunks cover all 16 bank quads) and
// ds_read_b64_tr_b16 column fragments (8 consecutive rows x one 32-byte pair cover all 8 bank
// octets).  The pair index (bits 5-6) changes, the chunk parity (bit 4) and byte (bits 0-3) stay.
template <typename T>
__device__ __forceinline__ int lds_off(int row, int byte) {
  if constexpr (std::is_same<T, bf16>::value)
    return row * 128 + (byte ^ (((row >> 1) & 3) << 5));
  else
    return row * AttnCfg<T>::ROWB + byte;
}

// keep-bit mask layout (the forward's register layout, so the forward and dQ kernels move one
// 16-bit word per lane and key tile): [B*H][KT = ceil(T/64)][4 lane groups g][ldm = roundup(T,64)]
// uint16; bit (kt*4 + r) of word (bh, tile, g, q) = keep(q, key = 64*tile + 16*kt + 4*g + r)
__host__ __device__ inline int64_t mask_ld(int T) { return ((int64_t)T + 63) / 64 * 64; }
__host__ __device__ inline int mask_kt(int T) { return (T + 63) / 64; }

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

// Attention dropout stream (include/rp_api.h, rp_attn_fwd): for query q, key tile `tile` and lane
// group g (keys 64*tile + 16*kt + 4*g + r, kt, r in 0..3) the state st = rp_hash(seed_bh,
// (q*KT + tile)*4 + g) is advanced by xorshift32 eight times; word j covers keys
// (kt = j>>1, r = 2*(j&1) + {0: low half, 1: high half}); a key is kept iff its half, read as a signed
// 16-bit integer, is >= round(p*65536) - 32768 (probability 1 - p, exact to 2^-16).
// Outputs dm[j] (0xFFFF in each dropped half: the AND-NOT mask of the packed bf16 P pair) and
// returns the 16 keep bits, bit (kt*4 + r).  Full-rate VALU only: a saturating packed 16-bit
// subtract + arithmetic shift per pair, no 32-bit multiplies beyond the one seeding hash.
__device__ __forceinline__ uint32_t drop_masks(uint32_t seed_bh, uint32_t q, uint32_t KT, uint32_t tile, uint32_t g,
                                               uint32_t thr, uint32_t dm[8]) {
  uint32_t st = rp_hash(seed_bh, (q * KT + tile) * 4u + g);
  const short ts = (short)((int)thr - 32768);
  const i16x2 t2 = {ts, ts};
  uint32_t acc = 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    st ^= st << 13;
    st ^= st >> 17;
    st ^= st << 5;
    const i16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(i16x2, st), t2);  // < 0 <=> dropped
    const uint32_t m = __builtin_bit_cast(uint32_t, (i16x2)(d >> (short)15));
    dm[j] = m;
    // keep bit of the low half -> bit 4*(j>>1) + 2*(j&1); high half -> 16 + that + 1 (folded below)
    const int b = 4 * (j >> 1) + 2 * (j & 1);
    acc |= ~m & ((1u << b) | (1u << (16 + b + 1)));
  }
  return (acc & 0xFFFFu) | (acc >> 16);
}

// =================================================================================================
// forward
// =================================================================================================
constexpr int FW_QB = NW * 32;  // queries per workgroup
constexpr int FW_KT = 64;       // keys per tile

template <typename T, bool DROP>
__global__ __launch_bounds__(NT, (std::is_same<T, bf16>::value && !DROP) ? 3 : 2) void attn_fwd_kernel(const T* __restrict__ qkv, const uint8_t* __restrict__ kvalid,
                                                        int B, int T_, int H, float scale, uint32_t drop_thresh,
                                                        float drop_scale, uint32_t seed, T* __restrict__ out,
                                                        float* __restrict__ lse, uint16_t* __restrict__ dmask) {
  using C = AttnCfg<T>;
  constexpr int TILE = FW_KT * C::ROWB;
  constexpr int BUF = 2 * TILE + FW_KT * 4 + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int nqb = (T_ + FW_QB - 1) / FW_QB;
  const int L = rp_xcd_remap(blockIdx.x, nqb * B * H);
  const int bh = L / nqb, qb = L % nqb;
  const int b = bh / H, h = bh % H;
  const int64_t ld = 3LL * H * HD;
  const T* seq = qkv + (int64_t)b * T_ * ld;
  const T* Qg = seq + h * HD;
  const T* Kg = seq + (int64_t)H * HD + h * HD;
  const T* Vg = seq + 2LL * H * HD + h * HD;
  const int q0 = qb * FW_QB + w * 32;  // this wave's first query
  const uint32_t seed_bh = rp_hash(seed, (uint32_t)bh);
  const float c = scale * LOG2E;
  const float rth = RESCALE_LOG2 / c;  // deferred-rescale threshold in score units
  const int KT = mask_kt(T_);
  const int64_t ldm = mask_ld(T_);
  uint16_t* mrow = dmask ? dmask + (int64_t)bh * KT * 4 * ldm : nullptr;

  // Q^T operand (B operand of S^T = K Q^T): lane holds Q[q0 + qt*16 + i][dk slots]
  constexpr bool BF = std::is_same<T, bf16>::value;
  bf16x8 qf[2][2];
  float qs[2][16];
  if constexpr (BF) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int s = 0; s < 2; ++s) qf[qt][s] = row_frag_gmem((const bf16*)Qg, ld, q0 + qt * 16, T_, s * 32, lane);
  } else {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      int q = q0 + qt * 16 + i;
#pragma unroll
      for (int s = 0; s < 16; ++s) qs[qt][s] = q < T_ ? (float)Qg[(int64_t)q * ld + 4 * s + g] : 0.f;
    }
  }

  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = zero4();
  float m[2] = {-INFINITY, -INFINITY}, lp[2] = {0.f, 0.f};

  Stage<T, FW_KT> sk, sv;
  const int nkt = (T_ + FW_KT - 1) / FW_KT;
  // key-valid flags of a tile: loaded with the K/V prefetch (wave 0, one byte per lane), staged as
  // an additive bias + a "no masked key" flag at the LDS write
  auto load_valid = [&](int k0) -> bool {
    const int k = k0 + lane;
    return w == 0 && k < T_ && kvalid[(int64_t)b * T_ + k];
  };
  auto stage_mask = [&](char* buf, bool ok) {
    float* kb = reinterpret_cast<float*>(buf + 2 * TILE);
    if (w == 0) {
      kb[lane] = ok ? 0.f : -INFINITY;
      const unsigned long long bal = __ballot(ok);
      if (lane == 0) *reinterpret_cast<int*>(buf + 2 * TILE + FW_KT * 4) = bal == ~0ull;
    }
  };
  sk.load(Kg, ld, 0, T_, tid);
  sv.load(Vg, ld, 0, T_, tid);
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
      sk.load(Kg, ld, k0 + FW_KT, T_, tid);
      sv.load(Vg, ld, k0 + FW_KT, T_, tid);
      kvn = load_valid(k0 + FW_KT);
    }
    const char* Kl = cur;
    const char* Vl = cur + TILE;
    const float* kbias = reinterpret_cast<const float*>(cur + 2 * TILE);
    const bool full = *reinterpret_cast<const int*>(cur + 2 * TILE + FW_KT * 4) != 0;

    // ---- S^T[key][q] = K Q^T ----
    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = zero4();
    if constexpr (BF) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          bf16x8 kf = row_frag_lds(Kl, kt * 16, ss * 32, lane);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) s[kt][qt] = mfma_bf16(kf, qf[qt][ss], s[kt][qt]);
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 16; ++ss) {
          float kf = ldsf(Kl, kt * 16 + i, 4 * ss + g);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) s[kt][qt] = mfma_f32(kf, qs[qt][ss], s[kt][qt]);
        }
    }
    // ---- mask (only tiles with masked keys) + column max ----
    // Deferred rescale: the running reference m only moves when the tile max exceeds it by more
    // than RESCALE_LOG2 (P <= 2^8 meanwhile, exact in fp32/bf16 range); l and O share the
    // reference, so out = O / l is unchanged and the lse uses the same m.
    float mnew[2];
    bool grow = false;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
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
      mx = quad_max(mx);
      mnew[qt] = mx;
      grow |= mx > m[qt] + rth;  // no NaN anywhere: m = -inf -> grows iff mx finite
    }
    if (__any(grow)) {  // wave-uniform branch, per-lane update
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const bool gq = mnew[qt] > m[qt] + rth;
        const float alpha = gq ? rp_exp2((m[qt] - mnew[qt]) * c) : 1.f;  // m = -inf -> 0
        lp[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        m[qt] = gq ? mnew[qt] : m[qt];
      }
    }
    // ---- P = exp2(S*c - m*c); per-lane partial row sums (before dropout), tree order ----
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float mc = (m[qt] == -INFINITY ? 0.f : m[qt]) * c;
      float t4[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kt][qt][r] = rp_exp2(fmaf(s[kt][qt][r], c, -mc));
        t4[kt] = (s[kt][qt][0] + s[kt][qt][1]) + (s[kt][qt][2] + s[kt][qt][3]);
      }
      lp[qt] += (t4[0] + t4[1]) + (t4[2] + t4[3]);
    }
    // ---- dropout: 8 drop masks per (query, tile) from one xorshift stream; keep bits stored ----
    uint32_t dm[2][8];
    if constexpr (DROP) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q = q0 + qt * 16 + i;
        const uint32_t word = drop_masks(seed_bh, (uint32_t)q, (uint32_t)KT, (uint32_t)kt_i, (uint32_t)g, drop_thresh, dm[qt]);
        if (q < T_) mrow[((int64_t)kt_i * 4 + g) * ldm + q] = (uint16_t)word;
      }
    }
    // ---- O^T[dk][q] += V^T P^T ----
    if constexpr (BF) {
      bf16x8 pf[2][2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
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
          for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma_bf16(vf, pf[qt][ks], o[qt][dt]);
        }
    } else {
      if constexpr (DROP) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
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
            for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma_f32(vf, s[kt][qt][r], o[qt][dt]);
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
  const int64_t ldo = (int64_t)H * HD;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float l = quad_sum(lp[qt]);
    const int q = q0 + qt * 16 + i;
    if (q >= T_) continue;
    const float inv = drop_scale / l;
    T* orow = out + ((int64_t)b * T_ + q) * ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) rp_st(orow + dt * 16 + 4 * g + r, o[qt][dt][r] * inv);
    if (g == 0) lse[(int64_t)bh * T_ + q] = m[qt] * scale + logf(l);
  }
}

// =================================================================================================
// backward pre-pass: delta[bh][q] = sum_d dO[q][d] * O[q][d]
// =================================================================================================
template <typename T>
__global__ void attn_delta_kernel(const T* __restrict__ out, const T* __restrict__ dout, int B, int T_, int H,
                                  float* __restrict__ delta) {
  // one wave per (b, t) row of H*64 elements; 8 lanes per head
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * T_) return;
  const int D = H * HD;
  for (int e = lane * 8; e < D; e += 512) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += rp_ld(out + row * D + e + j) * rp_ld(dout + row * D + e + j);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if ((lane & 7) == 0) {
      const int b = (int)(row / T_), t = (int)(row % T_);
      delta[((int64_t)b * H + e / HD) * T_ + t] = s;
    }
  }
}

// =================================================================================================
// backward: dK, dV per 128-key block (4 waves x 32 keys), sweep over 64-query tiles
// =================================================================================================
constexpr int KV_KB = NW * 32;
constexpr int KV_QT = 64;

template <typename T, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_bwd_kv_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                           const float* __restrict__ lse, const float* __restrict__ delta,
                                                           const uint8_t* __restrict__ kvalid, int B, int T_, int H,
                                                           float scale, int use_drop, float drop_scale,
                                                           const uint16_t* __restrict__ dmask, T* __restrict__ dqkv) {
  using C = AttnCfg<T>;
  constexpr bool BF = std::is_same<T, bf16>::value;
  constexpr int TILE = KV_QT * C::ROWB;
  constexpr int MASKB = (KV_KB / 64) * 4 * KV_QT * 2;    // 2 key tiles x 4 groups x 64 queries, u16
  constexpr int BUF = 2 * TILE + 2 * KV_QT * 4 + MASKB;  // Q, dO, lse*log2e, delta, keep bits
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int nkb = (T_ + KV_KB - 1) / KV_KB;
  const int L = rp_xcd_remap(blockIdx.x, nkb * B * H);
  const int bh = L / nkb, kb = L % nkb;
  const int b = bh / H, h = bh % H;
  const int64_t ld = 3LL * H * HD;
  const int64_t ldo = (int64_t)H * HD;
  const T* seq = qkv + (int64_t)b * T_ * ld;
  const T* Qg = seq + h * HD;
  const T* Kg = seq + (int64_t)H * HD + h * HD;
  const T* Vg = seq + 2LL * H * HD + h * HD;
  const T* dOg = dout + (int64_t)b * T_ * ldo + h * HD;
  const float* lse_bh = lse + (int64_t)bh * T_;
  const float* del_bh = delta + (int64_t)bh * T_;
  const int kw0 = kb * KV_KB + w * 32;
  const float c = scale * LOG2E;
  const float inv_ds = DROP ? 1.f / drop_scale : 1.f;
  const int KT = mask_kt(T_);
  const int64_t ldm = mask_ld(T_);

  // K, V as B operands of S = Q K^T and dP = dO V^T: lane holds X[kw0 + kt*16 + i][dk slots]
  bf16x8 kf[2][2], vf[2][2];
  float ks_[2][16], vs_[2][16];
  if constexpr (BF) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        kf[kt][s] = row_frag_gmem((const bf16*)Kg, ld, kw0 + kt * 16, T_, s * 32, lane);
        vf[kt][s] = row_frag_gmem((const bf16*)Vg, ld, kw0 + kt * 16, T_, s * 32, lane);
      }
  } else {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int k = kw0 + kt * 16 + i;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        ks_[kt][s] = k < T_ ? (float)Kg[(int64_t)k * ld + 4 * s + g] : 0.f;
        vs_[kt][s] = k < T_ ? (float)Vg[(int64_t)k * ld + 4 * s + g] : 0.f;
      }
    }
  }

  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kt][dt] = dv[kt][dt] = zero4();

  Stage<T, KV_QT> sq, sdo;
  uint4 mreg = make_uint4(0u, 0u, 0u, 0u);
  // keep-bit words of this workgroup's 2 key tiles x 4 groups x 64 queries: thread t < 64 moves
  // 16 bytes (row = tile*4 + g, 8 queries)
  auto load_mask = [&](int qs0) {
    if (DROP && tid < 64) {
      const int r = tid >> 3, cch = tid & 7;
      const int tile = kb * (KV_KB / 64) + (r >> 2);
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
      lse_r = q < T_ ? lse_bh[q] * LOG2E : INFINITY;  // +inf -> P = 0 for padded rows
      del_r = q < T_ ? -del_bh[q] * inv_ds : 0.f;     // -delta/ds: the dP accumulators' start
    }
  };
  auto stage_rows = [&](char* buf) {
    float* lb = reinterpret_cast<float*>(buf + 2 * TILE);
    if (tid < KV_QT) {
      lb[tid] = lse_r;
      lb[KV_QT + tid] = del_r;
    }
    if (DROP && tid < 64) *reinterpret_cast<uint4*>(buf + 2 * TILE + 2 * KV_QT * 4 + tid * 16) = mreg;
  };
  const int nqt = (T_ + KV_QT - 1) / KV_QT;
  sq.load(Qg, ld, 0, T_, tid);
  sdo.load(dOg, ldo, 0, T_, tid);
  load_mask(0);
  load_rows(0);
  sq.store(lds, tid);
  sdo.store(lds + TILE, tid);
  stage_rows(lds);
  __syncthreads();

  for (int it = 0; it < nqt; ++it) {
    char* cur = lds + (it & 1) * BUF;
    char* nxt = lds + ((it + 1) & 1) * BUF;
    const bool more = it + 1 < nqt;
    const int qs0 = it * KV_QT;
    if (more) {
      sq.load(Qg, ld, qs0 + KV_QT, T_, tid);
      sdo.load(dOg, ldo, qs0 + KV_QT, T_, tid);
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
      f32x4 s[2][2], dp[2][2], ndq[2];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        ndq[qq] = *reinterpret_cast<const f32x4*>(drow + (2 * hf + qq) * 16 + 4 * g);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[qq][kt] = zero4();
          dp[qq][kt] = ndq[qq];
        }
      }
      if constexpr (BF) {
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            bf16x8 qa = row_frag_lds(Ql, (2 * hf + qq) * 16, ss * 32, lane);
            bf16x8 da = row_frag_lds(dOl, (2 * hf + qq) * 16, ss * 32, lane);
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
              s[qq][kt] = mfma_bf16(qa, kf[kt][ss], s[qq][kt]);
              dp[qq][kt] = mfma_bf16(da, vf[kt][ss], dp[qq][kt]);
            }
          }
      } else {
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int ss = 0; ss < 16; ++ss) {
            float qa = ldsf(Ql, (2 * hf + qq) * 16 + i, 4 * ss + g);
            float da = ldsf(dOl, (2 * hf + qq) * 16 + i, 4 * ss + g);
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
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
        const float4 lq4 = *reinterpret_cast<const float4*>(lrow + qrow);
        const float lq[4] = {lq4.x, lq4.y, lq4.z, lq4.w};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          // this lane's key: ko = key % 64 -> word row (tile half, group (ko%16)/4), bit (ko/16)*4 + ko%4
          const int ko = (w * 32 + kt * 16 + i) & 63;
          const int mrow_l = ((w * 32 + kt * 16) >> 6) * 4 + ((ko & 15) >> 2);
          const int bit = (ko >> 4) * 4 + (ko & 3);
          uint2 bits = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
          if constexpr (DROP) bits = *reinterpret_cast<const uint2*>(mw + mrow_l * KV_QT + qrow);
          const uint32_t wd[4] = {bits.x & 0xFFFFu, bits.x >> 16, bits.y & 0xFFFFu, bits.y >> 16};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = rp_exp2(fmaf(s[qq][kt][r], c, -lq[r]));
            if constexpr (DROP) {  // dS = p*(keep*ds*dP - delta) = p*ds*(keep ? acc : -delta/ds)
              const bool keep = (wd[r] >> bit) & 1u;
              const float pds = p * drop_scale;
              s[qq][kt][r] = keep ? pds : 0.f;
              dp[qq][kt][r] = pds * (keep ? dp[qq][kt][r] : ndq[qq][r]);
            } else {
              s[qq][kt][r] = p;
              dp[qq][kt][r] = p * dp[qq][kt][r];
            }
          }
        }
      }
      // dV[key][dk] += P_d^T dO ; dK[key][dk] += dS^T Q     (key on the row, k = query slots)
      if constexpr (BF) {
        bf16x8 pa[2], sa[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          pa[kt] = pack8(s[0][kt], s[1][kt]);
          sa[kt] = pack8(dp[0][kt], dp[1][kt]);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const bf16x8 dob = col_frag_lds(dOl, hf * 32, dt * 16, lane);
          const bf16x8 qb = col_frag_lds(Ql, hf * 32, dt * 16, lane);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
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
              for (int kt = 0; kt < 2; ++kt) {
                dv[kt][dt] = mfma_f32(s[qq][kt][r], dob, dv[kt][dt]);
                dk[kt][dt] = mfma_f32(dp[qq][kt][r], qb, dk[kt][dt]);
              }
            }
      }
    }
    if (more) {
      sq.store(nxt, tid);
      sdo.store(nxt + TILE, tid);
      stage_rows(nxt);
    }
    __syncthreads();
  }
  // store: dk[kt][dt][r] = dK[key = kw0 + kt*16 + 4g + r][dk = dt*16 + i]; masked keys -> 0
  T* dK = dqkv + (int64_t)b * T_ * ld + (int64_t)H * HD + h * HD;
  T* dV = dqkv + (int64_t)b * T_ * ld + 2LL * H * HD + h * HD;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kw0 + kt * 16 + 4 * g + r;
      if (key >= T_) continue;
      const bool ok = kvalid[(int64_t)b * T_ + key] != 0;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        rp_st(dK + (int64_t)key * ld + dt * 16 + i, ok ? dk[kt][dt][r] * scale : 0.f);
        rp_st(dV + (int64_t)key * ld + dt * 16 + i, ok ? dv[kt][dt][r] : 0.f);
      }
    }
}

// =================================================================================================
// backward: dQ per 128-query block (4 waves x 32 queries), sweep over 64-key tiles
// =================================================================================================
template <typename T, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_bwd_q_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                          const float* __restrict__ lse, const float* __restrict__ delta,
                                                          const uint8_t* __restrict__ kvalid, int B, int T_, int H,
                                                          float scale, int use_drop, float drop_scale,
                                                          const uint16_t* __restrict__ dmask, T* __restrict__ dqkv) {
  using C = AttnCfg<T>;
  constexpr bool BF = std::is_same<T, bf16>::value;
  constexpr int TILE = FW_KT * C::ROWB;
  constexpr int BUF = 2 * TILE + FW_KT * 4 + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int nqb = (T_ + FW_QB - 1) / FW_QB;
  const int L = rp_xcd_remap(blockIdx.x, nqb * B * H);
  const int bh = L / nqb, qb = L % nqb;
  const int b = bh / H, h = bh % H;
  const int64_t ld = 3LL * H * HD;
  const int64_t ldo = (int64_t)H * HD;
  const T* seq = qkv + (int64_t)b * T_ * ld;
  const T* Qg = seq + h * HD;
  const T* Kg = seq + (int64_t)H * HD + h * HD;
  const T* Vg = seq + 2LL * H * HD + h * HD;
  const T* dOg = dout + (int64_t)b * T_ * ldo + h * HD;
  const int q0 = qb * FW_QB + w * 32;
  const float c = scale * LOG2E;
  const int KT = mask_kt(T_);
  const int64_t ldm = mask_ld(T_);
  const uint16_t* mrow = dmask ? dmask + (int64_t)bh * KT * 4 * ldm : nullptr;

  bf16x8 qf[2][2], df[2][2];
  float qs[2][16], dsv[2][16];
  float lq[2], dq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + qt * 16 + i;
    lq[qt] = q < T_ ? lse[(int64_t)bh * T_ + q] * LOG2E : INFINITY;
    dq[qt] = q < T_ ? -delta[(int64_t)bh * T_ + q] * (DROP ? 1.f / drop_scale : 1.f) : 0.f;  // -delta/ds
    if constexpr (BF) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        qf[qt][s] = row_frag_gmem((const bf16*)Qg, ld, q0 + qt * 16, T_, s * 32, lane);
        df[qt][s] = row_frag_gmem((const bf16*)dOg, ldo, q0 + qt * 16, T_, s * 32, lane);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        qs[qt][s] = q < T_ ? (float)Qg[(int64_t)q * ld + 4 * s + g] : 0.f;
        dsv[qt][s] = q < T_ ? (float)dOg[(int64_t)q * ldo + 4 * s + g] : 0.f;
      }
    }
  }

  f32x4 dqa[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dqa[qt][dt] = zero4();

  Stage<T, FW_KT> sk, sv;
  auto load_valid = [&](int k0) -> bool {
    const int k = k0 + lane;
    return w == 0 && k < T_ && kvalid[(int64_t)b * T_ + k];
  };
  auto stage_mask = [&](char* buf, bool ok) {
    float* kbm = reinterpret_cast<float*>(buf + 2 * TILE);
    if (w == 0) kbm[lane] = ok ? 0.f : -INFINITY;  // key bias: the S^T accumulators' start
  };
  const int nkt = (T_ + FW_KT - 1) / FW_KT;
  sk.load(Kg, ld, 0, T_, tid);
  sv.load(Vg, ld, 0, T_, tid);
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
    uint32_t kwd[2] = {0u, 0u};
    if constexpr (DROP) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q = q0 + qt * 16 + i;
        kwd[qt] = q < T_ ? (uint32_t)mrow[((int64_t)it * 4 + g) * ldm + q] : 0u;
      }
    }
    if (more) {
      sk.load(Kg, ld, k0 + FW_KT, T_, tid);
      sv.load(Vg, ld, k0 + FW_KT, T_, tid);
      kvn = load_valid(k0 + FW_KT);
    }
    const char* Kl = cur;
    const char* Vl = cur + TILE;
    const float* kbias = reinterpret_cast<const float*>(cur + 2 * TILE);

    // S^T[key][q] = K Q^T, dP^T[key][q] = V dO^T : row key = kt*16 + 4g + r, col q = qt*16 + i.
    // Row constants as the initial accumulators: S^T starts at the key bias (0 / -inf: masked keys
    // give P = 0 with no select), dP^T at -delta/ds.
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const f32x4 kb4 = *reinterpret_cast<const f32x4*>(kbias + kt * 16 + 4 * g);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        s[kt][qt] = kb4;
        dp[kt][qt] = f32x4{dq[qt], dq[qt], dq[qt], dq[qt]};
      }
    }
    if constexpr (BF) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          bf16x8 ka = row_frag_lds(Kl, kt * 16, ss * 32, lane);
          bf16x8 va = row_frag_lds(Vl, kt * 16, ss * 32, lane);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) {
            s[kt][qt] = mfma_bf16(ka, qf[qt][ss], s[kt][qt]);
            dp[kt][qt] = mfma_bf16(va, df[qt][ss], dp[kt][qt]);
          }
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ss = 0; ss < 16; ++ss) {
          float ka = ldsf(Kl, kt * 16 + i, 4 * ss + g);
          float va = ldsf(Vl, kt * 16 + i, 4 * ss + g);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) {
            s[kt][qt] = mfma_f32(ka, qs[qt][ss], s[kt][qt]);
            dp[kt][qt] = mfma_f32(va, dsv[qt][ss], dp[kt][qt]);
          }
        }
    }
    // dS^T = P^T (keep*ds*dP^T - delta) = P^T*ds*(keep ? acc : -delta/ds)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = rp_exp2(fmaf(s[kt][qt][r], c, -lq[qt]));
          if constexpr (DROP) {
            const bool keep = (kwd[qt] >> (4 * kt + r)) & 1u;
            s[kt][qt][r] = (p * drop_scale) * (keep ? dp[kt][qt][r] : dq[qt]);
          } else {
            s[kt][qt][r] = p * dp[kt][qt][r];
          }
        }
    }
    // dQ[q][dk] += dS K : A = dS (q on row = lane i, key slots), B = K columns (tr read)
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 sa[2];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) sa[qt] = pack8(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          bf16x8 kb = col_frag_lds(Kl, ks * 32, dt * 16, lane);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) dqa[qt][dt] = mfma_bf16(sa[qt], kb, dqa[qt][dt]);
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
            for (int qt = 0; qt < 2; ++qt) dqa[qt][dt] = mfma_f32(s[kt][qt][r], kb, dqa[qt][dt]);
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
  T* dQ = dqkv + (int64_t)b * T_ * ld + h * HD;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + qt * 16 + 4 * g + r;
      if (q >= T_) continue;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) rp_st(dQ + (int64_t)q * ld + dt * 16 + i, dqa[qt][dt][r] * scale);
    }
}

template <typename T>
int launch_fwd(const void* qkv, const uint8_t* kv, int B, int T_, int H, float scale, float p, uint32_t seed,
               void* out, float* lse, uint16_t* dmask, hipStream_t s) {
  const int nqb = (T_ + FW_QB - 1) / FW_QB;
  const uint32_t thr = rp_dropout_thresh(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (thr)
    hipLaunchKernelGGL((attn_fwd_kernel<T, true>), dim3((unsigned)(nqb * B * H)), dim3(NT), 0, s, (const T*)qkv, kv, B,
                       T_, H, scale, thr, ds, seed, (T*)out, lse, dmask);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<T, false>), dim3((unsigned)(nqb * B * H)), dim3(NT), 0, s, (const T*)qkv, kv, B,
                       T_, H, scale, thr, ds, seed, (T*)out, lse, nullptr);
  return rp_check_launch("rp_attn_fwd");
}

// phases: bit 0 = delta pre-pass, bit 1 = dK/dV kernel, bit 2 = dQ kernel
template <typename T>
int launch_bwd(int phases, const void* qkv, const void* out, const void* dout, const float* lse, const uint8_t* kv,
               int B, int T_, int H, float scale, float p, const uint16_t* dmask, void* dqkv, float* delta,
               hipStream_t s) {
  const int use = rp_dropout_thresh(p) != 0;
  const float dsc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int64_t rows = (int64_t)B * T_;
  if (phases & 1)
    hipLaunchKernelGGL(attn_delta_kernel<T>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, (const T*)out,
                       (const T*)dout, B, T_, H, delta);
  const int nkb = (T_ + KV_KB - 1) / KV_KB;
  const int nqb = (T_ + FW_QB - 1) / FW_QB;
  if (phases & 2) {
    if (use)
      hipLaunchKernelGGL((attn_bwd_kv_kernel<T, true>), dim3((unsigned)(nkb * B * H)), dim3(NT), 0, s, (const T*)qkv,
                         (const T*)dout, lse, delta, kv, B, T_, H, scale, use, dsc, dmask, (T*)dqkv);
    else
      hipLaunchKernelGGL((attn_bwd_kv_kernel<T, false>), dim3((unsigned)(nkb * B * H)), dim3(NT), 0, s, (const T*)qkv,
                         (const T*)dout, lse, delta, kv, B, T_, H, scale, use, dsc, dmask, (T*)dqkv);
  }
  if (phases & 4) {
    if (use)
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, true>), dim3((unsigned)(nqb * B * H)), dim3(NT), 0, s, (const T*)qkv,
                         (const T*)dout, lse, delta, kv, B, T_, H, scale, use, dsc, dmask, (T*)dqkv);
    else
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, false>), dim3((unsigned)(nqb * B * H)), dim3(NT), 0, s, (const T*)qkv,
                         (const T*)dout, lse, delta, kv, B, T_, H, scale, use, dsc, dmask, (T*)dqkv);
  }
  return rp_check_launch("rp_attn_bwd");
}

int attn_bwd_entry(int phases, int dtype, const void* qkv, const void* out, const void* dout, const float* lse,
                   const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                   const uint16_t* dropmask, void* dqkv, float* delta_ws, void* stream) {
  RP_REQUIRE(dk == HD, "rp_attn_bwd: head dim %d unsupported (64)", dk);
  RP_REQUIRE(B >= 0 && T >= 0 && H > 0, "rp_attn_bwd: bad shape");
  if (B == 0 || T == 0) return RP_OK;
  RP_REQUIRE(qkv && dout && lse && key_valid && dqkv && delta_ws && (out || !(phases & 1)), "rp_attn_bwd: null pointer");
  RP_REQUIRE(rp_aligned16(qkv) && rp_aligned16(dout) && rp_aligned16(dqkv), "rp_attn_bwd: 16-byte alignment required");
  RP_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "rp_attn_bwd: dropout_p out of range");
  RP_REQUIRE(rp_dropout_thresh(dropout_p) == 0 || (dropmask && rp_aligned16(dropmask)),
             "rp_attn_bwd: dropout needs the forward's dropmask");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RP_BF16)
    return launch_bwd<bf16>(phases, qkv, out, dout, lse, key_valid, B, T, H, scale, dropout_p, dropmask, dqkv,
                            delta_ws, s);
  if (dtype == RP_F32)
    return launch_bwd<float>(phases, qkv, out, dout, lse, key_valid, B, T, H, scale, dropout_p, dropmask, dqkv,
                             delta_ws, s);
  rp_set_error("rp_attn_bwd: bad dtype");
  return RP_ERR_ARG;
}

}  // namespace

extern "C" int64_t rp_attn_dropmask_elems(int B, int T, int H) {
  if (B <= 0 || T <= 0 || H <= 0) return 0;
  return (int64_t)B * H * mask_kt(T) * 4 * mask_ld(T);
}

extern "C" int rp_attn_fwd(int dtype, const void* qkv, const uint8_t* key_valid, int B, int T, int H, int dk, float scale,
                           float dropout_p, uint32_t seed, void* out, float* lse, uint16_t* dropmask, void* stream) {
  RP_REQUIRE(dk == HD, "rp_attn_fwd: head dim %d unsupported (64)", dk);
  RP_REQUIRE(B >= 0 && T >= 0 && H > 0, "rp_attn_fwd: bad shape");
  if (B == 0 || T == 0) return RP_OK;
  RP_REQUIRE(qkv && key_valid && out && lse, "rp_attn_fwd: null pointer");
  RP_REQUIRE(rp_aligned16(qkv) && rp_aligned16(out), "rp_attn_fwd: 16-byte alignment required");
  RP_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "rp_attn_fwd: dropout_p out of range");
  RP_REQUIRE((int64_t)T * T < (int64_t)UINT32_MAX, "rp_attn_fwd: T too large");
  RP_REQUIRE(rp_dropout_thresh(dropout_p) == 0 || (dropmask && rp_aligned16(dropmask)),
             "rp_attn_fwd: dropout needs a 16-byte aligned dropmask buffer (rp_attn_dropmask_elems)");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RP_BF16) return launch_fwd<bf16>(qkv, key_valid, B, T, H, scale, dropout_p, seed, out, lse, dropmask, s);
  if (dtype == RP_F32) return launch_fwd<float>(qkv, key_valid, B, T, H, scale, dropout_p, seed, out, lse, dropmask, s);
  rp_set_error("rp_attn_fwd: bad dtype");
  return RP_ERR_ARG;
}

extern "C" int rp_attn_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse,
                           const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                           const uint16_t* dropmask, void* dqkv, float* delta_ws, void* stream) {
  return attn_bwd_entry(7, dtype, qkv, out, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask, dqkv,
                        delta_ws, stream);
}

extern "C" int rp_attn_bwd_delta(int dtype, const void* out, const void* dout, int B, int T, int H, int dk,
                                 float* delta_ws, void* stream) {
  RP_REQUIRE(dk == HD, "rp_attn_bwd_delta: head dim %d unsupported (64)", dk);
  RP_REQUIRE(B >= 0 && T >= 0 && H > 0, "rp_attn_bwd_delta: bad shape");
  if (B == 0 || T == 0) return RP_OK;
  RP_REQUIRE(out && dout && delta_ws, "rp_attn_bwd_delta: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * T;
  if (dtype == RP_BF16)
    hipLaunchKernelGGL(attn_delta_kernel<bf16>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, (const bf16*)out,
                       (const bf16*)dout, B, T, H, delta_ws);
  else if (dtype == RP_F32)
    hipLaunchKernelGGL(attn_delta_kernel<float>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, (const float*)out,
                       (const float*)dout, B, T, H, delta_ws);
  else {
    rp_set_error("rp_attn_bwd_delta: bad dtype");
    return RP_ERR_ARG;
  }
  return rp_check_launch("rp_attn_bwd_delta");
}

extern "C" int rp_attn_bwd_dkdv(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                                const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                                const uint16_t* dropmask, void* dqkv, void* stream) {
  return attn_bwd_entry(2, dtype, qkv, nullptr, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask, dqkv,
                        (float*)delta_ws, stream);
}

extern "C" int rp_attn_bwd_dq(int dtype, const void* qkv, const void* dout, const float* lse, const float* delta_ws,
                              const uint8_t* key_valid, int B, int T, int H, int dk, float scale, float dropout_p,
                              const uint16_t* dropmask, void* dqkv, void* stream) {
  return attn_bwd_entry(4, dtype, qkv, nullptr, dout, lse, key_valid, B, T, H, dk, scale, dropout_p, dropmask, dqkv,
                        (float*)delta_ws, stream);
}
