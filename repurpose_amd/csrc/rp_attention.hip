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

template <typename T>
struct AttnCfg {
  static constexpr int ROWB = HD * (int)sizeof(T) + 16;  // padded LDS row (bytes)
  static constexpr int CPR = HD * (int)sizeof(T) / 16;   // 16-byte chunks per row
};

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
      *reinterpret_cast<uint4*>(lds + row * AttnCfg<T>::ROWB + c * 16) = r[i];
    }
  }
};

// ----- fragment helpers -------------------------------------------------------------------------
// bf16 row fragment: lane holds X[r0 + (l&15)][k0 + 8*(l>>4) + j]   (MFMA 16x16x32 A/B operand)
__device__ __forceinline__ bf16x8 row_frag_lds(const char* lds, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + (r0 + (lane & 15)) * AttnCfg<bf16>::ROWB + (k0 + 8 * (lane >> 4)) * 2);
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
  const char* p0 = lds + (R + 4 * g + q) * AttnCfg<bf16>::ROWB + (c0 + 4 * p) * 2;
  const char* p1 = p0 + 16 * AttnCfg<bf16>::ROWB;
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

// keep bits of 4 consecutive keys kb..kb+3 (kb even) of query q: one hash per key pair
// (element (q, k): 16-bit half (k & 1) of rp_hash(seed_bh, q*T + (k & ~1)))
__device__ __forceinline__ uint32_t keep_nibble(uint32_t seed_bh, uint32_t q, uint32_t T_, uint32_t kb,
                                                uint32_t thr) {
  const uint32_t h0 = rp_hash(seed_bh, q * T_ + kb);
  const uint32_t h1 = rp_hash(seed_bh, q * T_ + kb + 2);
  return ((h0 & 0xFFFFu) >= thr ? 1u : 0u) | ((h0 >> 16) >= thr ? 2u : 0u) | ((h1 & 0xFFFFu) >= thr ? 4u : 0u) |
         ((h1 >> 16) >= thr ? 8u : 0u);
}

// =================================================================================================
// forward
// =================================================================================================
constexpr int FW_QB = NW * 32;  // queries per workgroup
constexpr int FW_KT = 64;       // keys per tile

template <typename T>
__global__ __launch_bounds__(NT, 2) void attn_fwd_kernel(const T* __restrict__ qkv, const uint8_t* __restrict__ kvalid,
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
  auto stage_mask = [&](char* buf, int k0) {
    float* kb = reinterpret_cast<float*>(buf + 2 * TILE);
    if (tid < FW_KT) {  // exactly wave 0
      const int k = k0 + tid;
      const bool ok = k < T_ && kvalid[(int64_t)b * T_ + k];
      kb[tid] = ok ? 0.f : -INFINITY;
      const unsigned long long bal = __ballot(ok);
      if (tid == 0) *reinterpret_cast<int*>(buf + 2 * TILE + FW_KT * 4) = bal == ~0ull;
    }
  };
  sk.load(Kg, ld, 0, T_, tid);
  sv.load(Vg, ld, 0, T_, tid);
  sk.store(lds, tid);
  sv.store(lds + TILE, tid);
  stage_mask(lds, 0);
  __syncthreads();

  for (int kt_i = 0; kt_i < nkt; ++kt_i) {
    char* cur = lds + (kt_i & 1) * BUF;
    char* nxt = lds + ((kt_i + 1) & 1) * BUF;
    const bool more = kt_i + 1 < nkt;
    const int k0 = kt_i * FW_KT;
    if (more) {
      sk.load(Kg, ld, k0 + FW_KT, T_, tid);
      sv.load(Vg, ld, k0 + FW_KT, T_, tid);
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
      float mx = s[0][qt][0];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      mnew[qt] = fmaxf(m[qt], mx);
      grow |= mnew[qt] > m[qt];
    }
    if (__any(grow)) {  // rescale only when some row max grew (wave-uniform branch)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const float mref = mnew[qt] == -INFINITY ? 0.f : mnew[qt];
        const float alpha = exp2f((m[qt] - mref) * c);  // m = -inf -> 0
        lp[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        m[qt] = mnew[qt];
      }
    }
    // ---- P = exp2(S*c - m*c); per-lane partial row sums; dropout bits ----
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float mc = (m[qt] == -INFINITY ? 0.f : m[qt]) * c;
      const int q = q0 + qt * 16 + i;
      uint32_t word = 0;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(fmaf(s[kt][qt][r], c, -mc));
          lp[qt] += p;
          s[kt][qt][r] = p;
        }
        if (drop_thresh) {
          const uint32_t nib =
              keep_nibble(seed_bh, (uint32_t)q, (uint32_t)T_, (uint32_t)(k0 + kt * 16 + 4 * g), drop_thresh);
#pragma unroll
          for (int r = 0; r < 4; ++r) s[kt][qt][r] = ((nib >> r) & 1u) ? s[kt][qt][r] : 0.f;
          word |= nib << (4 * kt);
        }
      }
      if (drop_thresh && q < T_) mrow[((int64_t)kt_i * 4 + g) * ldm + q] = (uint16_t)word;
    }
    // ---- O^T[dk][q] += V^T P^T ----
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 pf[2];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) pf[qt] = pack8(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          bf16x8 vf = col_frag_lds(Vl, ks * 32, dt * 16, lane);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma_bf16(vf, pf[qt], o[qt][dt]);
        }
      }
    } else {
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
      stage_mask(nxt, k0 + FW_KT);
    }
    __syncthreads();
  }

  // ---- epilogue: O[q][dk] = O^T / l ; lse ----
  const int64_t ldo = (int64_t)H * HD;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = lp[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
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

template <typename T>
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
  bool kok[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int k = kw0 + kt * 16 + i;
    kok[kt] = k < T_ && kvalid[(int64_t)b * T_ + k];
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
    if (use_drop && tid < 64) {
      const int r = tid >> 3, cch = tid & 7;
      const int tile = kb * (KV_KB / 64) + (r >> 2);
      if (tile < KT)
        mreg = *reinterpret_cast<const uint4*>(dmask + (((int64_t)bh * KT + tile) * 4 + (r & 3)) * ldm + qs0 + cch * 8);
      else
        mreg = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto stage_rows = [&](char* buf, int qs0) {
    float* lb = reinterpret_cast<float*>(buf + 2 * TILE);
    if (tid < KV_QT) {
      int q = qs0 + tid;
      lb[tid] = q < T_ ? lse_bh[q] * LOG2E : INFINITY;  // +inf -> P = 0 for padded rows
      lb[KV_QT + tid] = q < T_ ? del_bh[q] : 0.f;
    }
    if (use_drop && tid < 64) *reinterpret_cast<uint4*>(buf + 2 * TILE + 2 * KV_QT * 4 + tid * 16) = mreg;
  };
  const int nqt = (T_ + KV_QT - 1) / KV_QT;
  sq.load(Qg, ld, 0, T_, tid);
  sdo.load(dOg, ldo, 0, T_, tid);
  load_mask(0);
  sq.store(lds, tid);
  sdo.store(lds + TILE, tid);
  stage_rows(lds, 0);
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
      f32x4 s[2][2], dp[2][2];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) s[qq][kt] = dp[qq][kt] = zero4();
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
      // P (dropped, for dV) -> s ; dS (for dK) -> dp
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int qrow = (2 * hf + qq) * 16 + 4 * g;
        const float4 lq4 = *reinterpret_cast<const float4*>(lrow + qrow);
        const float4 dq4 = *reinterpret_cast<const float4*>(drow + qrow);
        const float lq[4] = {lq4.x, lq4.y, lq4.z, lq4.w};
        const float dq[4] = {dq4.x, dq4.y, dq4.z, dq4.w};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          // this lane's key: ko = key % 64 -> word row (tile half, group (ko%16)/4), bit (ko/16)*4 + ko%4
          const int ko = (w * 32 + kt * 16 + i) & 63;
          const int mrow_l = ((w * 32 + kt * 16) >> 6) * 4 + ((ko & 15) >> 2);
          const int bit = (ko >> 4) * 4 + (ko & 3);
          uint2 bits = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
          if (use_drop) bits = *reinterpret_cast<const uint2*>(mw + mrow_l * KV_QT + qrow);
          const uint32_t wd[4] = {bits.x & 0xFFFFu, bits.x >> 16, bits.y & 0xFFFFu, bits.y >> 16};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = kok[kt] ? exp2f(fmaf(s[qq][kt][r], c, -lq[r])) : 0.f;
            float gp = dp[qq][kt][r];
            float pd = p;
            if (use_drop) {
              const bool keep = (wd[r] >> bit) & 1u;
              pd = keep ? p * drop_scale : 0.f;
              gp = keep ? gp * drop_scale : 0.f;
            }
            s[qq][kt][r] = pd;
            dp[qq][kt][r] = p * (gp - dq[r]);
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
      stage_rows(nxt, qs0 + KV_QT);
    }
    __syncthreads();
  }
  // store: dk[kt][dt][r] = dK[key = kw0 + kt*16 + 4g + r][dk = dt*16 + i]
  T* dK = dqkv + (int64_t)b * T_ * ld + (int64_t)H * HD + h * HD;
  T* dV = dqkv + (int64_t)b * T_ * ld + 2LL * H * HD + h * HD;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kw0 + kt * 16 + 4 * g + r;
      if (key >= T_) continue;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        rp_st(dK + (int64_t)key * ld + dt * 16 + i, dk[kt][dt][r] * scale);
        rp_st(dV + (int64_t)key * ld + dt * 16 + i, dv[kt][dt][r]);
      }
    }
}

// =================================================================================================
// backward: dQ per 128-query block (4 waves x 32 queries), sweep over 64-key tiles
// =================================================================================================
template <typename T>
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
    dq[qt] = q < T_ ? delta[(int64_t)bh * T_ + q] : 0.f;
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
  auto stage_mask = [&](char* buf, int k0) {
    float* kbm = reinterpret_cast<float*>(buf + 2 * TILE);
    if (tid < FW_KT) {
      int k = k0 + tid;
      kbm[tid] = (k < T_ && kvalid[(int64_t)b * T_ + k]) ? 1.f : 0.f;
    }
  };
  const int nkt = (T_ + FW_KT - 1) / FW_KT;
  sk.load(Kg, ld, 0, T_, tid);
  sv.load(Vg, ld, 0, T_, tid);
  sk.store(lds, tid);
  sv.store(lds + TILE, tid);
  stage_mask(lds, 0);
  __syncthreads();

  for (int it = 0; it < nkt; ++it) {
    char* cur = lds + (it & 1) * BUF;
    char* nxt = lds + ((it + 1) & 1) * BUF;
    const bool more = it + 1 < nkt;
    const int k0 = it * FW_KT;
    // keep-bit word of this lane's queries for the tile (same register layout as the forward)
    uint32_t kwd[2] = {0u, 0u};
    if (use_drop) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q = q0 + qt * 16 + i;
        kwd[qt] = q < T_ ? (uint32_t)mrow[((int64_t)it * 4 + g) * ldm + q] : 0u;
      }
    }
    if (more) {
      sk.load(Kg, ld, k0 + FW_KT, T_, tid);
      sv.load(Vg, ld, k0 + FW_KT, T_, tid);
    }
    const char* Kl = cur;
    const char* Vl = cur + TILE;
    const float* kok = reinterpret_cast<const float*>(cur + 2 * TILE);

    // S^T[key][q] = K Q^T, dP^T[key][q] = V dO^T : row key = kt*16 + 4g + r, col q = qt*16 + i
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = dp[kt][qt] = zero4();
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
    // dS^T = P^T (gP^T - delta)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const float4 ok4 = *reinterpret_cast<const float4*>(kok + kt * 16 + 4 * g);
      const float okr[4] = {ok4.x, ok4.y, ok4.z, ok4.w};
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = okr[r] != 0.f ? exp2f(fmaf(s[kt][qt][r], c, -lq[qt])) : 0.f;
          float gp = dp[kt][qt][r];
          if (use_drop) gp = ((kwd[qt] >> (4 * kt + r)) & 1u) ? gp * drop_scale : 0.f;
          s[kt][qt][r] = p * (gp - dq[qt]);
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
      stage_mask(nxt, k0 + FW_KT);
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
  hipLaunchKernelGGL(attn_fwd_kernel<T>, dim3((unsigned)(nqb * B * H)), dim3(NT), 0, s, (const T*)qkv, kv, B, T_, H,
                     scale, thr, ds, seed, (T*)out, lse, thr ? dmask : nullptr);
  return rp_check_launch("rp_attn_fwd");
}

template <typename T>
int launch_bwd(const void* qkv, const void* out, const void* dout, const float* lse, const uint8_t* kv, int B, int T_,
               int H, float scale, float p, const uint16_t* dmask, void* dqkv, float* delta, hipStream_t s) {
  const int use = rp_dropout_thresh(p) != 0;
  const float dsc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int64_t rows = (int64_t)B * T_;
  hipLaunchKernelGGL(attn_delta_kernel<T>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, (const T*)out,
                     (const T*)dout, B, T_, H, delta);
  const int nkb = (T_ + KV_KB - 1) / KV_KB;
  hipLaunchKernelGGL(attn_bwd_kv_kernel<T>, dim3((unsigned)(nkb * B * H)), dim3(NT), 0, s, (const T*)qkv,
                     (const T*)dout, lse, delta, kv, B, T_, H, scale, use, dsc, dmask, (T*)dqkv);
  const int nqb = (T_ + FW_QB - 1) / FW_QB;
  hipLaunchKernelGGL(attn_bwd_q_kernel<T>, dim3((unsigned)(nqb * B * H)), dim3(NT), 0, s, (const T*)qkv,
                     (const T*)dout, lse, delta, kv, B, T_, H, scale, use, dsc, dmask, (T*)dqkv);
  return rp_check_launch("rp_attn_bwd");
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
  RP_REQUIRE(dk == HD, "rp_attn_bwd: head dim %d unsupported (64)", dk);
  RP_REQUIRE(B >= 0 && T >= 0 && H > 0, "rp_attn_bwd: bad shape");
  if (B == 0 || T == 0) return RP_OK;
  RP_REQUIRE(qkv && out && dout && lse && key_valid && dqkv && delta_ws, "rp_attn_bwd: null pointer");
  RP_REQUIRE(rp_aligned16(qkv) && rp_aligned16(dout) && rp_aligned16(dqkv), "rp_attn_bwd: 16-byte alignment required");
  RP_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "rp_attn_bwd: dropout_p out of range");
  RP_REQUIRE(rp_dropout_thresh(dropout_p) == 0 || (dropmask && rp_aligned16(dropmask)),
             "rp_attn_bwd: dropout needs the forward's dropmask");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RP_BF16)
    return launch_bwd<bf16>(qkv, out, dout, lse, key_valid, B, T, H, scale, dropout_p, dropmask, dqkv, delta_ws, s);
  if (dtype == RP_F32)
    return launch_bwd<float>(qkv, out, dout, lse, key_valid, B, T, H, scale, dropout_p, dropmask, dqkv, delta_ws, s);
  rp_set_error("rp_attn_bwd: bad dtype");
  return RP_ERR_ARG;
}
