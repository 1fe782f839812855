// rp_gemm — MFMA GEMM with fused epilogues for every nn.Linear on the Repurpose hot path
// (input projection, MHA in/out projections, FFN linear1/linear2, feature_map, head hidden
// layers; reference models/MMCTransformer.py:32-93 and the stock encoder layer built at :41-55).
//
// One kernel template serves the three shapes autograd needs for y = x W^T:
//   forward  C = X  . W^T      A k-major (X [M,K]),    B k-major (W [N,K])
//   dgrad    dX = dY . W       A k-major (dY [M,N]),   B n-major (W [N,K] read as [K][N])
//   wgrad    dW = dY^T . X     A m-major (dY^T),       B n-major (X)
// Layout-aware LDS staging: tiles are copied to LDS in their memory order (16-byte coalesced
// loads), and fragments are read either row-wise (ds_read_b128) or column-wise with the gfx950
// transposed read ds_read_b64_tr_b16 — no transposed copies of activations are ever written.
//
// Tile 128x128, 4 waves (2x2), each wave 64x64 = 4x4 MFMA 16x16 tiles, register-staged double
// buffer (one barrier per K step), XCD-aware tile order.  bf16: v_mfma_f32_16x16x32_bf16, K-step
// 64; f32 parity mode: exact v_mfma_f32_16x16x4_f32, K-step 32.
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "rp_common.h"

namespace {

constexpr int BM = 128, BN = 128;
constexpr int NT = 256;
constexpr int PAD = 16;  // bytes of padding per LDS row

template <typename T>
struct GemmCfg {
  static constexpr int BK = 128 / (int)sizeof(T);          // 64 bf16 / 32 f32 -> 128-byte rows
  static constexpr int KROW = BK * (int)sizeof(T) + PAD;   // bytes per k-major LDS row (144)
  static constexpr int MROW = BM * (int)sizeof(T) + PAD;   // bytes per m-major LDS row
  static constexpr int KTILE = BM * KROW;                  // bytes of a k-major tile
  static constexpr int MTILE = BK * MROW;                  // bytes of an m-major tile
  static constexpr int VEC = 16 / (int)sizeof(T);          // elements per 16-byte chunk
};

struct EpiDev {
  const float* bias;
  int relu;
  uint32_t drop_thresh;
  float drop_scale;
  uint32_t drop_seed;
  const uint32_t* seed_base;  // graph-replayable dropout base word (the launch's seed_base argument), or null
  const float* residual;
  int64_t ldr;
  const void* gate;
  int gate_bf16;
  int64_t ldg;
  float gate_scale;
  int accumulate;
  int64_t col_scale_n;  // columns n < col_scale_n are multiplied by col_scale after the bias
  float col_scale;
  int split_major;  // split-K: deal the (split, tile) work items split-major over the XCDs (see tile_split)
  int prefetch_gate;  // 256-row kernel: touch the tile's bf16 gate lines one K-tile before the epilogue
  // attention delta fused into the attention-output gradient GEMM (rp_gemm_attn_dout_delta; bf16 C, the
  // RESB 2 epilogue of gemm_epilogue, M % 128 == N % 128 == 0): per (row, 64-column head) the row dot of
  // the STORED bf16 output with (dot_hi + dot_lo) -> the delta workspace planes, exactly as
  // attn_delta_kernel forms them
  const bf16* dot_hi;
  const bf16* dot_lo;  // may be null
  int64_t ld_dot;
  float* delta;        // [3, B, H, T] fp32
  const float* lse;    // [B, H, T]
  int dT, dH;          // rows are b * dT + t; dH heads of 64 columns
  float dscale;        // 1 / (1 - p)
  int st_pol;          // output store cache policy (rp_st16)
  int ld_pol;          // residual load cache policy (rp_ld16f)
};

// Work item of a workgroup: output tile t (XCD-aware: consecutive tiles share an XCD's L2) and, for
// split-K (MODE 1), the K split.  split_major: the (split, tile) pairs are numbered split-major and
// dealt in contiguous ranges per XCD, so the workgroups of one XCD share K ranges (the wgrad
// operands dY and X are then fetched once per XCD instead of once per output tile column / row).
template <int MODE>
__device__ __forceinline__ void tile_split(int tiles, int split_major, int& t, int& split) {
  if (MODE == 1 && split_major) {
    const int nwg = (int)(gridDim.x * gridDim.y);
    const int w = rp_xcd_remap((int)(blockIdx.y * gridDim.x + blockIdx.x), nwg);
    split = w / tiles;
    t = w % tiles;
  } else {
    t = rp_xcd_remap(blockIdx.x, tiles);
    split = MODE == 1 ? (int)blockIdx.y : 0;
  }
}

// --- global -> register staging -----------------------------------------------------------
// Each operand tile is 1024 chunks of 16 bytes; 256 threads own 4 chunks each.
template <typename T, bool KMAJ>
__device__ __forceinline__ void stage_load(uint4 (&r)[4], const T* __restrict__ base, int64_t ld,
                                           int64_t rows_lim /* M or N */, int64_t k_lim, int64_t row0,
                                           int64_t k0, int tid) {
  using C = GemmCfg<T>;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int id = tid + NT * i;
    int64_t rr, cc;  // memory row / element column of this chunk
    bool ok;
    if (KMAJ) {  // tile [BM rows][BK] ; chunks per row = BK / VEC = 8
      int row = id >> 3, c = id & 7;
      rr = row0 + row;
      cc = k0 + c * C::VEC;
      ok = (rr < rows_lim) && (cc < k_lim);
    } else {  // tile [BK rows (k)][BM cols] ; chunks per row = BM / VEC
      constexpr int CPR = BM / C::VEC;
      int row = id / CPR, c = id % CPR;
      rr = k0 + row;
      cc = row0 + c * C::VEC;
      ok = (rr < k_lim) && (cc < rows_lim);
    }
    if (ok)
      r[i] = *reinterpret_cast<const uint4*>(base + rr * ld + cc);
    else
      r[i] = make_uint4(0u, 0u, 0u, 0u);
  }
}

template <typename T, bool KMAJ>
__device__ __forceinline__ void stage_store(const uint4 (&r)[4], char* lds, int tid) {
  using C = GemmCfg<T>;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int id = tid + NT * i;
    int off;
    if (KMAJ) {
      int row = id >> 3, c = id & 7;
      off = row * C::KROW + c * 16;
    } else {
      constexpr int CPR = BM / C::VEC;
      int row = id / CPR, c = id % CPR;
      off = row * C::MROW + c * 16;
    }
    *reinterpret_cast<uint4*>(lds + off) = r[i];
  }
}

// --- fragment reads ----------------------------------------------------------------------
// bf16: fragment of 16 rows x 32 k for v_mfma_f32_16x16x32_bf16:
//   lane l holds X[row = l&15][k = 8*(l>>4) + j], j = 0..7
__device__ __forceinline__ bf16x8 frag_bf16(const char* lds, bool kmaj, int rbase, int kbase, int lane) {
  using C = GemmCfg<bf16>;
  int g = lane >> 4, i = lane & 15;
  if (kmaj) {
    const char* p = lds + (rbase + i) * C::KROW + (kbase + 8 * g) * 2;
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    int q = i >> 2, pp = i & 3;
    const char* p0 = lds + (kbase + 8 * g + q) * C::MROW + (rbase + 4 * pp) * 2;
    const char* p1 = p0 + 4 * C::MROW;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p1));
    bf16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

// f32: fragment for v_mfma_f32_16x16x4_f32: lane l holds X[row = l&15][k = l>>4]
__device__ __forceinline__ float frag_f32(const char* lds, bool kmaj, int rbase, int kbase, int lane) {
  using C = GemmCfg<float>;
  int g = lane >> 4, i = lane & 15;
  if (kmaj) return *reinterpret_cast<const float*>(lds + (rbase + i) * C::KROW + (kbase + g) * 4);
  return *reinterpret_cast<const float*>(lds + (kbase + g) * C::MROW + (rbase + i) * 4);
}

template <typename T, bool AK, bool BKM>
__device__ __forceinline__ void compute_tile(f32x4 (&acc)[4][4], const char* ldsA, const char* ldsB,
                                             int wm, int wn, int lane) {
  using C = GemmCfg<T>;
  if constexpr (std::is_same<T, bf16>::value) {
#pragma unroll
    for (int ks = 0; ks < C::BK; ks += 32) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag_bf16(ldsA, AK, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag_bf16(ldsB, BKM, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < C::BK; ks += 4) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag_f32(ldsA, AK, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag_f32(ldsB, BKM, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
}

// accumulate the column sums of an m-major A tile straight from the staging registers
// (bias gradient of the wgrad GEMM: db[m] = sum_k dY[k][m]); a thread always owns the same
// 16-byte column chunk because NT is a multiple of the chunks per row
template <typename T>
__device__ __forceinline__ void accum_chunks(float (&b)[GemmCfg<T>::VEC], const uint4 (&r)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const T* e = reinterpret_cast<const T*>(&r[i]);
#pragma unroll
    for (int j = 0; j < GemmCfg<T>::VEC; ++j) b[j] += (float)e[j];
  }
}

constexpr int CST = BN + 4;                 // fp32 LDS row stride of the staged C tile
constexpr int CTILE_BYTES = BM * CST * 4;   // whole staged C tile
constexpr int CHALF_BYTES = CTILE_BYTES / 2;  // C tile staged in two 64-row halves (low-LDS configs)

template <typename T, bool AK, bool BKM>
constexpr int gemm_lds_bytes() {
  using C = GemmCfg<T>;
  constexpr int TA = AK ? C::KTILE : C::MTILE;
  constexpr int TB = BKM ? C::KTILE : C::MTILE;
  return 2 * (TA + TB) > CTILE_BYTES ? 2 * (TA + TB) : CTILE_BYTES;
}

// ---- shared epilogue: stage the 128x128 fp32 tile in LDS, then 16-byte row chunks per thread ----
// MODE 0 applies the fused epilogue (bias, relu, dropout, gate, residual, accumulate) and converts;
// MODE 1 stores the raw fp32 partial tile into split blockIdx.y's slab.
// RESB (fp32 C with a residual, MODE 0): every LDS read and residual load of a pass is issued before
// the pass's first store.  In the interleaved loop each chunk's residual load waited behind the
// previous chunk's store (the compiler cannot prove the output and residual rows apart): one HBM
// round trip per chunk — s_memtime stamps put that epilogue at 1.5x the K = 512 main loop
// (out_proj forward).  Only the residual shapes take it: the batched registers cost the others
// their occupancy.  RESB == 2 (bf16 C with the attention delta, rp_gemm_attn_dout_delta): the tile's
// attention-output chunks (hi, lo) are requested by the kernel BEFORE its main loop (gemm_bf16_dma_kernel)
// and land while it runs.  Per chunk after its store they cost one HBM round trip each (28.8 us for the
// metric shape's launch), batched at the epilogue's start 23.2 us, before the main loop 21.8 us (the
// plain dgrad alone: 14.9 us; profiles/r06_dout_delta_ab.txt).
template <typename TC, int MODE, bool HALVES = false, int RESB = 0, int MI = 4>
__device__ __forceinline__ void gemm_epilogue(const f32x4 (&acc)[MI][4], char* lds, int tid, int lane, int wm, int wn,
                                              int64_t m0, int64_t n0, int64_t M, int64_t N, TC* __restrict__ Cout,
                                              int64_t ldc, float alpha, const EpiDev& ep, int split,
                                              const bf16x8* poh = nullptr, const bf16x8* pol = nullptr) {
  static_assert(MI == 4 || !HALVES, "64-row tiles stage whole");
  float* cs = reinterpret_cast<float*>(lds);
  constexpr int OV = 16 / (int)sizeof(TC);
  constexpr int CPRO = BN / OV;
  TC* Cbase = Cout + (MODE == 1 ? (int64_t)split * M * ldc : 0);
  const uint32_t dseed = (MODE == 0 && ep.drop_thresh) ? rp_seed_eff(ep.seed_base, ep.drop_seed) : 0u;
  // a thread's output chunk column is the same in every pass and iteration (NT % CPRO == 0): its bias
  // chunk is loaded once, not per chunk (the stores through C may alias it, so the compiler reloads)
  static_assert(NT % CPRO == 0, "fixed chunk column per thread");
  float bv[OV];
#pragma unroll
  for (int e = 0; e < OV; ++e) bv[e] = 0.f;
  if (MODE == 0 && ep.bias && n0 + (tid % CPRO) * OV < N) {
#pragma unroll
    for (int e = 0; e < OV; e += 4) {
      const float4 q = *reinterpret_cast<const float4*>(ep.bias + n0 + (tid % CPRO) * OV + e);
      bv[e] = q.x; bv[e + 1] = q.y; bv[e + 2] = q.z; bv[e + 3] = q.w;
    }
  }
  constexpr int NH = HALVES ? 2 : 1;  // staging passes
  constexpr int HR = MI * 32 / NH;     // rows per pass
#pragma unroll 1
  for (int half = 0; half < NH; ++half) {
  if (half) __syncthreads();  // the first half's rows are consumed
  if (!HALVES || wm == half) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[((HALVES ? 0 : wm * (MI * 16)) + i * 16 + g * 4 + r) * CST + wn * 64 + j * 16 + cl] = acc[i][j][r];
  }
  __syncthreads();
  if constexpr (RESB == 2) {
    // the out_proj dgrad with the delta epilogue: alpha only (no bias / relu / dropout / gate / residual,
    // rp_gemm_attn_dout_delta sets none), M and N whole tiles; the arithmetic of the per-chunk loop below
    static_assert(std::is_same<TC, bf16>::value && MODE == 0 && OV == 8, "delta epilogue: bf16 C, MODE 0");
    constexpr int ITER = HR * CPRO / NT;
    static_assert(HR * CPRO % NT == 0, "whole chunks per thread");
    bf16x8 oh[ITER], ol[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {  // loaded by the kernel before its main loop
      oh[it] = poh[it];
      if (ep.dot_lo) ol[it] = pol[it];
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int id = tid + it * NT;
      const int row = id / CPRO + half * HR, cc = (id % CPRO) * OV;
      const int64_t m = m0 + row, n = n0 + cc;
      uint4 o;
      bf16* ob = reinterpret_cast<bf16*>(&o);
#pragma unroll
      for (int e = 0; e < OV; e += 4) {
        const float4 q = *reinterpret_cast<const float4*>(cs + (row - half * HR) * CST + cc + e);
        ob[e] = (bf16)(q.x * alpha); ob[e + 1] = (bf16)(q.y * alpha);
        ob[e + 2] = (bf16)(q.z * alpha); ob[e + 3] = (bf16)(q.w * alpha);
      }
      rp_st16((TC*)Cbase + m * ldc + n, o, ep.st_pol);
      float dsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += ((float)oh[it][e] + (ep.dot_lo ? (float)ol[it][e] : 0.f)) * (float)ob[e];
      dsum = rp_sum8(dsum);
      if ((n & 63) == 0) {
        const int b = (int)(m / ep.dT), t = (int)(m % ep.dT);
        const int64_t at = ((int64_t)b * ep.dH + n / 64) * ep.dT + t, plane = (M / ep.dT) * ep.dH * ep.dT;
        ep.delta[at] = dsum;
        ep.delta[plane + at] = -dsum / ep.dscale;
        ep.delta[2 * plane + at] = -(ep.lse[at] * 1.4426950408889634f - log2f(ep.dscale));
      }
    }
    continue;
  } else if constexpr (RESB && std::is_same<TC, bf16>::value) {
    // bf16 C gated by a bf16 tensor (the d_ff dgrad through ReLU + dropout; no residual, no delta): the
    // pass's gate chunks loaded before its first store, as the residual below
    static_assert(MODE == 0 && OV == 8, "RESB bf16: MODE 0");
    constexpr int ITER = HR * CPRO / NT;
    static_assert(HR * CPRO % NT == 0, "whole chunks per thread");
    bf16x8 gv[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int id = tid + it * NT;
      const int64_t m = m0 + id / CPRO + half * HR, n = n0 + (id % CPRO) * OV;
      if (m < M && n < N) gv[it] = *reinterpret_cast<const bf16x8*>((const bf16*)ep.gate + m * ep.ldg + n);
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int id = tid + it * NT;
      const int row = id / CPRO + half * HR, cc = (id % CPRO) * OV;
      const int64_t m = m0 + row, n = n0 + cc;
      if (m >= M || n >= N) continue;
      float v[OV];
#pragma unroll
      for (int e = 0; e < OV; e += 4) {
        float4 q = *reinterpret_cast<const float4*>(cs + (row - half * HR) * CST + cc + e);
        v[e] = q.x * alpha; v[e + 1] = q.y * alpha; v[e + 2] = q.z * alpha; v[e + 3] = q.w * alpha;
      }
      if (ep.bias) {
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] += bv[e];
      }
      if (n < ep.col_scale_n) {
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] *= ep.col_scale;
      }
      if (ep.relu) {
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (ep.drop_thresh) {
        const uint32_t kb = rp_keep_bits<OV>(dseed, (uint32_t)(m * N + n), ep.drop_thresh);
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] = ((kb >> e) & 1u) ? v[e] * ep.drop_scale : 0.f;
      }
#pragma unroll
      for (int e = 0; e < OV; ++e) v[e] = (float)gv[it][e] > 0.f ? v[e] * ep.gate_scale : 0.f;
      uint4 o;
      bf16* ob = reinterpret_cast<bf16*>(&o);
#pragma unroll
      for (int e = 0; e < 8; ++e) ob[e] = (bf16)v[e];
      rp_st16((TC*)Cbase + m * ldc + n, o, ep.st_pol);
    }
    continue;
  } else if constexpr (RESB) {
    static_assert(std::is_same<TC, float>::value && MODE == 0, "RESB: fp32 C, MODE 0");
    constexpr int ITER = HR * CPRO / NT;
    static_assert(HR * CPRO % NT == 0, "whole chunks per thread");
    float4 v[ITER], r[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int id = tid + it * NT;
      const int row = id / CPRO, cc = (id % CPRO) * OV;
      const int64_t m = m0 + row + half * HR, n = n0 + cc;
      v[it] = *reinterpret_cast<const float4*>(cs + row * CST + cc);
      r[it] = (m < M && n < N) ? rp_ld16f(ep.residual + m * ep.ldr + n, ep.ld_pol)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int id = tid + it * NT;
      const int row = id / CPRO + half * HR, cc = (id % CPRO) * OV;
      const int64_t m = m0 + row, n = n0 + cc;
      if (m >= M || n >= N) continue;
      float e4[4] = {v[it].x * alpha, v[it].y * alpha, v[it].z * alpha, v[it].w * alpha};
      if (ep.bias) {
        e4[0] += bv[0]; e4[1] += bv[1]; e4[2] += bv[2]; e4[3] += bv[3];
      }
      if (n < ep.col_scale_n) {
#pragma unroll
        for (int e = 0; e < 4; ++e) e4[e] *= ep.col_scale;
      }
      if (ep.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) e4[e] = fmaxf(e4[e], 0.f);
      }
      if (ep.drop_thresh) {
        const uint32_t kb = rp_keep_bits<4>(dseed, (uint32_t)(m * N + n), ep.drop_thresh);
#pragma unroll
        for (int e = 0; e < 4; ++e) e4[e] = ((kb >> e) & 1u) ? e4[e] * ep.drop_scale : 0.f;
      }
      if (ep.gate) {
        if (ep.gate_bf16) {
          const bf16* gp = (const bf16*)ep.gate + m * ep.ldg + n;
#pragma unroll
          for (int e = 0; e < 4; ++e) e4[e] = (float)gp[e] > 0.f ? e4[e] * ep.gate_scale : 0.f;
        } else {
          const float* gp = (const float*)ep.gate + m * ep.ldg + n;
#pragma unroll
          for (int e = 0; e < 4; ++e) e4[e] = gp[e] > 0.f ? e4[e] * ep.gate_scale : 0.f;
        }
      }
      e4[0] += r[it].x; e4[1] += r[it].y; e4[2] += r[it].z; e4[3] += r[it].w;
      float* dst = (float*)Cbase + m * ldc + n;
      if (ep.accumulate) {
        const float4 q = *reinterpret_cast<const float4*>(dst);
        e4[0] += q.x; e4[1] += q.y; e4[2] += q.z; e4[3] += q.w;
      }
      rp_st16(dst, make_float4(e4[0], e4[1], e4[2], e4[3]), ep.st_pol);
    }
    continue;
  }
  for (int id = tid; id < HR * CPRO; id += NT) {
    const int row = id / CPRO + half * HR, cc = (id % CPRO) * OV;
    const int64_t m = m0 + row, n = n0 + cc;
    if (m >= M || n >= N) continue;
    float v[OV];
#pragma unroll
    for (int e = 0; e < OV; e += 4) {
      float4 q = *reinterpret_cast<const float4*>(cs + (row - half * HR) * CST + cc + e);
      v[e] = q.x * alpha; v[e + 1] = q.y * alpha; v[e + 2] = q.z * alpha; v[e + 3] = q.w * alpha;
    }
    if (MODE == 0) {
      if (ep.bias) {
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] += bv[e];
      }
      if (n < ep.col_scale_n) {  // chunks never straddle col_scale_n (a multiple of 8)
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] *= ep.col_scale;
      }
      if (ep.relu) {
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (ep.drop_thresh) {
        const uint32_t kb = rp_keep_bits<OV>(dseed, (uint32_t)(m * N + n), ep.drop_thresh);
#pragma unroll
        for (int e = 0; e < OV; ++e) v[e] = ((kb >> e) & 1u) ? v[e] * ep.drop_scale : 0.f;
      }
      if (ep.gate) {
        if (ep.gate_bf16) {
          const bf16* gp = (const bf16*)ep.gate + m * ep.ldg + n;
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] = (float)gp[e] > 0.f ? v[e] * ep.gate_scale : 0.f;
        } else {
          const float* gp = (const float*)ep.gate + m * ep.ldg + n;
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] = gp[e] > 0.f ? v[e] * ep.gate_scale : 0.f;
        }
      }
      if (ep.residual) {
#pragma unroll
        for (int e = 0; e < OV; e += 4) {
          float4 q = rp_ld16f(ep.residual + m * ep.ldr + n + e, ep.ld_pol);
          v[e] += q.x; v[e + 1] += q.y; v[e + 2] += q.z; v[e + 3] += q.w;
        }
      }
    }
    TC* dst = Cbase + m * ldc + n;
    if constexpr (std::is_same<TC, float>::value) {
      if (MODE == 0 && ep.accumulate) {
        float4 q = *reinterpret_cast<const float4*>(dst);
        v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
      }
      rp_st16(dst, make_float4(v[0], v[1], v[2], v[3]), ep.st_pol);
    } else {
      uint4 o;
      bf16* ob = reinterpret_cast<bf16*>(&o);
#pragma unroll
      for (int e = 0; e < 8; ++e) ob[e] = (bf16)v[e];
      rp_st16(dst, o, ep.st_pol);
    }
  }
  }
}

// bias-gradient partials: thread t holds VEC column sums of column chunk t % (BM/VEC); reduce the
// threads sharing a chunk through LDS and write this split's partial row
template <int VEC>
__device__ __forceinline__ void bias_reduce(const float (&bacc)[VEC], char* lds, int tid, int64_t m0, int64_t M,
                                            float* __restrict__ bslab, int split) {
  __syncthreads();
  constexpr int CPR = BM / VEC;
  float* red = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[tid * VEC + j] = bacc[j];
  __syncthreads();
  if (tid < BM && m0 + tid < M) {
    const int c = tid / VEC, e = tid % VEC;
    float sum = 0.f;
    for (int j = 0; j < NT / CPR; ++j) sum += red[(c + CPR * j) * VEC + e];
    bslab[(int64_t)split * M + m0 + tid] = sum;
  }
}

// MODE 0: full-K tile with the fused epilogue;  MODE 1: split-K partial tile -> fp32 slab
// (blockIdx.y = split), optional bias column sums of A -> bias slab.
template <typename T, bool AK, bool BKM, typename TC, int MODE>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(int64_t M, int64_t N, int64_t K, const T* __restrict__ A,
                                                     int64_t lda, const T* __restrict__ B, int64_t ldb,
                                                     TC* __restrict__ Cout, int64_t ldc, float alpha,
                                                     EpiDev ep, int64_t kchunk, float* __restrict__ bslab) {
  using C = GemmCfg<T>;
  constexpr int TA = AK ? C::KTILE : C::MTILE;
  constexpr int TB = BKM ? C::KTILE : C::MTILE;
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<T, AK, BKM>()];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (int)((N + BN - 1) / BN);
  const int tiles_m = (int)((M + BM - 1) / BM);
  int t, split;
  tile_split<MODE>(tiles_m * tiles_n, ep.split_major, t, split);
  const int64_t m0 = (int64_t)(t / tiles_n) * BM;
  const int64_t n0 = (int64_t)(t % tiles_n) * BN;
  int64_t kbeg = 0, kend = K;
  if (MODE == 1) {
    kbeg = (int64_t)split * kchunk;
    kend = kbeg + kchunk < K ? kbeg + kchunk : K;
  }
  const bool want_bias = MODE == 1 && !AK && bslab != nullptr && n0 == 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[C::VEC];
#pragma unroll
  for (int j = 0; j < C::VEC; ++j) bacc[j] = 0.f;

  uint4 ra[4], rb[4];
  const int nk = kend > kbeg ? (int)((kend - kbeg + C::BK - 1) / C::BK) : 0;
  if (nk > 0) {
    stage_load<T, AK>(ra, A, lda, M, kend, m0, kbeg, tid);
    stage_load<T, BKM>(rb, B, ldb, N, kend, n0, kbeg, tid);
    if (want_bias) accum_chunks<T>(bacc, ra);
    stage_store<T, AK>(ra, lds, tid);
    stage_store<T, BKM>(rb, lds + TA, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = lds + (kt & 1) * (TA + TB);
    char* nxt = lds + ((kt + 1) & 1) * (TA + TB);
    const bool more = (kt + 1) < nk;
    if (more) {
      const int64_t k1 = kbeg + (int64_t)(kt + 1) * C::BK;
      stage_load<T, AK>(ra, A, lda, M, kend, m0, k1, tid);
      stage_load<T, BKM>(rb, B, ldb, N, kend, n0, k1, tid);
      if (want_bias) accum_chunks<T>(bacc, ra);
    }
    compute_tile<T, AK, BKM>(acc, cur, cur + TA, wm, wn, lane);
    if (more) {
      stage_store<T, AK>(ra, nxt, tid);
      stage_store<T, BKM>(rb, nxt + TA, tid);
    }
    __syncthreads();
  }

  gemm_epilogue<TC, MODE>(acc, lds, tid, lane, wm, wn, m0, n0, M, N, Cout, ldc, alpha, ep, split);
  if (MODE == 1 && want_bias) bias_reduce<C::VEC>(bacc, lds, tid, m0, M, bslab, split);
}

// ============================ bf16 fast path: LDS-DMA staged main loop ============================
// global_load_lds_dwordx4 writes each wave-instruction's 64 x 16 B lane-linearly into LDS, so the
// LDS images are unpadded and the bank-conflict XOR swizzle goes on the per-lane SOURCE address
// (guide §5.4 rule 21); the fragment reads apply the same involution:
//   k-major tile [128 rows][64 k] (128-B rows): 16-B chunk c of row r lives at chunk c ^ ((r>>1)&7)
//     -> every ds_read_b128 lane group of the 16x16x32 A/B fragment read hits 16 distinct slots;
//   k-major tile [128 rows][32 k] (64-B rows): chunk c of row r lives at c ^ f((r>>2)&3),
//     f = {0,2,3,1} -> the four rows of each residue r&3 in a ds_read_b128 lane group (two with
//     k-chunk g, two with g^1) land on four distinct chunks: 16 distinct slots again;
//   m-major tile [BK k][128 cols] (256-B rows): chunk c of row k lives at c ^ 2*s(k),
//     s(k) = (k&3) | ((k>>3)&1)<<2 -> the 8 rows of a ds_read_b64_tr_b16 half-wave read hit
//     8 distinct 32-B slots.
// Configurations (the 16 KiB-per-stage k=64 images, or 8 KiB k=32 ones):
//   CFG 0  BK 64, two LDS stages, whole-tile C staging: 67.6 KiB, 2 workgroups / CU
//   CFG 1  BK 64, one LDS stage (load, barrier, compute, barrier), C in halves: 33.8 KiB, 4 / CU
//   CFG 2  BK 32, two LDS stages, C in halves: 33.8 KiB, 4 / CU
// Measured on MI355X (scripts/microbench.py, M = 16384): K <= 1024 runs best on CFG 1, whose four
// co-resident workgroups hide each other's load latency (qkv fwd 43.1 -> 41.3 us, linear1 fwd
// 54.3 -> 50.5, K = 512 dgrad into d_ff 64.3 -> 52.8), deeper K on CFG 0 (linear2 fwd 39.5 vs 43.0);
// CFG 2 lost to CFG 1 everywhere and serves only K % 64 == 32.  In the whole training step, though,
// CFG 1 on the K = 512, N >= 1536 shapes measured 20.30 vs 20.15 ms per step in round 1 (eager step,
// per-kernel events inside the timed region); in the graph-replayed step of round 2 it measures 16.03
// vs 16.21 ms (three interleaved pairs, one box), so it is the default (rp_gemm_cfg).  CFG 1 on every
// short-K shape (N = 512 too) measured the same as on the wide ones only; CFG 1 everywhere 16.52 ms.
// Rows past M/N are clamped to the last valid row (their outputs are discarded), so the path needs
// whole BK-deep K steps.
typedef __attribute__((address_space(3))) void lds_void;

template <int CFG>
struct DmaCfg {
  static constexpr int BK = CFG == 2 ? 32 : 64;
  static constexpr int STAGES = CFG == 1 ? 1 : 2;
  static constexpr bool HALVES = CFG != 0;
  static constexpr int GT = BM * BK * 2;  // bytes of one operand tile (one stage)
  static constexpr int PER_WAVE = GT / 1024 / (NT / 64);  // 1-KiB DMA pieces per wave per operand
  static constexpr int LDS_MAIN = 2 * STAGES * GT;
  static constexpr int LDS_EPI = HALVES ? CHALF_BYTES : CTILE_BYTES;
  static constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
};

__device__ __forceinline__ int kswz(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ int kswz32(int r, int c) { return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3); }
__device__ __forceinline__ int mswz(int k, int c) { return c ^ (2 * ((k & 3) | (((k >> 3) & 1) << 2))); }

template <bool KMAJ, int BK, int ROWS = BM>
__device__ __forceinline__ void glds_tile(const bf16* __restrict__ base, int64_t ld, int64_t rows_lim, int64_t row0,
                                          int64_t k0, char* tile, int wid, int lane) {
  static_assert(KMAJ || ROWS == 128, "m-major images are 128 columns wide");
  constexpr int PER = ROWS * BK * 2 / 1024 / (NT / 64);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int I = wid * PER + j;  // wave-instruction index (1 KiB of the tile)
    const bf16* src;
    if (KMAJ) {
      int r, lc;
      if constexpr (BK == 64) {
        r = I * 8 + (lane >> 3);
        lc = kswz(r, lane & 7);
      } else {
        r = I * 16 + (lane >> 2);
        lc = kswz32(r, lane & 3);
      }
      int64_t rr = row0 + r;
      if (rr >= rows_lim) rr = rows_lim - 1;
      src = base + rr * ld + k0 + lc * 8;
    } else {
      const int k = I * 4 + (lane >> 4);
      const int lc = mswz(k, lane & 15);
      int64_t cc = row0 + lc * 8;
      if (cc >= rows_lim) cc = rows_lim - 8;
      src = base + (k0 + k) * ld + cc;
    }
    __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + I * 1024), 16, 0, 0);
  }
}

template <int BK>
__device__ __forceinline__ bf16x8 frag_k_swz(const char* t, int rbase, int kbase, int lane) {
  const int r = rbase + (lane & 15);
  const int lc = (kbase >> 3) + (lane >> 4);
  if constexpr (BK == 64) return *reinterpret_cast<const bf16x8*>(t + r * 128 + kswz(r, lc) * 16);
  return *reinterpret_cast<const bf16x8*>(t + r * 64 + kswz32(r, lc) * 16);
}

__device__ __forceinline__ bf16x8 frag_m_swz(const char* t, int rbase, int kbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k0 = kbase + 8 * g + q, k1 = k0 + 4;
  const int lc = (rbase >> 3) + (p >> 1);
  const char* p0 = t + k0 * 256 + mswz(k0, lc) * 16 + (p & 1) * 8;
  const char* p1 = t + k1 * 256 + mswz(k1, lc) * 16 + (p & 1) * 8;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// main loop of the (32 MI) x 128 LDS-DMA tile over the K range [kbeg, kend) (whole BK steps): acc
// gets the tile's products; with want_bias, bacc the column sums of the staged m-major A tiles.  MI = 4:
// 128 x 128 (each wave 64 x 64); MI = 2: 64 x 128 (each wave 32 x 64; k-major A only) for grids of
// 128-row tiles that leave CUs idle (DmaTile)
template <bool AK, bool BKM, int CFG, int MI = 4>
__device__ __forceinline__ void dma_mainloop(const bf16* __restrict__ A, int64_t lda, int64_t M,
                                             const bf16* __restrict__ B, int64_t ldb, int64_t N, int64_t m0,
                                             int64_t n0, int64_t kbeg, int64_t kend, bool want_bias,
                                             f32x4 (&acc)[MI][4], float (&bacc)[8], char* lds, int tid, int lane,
                                             int wid, int wm, int wn) {
  using D = DmaCfg<CFG>;
  constexpr int BK = D::BK, GT = D::GT;
  constexpr int ROWS = MI * 32, GTA = ROWS * BK * 2, SG = GTA + GT;  // A image, stage bytes
  static_assert(MI == 4 || (AK && D::STAGES == 2), "64-row tiles: k-major A, two stages");
  const int nk = kend > kbeg ? (int)((kend - kbeg) / BK) : 0;
  if (D::STAGES == 2 && nk > 0) {
    glds_tile<AK, BK, ROWS>(A, lda, M, m0, kbeg, lds, wid, lane);
    glds_tile<BKM, BK>(B, ldb, N, n0, kbeg, lds + GTA, wid, lane);
  }
  if (D::STAGES == 2) __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = lds + (D::STAGES == 2 ? (kt & 1) * SG : 0);
    char* nxt = lds + ((kt + 1) & 1) * SG;
    if (D::STAGES == 1) {  // one LDS stage: the co-resident workgroups hide the load latency
      if (kt > 0) __syncthreads();
      glds_tile<AK, BK, ROWS>(A, lda, M, m0, kbeg + (int64_t)kt * BK, lds, wid, lane);
      glds_tile<BKM, BK>(B, ldb, N, n0, kbeg + (int64_t)kt * BK, lds + GTA, wid, lane);
      __syncthreads();
    } else if (kt + 1 < nk) {
      const int64_t k1 = kbeg + (int64_t)(kt + 1) * BK;
      glds_tile<AK, BK, ROWS>(A, lda, M, m0, k1, nxt, wid, lane);
      glds_tile<BKM, BK>(B, ldb, N, n0, k1, nxt + GTA, wid, lane);
    }
    if (want_bias) {  // column sums of the staged dY tile (bias gradient), BK/16 x 16 B per thread
      const int cg = tid & 15;
#pragma unroll
      for (int j = 0; j < BK / 16; ++j) {
        const int k = (tid >> 4) + 16 * j;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(cur + k * 256 + mswz(k, cg) * 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) bacc[e] += (float)v[e];
      }
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 a[MI], b[4];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        a[i] = AK ? frag_k_swz<BK>(cur, wm * (MI * 16) + i * 16, ks, lane)
                  : frag_m_swz(cur, wm * (MI * 16) + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = BKM ? frag_k_swz<BK>(cur + GTA, wn * 64 + j * 16, ks, lane)
                   : frag_m_swz(cur + GTA, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (D::STAGES == 2) __syncthreads();
  }
  if (D::STAGES == 1) __syncthreads();
}

// LDS of a (32 MI) x 128 DMA tile: two (or one) stages of the A and B images, or the staged C tile
template <int CFG, int MI>
constexpr int dma_tile_lds() {
  using D = DmaCfg<CFG>;
  constexpr int MAIN = D::STAGES * (MI * 32 * D::BK * 2 + D::GT);
  constexpr int EPI = D::HALVES ? CHALF_BYTES : MI * 32 * CST * 4;
  return MAIN > EPI ? MAIN : EPI;
}

#ifdef RP_GEMM_PROBE
constexpr int RP_PROBE_MAX = 8192;
__device__ uint64_t g_gemm_probe[RP_PROBE_MAX * 4];
__device__ uint64_t g_lnx_probe[RP_PROBE_MAX * 8];  // exchange kernels: 6 stamps per workgroup
#define LX_STAMP(i) if (tid == 0 && blockIdx.x < RP_PROBE_MAX) g_lnx_probe[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime()
#else
#define LX_STAMP(i)
#endif

template <bool AK, bool BKM, typename TC, int MODE, int CFG, int RESB = 0, int MI = 4>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_dma_kernel(int64_t M, int64_t N, int64_t K,
                                                              const bf16* __restrict__ A, int64_t lda,
                                                              const bf16* __restrict__ B, int64_t ldb,
                                                              TC* __restrict__ Cout, int64_t ldc, float alpha,
                                                              EpiDev ep, int64_t kchunk, float* __restrict__ bslab) {
  using D = DmaCfg<CFG>;
  static_assert(MI != 4 || dma_tile_lds<CFG, 4>() == D::LDS, "128-row LDS as before");
  __shared__ __attribute__((aligned(16))) char lds[dma_tile_lds<CFG, MI>()];
  constexpr int TBM = MI * 32;  // tile rows
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (int)((N + BN - 1) / BN);
  const int tiles_m = (int)((M + TBM - 1) / TBM);
  int t, split;
  tile_split<MODE>(tiles_m * tiles_n, ep.split_major, t, split);
  const int64_t m0 = (int64_t)(t / tiles_n) * TBM;
  const int64_t n0 = (int64_t)(t % tiles_n) * BN;
  int64_t kbeg = 0, kend = K;
  if (MODE == 1) {
    kbeg = (int64_t)split * kchunk;
    kend = kbeg + kchunk < K ? kbeg + kchunk : K;
  }
  const bool want_bias = MODE == 1 && !AK && bslab != nullptr && n0 == 0;
  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  // RESB == 2: the delta epilogue's attention-output chunks requested before the main loop
  constexpr int PRE = RESB == 2 ? 2 * MI : 1;
  bf16x8 poh[PRE], pol[PRE];
  if constexpr (RESB == 2) {
    static_assert(!D::HALVES && MI * 32 * (BN / 8) == PRE * NT, "one staging pass, whole chunks");
#pragma unroll
    for (int it = 0; it < PRE; ++it) {
      const int id = tid + it * NT;
      const int64_t m = m0 + id / (BN / 8), n = n0 + (id % (BN / 8)) * 8;
      poh[it] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(ep.dot_hi + m * ep.ld_dot + n));
      if (ep.dot_lo) pol[it] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(ep.dot_lo + m * ep.ld_dot + n));
    }
  }
#ifdef RP_GEMM_PROBE
  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();
#endif
  dma_mainloop<AK, BKM, CFG, MI>(A, lda, M, B, ldb, N, m0, n0, kbeg, kend, want_bias, acc, bacc, lds, tid, lane, wid,
                                 wm, wn);
#ifdef RP_GEMM_PROBE
  const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();
#endif
  gemm_epilogue<TC, MODE, D::HALVES, RESB, MI>(acc, lds, tid, lane, wm, wn, m0, n0, M, N, Cout, ldc, alpha, ep,
                                               split, poh, pol);
  if (MODE == 1 && want_bias) bias_reduce<8>(bacc, lds, tid, m0, M, bslab, split);
#ifdef RP_GEMM_PROBE
  // tuning build only (never the shipping library): per-workgroup phase stamps of wave 0 at the
  // 100 MHz real-time counter, stored by lanes 0..3 (vector stores)
  const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t ts3 = __builtin_amdgcn_s_memrealtime();
  const int bid = blockIdx.x + blockIdx.y * gridDim.x;
  if (wid == 0 && lane < 4 && bid < RP_PROBE_MAX)
    g_gemm_probe[bid * 4 + lane] = lane == 0 ? ts0 : lane == 1 ? ts1 : lane == 2 ? ts2 : ts3;
#endif
}

// ============ grouped weight gradients: many (dY, X) pairs over the same token range ============
// One launch computes up to WG_MAX weight gradients dW_i = dY_i^T X_i (+ db_i = colsum dY_i) that
// share the token count K, every output tile over the WHOLE K range (no split-K slabs, no reduce
// pass).  The deferred per-layer weight gradients of the encoder (16 layers x {linear2, linear1,
// out_proj, in_proj}) are the intended use, on 256 x 256 tiles (wgrad8_grouped_kernel below, 48
// tiles per layer, all 16 layers = 768 tiles = three per CU; the 128 x 128 form of rounds 2-4 ran
// ~0.3 ms slower per step and was removed in round 6); the XCD remap deals each XCD consecutive tiles,
// i.e. whole layers, whose operand panels its L2 then shares.
constexpr int WG_MAX = 64;
struct WgItem {
  const bf16* dY;
  const bf16* X;
  float* dW;
  float* db;
  int M, N, ldy, ldx;
};
struct WgGroup {
  int n, accumulate, tiles_total;
  int order;  // tile order: 0 XCD chunks, m-major (orders 1 n-major / 2 no remap measured alike)
  int st_pol;  // output store cache policy (rp_st16)
  int64_t K;
  int start[WG_MAX + 1];
  WgItem it[WG_MAX];
};

// ====================== 256-row tiles: 8 waves, whole-K-tile LDS-DMA ring =======================
// One workgroup of 512 threads (8 waves as 2 (M) x 4 (N)) owns a 256 x BNT output tile (BNT = 256
// or 128); each wave accumulates 128 x BNT/4 (8 x BNT/64 MFMA 16x16 tiles).  A K-tile (BK = 64) is
// staged as 128-row "half images" in exactly the formats of the kernel above (k-major 128 x 64
// kswz, m-major [64 k][128] mswz), so the fragment readers are shared; two K-tile stages
// (A 32 KiB + B 16/32 KiB each) at one workgroup per CU.  Arithmetic intensity per staged byte is
// 2x (BNT = 256) or 1.33x that of the 128x128 tile, which is what the per-CU L2 -> LDS rate bounds.
// Pipeline (guide §5, 'Pipelining across barriers'): the LDS-DMA of K-tile t+2 is issued right
// after the barrier that ends every wave's reads of K-tile t, so each fill has one whole K-tile of
// MFMA time (8 waves x 64 MFMAs) to land; the loop waits with a counted s_waitcnt vmcnt and a raw
// s_barrier (never __syncthreads(), whose fence would drain the DMA in flight), and all LDS lives
// in one __shared__ array (guide item 4(a)).
constexpr int NT8 = 512;
constexpr int HIMG = 16384;  // one 128 x 64 bf16 half image

template <int VM, int LGKM>
__device__ __forceinline__ void rp_waitcnt() {
  // gfx9 s_waitcnt immediate: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((VM & 15) | ((VM >> 4) << 14) | (7 << 4) | ((LGKM & 15) << 8));
}

__device__ __forceinline__ void rp_raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// one 1 KiB piece (wave-instruction index I) of a half image
template <bool KMAJ, int KD>
__device__ __forceinline__ void glds_piece8(const bf16* __restrict__ base, int64_t ld, int64_t rows_lim, int64_t row0,
                                            int64_t k0, char* img, int I, int lane) {
  const bf16* src;
  if (KMAJ) {
    int r, lc;
    if constexpr (KD == 64) {
      r = I * 8 + (lane >> 3);
      lc = kswz(r, lane & 7);
    } else {
      r = I * 16 + (lane >> 2);
      lc = kswz32(r, lane & 3);
    }
    int64_t rr = row0 + r;
    if (rr >= rows_lim) rr = rows_lim - 1;
    src = base + rr * ld + k0 + lc * 8;
  } else {
    const int k = I * 4 + (lane >> 4);
    const int lc = mswz(k, lane & 15);
    int64_t cc = row0 + lc * 8;
    if (cc >= rows_lim) cc = rows_lim - 8;
    src = base + (k0 + k) * ld + cc;
  }
  __builtin_amdgcn_global_load_lds(src, (lds_void*)(img + I * 1024), 16, 0, 0);
}

template <int BNT, int KD = 64, int S = 2>
struct G8 {
  static constexpr int NBH = BNT / 128;               // B half images per slot
  static constexpr int HB = 128 * KD * 2;             // bytes of one half image
  static constexpr int SLOT = (2 + NBH) * HB;         // bytes of one K-slab slot (A 256 rows + B BNT rows)
  static constexpr int LPT = (2 + NBH) * KD / 32;     // LDS-DMA instructions per thread per slot
  static constexpr int WN = BNT / 4;                  // output columns per wave
  static constexpr int JT = WN / 16;                  // MFMA column tiles per wave
  static constexpr int CST = BNT + 4;                 // fp32 row stride of an epilogue pass
  static constexpr int PR = 128;                      // rows per epilogue pass (one wave row half)
  static constexpr int EPI = PR * CST * 4;            // one epilogue pass
  static constexpr int LDS = S * SLOT > EPI ? S * SLOT : EPI;
};

// epilogue: two passes of 128 rows (one wave row half each) staged as fp32 in LDS, then 16-byte row
// chunks per thread (four 64-row passes before round 5: twice the barriers, half the stores in flight).
// GATEB (bf16 C, bf16 gate: the linear2 dgrad): a pass's gate chunks are loaded before its stores
// (16 bytes per chunk; inline, each waited behind the previous chunk's store, as the residual did in
// the 128 x 128 epilogue)
template <typename TC, int MODE, int BNT, bool GATEB = false>
__device__ __forceinline__ void gemm8_epilogue(const f32x4 (&acc)[8][BNT / 64], char* lds, int tid, int lane, int wm,
                                               int wn, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                               TC* __restrict__ Cout, int64_t ldc, float alpha, const EpiDev& ep,
                                               int split) {
  using G = G8<BNT>;
  float* cs = reinterpret_cast<float*>(lds);
  constexpr int OV = 16 / (int)sizeof(TC);
  constexpr int CPRO = BNT / OV;
  TC* Cbase = Cout + (MODE == 1 ? (int64_t)split * M * ldc : 0);
  const uint32_t dseed = (MODE == 0 && ep.drop_thresh) ? rp_seed_eff(ep.seed_base, ep.drop_seed) : 0u;
  const int g = lane >> 4, cl = lane & 15;
  // the thread's chunk column is fixed (NT8 % CPRO == 0): its bias chunk loaded once (gemm_epilogue)
  static_assert(NT8 % CPRO == 0, "fixed chunk column per thread");
  float bv[OV];
#pragma unroll
  for (int e = 0; e < OV; ++e) bv[e] = 0.f;
  if (MODE == 0 && ep.bias && n0 + (tid % CPRO) * OV < N) {
#pragma unroll
    for (int e = 0; e < OV; e += 4) {
      const float4 q = *reinterpret_cast<const float4*>(ep.bias + n0 + (tid % CPRO) * OV + e);
      bv[e] = q.x; bv[e + 1] = q.y; bv[e + 2] = q.z; bv[e + 3] = q.w;
    }
  }
  constexpr int PPW = G::PR / 64;  // 64-row accumulator groups of a wave per pass
#pragma unroll
  for (int pass = 0; pass < 256 / G::PR; ++pass) {
    constexpr int ITER = G::PR * CPRO / NT8;
    // fp32 C with a residual (the 256 x 128 tile's linear2 forward) / a bf16 gate (linear2 dgrad): the
    // pass's chunks are loaded before its staging (in flight across the staging and its barriers) and
    // before its first store (inline, each load would wait behind the previous chunk's store)
    constexpr bool RESV = std::is_same<TC, float>::value && MODE == 0;
    float4 rv[RESV ? ITER : 1];
    if constexpr (RESV) {
      if (ep.residual) {
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
          const int id = tid + it * NT8;
          const int64_t m = m0 + pass * G::PR + id / CPRO, n = n0 + (id % CPRO) * OV;
          rv[it] = (m < M && n < N) ? rp_ld16f(ep.residual + m * ep.ldr + n, ep.ld_pol)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    bf16x8 gv[GATEB ? ITER : 1];
    if constexpr (GATEB) {
      static_assert(OV == 8 && MODE == 0, "GATEB: bf16 C");
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        const int id = tid + it * NT8;
        const int64_t m = m0 + pass * G::PR + id / CPRO, n = n0 + (id % CPRO) * OV;
        if (m < M && n < N) gv[it] = *reinterpret_cast<const bf16x8*>((const bf16*)ep.gate + m * ep.ldg + n);
      }
    }
    if (pass) __syncthreads();
    if (wm == pass * G::PR / 128) {
#pragma unroll
      for (int i = 0; i < 4 * PPW; ++i)
#pragma unroll
        for (int j = 0; j < G::JT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cs[(i * 16 + g * 4 + r) * G::CST + wn * G::WN + j * 16 + cl] =
                acc[((pass * G::PR / 64) & 1) * 4 + i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int id = tid + it * NT8;
      const int row = id / CPRO, cc = (id % CPRO) * OV;
      const int64_t m = m0 + pass * G::PR + row, n = n0 + cc;
      if (m >= M || n >= N) continue;
      float v[OV];
#pragma unroll
      for (int e = 0; e < OV; e += 4) {
        float4 q = *reinterpret_cast<const float4*>(cs + row * G::CST + cc + e);
        v[e] = q.x * alpha; v[e + 1] = q.y * alpha; v[e + 2] = q.z * alpha; v[e + 3] = q.w * alpha;
      }
      if (MODE == 0) {
        if (ep.bias) {
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] += bv[e];
        }
        if (n < ep.col_scale_n) {
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] *= ep.col_scale;
        }
        if (ep.relu) {
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (ep.drop_thresh) {
          const uint32_t kb = rp_keep_bits<OV>(dseed, (uint32_t)(m * N + n), ep.drop_thresh);
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] = ((kb >> e) & 1u) ? v[e] * ep.drop_scale : 0.f;
        }
        if constexpr (GATEB) {
#pragma unroll
          for (int e = 0; e < OV; ++e) v[e] = (float)gv[it][e] > 0.f ? v[e] * ep.gate_scale : 0.f;
        } else if (ep.gate) {
          if (ep.gate_bf16) {
            const bf16* gp = (const bf16*)ep.gate + m * ep.ldg + n;
#pragma unroll
            for (int e = 0; e < OV; ++e) v[e] = (float)gp[e] > 0.f ? v[e] * ep.gate_scale : 0.f;
          } else {
            const float* gp = (const float*)ep.gate + m * ep.ldg + n;
#pragma unroll
            for (int e = 0; e < OV; ++e) v[e] = gp[e] > 0.f ? v[e] * ep.gate_scale : 0.f;
          }
        }
        if (ep.residual) {
          if constexpr (RESV) {
            v[0] += rv[it].x; v[1] += rv[it].y; v[2] += rv[it].z; v[3] += rv[it].w;
          } else {
#pragma unroll
            for (int e = 0; e < OV; e += 4) {
              float4 q = rp_ld16f(ep.residual + m * ep.ldr + n + e, ep.ld_pol);
              v[e] += q.x; v[e + 1] += q.y; v[e + 2] += q.z; v[e + 3] += q.w;
            }
          }
        }
      }
      TC* dst = Cbase + m * ldc + n;
      if constexpr (std::is_same<TC, float>::value) {
        if (MODE == 0 && ep.accumulate) {
          float4 q = *reinterpret_cast<const float4*>(dst);
          v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
        }
        rp_st16(dst, make_float4(v[0], v[1], v[2], v[3]), ep.st_pol);
      } else {
        uint4 o;
        bf16* ob = reinterpret_cast<bf16*>(&o);
#pragma unroll
        for (int e = 0; e < 8; ++e) ob[e] = (bf16)v[e];
        rp_st16(dst, o, ep.st_pol);
      }
    }
  }
}

// Phased main loop (cdna_hip_programming.md §5 'The 256² 8-phase template', written for this
// tile): a 64-deep K-tile is four phases, one per quadrant (64 rows x 32 columns) of the wave's
// 128 x 64 output: 16 MFMAs each.  A phase is a READ segment (its new fragments by ds_read, plus
// any LDS-DMA pieces) and a COMPUTE segment (its MFMAs), each closed by a raw s_barrier.  Waves
// 4-7 (wm = 1; the second wave of every SIMD) run one barrier behind waves 0-3, so on every SIMD
// one wave reads while its partner computes.  Quadrant order (0,0) (0,1) (1,1) (1,0): phase 0
// reads A rows 0-63 + B columns 0-31 of the wave's block, phase 1 B columns 32-63, phase 2 A rows
// 64-127, phase 3 nothing.  Two LDS slots of one K-tile (A 2 x 16 KiB + B 2 x 16 KiB).
// Slot reuse (barrier b(8t + j) = the j-th barrier of K-tile t's phases, G0's clock): the B
// images of K-tile t are dead after b(8t+4), the A images after b(8t+6); the B pieces of K-tile
// t+2 are issued in phase 3 of K-tile t, the A pieces of K-tile t+1 in phase 0 of K-tile t.
// INVARIANT (cross-wave: each wave's wait covers only its OWN fills): every fill piece of K-tile
// t+1 has landed by G0-clock barrier b(8t+8), the first barrier any wave passes before reading
// K-tile t+1.  b(8t+8) is the LEADING half's last barrier of K-tile t and the LAGGING half's first
// barrier of phase 3, so the lagging half (waves 4-7) waits (vmcnt(4): only B(t+2) may stay in
// flight) before its phase-3 first barrier and the leading half (waves 0-3) before its phase-3
// SECOND barrier — both are event b(8t+8).  Moving either wait later lets a wave read K-tile t+1
// before another wave's pieces land (the round-2 race, caught by the wgrad/dgrad relaunch tests).
__device__ __forceinline__ void rp_lgkm0() {
  __builtin_amdgcn_s_waitcnt((15) | (3 << 14) | (7 << 4) | (0 << 8));
}

// One 256 x BNT output tile over the K range [kbeg, kend): the phased main loop, the epilogue and
// (bias_dst != null, m-major A) the tile rows' column sums of the staged A: bias_dst[m0 + r] (+)=.
template <bool AK, bool BKM, typename TC, int MODE, int BNT, bool GATEB = false>
__device__ __forceinline__ void gemm8_tile(int64_t M, int64_t N, const bf16* __restrict__ A, int64_t lda,
                                           const bf16* __restrict__ B, int64_t ldb, TC* __restrict__ Cout,
                                           int64_t ldc, float alpha, const EpiDev& ep, int64_t kbeg, int64_t kend,
                                           int64_t m0, int64_t n0, int split, float* __restrict__ bias_dst,
                                           int bias_acc, char* lds) {
  static_assert(BNT == 256, "phased 256-row kernel: 256 x 256 tiles");
  using G = G8<BNT, 64, 2>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
#ifdef RP_GEMM_PROBE
  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();
#endif
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int bimg = wn >> 1, bcol = (wn & 1) * 64;
  const int nk = kend > kbeg ? (int)((kend - kbeg) / 64) : 0;
  const bool pf = MODE == 0 && ep.prefetch_gate && ep.gate && ep.gate_bf16 && nk >= 2;
  uint16_t pfd[2] = {0, 0};
  const bool want_bias = !AK && bias_dst != nullptr;
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  // A pieces (2 half images x 2) and B pieces of K-tile kt into slot kt & 1
  auto fill_a = [&](int kt) {
    char* buf = lds + (kt & 1) * G::SLOT;
    const int64_t k0 = kbeg + (int64_t)kt * 64;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        glds_piece8<AK, 64>(A, lda, M, m0 + 128 * h, k0, buf + h * G::HB, wid * 2 + j, lane);
  };
  auto fill_b = [&](int kt) {
    char* buf = lds + (kt & 1) * G::SLOT;
    const int64_t k0 = kbeg + (int64_t)kt * 64;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        glds_piece8<BKM, 64>(B, ldb, N, n0 + 128 * h, k0, buf + (2 + h) * G::HB, wid * 2 + j, lane);
  };
  auto ra = [&](const char* img, int i, int kk) -> bf16x8 {
    return AK ? frag_k_swz<64>(img, i * 16, kk, lane) : frag_m_swz(img, i * 16, kk, lane);
  };
  auto rb = [&](const char* img, int j, int kk) -> bf16x8 {
    return BKM ? frag_k_swz<64>(img, bcol + j * 16, kk, lane) : frag_m_swz(img, bcol + j * 16, kk, lane);
  };
  if (nk > 0) {
    fill_a(0);
    fill_b(0);
    if (nk > 1) {
      fill_b(1);
      rp_waitcnt<4, 15>();
    } else {
      rp_waitcnt<0, 15>();
    }
  }
  rp_raw_barrier();
  if (wm == 1) rp_raw_barrier();  // the second wave of each SIMD runs one barrier behind

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = lds + (kt & 1) * G::SLOT;
    const char* ai = cur + wm * G::HB;
    const char* bi = cur + (2 + bimg) * G::HB;
    // ---- phase 0: A rows 0-63, B columns 0-31; A pieces of K-tile kt+1 ----
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = ra(ai, i, kk * 32);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb0[j][kk] = rb(bi, j, kk * 32);
    if (kt + 1 < nk) fill_a(kt + 1);
    if (pf && kt == nk - 2) {
      // the gate (the forward's saved activation, cold by now) read by the epilogue: one 2-byte load
      // per 128-byte line of the 256 x 256 bf16 tile, two lines per thread, issued after the last
      // LDS-DMA fill so the counted waits below can leave them in flight into the epilogue
      const bf16* gb = (const bf16*)ep.gate;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int L = tid * 2 + j, row = L >> 2;
        const int64_t m = m0 + row < M ? m0 + row : M - 1;
        const int64_t n = n0 + (L & 3) * 64 < N ? n0 + (L & 3) * 64 : n0;
        pfd[j] = *(const __attribute__((address_space(1))) uint16_t*)(uintptr_t)(gb + m * ep.ldg + n);
      }
    }
    rp_raw_barrier();
    rp_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb0[j][kk], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    rp_raw_barrier();
    // ---- phase 1: B columns 32-63 ----
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb1[j][kk] = rb(bi, 2 + j, kk * 32);
    rp_raw_barrier();
    rp_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb1[j][kk], acc[i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    rp_raw_barrier();
    // ---- phase 2: A rows 64-127 ----
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = ra(ai, 4 + i, kk * 32);
    rp_raw_barrier();
    rp_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb1[j][kk], acc[4 + i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    rp_raw_barrier();
    // ---- phase 3: no fragment reads; B pieces of K-tile kt+2; own pieces of K-tile kt+1 landed by its end ----
    if (want_bias) {  // wgrad bias: column sums of the staged m-major dY tile, 4 x 16 B per thread
      const char* hi = cur + (tid >> 8) * G::HB;
      const int cg = tid & 15;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = ((tid >> 4) & 15) + 16 * j;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(hi + k * 256 + mswz(k, cg) * 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) bacc[e] += (float)v[e];
      }
      rp_lgkm0();  // retired before the barrier after which the next A pieces may overwrite them
    }
    if (kt + 2 < nk) fill_b(kt + 2);
    // every wave's pieces of K-tile kt+1 must have landed by barrier event 8kt+8 (G0's clock), after
    // which the leading half reads K-tile kt+1.  That event is the leading half's LAST barrier of
    // this K-tile but the lagging half's FIRST barrier of this phase: the lagging half waits here,
    // the leading half after this phase's MFMA segment (which gives its fills that segment too)
    auto wait_next = [&]() {
      if (kt + 2 < nk)
        rp_waitcnt<4, 15>();  // only B(kt+2) may stay in flight
      else if (pf)
        rp_waitcnt<2, 15>();  // every fill landed; the two gate loads may stay in flight
      else
        rp_waitcnt<0, 15>();
    };
    if (wm == 1) wait_next();
    rp_raw_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb0[j][kk], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (wm == 0) wait_next();
    rp_raw_barrier();
  }
  if (wm == 0) rp_raw_barrier();  // match the lagging half's barrier count
  __syncthreads();
#ifdef RP_GEMM_PROBE
  const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();
#endif
  gemm8_epilogue<TC, MODE, BNT, GATEB>(acc, lds, tid, lane, wm, wn, m0, n0, M, N, Cout, ldc, alpha, ep, split);
  if (pf) asm volatile("" ::"v"(pfd[0]), "v"(pfd[1]));
#ifdef RP_GEMM_PROBE
  {  // tuning build only: per-workgroup phase stamps (start, main loop done, epilogue issued, drained)
    const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t ts3 = __builtin_amdgcn_s_memrealtime();
    const int bid = blockIdx.x + blockIdx.y * gridDim.x;
    if (tid < 4 && bid < RP_PROBE_MAX)
      g_gemm_probe[bid * 4 + tid] = tid == 0 ? ts0 : tid == 1 ? ts1 : tid == 2 ? ts2 : ts3;
  }
#endif
  if (want_bias) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bacc[j];
    __syncthreads();
    if (tid < 256 && m0 + tid < M) {
      const int h = tid >> 7, cg = (tid & 127) >> 3, e = tid & 7;
      float sum = 0.f;
      for (int r = 0; r < 16; ++r) sum += red[((h << 8) + cg + 16 * r) * 8 + e];
      bias_dst[m0 + tid] = bias_acc ? bias_dst[m0 + tid] + sum : sum;
    }
  }
}

template <bool AK, bool BKM, typename TC, int MODE, int BNT, bool GATEB = false>
__global__ __launch_bounds__(NT8, 2) void gemm8_kernel(int64_t M, int64_t N, int64_t K, const bf16* __restrict__ A,
                                                       int64_t lda, const bf16* __restrict__ B, int64_t ldb,
                                                       TC* __restrict__ Cout, int64_t ldc, float alpha, EpiDev ep,
                                                       int64_t kchunk, float* __restrict__ bslab) {
  __shared__ __attribute__((aligned(16))) char lds[G8<BNT, 64, 2>::LDS];
  const int tiles_n = (int)((N + BNT - 1) / BNT);
  const int tiles_m = (int)((M + 255) / 256);
  int t, split;
  tile_split<MODE>(tiles_m * tiles_n, ep.split_major, t, split);
  const int64_t m0 = (int64_t)(t / tiles_n) * 256;
  const int64_t n0 = (int64_t)(t % tiles_n) * BNT;
  int64_t kbeg = 0, kend = K;
  if (MODE == 1) {
    kbeg = (int64_t)split * kchunk;
    kend = kbeg + kchunk < K ? kbeg + kchunk : K;
  }
  float* bias_dst = (MODE == 1 && bslab != nullptr && n0 == 0) ? bslab + (int64_t)split * M : nullptr;
  gemm8_tile<AK, BKM, TC, MODE, BNT, GATEB>(M, N, A, lda, B, ldb, Cout, ldc, alpha, ep, kbeg, kend, m0, n0, split,
                                            bias_dst, 0, lds);
}

// grouped weight gradients on 256 x 256 tiles (a WgGroup, every tile over the whole K): twice
// the MFMA work per staged operand byte of the 128 x 128 tile, which the whole-K L2 -> LDS stream of
// the grouped launch is bound by; one workgroup of 8 waves per CU
__global__ __launch_bounds__(NT8, 1) void wgrad8_grouped_kernel(const WgGroup g) {
  __shared__ __attribute__((aligned(16))) char lds[G8<256, 64, 2>::LDS];
  const int t = g.order == 2 ? (int)blockIdx.x : rp_xcd_remap(blockIdx.x, g.tiles_total);
  int k = 0;
  while (k + 1 < g.n && t >= g.start[k + 1]) ++k;
  const WgItem w = g.it[k];
  const int local = t - g.start[k];
  const int tiles_n = (w.N + 255) / 256, tiles_m = (w.M + 255) / 256;
  const int64_t m0 = (int64_t)(g.order == 1 ? local % tiles_m : local / tiles_n) * 256;
  const int64_t n0 = (int64_t)(g.order == 1 ? local / tiles_m : local % tiles_n) * 256;
  EpiDev ep{};
  ep.gate_scale = 1.f;
  ep.accumulate = g.accumulate;
  ep.st_pol = g.st_pol;
  gemm8_tile<false, false, float, 0, 256>(w.M, w.N, w.dY, w.ldy, w.X, w.ldx, w.dW, w.N, 1.f, ep, 0, g.K, m0, n0, 0,
                                          n0 == 0 ? w.db : nullptr, g.accumulate, lds);
}

// compute units of the current device (cached per device); the tile-shape rules below count workgroups
// per CU in units of it (256 on a whole MI355X)
static int64_t gemm_cu_count() {
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

// 256-row phased path selection.  RP_GEMM8=0 disables it, RP_GEMM8=1 forces it wherever legal
// (read per call: scripts/gemm_ab.py switches it between launches).  Default: the wide short-K
// shapes with at least one 256 x 256 tile per CU (MI355X, M = 16384: linear1 forward 54.6 ->
// 48.9 us, the K = 512 dgrad into d_ff 61.0 -> 50.1 us); N = 512 shapes have only 128 tiles, and
// N = 1536 ones 1.5 tiles per CU.
static int rp_gemm8_mode() {
  const char* e = getenv("RP_GEMM8");
  return e ? (e[0] == '0' ? 0 : (e[0] == '1' ? 1 : -1)) : -1;
}
static int rp_gemm8_bn(int64_t M, int64_t N, int64_t kext) {
  if (kext % 64 != 0 || kext < 128 || M < 256 || N % 8 != 0) return 0;
  const int mode = rp_gemm8_mode();
  if (mode == 0) return 0;
  if (mode == 1) return 256;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  return (N >= 2048 && kext <= 1024 && tiles >= gemm_cu_count()) ? 256 : 0;
}

// dst[i] (+)= sum_s slab[s][i] in fixed slab order (deterministic), for the weight slabs (n
// elements) and, in the same launch, the bias slabs (n2 elements, blocks past nb1).  Four slab
// loads in flight per step.
__device__ __forceinline__ void splitk_sum4(const float* __restrict__ slab, int S, int64_t n, int64_t i,
                                            float* __restrict__ dst, int accumulate) {
  float4 acc = accumulate ? reinterpret_cast<const float4*>(dst)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* p = reinterpret_cast<const float4*>(slab) + i;
  const int64_t st = n / 4;
  int s = 0;
  for (; s + 4 <= S; s += 4) {
    const float4 a = p[(int64_t)s * st], b = p[(int64_t)(s + 1) * st], c = p[(int64_t)(s + 2) * st],
                 d = p[(int64_t)(s + 3) * st];
    acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
    acc.x += c.x; acc.y += c.y; acc.z += c.z; acc.w += c.w;
    acc.x += d.x; acc.y += d.y; acc.z += d.z; acc.w += d.w;
  }
  for (; s < S; ++s) {
    const float4 a = p[(int64_t)s * st];
    acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
  }
  reinterpret_cast<float4*>(dst)[i] = acc;
}

__global__ void splitk_reduce_kernel(const float* __restrict__ slab, int S, int64_t n, float* __restrict__ dst,
                                     const float* __restrict__ slab2, int64_t n2, float* __restrict__ dst2,
                                     int nb1, int accumulate) {
  // n, n2 are multiples of 4 (M, N multiples of 8)
  if ((int)blockIdx.x < nb1) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += (int64_t)nb1 * blockDim.x)
      splitk_sum4(slab, S, n, i, dst, accumulate);
  } else {
    const int64_t i = (int64_t)(blockIdx.x - nb1) * blockDim.x + threadIdx.x;
    if (i < n2 / 4) splitk_sum4(slab2, S, n2, i, dst2, accumulate);
  }
}

#define RP_GEMM_LAUNCH(AKV, BKV, MODEV, GRID)                                                              \
  hipLaunchKernelGGL((gemm_kernel<T, AKV, BKV, TC, MODEV>), GRID, dim3(NT), 0, s, M, N, K, a, lda, b, ldb, c, \
                     ldc, alpha, ep, kchunk, bslab)

// DMA kernel configuration for a K extent (per split): 2 for K % 64 == 32; configuration 1 (one stage,
// four workgroups per CU) for short-K wide shapes where the 128 x 128 grid exceeds two workgroups per CU
// (the metric shape's QKV forward: 15.46 -> 15.66 ms per step with configuration 0 everywhere); at fewer
// (config 4, M = 4096: the QKV forward's 384 and the d_ff = 2048 shapes' 512 tiles) configuration 0 —
// which also opens the 64-row tiles to the QKV forward — measured 7.08 / 7.07 -> 6.93 / 6.97 ms per step.
static int rp_gemm_cfg(int64_t kext, int64_t n, int64_t m) {
  if (kext % 64 != 0) return 2;
  const int64_t tiles = ((m + BM - 1) / BM) * ((n + BN - 1) / BN);
  return (kext <= 1024 && n >= 1536 && tiles > 2 * gemm_cu_count()) ? 1 : 0;
}


// the GEMM epilogues' output stores non-temporal (policy 2; plain 15.47, sc1 write-through 15.26 vs nt
// 15.08 ms per step), their fp32 residual loads too (-0.09 ms per step: the residual
// stream is next read in the backward)
static int rp_store_policy() { return 2; }
static int rp_residual_load_policy() { return 2; }

template <typename TC>
int launch_gemm8(int bn, int64_t M, int64_t N, int64_t K, const bf16* a, int64_t lda, int ak, const bf16* b,
                 int64_t ldb, int bk, TC* c, int64_t ldc, float alpha, const EpiDev& ep, hipStream_t s, int splits,
                 int64_t kchunk, float* bslab) {
  const int64_t tiles = ((M + 255) / 256) * ((N + bn - 1) / bn);
#define RP_G8_LAUNCH1(AKV, BKV, MODEV, BNV, GRID)                                                            \
  hipLaunchKernelGGL((gemm8_kernel<AKV, BKV, TC, MODEV, 256>), GRID, dim3(NT8), 0, s, M, N, K, a, lda, b, ldb, c, \
                     ldc, alpha, ep, kchunk, bslab)
#define RP_G8_LAUNCH(AKV, BKV, MODEV, GRID) RP_G8_LAUNCH1(AKV, BKV, MODEV, 256, GRID)
  if constexpr (!std::is_same<TC, float>::value) {
    if (splits == 0 && ak && !bk && ep.gate && ep.gate_bf16) {  // the linear2 dgrad: see GATEB
      hipLaunchKernelGGL((gemm8_kernel<true, false, TC, 0, 256, true>), dim3((unsigned)tiles), dim3(NT8), 0, s, M, N, K,
                         a, lda, b, ldb, c, ldc, alpha, ep, kchunk, bslab);
      return rp_check_launch("rp_gemm");
    }
  }
  if (splits == 0) {
    dim3 grid((unsigned)tiles);
    if (ak && bk) RP_G8_LAUNCH(true, true, 0, grid);
    else if (ak && !bk) RP_G8_LAUNCH(true, false, 0, grid);
    else if (!ak && !bk) RP_G8_LAUNCH(false, false, 0, grid);
    else RP_G8_LAUNCH(false, true, 0, grid);
  } else {
    dim3 grid((unsigned)tiles, (unsigned)splits);
    RP_G8_LAUNCH(false, false, 1, grid);  // split-K serves the wgrad layout only
  }
#undef RP_G8_LAUNCH
#undef RP_G8_LAUNCH1
  return rp_check_launch("rp_gemm");
}

// 64 x 128 tiles (k-major A, two-stage K = 64 configuration) where the grid of 128 x 128 tiles gives
// fewer than two workgroups per CU: config 4 (M = 4096) has 128 such tiles on its d_model = 512 GEMMs
// (half the CUs idle; step 7.92 -> 7.60 ms), config 2 (M = 8192) 256 (7.95 -> 7.66 ms).  RP_GEMM_BM64=0
// never, =1 wherever legal (tests, A/B), unset: fewer 128 x 128 tiles than twice the CUs.  Per call.
// RP_GEMM_GATEB=0 (A/B, read per call): the gated bf16 dgrads on the per-chunk epilogue
static bool rp_gate_batch() {
  const char* e = getenv("RP_GEMM_GATEB");
  return !(e && e[0] == '0');
}

static bool rp_gemm_bm64(int64_t M, int64_t N) {
  const char* e = getenv("RP_GEMM_BM64");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return ((M + BM - 1) / BM) * ((N + BN - 1) / BN) < 2 * gemm_cu_count();
}

// 32 x 128 tiles (each wave 16 x 64; the same K order per output element, so bitwise the 64- and
// 128-row kernels) where even the 64 x 128 grid gives fewer than two workgroups per CU: config 4's
// d_model = 512 GEMMs (M = 4096: 256 -> 512 tiles; step 7.36 -> 7.17 ms).  RP_GEMM_BM32=0 never, =1
// wherever the 64-row tiles run (tests, A/B), unset: fewer 64 x 128 tiles than twice the CUs.  Per call.
static bool rp_gemm_bm32(int64_t M, int64_t N) {
  const char* e = getenv("RP_GEMM_BM32");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return ((M + 63) / 64) * ((N + BN - 1) / BN) < 2 * gemm_cu_count();
}

template <typename T, typename TC>
int launch_gemm_t(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, int ak, const void* B,
                  int64_t ldb, int bk, void* Cp, int64_t ldc, float alpha, const EpiDev& ep,
                  hipStream_t s, int splits = 0, int64_t kchunk = 0, float* bslab = nullptr) {
  int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  TC* c = (TC*)Cp;
  if constexpr (std::is_same<T, bf16>::value) {
    const int bn8 = splits == 0 ? rp_gemm8_bn(M, N, K) : 0;
    if (bn8 > 0)
      return launch_gemm8<TC>(bn8, M, N, K, (const bf16*)A, lda, ak, (const bf16*)B, ldb, bk, c, ldc, alpha, ep, s,
                              splits, kchunk, bslab);
    const bool full_k = K % 32 == 0 && (splits == 0 || kchunk % 32 == 0);
    if (full_k) {
      const int cfg = rp_gemm_cfg(splits == 0 ? K : kchunk, N, M);
      const bf16* ab = (const bf16*)A;
      const bf16* bb = (const bf16*)B;
#define RP_DMA_LAUNCH1(AKV, BKV, MODEV, CFGV, GRID)                                                        \
  hipLaunchKernelGGL((gemm_bf16_dma_kernel<AKV, BKV, TC, MODEV, CFGV>), GRID, dim3(NT), 0, s, M, N, K, ab, lda, \
                     bb, ldb, c, ldc, alpha, ep, kchunk, bslab)
#define RP_DMA_LAUNCH(AKV, BKV, MODEV, GRID)                                  \
  do {                                                                        \
    switch (cfg) {                                                            \
      case 0: RP_DMA_LAUNCH1(AKV, BKV, MODEV, 0, GRID); break;                \
      case 1: RP_DMA_LAUNCH1(AKV, BKV, MODEV, 1, GRID); break;                \
      default: RP_DMA_LAUNCH1(AKV, BKV, MODEV, 2, GRID); break;               \
    }                                                                         \
  } while (0)
      // bf16 C gated by a bf16 tensor, nothing else read (the d_ff dgrad): the gate-batched epilogue
      bool gateb = false;
      if constexpr (std::is_same<TC, bf16>::value)
        gateb = splits == 0 && ak && !bk && ep.gate && ep.gate_bf16 && !ep.residual && !ep.delta && !ep.accumulate &&
                rp_gate_batch();
      if (splits == 0 && ak && cfg == 0 && rp_gemm_bm64(M, N) && rp_gemm_bm32(M, N)) {  // 32 x 128 tiles
        const dim3 grid((unsigned)(((M + 31) / 32) * ((N + BN - 1) / BN)));
        bool done = false;
        if constexpr (std::is_same<TC, float>::value) {
          if (bk && ep.residual) {
            hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 0, true, 1>), grid, dim3(NT), 0, s, M, N, K,
                               ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
            done = true;
          }
        } else if (gateb) {
          hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 0, true, 1>), grid, dim3(NT), 0, s, M, N, K, ab,
                             lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
          done = true;
        }
        if (!done) {
          if (bk)
            hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 0, false, 1>), grid, dim3(NT), 0, s, M, N, K,
                               ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
          else
            hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 0, false, 1>), grid, dim3(NT), 0, s, M, N, K,
                               ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
        }
        return rp_check_launch("rp_gemm");
      }
      if (splits == 0 && ak && cfg == 0 && rp_gemm_bm64(M, N)) {
        const dim3 grid((unsigned)(((M + 63) / 64) * ((N + BN - 1) / BN)));
        bool done = false;
        if constexpr (std::is_same<TC, float>::value) {
          if (bk && ep.residual) {
            hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 0, true, 2>), grid, dim3(NT), 0, s, M, N, K,
                               ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
            done = true;
          }
        } else if (gateb) {
          hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 0, true, 2>), grid, dim3(NT), 0, s, M, N, K, ab,
                             lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
          done = true;
        }
        if (!done) {
          if (bk)
            hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 0, false, 2>), grid, dim3(NT), 0, s, M, N, K,
                               ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
          else
            hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 0, false, 2>), grid, dim3(NT), 0, s, M, N, K,
                               ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab);
        }
        return rp_check_launch("rp_gemm");
      }
      if constexpr (std::is_same<TC, float>::value) {
        if (splits == 0 && ak && bk && ep.residual) {  // the residual (fp32) forward shapes: see RESB
          dim3 grid((unsigned)tiles);
          switch (cfg) {
            case 0: hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 0, true>), grid, dim3(NT), 0, s, M, N, K, ab,
                                       lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab); break;
            case 1: hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 1, true>), grid, dim3(NT), 0, s, M, N, K, ab,
                                       lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab); break;
            default: hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, true, TC, 0, 2, true>), grid, dim3(NT), 0, s, M, N, K,
                                        ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab); break;
          }
          return rp_check_launch("rp_gemm");
        }
      }
      if (gateb) {
        dim3 grid((unsigned)tiles);
        switch (cfg) {
          case 0: hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 0, true>), grid, dim3(NT), 0, s, M, N, K, ab,
                                     lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab); break;
          case 1: hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 1, true>), grid, dim3(NT), 0, s, M, N, K, ab,
                                     lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab); break;
          default: hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, TC, 0, 2, true>), grid, dim3(NT), 0, s, M, N, K,
                                      ab, lda, bb, ldb, c, ldc, alpha, ep, kchunk, bslab); break;
        }
        return rp_check_launch("rp_gemm");
      }
      if (splits == 0) {
        dim3 grid((unsigned)tiles);
        if (ak && bk) RP_DMA_LAUNCH(true, true, 0, grid);
        else if (ak && !bk) RP_DMA_LAUNCH(true, false, 0, grid);
        else if (!ak && !bk) RP_DMA_LAUNCH(false, false, 0, grid);
        else RP_DMA_LAUNCH(false, true, 0, grid);
      } else {
        dim3 grid((unsigned)tiles, (unsigned)splits);
        if (ak && bk) RP_DMA_LAUNCH(true, true, 1, grid);
        else if (ak && !bk) RP_DMA_LAUNCH(true, false, 1, grid);
        else if (!ak && !bk) RP_DMA_LAUNCH(false, false, 1, grid);
        else RP_DMA_LAUNCH(false, true, 1, grid);
      }
#undef RP_DMA_LAUNCH
#undef RP_DMA_LAUNCH1
      return rp_check_launch("rp_gemm");
    }
  }
  if (splits == 0) {
    dim3 grid((unsigned)tiles);
    if (ak && bk) RP_GEMM_LAUNCH(true, true, 0, grid);
    else if (ak && !bk) RP_GEMM_LAUNCH(true, false, 0, grid);
    else if (!ak && !bk) RP_GEMM_LAUNCH(false, false, 0, grid);
    else RP_GEMM_LAUNCH(false, true, 0, grid);
  } else {
    dim3 grid((unsigned)tiles, (unsigned)splits);
    if (ak && bk) RP_GEMM_LAUNCH(true, true, 1, grid);
    else if (ak && !bk) RP_GEMM_LAUNCH(true, false, 1, grid);
    else if (!ak && !bk) RP_GEMM_LAUNCH(false, false, 1, grid);
    else RP_GEMM_LAUNCH(false, true, 1, grid);
  }
  return rp_check_launch("rp_gemm");
}

// split count for the wgrad shape (tokens are the reduction): aim at ~2 workgroups per CU,
// each split at least 8 K-steps long
void wgrad_plan(int64_t M, int64_t N, int64_t K, int bk, int& splits, int64_t& kchunk) {
  if (K <= 0) {
    splits = 1;
    kchunk = bk;
    return;
  }
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int64_t target = 512;  // workgroups to aim at (256 / 384 / 768 / 1024 measured slower)
  int64_t sp = target / (tiles > 0 ? tiles : 1);
  const int64_t maxsp = K / (8 * bk);
  if (sp > maxsp) sp = maxsp;
  if (sp < 1) sp = 1;
  kchunk = ((K + sp - 1) / sp + bk - 1) / bk * bk;
  splits = (int)((K + kchunk - 1) / kchunk);
  if (splits < 1) splits = 1;
}

// the 256 x 256 phased kernel's wgrad plan (only under RP_GEMM8=1): ~one workgroup per CU, splits of whole 64-deep K-tiles, at least 8 per split; returns 0
// when the 128 x 128 kernel runs.  Measured (scripts/gemm_ab.py, M = 16384, split-major mapping on
// both): 46.0 / 31.2 / 53.2 / 53.4 / 67.3 us for the qkv / out_proj / linear1 / linear2 / input
// projection weight gradients against 40.9 / 23.9 / 49.2 / 47.5 / 68.1 us on the 128 x 128 kernel
// at two workgroups per CU — the m-major x m-major fragment reads (two transposed reads each) and
// the 16-32 x larger fp32 slabs per tile cost more than the tile's operand reuse gains.
int wgrad8_plan(int64_t M, int64_t N, int64_t K, int& splits, int64_t& kchunk) {
  const int mode = rp_gemm8_mode();
  if (mode != 1 || K % 64 != 0 || K < 512 || M < 256) return 0;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int64_t target = 256;
  int64_t sp = target / tiles;
  const int64_t maxsp = K / (8 * 64);
  if (sp > maxsp) sp = maxsp;
  if (sp < 1) sp = 1;
  kchunk = ((K + sp - 1) / sp + 63) / 64 * 64;
  splits = (int)((K + kchunk - 1) / kchunk);
  return 256;
}


// ============== GEMM + LayerNorm with full-row tiles (d_model = 512 output columns) ==============
// The four N = 512 GEMMs of an encoder layer feed a LayerNorm (reference: the pre-LN encoder layer
// built at models/MMCTransformer.py:41-55 — x1 = x + drop(out_proj(.)), norm2(x1); x2 = x1 +
// drop(linear2(.)), next layer's norm1(x2) / encoder_norm; and their backward).  With 128 x 128 tiles
// the GEMM wrote the fp32 rows and a separate LayerNorm pass read them back (33.5 MB each way per
// launch at M = 16384), and the LayerNorm backward read the fp32 dgrad output back the same way.
// Here one workgroup owns 64 WHOLE rows (64 x 512 outputs, 8 waves, wave w the 64 columns
// [64w, 64w + 64)), so the LayerNorm runs in the GEMM's epilogue on rows staged in LDS:
//   fwd: x_out = dropout(A W^T + bias) + residual (fp32, the residual stream), h = LN(x_out) (bf16),
//        mean / rstd saved — the arithmetic of gemm_epilogue followed by ln_fwd_kernel<8>, op for op;
//   bwd: dh = dY W (kept in LDS, never written), then ln_bwd_kernel<8>'s row loop on it (dx fp32 with
//        the residual gradient added, the dropout-masked bf16 copy for the next GEMM, gamma / beta
//        partials per 32-row block in that kernel's order and layout).
// The MFMA products are the 128 x 128 kernel's (16x16x32 bf16, K in 64-deep steps, k ascending), so
// every output is bitwise the unfused pair's.  Main loop: two LDS stages of (A 64 x 64, B 512 x 64)
// = 72 KiB each, one barrier per K step, one workgroup per CU (256 row blocks at M = 16384).
constexpr int GL_BM = 64, GL_N = 512, GL_NT = 512, GL_BK = 64;
constexpr int GL_AB = GL_BM * GL_BK * 2;  // A image of a stage (8 KiB)
constexpr int GL_BB = GL_N * GL_BK * 2;   // B image(s) of a stage (64 KiB)
constexpr int GL_STAGE = GL_AB + GL_BB;
constexpr int GL_CST = GL_N + 4;          // fp32 row stride of the staged output rows
constexpr int GL_LDS = 2 * GL_STAGE;
static_assert(GL_BM * GL_CST * 4 <= GL_LDS, "staged rows fit the main-loop LDS");

struct GlnDev {
  const bf16* A; int64_t lda;
  const bf16* W; int64_t ldw;  // fwd: W [512][K] (k-major, nn.Linear weight); bwd: W [K][512] (n-major)
  const float* bias;
  uint32_t drop_thresh; float drop_scale; uint32_t drop_seed; const uint32_t* seed_base;
  const float* residual; int64_t ldr;
  float* xo; int64_t ldxo;
  const float* gamma; const float* beta; float eps;
  bf16* h; int64_t ldh;
  float* mean; float* rstd;
  const float* x; int64_t ldx;
  const float* dres; int64_t lddres;
  float* dx; int64_t lddx;
  bf16* dx_lp; int64_t lddx_lp; uint32_t lp_thresh; float lp_scale; uint32_t lp_seed;
  float* dgamma_part; float* dbeta_part; int64_t ld_part;
};

// Main loop: a four-slot ring of 32-deep K steps (A 64 x 32 = 4 KiB, B 512 x 32 = 32 KiB per slot),
// three steps in flight (the DMA of step t + 3 goes into the slot step t - 1 read, issued right after
// the barrier that ends those reads), counted s_waitcnt vmcnt + raw barrier per step.  A two-stage
// 64-deep version with a full drain per step measured slower than the unfused pair at K = 2048 (one
// workgroup per CU cannot hide a 72 KiB fill per step): this one keeps ~108 KiB in flight per CU.
// Pieces per slot: A 4 (waves 0-3), B 32 (four per wave) -> 5 DMA instructions for waves 0-3, 4 for 4-7.
constexpr int GL_KS = 32;                    // K per ring slot
constexpr int GL_SA = GL_BM * GL_KS * 2;     // A image of a slot (4 KiB)
constexpr int GL_SLOT = GL_SA + GL_N * GL_KS * 2;
constexpr int GL_RING = 4;
static_assert(GL_RING * GL_SLOT <= GL_LDS, "ring fits");

template <bool BKM>
__device__ __forceinline__ void gln_issue(const GlnDev& a, int64_t m0, int64_t k0, uint32_t slot, int w, int lane) {
  if (w < 4) {  // A: [64 rows][32 k], 64-B rows, kswz32
    const int r = w * 16 + (lane >> 2);
    rp_dma16(a.A + (m0 + r) * a.lda + k0 + kswz32(r, lane & 3) * 8, slot + w * 1024);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int I = w * 4 + j;
    const bf16* src;
    if constexpr (BKM) {  // [512 rows][32 k], 64-B rows, kswz32
      const int r = I * 16 + (lane >> 2);
      src = a.W + (int64_t)r * a.ldw + k0 + kswz32(r, lane & 3) * 8;
    } else {  // four [32 k][128 cols] images (8 KiB), 256-B rows, mswz
      const int k = (I & 7) * 4 + (lane >> 4);
      src = a.W + (k0 + k) * a.ldw + (I >> 3) * 128 + mswz(k, lane & 15) * 8;
    }
    rp_dma16(src, slot + GL_SA + I * 1024);
  }
}

// acc[i][j][r] = C[m0 + 16 i + 4 g + r][64 w + 16 j + c] over the whole K
template <bool BKM>
__device__ __forceinline__ void gln_mainloop(const GlnDev& a, int64_t m0, int64_t K, char* lds, f32x4 (&acc)[4][4],
                                             int w, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (int)(K / GL_KS);
  const uint32_t base = rp_lds_addr(lds);
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (t < nk) gln_issue<BKM>(a, m0, (int64_t)t * GL_KS, base + t * GL_SLOT, w, lane);
  for (int t = 0; t < nk; ++t) {
    // DMA instructions issued after step t's: those of steps t+1, t+2 (if they exist)
    const int after = (nk - 1 - t) < 2 ? (nk - 1 - t) : 2;
    if (w < 4) {
      if (after == 2) rp_waitcnt<10, 15>(); else if (after == 1) rp_waitcnt<5, 15>(); else rp_waitcnt<0, 15>();
    } else {
      if (after == 2) rp_waitcnt<8, 15>(); else if (after == 1) rp_waitcnt<4, 15>(); else rp_waitcnt<0, 15>();
    }
    rp_raw_barrier();
    if (t + 3 < nk) gln_issue<BKM>(a, m0, (int64_t)(t + 3) * GL_KS, base + ((t + 3) & 3) * GL_SLOT, w, lane);
    const char* cur = lds + (t & 3) * GL_SLOT;
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag_k_swz<32>(cur, i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = BKM ? frag_k_swz<32>(cur + GL_SA, 64 * w + 16 * j, 0, lane)
                   : frag_m_swz(cur + GL_SA + (w >> 1) * 8192, (w & 1) * 64 + 16 * j, 0, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // every wave's reads of the ring are done before the epilogue reuses the LDS
}

__device__ __forceinline__ void gln_stage(const f32x4 (&acc)[4][4], float* cs, int w, int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[(i * 16 + g * 4 + r) * GL_CST + 64 * w + j * 16 + c] = acc[i][j][r];
}

__device__ __forceinline__ void ld8(float (&v)[8], const float* p) {
  const float4 q0 = *reinterpret_cast<const float4*>(p), q1 = *reinterpret_cast<const float4*>(p + 4);
  v[0] = q0.x; v[1] = q0.y; v[2] = q0.z; v[3] = q0.w; v[4] = q1.x; v[5] = q1.y; v[6] = q1.z; v[7] = q1.w;
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void st8bf(bf16* p, const float (&v)[8]) {
  uint4 q;
  bf16* e = reinterpret_cast<bf16*>(&q);
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = (bf16)v[j];
  *reinterpret_cast<uint4*>(p) = q;
}

__global__ __launch_bounds__(GL_NT, 1) void gemm_ln_fwd_kernel(int64_t M, int64_t K, const GlnDev a) {
  __shared__ __attribute__((aligned(1024))) char lds[GL_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * GL_BM;
  f32x4 acc[4][4];
  gln_mainloop<true>(a, m0, K, lds, acc, w, lane);
  // this wave's rows w*8 .. w*8+7, lane l holds columns 8l .. 8l+7 (ln_fwd_kernel<8>'s layout)
  const int c0 = lane * 8;
  float res[8][8];
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) ld8(res[rr], a.residual + (m0 + w * 8 + rr) * a.ldr + c0);
  float bi[8], gm[8], bt[8];
  ld8(bi, a.bias + c0);
  ld8(gm, a.gamma + c0);
  ld8(bt, a.beta + c0);
  float* cs = reinterpret_cast<float*>(lds);
  gln_stage(acc, cs, w, lane);
  __syncthreads();
  const uint32_t dseed = a.drop_thresh ? rp_seed_eff(a.seed_base, a.drop_seed) : 0u;
#pragma unroll 2
  for (int rr = 0; rr < 8; ++rr) {
    const int row = w * 8 + rr;
    const int64_t m = m0 + row;
    float v[8];
    ld8(v, cs + row * GL_CST + c0);
    // gemm_epilogue (MODE 0, fp32 C): alpha (1) * acc + bias, dropout, + residual
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bi[e];
    if (a.drop_thresh) {
      const uint32_t kb = rp_keep_bits<8>(dseed, (uint32_t)(m * GL_N + c0), a.drop_thresh);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((kb >> e) & 1u) ? v[e] * a.drop_scale : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += res[rr][e];
    st8(a.xo + m * a.ldxo + c0, v);
    // ln_fwd_kernel<8>
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    const float mean = rp_wave_sum(s) * (1.f / GL_N);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = v[i] - mean;
      q += d * d;
    }
    const float var = rp_wave_sum(q) * (1.f / GL_N);
    const float rstd = rsqrtf(var + a.eps);
    float y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = (v[i] - mean) * rstd * gm[i] + bt[i];
    st8bf(a.h + m * a.ldh + c0, y);
    if (lane == 0) {
      a.mean[m] = mean;
      a.rstd[m] = rstd;
    }
  }
}

__global__ __launch_bounds__(GL_NT, 1) void gemm_ln_bwd_kernel(int64_t M, int64_t K, const GlnDev a) {
  __shared__ __attribute__((aligned(1024))) char lds[GL_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * GL_BM;
  f32x4 acc[4][4];
  gln_mainloop<false>(a, m0, K, lds, acc, w, lane);
  const int c0 = lane * 8;
  float gam[8];
  ld8(gam, a.gamma + c0);
  float* cs = reinterpret_cast<float*>(lds);
  gln_stage(acc, cs, w, lane);
  __syncthreads();
  const uint32_t lseed = a.lp_thresh ? rp_seed_eff(a.seed_base, a.lp_seed) : 0u;
  // ln_bwd_kernel<8>, one 32-row block at a time (its rows w, w+8, w+16, w+24 per wave, in that order)
#pragma unroll 1
  for (int blk = 0; blk < 2; ++blk) {
    float pg[8], pb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) pg[i] = pb[i] = 0.f;
#pragma unroll 1
    for (int rr = w; rr < 32; rr += 8) {
      const int row = blk * 32 + rr;
      const int64_t m = m0 + row;
      float g[8], x[8], r[8];
      ld8(x, a.x + m * a.ldx + c0);
      if (a.dres) ld8(r, a.dres + m * a.lddres + c0);
      ld8(g, cs + row * GL_CST + c0);
      const float mu = a.mean[m], rs = a.rstd[m];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        x[i] = (x[i] - mu) * rs;
        const float gg = g[i] * gam[i];
        s1 += gg;
        s2 += gg * x[i];
        pg[i] += g[i] * x[i];
        pb[i] += g[i];
      }
      s1 = rp_wave_sum(s1) * (1.f / GL_N);
      s2 = rp_wave_sum(s2) * (1.f / GL_N);
      float dx[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) dx[i] = rs * (g[i] * gam[i] - s1 - x[i] * s2);
      if (a.dres) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dx[i] += r[i];
      }
      st8(a.dx + m * a.lddx + c0, dx);
      if (a.dx_lp) {
        if (a.lp_thresh) {
          const uint32_t kb = rp_keep_bits<8>(lseed, (uint32_t)(m * GL_N + c0), a.lp_thresh);
#pragma unroll
          for (int i = 0; i < 8; ++i) dx[i] = ((kb >> i) & 1u) ? dx[i] * a.lp_scale : 0.f;
        }
        st8bf(a.dx_lp + m * a.lddx_lp + c0, dx);
      }
    }
    // the block's gamma / beta partial row (rows 0..31 of the staging area are consumed by now)
    __syncthreads();
    float* red = cs;  // [2][8 waves][512]
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(0 * 8 + w) * GL_N + c0 + i] = pg[i];
      red[(1 * 8 + w) * GL_N + c0 + i] = pb[i];
    }
    __syncthreads();
    {
      const int c = tid;  // GL_NT == GL_N: one column per thread
      float sg = 0.f, sb = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sg += red[(0 * 8 + k) * GL_N + c];
        sb += red[(1 * 8 + k) * GL_N + c];
      }
      const int64_t pr = m0 / 32 + blk;
      if (a.dgamma_part) a.dgamma_part[pr * a.ld_part + c] = sg;
      if (a.dbeta_part) a.dbeta_part[pr * a.ld_part + c] = sb;
    }
    __syncthreads();
  }
}

// ======= GEMM + LayerNorm on 128 x 128 tiles: row statistics exchanged between the column tiles =======
// The 64 x 512 full-row kernels above keep a row in one workgroup but stream the whole weight per 64 rows
// at one workgroup per CU.  These keep the 128 x 128 LDS-DMA GEMM (dma_mainloop, two workgroups per CU),
// and the four column tiles of a 128-row block trade per-row partial statistics through a small global
// workspace (rp_gemm_ln_xchg_bytes):
//   fwd: per row (sum, M2 about the tile's own mean) of x_out over the tile's 128 columns, combined as a
//        parallel variance: mean = sum / 512, M2 = sum_k M2_k + 128 (mean_k - mean)^2, var = M2 / 512;
//   bwd: per row (sum g gamma, sum g gamma xhat) over the tile's columns (ln_bwd_kernel's s1, s2).
// Protocol (cdna_hip_programming.md §6 Guideline 16, recipe R1): the payload stored write-through (sc1)
// and drained by every storing wave, a barrier, one relaxed agent-scope arrive add per workgroup, one
// polling lane (relaxed agent-scope loads + s_sleep, bounded in time: a wait that gives up sets the
// workspace's error word and the library's host-mapped fault word, which every later rp_gemm_ln_* call
// and rp_gemm_ln_status() report as RP_ERR_LAUNCH until rp_gemm_ln_reset), a barrier; the partners'
// payload read back with sc1 loads only.  The last of the four to finish reading resets the row block's
// counters, so each launch starts from and leaves a zeroed workspace.
// Forward progress (co-residency rule): the host splits a seam into launches whose grid is
// at most the co-resident capacity (CUs x workgroups per CU, from the occupancy query, at most 2), so
// every workgroup of a launch is resident at once, or becomes resident as soon as other streams' kernels
// retire, whatever the dispatch order; lx_tile also places the four column tiles of a row block back to
// back in dispatch order on one XCD (speed and a second line of defence, never relied on alone).
// x_out is bitwise the unfused GEMM's; h / mean / rstd / dx agree with the unfused LayerNorm to fp32
// rounding of the row sums (associated per column tile, not per lane).
constexpr int LX_TN = GL_N / BN;  // column tiles of a 512-wide row
// Workspace: a 256-byte error word, then one record per 128 rows (its layout independent of M and of the
// tile height, so launches of any row counts and tile heights can share the workspace): four pairs of
// arrive / done counters (one per 32-row block: a 128-row tile uses the first, a 64-row tile the first
// of its half), 224 bytes of padding, then the [LX_TN][128] per-row partial pairs.
constexpr int64_t LX_REC = 256 + LX_TN * BM * 8;
struct LnxWs {
  uint32_t* err;    // 1 when a wait gave up (never in a correct launch)
  char* rec;        // rows [128 r, 128 r + 128): record r at rec + r * LX_REC
  uint32_t* fault;  // the library's host-mapped fault word (lx_fault_word), also set on a give-up
  uint64_t limit;   // give-up bound of a wait, s_memrealtime ticks (100 MHz)
  int rb0, nrb;     // this launch's row blocks: [rb0, rb0 + nrb) of the seam (TR-row blocks)
  // the arrive / done counters of the row block (tile row group) that starts at row m0
  __device__ uint32_t* cnt(int64_t m0) const { return (uint32_t*)(rec + (m0 / BM) * LX_REC) + 2 * ((m0 / 32) & 3); }
  // row m's pair of column tile 0 (column tile nt's at + nt * BM)
  __device__ f32x2* part(int64_t m) const { return (f32x2*)(rec + (m / BM) * LX_REC + 256) + m % BM; }
};

__device__ __forceinline__ void lx_store_sc1(f32x2* p, f32x2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// the row's pair from each of the row block's column tiles (sc1 loads, one wait)
__device__ __forceinline__ void lx_load_sc1(const f32x2* base, f32x2 (&o)[LX_TN]) {
  static_assert(LX_TN == 4, "four column tiles");
  asm volatile(
      "global_load_dwordx2 %0, %4, off sc1\n\t"
      "global_load_dwordx2 %1, %5, off sc1\n\t"
      "global_load_dwordx2 %2, %6, off sc1\n\t"
      "global_load_dwordx2 %3, %7, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3])
      : "v"(base), "v"(base + BM), "v"(base + 2 * BM), "v"(base + 3 * BM)
      : "memory");
}

// every thread, after its payload stores: drain them, arrive, wait for the row block's column tiles
__device__ __forceinline__ void lx_drain_arrive(uint32_t* cnt, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lx_wait(const LnxWs& ws, uint32_t* cnt, int tid) {
  if (tid == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)LX_TN) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > ws.limit) {
        __hip_atomic_store(ws.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ws.fault) __hip_atomic_store(ws.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
}

// (row block, column tile) of workgroup bid: the four column tiles of a row block are dispatched back to
// back on one XCD under round-robin placement — blocks b, b + 8, b + 16, b + 24 of each 32-block chunk of
// eight row blocks — whatever the grid size (the XCD remap of consecutive tiles split a row block across
// two XCDs at chunk edges); a last partial chunk keeps them adjacent (b .. b + 3).  The A row panel stays
// on the XCD of its four tiles, as before; W is read by every tile either way.
__device__ __forceinline__ void lx_tile(int bid, const LnxWs& ws, int& rb, int& nt) {
  const int g = bid >> 5;
  if ((g + 1) * 8 <= ws.nrb) {
    rb = g * 8 + (bid & 7);
    nt = (bid >> 3) & 3;
  } else {
    const int l = bid - g * 32;
    rb = g * 8 + (l >> 2);
    nt = l & 3;
  }
  rb += ws.rb0;
}
// after a barrier that follows every thread's partner reads: the last of the four resets the counters
__device__ __forceinline__ void lx_done(uint32_t* c, int tid) {
  if (tid == 0) {
    if (__hip_atomic_fetch_add(c + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(LX_TN - 1)) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Cross-lane sums on the VALU (DPP lane moves + one v_permlane16_swap) instead of __shfl_xor, which
// compiles to ds_bpermute: an LDS round trip per step, five dependent ones for a 32-lane sum
__device__ __forceinline__ float lx_sum2(float v) { return v + rp_dpp<0xB1>(v); }  // lanes l, l ^ 1
__device__ __forceinline__ float lx_sum4(float v) {  // the lane's quad
  v += rp_dpp<0xB1>(v);
  return v + rp_dpp<0x4E>(v);
}
// Row sums of a half-wave's partials: each of the 32 lanes holds IT partials per sum (a, b), one per row
// r0 + RS it, and every row's total over the 32 lanes is wanted.  Recursive halving instead of one
// 32-lane reduction per row: at each lane bit (4, then 3 .. 0) a lane pair splits its rows, each lane keeping
// one half and adding its partner's values for that half, until one row is left; the remaining bits add
// plainly.  Bit 4 pairs lanes l, l ^ 16 through v_permlane16_swap (odd 16-lane rows of the first operand
// trade with even rows of the second: one instruction moves both halves of a pair of rows), bits 3 .. 0
// through DPP row_mirror, row_half_mirror and quad perms (partners differ in that bit; the rows a lane
// holds depend only on the bits above, which partners share).  2 (IT - 1) + 3 adds / selects per sum
// instead of 6 IT.  Returns the row index (it) whose totals land in a[0] / b[0], in lanes l and l ^ 1.
template <int N, int CTRL, int IT>
__device__ __forceinline__ void lx_halve(float (&a)[IT], float (&b)[IT], int l, int bit, int& row) {
  const bool hi = (l >> bit) & 1;
  if constexpr (N > 1) {  // N rows held: keep half, add the partner's values for it
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
      const float ka = hi ? a[j + N / 2] : a[j], sa = hi ? a[j] : a[j + N / 2];
      const float kb = hi ? b[j + N / 2] : b[j], sb = hi ? b[j] : b[j + N / 2];
      a[j] = ka + rp_dpp<CTRL>(sa);
      b[j] = kb + rp_dpp<CTRL>(sb);
    }
    row += hi ? N / 2 : 0;
  } else {  // one row left: plain add
    a[0] += rp_dpp<CTRL>(a[0]);
    b[0] += rp_dpp<CTRL>(b[0]);
  }
}
template <int IT>
__device__ __forceinline__ int lx_rowsums(float (&a)[IT], float (&b)[IT], int l) {
  static_assert(IT >= 2 && (IT & (IT - 1)) == 0, "a power-of-two row count");
#pragma unroll
  for (int j = 0; j < IT / 2; ++j) {
    const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[j]), __float_as_uint(a[j + IT / 2]), false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(b[j]), __float_as_uint(b[j + IT / 2]), false, false);
    a[j] = __uint_as_float(x[0]) + __uint_as_float(x[1]);
    b[j] = __uint_as_float(y[0]) + __uint_as_float(y[1]);
  }
  int row = ((l >> 4) & 1) * (IT / 2);
  constexpr int N3 = IT / 2, N2 = N3 > 1 ? N3 / 2 : 1, N1 = N2 > 1 ? N2 / 2 : 1, N0 = N1 > 1 ? N1 / 2 : 1;
  lx_halve<N3, 0x140>(a, b, l, 3, row);  // row_mirror: partner l ^ 15 within 16
  lx_halve<N2, 0x141>(a, b, l, 2, row);  // row_half_mirror: l ^ 7 within 8
  lx_halve<N1, 0x4E>(a, b, l, 1, row);   // quad_perm [2,3,0,1]: l ^ 2
  lx_halve<N0, 0xB1>(a, b, l, 0, row);   // quad_perm [1,0,3,2]: l ^ 1
  return row;
}

// dma_mainloop's (32 MI) x 128 accumulator tile -> cs[row][CST]
template <int MI>
__device__ __forceinline__ void lx_stage(const f32x4 (&acc)[MI][4], float* cs, int lane, int wm, int wn) {
  const int g = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * (MI * 16) + i * 16 + g * 4 + r) * CST + wn * 64 + j * 16 + cl] = acc[i][j][r];
}

constexpr int LX_CPR = BN / 4;  // float4 chunks per tile row (a half-wave)
static_assert(DmaCfg<0>::LDS <= CTILE_BYTES, "main loop fits the staging area");
// An exchange epilogue over a staged TR x 128 tile with TNT threads: thread tid owns chunk column
// tid % 32 of the rows tid / 32 + RS it, it < IT; the forward's row statistics take TPR threads per row.
// Row m's partials go to its record (LnxWs::part); the four column tiles of rows [m0, m0 + TR) arrive on
// LnxWs::cnt(m0).
template <int TR, int TNT>
struct LxG {
  static constexpr int RS = TNT / LX_CPR;                // rows per chunk step
  static constexpr int IT = TR / RS;                     // chunks per thread
  static constexpr int TPR = TNT / TR;                   // threads per row (forward statistics)
  static constexpr int LDS = TR * CST * 4 + 4 * TR * 4;  // staged tile, per-row totals, (bwd) mean / rstd
  static_assert((TPR == 2 || TPR == 4 || TPR == 8) && TR % 32 == 0 && TR <= BM, "row statistics lanes, row blocks");
};
constexpr int LX_IT = LxG<BM, NT>::IT;  // 16: row = tid / 32 + 8 it

// glds_tile's fills issued through inline asm (rp_dma16): the compiler does not track them, so it adds
// no vmcnt(0) ahead of the LDS reads, and loads the caller issues between fills stay in flight across
// the loop's barriers; the caller orders every fill before its readers (counted vmcnt + barrier)
template <bool KMAJ, int ROWS = BM>
__device__ __forceinline__ void glds_tile_u(const bf16* __restrict__ base, int64_t ld, int64_t rows_lim, int64_t row0,
                                            int64_t k0, char* tile, int wid, int lane) {
  constexpr int PER = ROWS * 64 * 2 / 1024 / (NT / 64);  // 1 KB pieces per wave
  static_assert(PER >= 1 && (KMAJ || ROWS == BM), "whole pieces; m-major images are 128 columns wide");
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int I = wid * PER + j;
    const bf16* src;
    if (KMAJ) {
      const int r = I * 8 + (lane >> 3), lc = kswz(r, lane & 7);
      int64_t rr = row0 + r;
      if (rr >= rows_lim) rr = rows_lim - 1;
      src = base + rr * ld + k0 + lc * 8;
    } else {
      const int k = I * 4 + (lane >> 4), lc = mswz(k, lane & 15);
      int64_t cc = row0 + lc * 8;
      if (cc >= rows_lim) cc = rows_lim - 8;
      src = base + (k0 + k) * ld + cc;
    }
    rp_dma16(src, rp_lds_addr(tile + I * 1024));
  }
}

// The (32 MI) x 128 main loop of dma_mainloop (two 64-deep LDS stages, one barrier per K step, the same
// MFMA order, so the same products bit for bit) with the fills untracked and a per-thread prefetch of
// the 4 MI 16-byte fp32 chunks of the epilogue's operand spread over the first K steps: LX_PF chunks
// issued right after step kt's fill of stage kt + 1, waited for only one step later (the counted
// vmcnt at the end of a step leaves exactly that step's prefetch in flight).  The lockstep grid keeps
// HBM idle through the main loop, so these bytes leave the HBM-bound epilogue.  Each step also waits
// for its own LDS reads (lgkmcnt(0)) before the barrier: after it another wave's fill of step kt + 1
// overwrites the stage read in step kt, and an LDS read still queued behind that traffic would read the
// new bytes (the compiler leaves the last reads of a step outstanding across the barrier otherwise).
constexpr int LX_PF = 2;  // prefetch chunks per K step
template <int MI>
constexpr int lx_pfs() { return LxG<32 * MI, NT>::IT / LX_PF; }  // K steps that carry them (8 at MI = 4)
template <bool AK, bool BKM, int MI = 4>
__device__ __forceinline__ void lx_mainloop(const bf16* __restrict__ A, int64_t lda, int64_t M,
                                            const bf16* __restrict__ B, int64_t ldb, int64_t m0, int64_t n0,
                                            int64_t K, f32x4 (&acc)[MI][4], char* lds, int lane, int wid, int wm,
                                            int wn, const float* __restrict__ pf_base, int64_t pf_ld,
                                            float4 (&pf)[LxG<32 * MI, NT>::IT], int tid) {
  constexpr int LX_PFS = lx_pfs<MI>();
  static_assert(AK || MI == 4, "64- / 32-row images: k-major A");
  constexpr int BK = 64, GTA = MI * 32 * BK * 2, GT = BM * BK * 2, SG = GTA + GT;
  const int nk = (int)(K / BK);
  const float* pfp = pf_base + (m0 + tid / LX_CPR) * pf_ld + n0 + (tid % LX_CPR) * 4;
  auto prefetch = [&](int c) { pf[c] = rp_ld16f(pfp + (int64_t)c * (NT / LX_CPR) * pf_ld, 2); };
  auto fill = [&](int kt) {
    char* buf = lds + (kt & 1) * SG;
    glds_tile_u<AK, MI * 32>(A, lda, M, m0, (int64_t)kt * BK, buf, wid, lane);
    glds_tile_u<BKM>(B, ldb, GL_N, n0, (int64_t)kt * BK, buf + GTA, wid, lane);
  };
  auto compute = [&](int kt) {
    const char* cur = lds + (kt & 1) * SG;
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 fa[MI], fb[4];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        fa[i] = AK ? frag_k_swz<BK>(cur, wm * (MI * 16) + i * 16, ks, lane)
                   : frag_m_swz(cur, wm * (MI * 16) + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = BKM ? frag_k_swz<BK>(cur + GTA, wn * 64 + j * 16, ks, lane)
                    : frag_m_swz(cur + GTA, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };
  // K >= 64 LX_PFS (the host's condition): every prefetch step is a main-loop step, straight-line code
  fill(0);
  rp_waitcnt<0, 15>();
  rp_raw_barrier();
  // steps that carry prefetch chunks: unrolled, so the chunk registers have compile-time indices
#pragma unroll
  for (int kt = 0; kt < LX_PFS; ++kt) {
    if (kt + 1 < LX_PFS || nk > LX_PFS) fill(kt + 1);
#pragma unroll
    for (int c = 0; c < LX_PF; ++c) prefetch(kt * LX_PF + c);
    compute(kt);
    rp_waitcnt<LX_PF, 0>();  // stage kt + 1 has landed; this step's prefetch may stay in flight
    rp_raw_barrier();
  }
  for (int kt = LX_PFS; kt < nk; ++kt) {
    if (kt + 1 < nk) fill(kt + 1);
    compute(kt);
    rp_waitcnt<0, 0>();
    rp_raw_barrier();
  }
}

// the exchange kernels' epilogue operand prefetched over the untracked main loop (lx_mainloop; the
// dma_mainloop form with the operand loaded after it measured 14.51 vs 14.46 ms per step)
static int lnx_prefetch() { return 1; }

// Forward epilogue of a staged TR x 128 accumulator tile cs (r: the thread's residual chunks)
template <int TR, int TNT>
__device__ __forceinline__ void lx_fwd_tail(const GlnDev& a, const LnxWs& ws, int64_t m0, int64_t n0, int nt,
                                            float* cs, const float4 (&r)[LxG<TR, TNT>::IT], int tid) {
  using L = LxG<TR, TNT>;
  float* st = cs + TR * CST;  // per-row mean, rstd
  uint32_t* const cnt = ws.cnt(m0);
  const int cc = (tid % LX_CPR) * 4;
  // x_out = dropout(acc + bias) + residual: gemm_epilogue's RESB arithmetic, op for op
  const float4 bi = *reinterpret_cast<const float4*>(a.bias + n0 + cc);
  const uint32_t dseed = a.drop_thresh ? rp_seed_eff(a.seed_base, a.drop_seed) : 0u;
  static_assert(L::IT % 2 == 0, "rows in pairs (rp_keep4_pair)");
  uint32_t knext = 0u;  // keep bits of the odd row of a pair, drawn with the even row's
#pragma unroll
  for (int it = 0; it < L::IT; ++it) {
    const int row = tid / LX_CPR + it * L::RS;
    const int64_t m = m0 + row, n = n0 + cc;
    float* c = cs + row * CST + cc;
    const float4 v = *reinterpret_cast<const float4*>(c);
    float e4[4] = {v.x * 1.f + bi.x, v.y * 1.f + bi.y, v.z * 1.f + bi.z, v.w * 1.f + bi.w};
    if (a.drop_thresh) {
      uint32_t kb = knext;
      if ((it & 1) == 0)
        rp_keep4_pair(dseed, (uint32_t)(m * GL_N + n), (uint32_t)((m + L::RS) * GL_N + n), a.drop_thresh, tid & 1, kb,
                      knext);
#pragma unroll
      for (int e = 0; e < 4; ++e) e4[e] = ((kb >> e) & 1u) ? e4[e] * a.drop_scale : 0.f;
    }
    e4[0] += r[it].x; e4[1] += r[it].y; e4[2] += r[it].z; e4[3] += r[it].w;
    const float4 o = make_float4(e4[0], e4[1], e4[2], e4[3]);
    rp_st16(a.xo + m * a.ldxo + n, o, 2);
    *reinterpret_cast<float4*>(c) = o;
  }
  LX_STAMP(7);
  __syncthreads();
  // the tile's per-row (sum, M2): TPR threads per row (adjacent lanes), 128 / TPR columns each
  constexpr int CPT = BN / L::TPR / 4;  // float4 chunks per thread
  const int row = tid / L::TPR, hf = tid % L::TPR;
  f32x2* rec = ws.part(m0 + row);  // the row's pair of column tile 0
  auto lane_sum = [](float v) { return L::TPR == 2 ? lx_sum2(v) : (L::TPR == 4 ? lx_sum4(v) : rp_sum8(v)); };
  {
    const float* rr = cs + row * CST + hf * (BN / L::TPR);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const float4 q = *reinterpret_cast<const float4*>(rr + 4 * j);
      s += (q.x + q.y) + (q.z + q.w);
    }
    s = lane_sum(s);
    const float mk = s * (1.f / BN);
    float q2 = 0.f;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const float4 q = *reinterpret_cast<const float4*>(rr + 4 * j);
      const float d0 = q.x - mk, d1 = q.y - mk, d2 = q.z - mk, d3 = q.w - mk;
      q2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
    q2 = lane_sum(q2);
    if (hf == 0) lx_store_sc1(rec + nt * BM, f32x2{s, q2});
  }
  LX_STAMP(2);
  lx_drain_arrive(cnt, tid);
  LX_STAMP(3);
  lx_wait(ws, cnt, tid);
  LX_STAMP(4);
  if (hf == 0) {
    f32x2 o[LX_TN];
    lx_load_sc1(rec, o);
    const float mean = ((o[0].x + o[1].x) + (o[2].x + o[3].x)) * (1.f / GL_N);
    float m2 = (o[0].y + o[1].y) + (o[2].y + o[3].y);
#pragma unroll
    for (int k = 0; k < LX_TN; ++k) {
      const float d = o[k].x * (1.f / BN) - mean;
      m2 += (float)BN * d * d;
    }
    st[row] = mean;
    st[TR + row] = rsqrtf(m2 * (1.f / GL_N) + a.eps);
  }
  __syncthreads();
  lx_done(cnt, tid);
  // h = LayerNorm(x_out): ln_fwd_kernel's (v - mean) * rstd * gamma + beta, 8 columns per thread
  const int c8 = (tid % (BN / 8)) * 8;
  float gm[8], bt[8];
  ld8(gm, a.gamma + n0 + c8);
  ld8(bt, a.beta + n0 + c8);
#pragma unroll 2
  for (int it = 0; it < TR * (BN / 8) / TNT; ++it) {
    const int rw = tid / (BN / 8) + it * (TNT / (BN / 8));
    float v[8];
    ld8(v, cs + rw * CST + c8);
    const float mean = st[rw], rstd = st[TR + rw];
    float y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = (v[i] - mean) * rstd * gm[i] + bt[i];
    st8bf(a.h + (m0 + rw) * a.ldh + n0 + c8, y);
  }
  if (nt == 0 && tid < TR) {
    a.mean[m0 + tid] = st[tid];
    a.rstd[m0 + tid] = st[TR + tid];
  }
#ifdef RP_GEMM_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  LX_STAMP(5);
#endif
}

// Backward epilogue of a staged TR x 128 gradient tile cs (rows' mean / rstd staged at
// cs + TR CST + 2 TR; xh: the thread's x chunks)
template <int TR, int TNT>
__device__ __forceinline__ void lx_bwd_tail(const GlnDev& a, const LnxWs& ws, int64_t m0, int64_t n0, int nt,
                                            float* cs, float4 (&xh)[LxG<TR, TNT>::IT], int tid) {
  using L = LxG<TR, TNT>;
  float* st = cs + TR * CST;  // per-row s1 / 512, s2 / 512
  const float* mr = st + 2 * TR;
  uint32_t* const cnt = ws.cnt(m0);
  const int cc = (tid % LX_CPR) * 4, r0 = tid / LX_CPR;
  const float4 gm = *reinterpret_cast<const float4*>(a.gamma + n0 + cc);
  const float gam[4] = {gm.x, gm.y, gm.z, gm.w};
  float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};  // the tile's gamma / beta partials
  float ps1[L::IT], ps2[L::IT];  // the thread's partials of each row's sums
#pragma unroll
  for (int it = 0; it < L::IT; ++it) {
    const int row = r0 + it * L::RS;
    const float mu = mr[row], rs = mr[TR + row];
    const float4 g4 = *reinterpret_cast<const float4*>(cs + row * CST + cc);
    const float g[4] = {g4.x, g4.y, g4.z, g4.w};
    float x[4] = {xh[it].x, xh[it].y, xh[it].z, xh[it].w};
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[e] = (x[e] - mu) * rs;
      const float gg = g[e] * gam[e];
      s1 += gg;
      s2 += gg * x[e];
      pg[e] += g[e] * x[e];
      pb[e] += g[e];
    }
    xh[it] = make_float4(x[0], x[1], x[2], x[3]);
    ps1[it] = s1;
    ps2[it] = s2;
  }
  static_assert(LX_CPR == 32, "a row's chunks fill a half-wave");
  {
    const int rit = lx_rowsums<L::IT>(ps1, ps2, tid % LX_CPR);
    if ((tid & 1) == 0) lx_store_sc1(ws.part(m0 + r0 + rit * L::RS) + nt * BM, f32x2{ps1[0], ps2[0]});
  }
  LX_STAMP(2);
  lx_drain_arrive(cnt, tid);
  LX_STAMP(3);
  float4 dr[L::IT];  // the residual gradient, in flight while the row block gathers
  if (a.dres) {
#pragma unroll
    for (int it = 0; it < L::IT; ++it) dr[it] = rp_ld16f(a.dres + (m0 + r0 + it * L::RS) * a.lddres + n0 + cc, 2);
  }
  lx_wait(ws, cnt, tid);
  LX_STAMP(4);
  if (tid < TR) {
    f32x2 o[LX_TN];
    lx_load_sc1(ws.part(m0 + tid), o);
    st[tid] = ((o[0].x + o[1].x) + (o[2].x + o[3].x)) * (1.f / GL_N);
    st[TR + tid] = ((o[0].y + o[1].y) + (o[2].y + o[3].y)) * (1.f / GL_N);
  }
  __syncthreads();
  lx_done(cnt, tid);
  const uint32_t lseed = a.lp_thresh ? rp_seed_eff(a.seed_base, a.lp_seed) : 0u;
  uint32_t knext = 0u;  // keep bits of the odd row of a pair (rp_keep4_pair)
#pragma unroll
  for (int it = 0; it < L::IT; ++it) {
    const int row = r0 + it * L::RS;
    const int64_t m = m0 + row, n = n0 + cc;
    const float rs = mr[TR + row], s1 = st[row], s2 = st[TR + row];
    const float4 g4 = *reinterpret_cast<const float4*>(cs + row * CST + cc);
    const float g[4] = {g4.x, g4.y, g4.z, g4.w}, x[4] = {xh[it].x, xh[it].y, xh[it].z, xh[it].w};
    float dx[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) dx[e] = rs * (g[e] * gam[e] - s1 - x[e] * s2);
    if (a.dres) {
      dx[0] += dr[it].x; dx[1] += dr[it].y; dx[2] += dr[it].z; dx[3] += dr[it].w;
    }
    *reinterpret_cast<float4*>(a.dx + m * a.lddx + n) = make_float4(dx[0], dx[1], dx[2], dx[3]);
    if (a.dx_lp) {
      if (a.lp_thresh) {
        uint32_t kb = knext;
        if ((it & 1) == 0)
          rp_keep4_pair(lseed, (uint32_t)(m * GL_N + n), (uint32_t)((m + L::RS) * GL_N + n), a.lp_thresh, tid & 1, kb,
                        knext);
#pragma unroll
        for (int e = 0; e < 4; ++e) dx[e] = ((kb >> e) & 1u) ? dx[e] * a.lp_scale : 0.f;
      }
      bf16x4 q;
#pragma unroll
      for (int e = 0; e < 4; ++e) q[e] = (bf16)dx[e];
      *reinterpret_cast<bf16x4*>(a.dx_lp + m * a.lddx_lp + n) = q;
    }
  }
  // gamma / beta partials: the tile's column sums (the RS threads of a column chunk summed in LDS) in
  // partial row m0 / 32, zeros in its other TR / 32 - 1 rows (the partial rows are 32-row blocks)
  if (a.dgamma_part || a.dbeta_part) {
    __syncthreads();  // every read of the staged tile is done
    float* red = cs;  // [2][RS row groups][128 columns]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[(0 * L::RS + r0) * BN + cc + e] = pg[e];
      red[(1 * L::RS + r0) * BN + cc + e] = pb[e];
    }
    __syncthreads();
    const int64_t pr = m0 / 32;
    if (tid < 2 * BN) {
      const int k = tid / BN, c = tid % BN;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < L::RS; ++q) s += red[(k * L::RS + q) * BN + c];
      float* dst = k ? a.dbeta_part : a.dgamma_part;
      if (dst) dst[pr * a.ld_part + n0 + c] = s;
    }
    if constexpr (TR > 32) {
      for (int id = tid; id < (TR / 32 - 1) * 2 * BN; id += TNT) {
        const int k = id / ((TR / 32 - 1) * BN), rr = (id / BN) % (TR / 32 - 1) + 1, c = id % BN;
        float* dst = k ? a.dbeta_part : a.dgamma_part;
        if (dst) dst[(pr + rr) * a.ld_part + n0 + c] = 0.f;
      }
    }
  }
#ifdef RP_GEMM_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  LX_STAMP(5);
#endif
}

__global__ __launch_bounds__(NT, 2) void gemm_lnx_fwd_kernel(int64_t M, int64_t K, const GlnDev a, const LnxWs ws,
                                                             int pf) {
  __shared__ __attribute__((aligned(16))) char lds[LxG<BM, NT>::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  int rb, nt;
  lx_tile(blockIdx.x, ws, rb, nt);
  const int64_t m0 = (int64_t)rb * BM, n0 = (int64_t)nt * BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8];
  const int cc = (tid % LX_CPR) * 4;
  float4 r[LX_IT];  // the residual tile
  LX_STAMP(0);
  if (pf) {
    lx_mainloop<true, true>(a.A, a.lda, M, a.W, a.ldw, m0, n0, K, acc, lds, lane, wid, wm, wn, a.residual, a.ldr, r,
                            tid);
  } else {
    dma_mainloop<true, true, 0, 4>(a.A, a.lda, M, a.W, a.ldw, GL_N, m0, n0, 0, K, false, acc, bacc, lds, tid, lane,
                                   wid, wm, wn);
#pragma unroll
    for (int it = 0; it < LX_IT; ++it)
      r[it] = rp_ld16f(a.residual + (m0 + tid / LX_CPR + it * (NT / LX_CPR)) * a.ldr + n0 + cc, 2);
  }
  LX_STAMP(1);
  float* cs = reinterpret_cast<float*>(lds);
  lx_stage(acc, cs, lane, wm, wn);
  __syncthreads();
  LX_STAMP(6);
  lx_fwd_tail<BM, NT>(a, ws, m0, n0, nt, cs, r, tid);
}

__global__ __launch_bounds__(NT, 2) void gemm_lnx_bwd_kernel(int64_t M, int64_t K, const GlnDev a, const LnxWs ws,
                                                             int pf) {
  __shared__ __attribute__((aligned(16))) char lds[LxG<BM, NT>::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  int rb, nt;
  lx_tile(blockIdx.x, ws, rb, nt);
  const int64_t m0 = (int64_t)rb * BM, n0 = (int64_t)nt * BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8];
  const int cc = (tid % LX_CPR) * 4, r0 = tid / LX_CPR;
  float4 xh[LX_IT];  // x, then xhat
  LX_STAMP(0);
  if (pf) {
    lx_mainloop<true, false>(a.A, a.lda, M, a.W, a.ldw, m0, n0, K, acc, lds, lane, wid, wm, wn, a.x, a.ldx, xh, tid);
  } else {
    dma_mainloop<true, false, 0, 4>(a.A, a.lda, M, a.W, a.ldw, GL_N, m0, n0, 0, K, false, acc, bacc, lds, tid, lane,
                                    wid, wm, wn);
#pragma unroll
    for (int it = 0; it < LX_IT; ++it)
      xh[it] = rp_ld16f(a.x + (m0 + r0 + it * (NT / LX_CPR)) * a.ldx + n0 + cc, 2);
  }
  LX_STAMP(1);
  float* cs = reinterpret_cast<float*>(lds);
  float* mr = cs + BM * CST + 2 * BM;  // the tile rows' mean, rstd: loaded once, read by both passes
  float mrv = 0.f;
  if (tid < 2 * BM) mrv = tid < BM ? a.mean[m0 + tid] : a.rstd[m0 + tid - BM];
  lx_stage(acc, cs, lane, wm, wn);
  if (tid < 2 * BM) mr[tid] = mrv;
  __syncthreads();
  LX_STAMP(6);
  lx_bwd_tail<BM, NT>(a, ws, m0, n0, nt, cs, xh, tid);
}

// 64 x 128 and 32 x 128 exchange tiles (dma_mainloop MI = 2 / 1: each wave 32 / 16 x 64) for grids whose
// 128-row tiles would leave CUs idle (config 4, M = 4096: 128 -> 256 / 512 workgroups): the same epilogue
// tails — the forward's row statistics four / eight threads per row — on the row block's own counter pair
// (LnxWs::cnt)
template <int MI>
constexpr int lx_small_lds() {
  return dma_tile_lds<0, MI>() > LxG<32 * MI, NT>::LDS ? dma_tile_lds<0, MI>() : LxG<32 * MI, NT>::LDS;
}
template <bool FWD, int MI>
__global__ __launch_bounds__(NT, 2) void gemm_lnx64_kernel(int64_t M, int64_t K, const GlnDev a, const LnxWs ws,
                                                           int pf) {
  constexpr int TR = 32 * MI;
  __shared__ __attribute__((aligned(16))) char lds[lx_small_lds<MI>()];
  using L = LxG<TR, NT>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  int rb, nt;
  lx_tile(blockIdx.x, ws, rb, nt);
  const int64_t m0 = (int64_t)rb * TR, n0 = (int64_t)nt * BN;
  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8];
  // the epilogue's fp32 operand (fwd: the residual, bwd: x): prefetched across the first K steps of the
  // untracked main loop (pf), or issued before dma_mainloop (in flight under its first fills); and (bwd)
  // the rows' mean / rstd
  const float* src = FWD ? a.residual : a.x;
  const int64_t ld = FWD ? a.ldr : a.ldx;
  const int cc = (tid % LX_CPR) * 4, r0 = tid / LX_CPR;
  float4 xr[L::IT];
  float mrv = 0.f;
  if (!FWD && tid < 2 * TR) mrv = tid < TR ? a.mean[m0 + tid] : a.rstd[m0 + tid - TR];
  if (pf) {
    lx_mainloop<true, FWD, MI>(a.A, a.lda, M, a.W, a.ldw, m0, n0, K, acc, lds, lane, wid, wm, wn, src, ld, xr, tid);
  } else {
#pragma unroll
    for (int it = 0; it < L::IT; ++it) xr[it] = rp_ld16f(src + (m0 + r0 + it * L::RS) * ld + n0 + cc, 2);
    dma_mainloop<true, FWD, 0, MI>(a.A, a.lda, M, a.W, a.ldw, GL_N, m0, n0, 0, K, false, acc, bacc, lds, tid, lane,
                                   wid, wm, wn);
  }
  float* cs = reinterpret_cast<float*>(lds);  // dma_mainloop ended on a barrier: its stages are free
  lx_stage<MI>(acc, cs, lane, wm, wn);
  if (!FWD && tid < 2 * TR) cs[TR * CST + 2 * TR + tid] = mrv;
  __syncthreads();
  if constexpr (FWD)
    lx_fwd_tail<TR, NT>(a, ws, m0, n0, nt, cs, xr, tid);
  else
    lx_bwd_tail<TR, NT>(a, ws, m0, n0, nt, cs, xr, tid);
}
}  // namespace

extern "C" int rp_gemm(int dtype, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, int a_kmajor,
                       const void* B, int64_t ldb, int b_kmajor, void* C, int64_t ldc, int c_dtype, float alpha,
                       const rp_gemm_epilogue* ep, void* stream) {
  RP_REQUIRE(dtype == RP_F32 || dtype == RP_BF16, "rp_gemm: bad dtype %d", dtype);
  RP_REQUIRE(c_dtype == RP_F32 || c_dtype == RP_BF16, "rp_gemm: bad c_dtype %d", c_dtype);
  RP_REQUIRE(M >= 0 && N >= 0 && K >= 0, "rp_gemm: negative size");
  if (M == 0 || N == 0) return RP_OK;
  RP_REQUIRE(A && B && C, "rp_gemm: null operand");
  const int64_t vec = 8;
  RP_REQUIRE((!a_kmajor && !b_kmajor) || K % vec == 0, "rp_gemm: K=%lld must be a multiple of 8", (long long)K);
  RP_REQUIRE(lda % vec == 0 && ldb % vec == 0 && ldc % vec == 0, "rp_gemm: leading dims must be multiples of 8");
  RP_REQUIRE(a_kmajor || M % vec == 0, "rp_gemm: m-major A needs M %% 8 == 0");
  RP_REQUIRE(b_kmajor || N % vec == 0, "rp_gemm: n-major B needs N %% 8 == 0");
  RP_REQUIRE(rp_aligned16(A) && rp_aligned16(B), "rp_gemm: operands must be 16-byte aligned");
  RP_REQUIRE(a_kmajor ? lda >= K : lda >= M, "rp_gemm: lda too small");
  RP_REQUIRE(b_kmajor ? ldb >= K : ldb >= N, "rp_gemm: ldb too small");
  RP_REQUIRE(ldc >= N, "rp_gemm: ldc too small");
  RP_REQUIRE(N % vec == 0, "rp_gemm: N=%lld must be a multiple of 8 (use rp_rowdot_* for N <= 4)", (long long)N);
  RP_REQUIRE(rp_aligned16(C), "rp_gemm: C must be 16-byte aligned");
  EpiDev e{};
  e.gate_scale = 1.f;
  e.st_pol = rp_store_policy();
  e.ld_pol = rp_residual_load_policy();
  if (ep) {
    e.bias = ep->bias;
    e.relu = ep->relu;
    e.drop_thresh = rp_dropout_thresh(ep->dropout_p);
    e.drop_scale = ep->dropout_p > 0.f ? 1.f / (1.f - ep->dropout_p) : 1.f;
    e.drop_seed = ep->dropout_seed;
    e.seed_base = e.drop_thresh ? ep->seed_base : nullptr;
    e.residual = ep->residual;
    e.ldr = ep->ldr;
    e.gate = ep->gate;
    e.gate_bf16 = ep->gate_dtype == RP_BF16;
    e.ldg = ep->ldg;
    e.gate_scale = ep->gate_scale;
    e.accumulate = ep->accumulate;
    e.col_scale_n = ep->col_scale_n;
    e.col_scale = ep->col_scale;
    e.prefetch_gate = 1;
    RP_REQUIRE(ep->dropout_p >= 0.f && ep->dropout_p < 1.f, "rp_gemm: dropout_p must be in [0, 1)");
    RP_REQUIRE(e.col_scale_n >= 0 && e.col_scale_n % 8 == 0, "rp_gemm: col_scale_n must be a multiple of 8");
    RP_REQUIRE(!e.accumulate || c_dtype == RP_F32, "rp_gemm: accumulate needs an fp32 C");
    RP_REQUIRE(!e.drop_thresh || M * N < (int64_t)UINT32_MAX, "rp_gemm: dropout index overflow");
    RP_REQUIRE(!e.bias || rp_aligned16(e.bias), "rp_gemm: bias must be 16-byte aligned");
    RP_REQUIRE(!e.residual || (rp_aligned16(e.residual) && e.ldr % 4 == 0), "rp_gemm: residual alignment");
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RP_BF16) {
    if (c_dtype == RP_BF16) return launch_gemm_t<bf16, bf16>(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, alpha, e, s);
    return launch_gemm_t<bf16, float>(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, alpha, e, s);
  }
  if (c_dtype == RP_BF16) return launch_gemm_t<float, bf16>(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, alpha, e, s);
  return launch_gemm_t<float, float>(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, alpha, e, s);
}

extern "C" int rp_gemm_wgrad_grouped(int64_t K, const rp_wgrad_item* items, int n_items, int accumulate,
                                     void* stream) {
  RP_REQUIRE(n_items >= 0 && n_items <= WG_MAX, "rp_gemm_wgrad_grouped: 0..%d items per launch", WG_MAX);
  RP_REQUIRE(K >= 0 && K % 64 == 0, "rp_gemm_wgrad_grouped: K=%lld must be a multiple of 64", (long long)K);
  if (n_items == 0) return RP_OK;
  RP_REQUIRE(items, "rp_gemm_wgrad_grouped: null items");
  WgGroup g{};
  g.n = n_items;
  g.accumulate = accumulate;
  g.K = K;
  g.order = 0;  // the XCD remap of consecutive tiles (orders 1 / 2 measured alike, profiles/r05_wgrad_order_probe.txt)
  g.st_pol = rp_store_policy();
  int64_t tiles = 0;
  for (int i = 0; i < n_items; ++i) {
    const rp_wgrad_item& it = items[i];
    RP_REQUIRE(it.M > 0 && it.N > 0 && it.M % 8 == 0 && it.N % 8 == 0 && it.ldy % 8 == 0 && it.ldx % 8 == 0 &&
                   it.ldy >= it.M && it.ldx >= it.N && it.M <= INT32_MAX && it.N <= INT32_MAX &&
                   it.ldy <= INT32_MAX && it.ldx <= INT32_MAX,
               "rp_gemm_wgrad_grouped: item %d: M, N, leading dims must be positive multiples of 8", i);
    RP_REQUIRE(it.dW && (K == 0 || (it.dY && it.X)), "rp_gemm_wgrad_grouped: item %d: null operand", i);
    RP_REQUIRE(rp_aligned16(it.dY) && rp_aligned16(it.X) && rp_aligned16(it.dW),
               "rp_gemm_wgrad_grouped: item %d: 16-byte alignment required", i);
    g.start[i] = (int)tiles;
    g.it[i] = WgItem{(const bf16*)it.dY, (const bf16*)it.X, it.dW, it.db, (int)it.M, (int)it.N, (int)it.ldy,
                     (int)it.ldx};
    tiles += ((it.M + 255) / 256) * ((it.N + 255) / 256);
  }
  RP_REQUIRE(tiles < (1 << 30), "rp_gemm_wgrad_grouped: too many tiles");
  g.start[n_items] = (int)tiles;
  g.tiles_total = (int)tiles;
  hipLaunchKernelGGL(wgrad8_grouped_kernel, dim3((unsigned)tiles), dim3(NT8), 0, (hipStream_t)stream, g);
  return rp_check_launch("rp_gemm_wgrad_grouped");
}

extern "C" int rp_gemm_attn_dout_delta(const void* dY, int64_t ldy, const void* W, int64_t ldw, int64_t M, int64_t K,
                                       void* dO, int64_t ldo, const void* out, const void* out_lo, int64_t ld_out,
                                       const float* lse, int B, int T, int H, float dropout_p, float* delta_ws,
                                       void* stream) {
  const int64_t N = (int64_t)H * 64;
  RP_REQUIRE(B > 0 && T > 0 && H > 0 && M == (int64_t)B * T, "rp_gemm_attn_dout_delta: M must be B*T");
  RP_REQUIRE(M % BM == 0 && N % BN == 0 && K % 64 == 0 && K > 0,
             "rp_gemm_attn_dout_delta: M and H*64 multiples of 128, K a multiple of 64");
  RP_REQUIRE(dY && W && dO && out && lse && delta_ws, "rp_gemm_attn_dout_delta: null pointer");
  RP_REQUIRE(rp_aligned16(dY) && rp_aligned16(W) && rp_aligned16(dO) && rp_aligned16(out) &&
                 (!out_lo || rp_aligned16(out_lo)),
             "rp_gemm_attn_dout_delta: 16-byte alignment required");
  RP_REQUIRE(ldy >= K && ldw >= N && ldo >= N && ld_out >= N && ldy % 8 == 0 && ldw % 8 == 0 && ldo % 8 == 0 &&
                 ld_out % 8 == 0,
             "rp_gemm_attn_dout_delta: leading dims");
  RP_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "rp_gemm_attn_dout_delta: dropout_p out of range");
  EpiDev e{};
  e.gate_scale = 1.f;
  e.st_pol = rp_store_policy();
  e.ld_pol = rp_residual_load_policy();
  e.dot_hi = (const bf16*)out;
  e.dot_lo = (const bf16*)out_lo;
  e.ld_dot = ld_out;
  e.delta = delta_ws;
  e.lse = lse;
  e.dT = T;
  e.dH = H;
  e.dscale = dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f;
  // dO = dY W: k-major A = dY [M, K], B = W [K, N] row-major (the nn.Linear weight's dgrad layout),
  // configuration 0 — the only path that carries the fused delta — on 128-, 64- or 32-row tiles by the
  // plain GEMMs' rule (rp_gemm_bm64 / rp_gemm_bm32: config 4's 128 tiles -> 512); the delta epilogue
  // (RESB 2) with its operand chunks requested before the main loop
  const int mi = rp_gemm_bm64(M, N) ? (rp_gemm_bm32(M, N) ? 1 : 2) : 4;
  const dim3 grid((unsigned)((M / (32 * mi)) * (N / BN)));
#define RP_DOUT_LAUNCH(MI_)                                                                                           \
  hipLaunchKernelGGL((gemm_bf16_dma_kernel<true, false, bf16, 0, 0, 2, MI_>), grid, dim3(NT), 0, (hipStream_t)stream, \
                     M, N, K, (const bf16*)dY, ldy, (const bf16*)W, ldw, (bf16*)dO, ldo, 1.f, e, (int64_t)0,           \
                     (float*)nullptr)
  if (mi == 4)
    RP_DOUT_LAUNCH(4);
  else if (mi == 2)
    RP_DOUT_LAUNCH(2);
  else
    RP_DOUT_LAUNCH(1);
#undef RP_DOUT_LAUNCH
  return rp_check_launch("rp_gemm_attn_dout_delta");
}

extern "C" int64_t rp_gemm_wgrad_workspace(int64_t M, int64_t N, int64_t K) {
  int splits;
  int64_t kchunk;
  wgrad_plan(M, N, K, GemmCfg<bf16>::BK, splits, kchunk);
  int s2;
  int64_t k2;
  wgrad_plan(M, N, K, GemmCfg<float>::BK, s2, k2);
  if (s2 > splits) splits = s2;
  if (wgrad8_plan(M, N, K, s2, k2) && s2 > splits) splits = s2;
  return (int64_t)splits * (M * N + M) * 4;
}

extern "C" int rp_gemm_wgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dY, int64_t ldy, const void* X,
                             int64_t ldx, float* dW, float* db, int accumulate, void* workspace, int64_t ws_bytes,
                             void* stream) {
  RP_REQUIRE(dtype == RP_F32 || dtype == RP_BF16, "rp_gemm_wgrad: bad dtype %d", dtype);
  RP_REQUIRE(M >= 0 && N >= 0 && K >= 0, "rp_gemm_wgrad: negative size");
  if (M == 0 || N == 0) return RP_OK;
  RP_REQUIRE(dW && workspace, "rp_gemm_wgrad: null output / workspace");
  RP_REQUIRE(K == 0 || (dY && X), "rp_gemm_wgrad: null operand");
  RP_REQUIRE(M % 8 == 0 && N % 8 == 0 && ldy % 8 == 0 && ldx % 8 == 0 && ldy >= M && ldx >= N,
             "rp_gemm_wgrad: M, N and leading dims must be multiples of 8");
  RP_REQUIRE(rp_aligned16(dY) && rp_aligned16(X) && rp_aligned16(dW) && rp_aligned16(workspace),
             "rp_gemm_wgrad: 16-byte alignment required");
  const int bk = dtype == RP_BF16 ? GemmCfg<bf16>::BK : GemmCfg<float>::BK;
  int splits;
  int64_t kchunk;
  const int bn8 = dtype == RP_BF16 ? wgrad8_plan(M, N, K, splits, kchunk) : 0;
  if (!bn8) wgrad_plan(M, N, K, bk, splits, kchunk);
  RP_REQUIRE(ws_bytes >= (int64_t)splits * (M * N + M) * 4, "rp_gemm_wgrad: workspace too small");
  float* slab = (float*)workspace;
  float* bslab = db ? slab + (int64_t)splits * M * N : nullptr;
  hipStream_t s = (hipStream_t)stream;
  EpiDev e{};
  e.gate_scale = 1.f;
  e.st_pol = rp_store_policy();
  e.ld_pol = rp_residual_load_policy();
  e.split_major = 1;
  int rc;
  if (bn8)
    rc = launch_gemm8<float>(bn8, M, N, K, (const bf16*)dY, ldy, 0, (const bf16*)X, ldx, 0, slab, N, 1.f, e, s, splits,
                             kchunk, bslab);
  else if (dtype == RP_BF16)
    rc = launch_gemm_t<bf16, float>(M, N, K, dY, ldy, 0, X, ldx, 0, slab, N, 1.f, e, s, splits, kchunk, bslab);
  else
    rc = launch_gemm_t<float, float>(M, N, K, dY, ldy, 0, X, ldx, 0, slab, N, 1.f, e, s, splits, kchunk, bslab);
  if (rc) return rc;
  const int64_t n = M * N;
  int64_t g = (n / 4 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  const int64_t g2 = db ? (M / 4 + 255) / 256 : 0;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)(g + g2)), dim3(256), 0, s, slab, splits, n, dW, bslab, M, db,
                     (int)g, accumulate);
  return rp_check_launch("rp_gemm_wgrad");
}

// ---- GEMM + LayerNorm entry points (include/rp_api.h) ----
// exchange workspace of the 128 x 128 GEMM + LayerNorm kernels: error word, counters, partial pairs
extern "C" int64_t rp_gemm_ln_xchg_bytes(int64_t M) {
  return 256 + (M > 0 ? (M + BM - 1) / BM : 0) * LX_REC;
}

// The fault word: one host-mapped word per process (allocated on the first exchange launch, never in a
// kernel), set by any exchange wait that gives up.  The host reads it without synchronising, so a fault
// is reported by the next rp_gemm_ln_* call (or rp_gemm_ln_status) after the faulting kernel ran.
static std::mutex g_lx_mu;
static uint32_t* g_lx_fault_host = nullptr;
static uint32_t* g_lx_fault_dev = nullptr;
constexpr double LX_TIMEOUT_S = 10.0;  // give-up bound of a partner wait (co-resident partners: microseconds)

static int lx_fault_word(uint32_t** dev) {
  std::lock_guard<std::mutex> lk(g_lx_mu);
  if (!g_lx_fault_host) {
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, 256, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        !h) {
      (void)hipGetLastError();
      rp_set_error("rp_gemm_ln: cannot allocate the exchange fault word (hipHostMalloc)");
      return RP_ERR_LAUNCH;
    }
    memset(h, 0, 256);
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
      (void)hipGetLastError();
      (void)hipHostFree(h);
      rp_set_error("rp_gemm_ln: no device address for the exchange fault word");
      return RP_ERR_LAUNCH;
    }
    g_lx_fault_host = (uint32_t*)h;
    g_lx_fault_dev = (uint32_t*)d;
  }
  *dev = g_lx_fault_dev;
  return RP_OK;
}

static int lx_fault_check(const char* fn) {
  const uint32_t* h = g_lx_fault_host;
  if (h && __atomic_load_n(h, __ATOMIC_ACQUIRE) != 0) {
    rp_set_error("%s: an earlier GEMM + LayerNorm exchange launch gave up waiting for the partner tiles of a row "
                 "block (a partner workgroup was not resident within %.0f s): its LayerNorm outputs are invalid and "
                 "its exchange workspace is inconsistent; call rp_gemm_ln_reset on that workspace",
                 fn, LX_TIMEOUT_S);
    return RP_ERR_LAUNCH;
  }
  return RP_OK;
}

extern "C" int rp_gemm_ln_status(void) { return lx_fault_check("rp_gemm_ln_status"); }

extern "C" int rp_gemm_ln_reset(void* xchg, int64_t M, void* stream) {
  RP_REQUIRE(M >= 0, "rp_gemm_ln_reset: negative M");
  RP_REQUIRE(!xchg || (((uintptr_t)xchg) & 255u) == 0, "rp_gemm_ln_reset: xchg must be 256-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  // the faulting launch may still run (its give-up workgroups finish their tiles): drain it first
  if (hipStreamSynchronize(s) != hipSuccess) return rp_check_launch("rp_gemm_ln_reset");
  if (xchg && hipMemsetAsync(xchg, 0, (size_t)rp_gemm_ln_xchg_bytes(M), s) != hipSuccess)
    return rp_check_launch("rp_gemm_ln_reset");
  if (hipStreamSynchronize(s) != hipSuccess) return rp_check_launch("rp_gemm_ln_reset");
  if (g_lx_fault_host) __atomic_store_n(g_lx_fault_host, 0u, __ATOMIC_RELEASE);
  return RP_OK;
}

// Exchange tile height: the tallest of 128 / 64 / 32 rows whose grid gives every CU two workgroups, else
// 32 (M is a multiple of 64).  Interleaved whole-step A/B (profiles/r05_lnx64_ab.txt): bench shape
// (M = 16384) 13.98 ms on 128-row tiles vs 15.11 on 64-row ones; config 2 (M = 8192, one 128-row tile per
// CU) 7.11 vs 7.04 on 64-row tiles; config 4 (M = 4096) 7.03 on 64-row tiles vs 7.12 unfused.
static int g_lnx_rows_forced = 0;  // rp_debug_set_lnx_rows (tests: every tile height at small M)
static int lnx_rows(int64_t M) {
  const int f = g_lnx_rows_forced;
  if (f == 32 || f == 64) return f;
  if (f == 128) return M % 128 == 0 ? 128 : 64;
  const int64_t two = 2 * gemm_cu_count();
  if (M % 128 == 0 && (M / 128) * LX_TN >= two) return 128;
  return (M / 64) * LX_TN >= two ? 64 : 32;
}

// Co-resident capacity of an exchange kernel: CUs x workgroups per CU (the occupancy query, at most 2 —
// the __launch_bounds__ residency the tile shapes are sized for).  A launch never exceeds it.
static int64_t lx_capacity(const void* kern) {
  static std::mutex mu;
  static const void* keys[16] = {nullptr};
  static int vals[16] = {0};
  int per = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 0; i < 16 && keys[i]; ++i)
      if (keys[i] == kern) per = vals[i];
    if (!per) {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, NT, 0) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = 1;
      }
      per = n < 2 ? n : 2;
      for (int i = 0; i < 16; ++i)
        if (!keys[i]) {
          keys[i] = kern;
          vals[i] = per;
          break;
        }
    }
  }
  return gemm_cu_count() * per;
}

// One seam as launches of at most the co-resident capacity (whole row blocks each); max_tiles < 0: all
// tiles (a debug launch passes fewer, leaving a row block without a partner)
template <typename Kern>
static int lx_launch(Kern kern, const char* fn, int tr, int64_t M, int64_t K, const GlnDev& d, void* xchg, int pf,
                     hipStream_t s, int64_t max_tiles, double timeout_s) {
  uint32_t* fault = nullptr;
  const int rc = lx_fault_word(&fault);
  if (rc) return rc;
  const int64_t nrb = M / tr;
  int64_t cap = lx_capacity(reinterpret_cast<const void*>(kern)) / LX_TN;
  if (cap < 1) cap = 1;
  const uint64_t limit = (uint64_t)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  for (int64_t r0 = 0; r0 < nrb; r0 += cap) {
    const int64_t n = nrb - r0 < cap ? nrb - r0 : cap;
    int64_t grid = n * LX_TN;
    if (max_tiles >= 0 && grid > max_tiles) grid = max_tiles;
    if (grid <= 0) break;
    const LnxWs ws{(uint32_t*)xchg, (char*)xchg + 256, fault, limit, (int)r0, (int)n};
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, s, M, K, d, ws, pf);
    if (max_tiles >= 0) max_tiles -= grid;
  }
  return rp_check_launch(fn);
}

// the exchange launch of a seam (tile height by lnx_rows)
static int lx_dispatch(bool fwd, int64_t M, int64_t K, const GlnDev& d, void* xchg, hipStream_t s, int64_t max_tiles,
                       double timeout_s) {
  const char* fn = fwd ? "rp_gemm_ln_fwd" : "rp_gemm_ln_bwd";
  const int xrows = lnx_rows(M);
  const int pf = lnx_prefetch();
  if (xrows == 64)
    return fwd ? lx_launch(gemm_lnx64_kernel<true, 2>, fn, 64, M, K, d, xchg, pf && K >= 64 * lx_pfs<2>(), s,
                           max_tiles, timeout_s)
               : lx_launch(gemm_lnx64_kernel<false, 2>, fn, 64, M, K, d, xchg, pf && K >= 64 * lx_pfs<2>(), s,
                           max_tiles, timeout_s);
  if (xrows == 32)
    return fwd ? lx_launch(gemm_lnx64_kernel<true, 1>, fn, 32, M, K, d, xchg, pf && K >= 64 * lx_pfs<1>(), s,
                           max_tiles, timeout_s)
               : lx_launch(gemm_lnx64_kernel<false, 1>, fn, 32, M, K, d, xchg, pf && K >= 64 * lx_pfs<1>(), s,
                           max_tiles, timeout_s);
  return fwd ? lx_launch(gemm_lnx_fwd_kernel, fn, BM, M, K, d, xchg, pf && K >= 64 * lx_pfs<4>(), s, max_tiles,
                         timeout_s)
             : lx_launch(gemm_lnx_bwd_kernel, fn, BM, M, K, d, xchg, pf && K >= 64 * lx_pfs<4>(), s, max_tiles,
                         timeout_s);
}

static int gemm_ln_common(const char* fn, int64_t M, int64_t K, const rp_gemm_ln_args* p, GlnDev& d) {
  const int fc = lx_fault_check(fn);
  if (fc) return fc;
  RP_REQUIRE(p, "%s: null args", fn);
  RP_REQUIRE(M >= 0 && K > 0 && M % GL_BM == 0 && K % GL_BK == 0, "%s: M must be a multiple of 64 and K of 64 (M=%lld K=%lld)",
             fn, (long long)M, (long long)K);
  RP_REQUIRE(p->A && p->W && p->gamma, "%s: null operand", fn);
  RP_REQUIRE(rp_aligned16(p->A) && rp_aligned16(p->W) && rp_aligned16(p->gamma), "%s: 16-byte alignment required", fn);
  RP_REQUIRE(p->lda >= K && p->lda % 8 == 0, "%s: bad lda", fn);
  RP_REQUIRE(p->dropout_p >= 0.f && p->dropout_p < 1.f, "%s: dropout_p must be in [0, 1)", fn);
  d = GlnDev{};
  d.A = (const bf16*)p->A; d.lda = p->lda; d.W = (const bf16*)p->W; d.ldw = p->ldw;
  d.gamma = p->gamma;
  d.drop_thresh = rp_dropout_thresh(p->dropout_p);
  d.drop_scale = p->dropout_p > 0.f ? 1.f / (1.f - p->dropout_p) : 1.f;
  d.drop_seed = p->dropout_seed;
  d.seed_base = p->seed_base;
  d.mean = p->mean; d.rstd = p->rstd;
  RP_REQUIRE(p->mean && p->rstd, "%s: null mean / rstd", fn);
  RP_REQUIRE(!p->xchg || (((uintptr_t)p->xchg) & 255u) == 0, "%s: xchg must be 256-byte aligned", fn);
  return RP_OK;
}

static int gemm_ln_fwd_prep(int64_t M, int64_t K, const rp_gemm_ln_args* p, GlnDev& d) {
  const int rc = gemm_ln_common("rp_gemm_ln_fwd", M, K, p, d);
  if (rc) return rc;
  RP_REQUIRE(p->ldw >= K && p->ldw % 8 == 0, "rp_gemm_ln_fwd: W must be [512][ldw >= K]");
  RP_REQUIRE(p->bias && p->beta && p->residual && p->x_out && p->h_out, "rp_gemm_ln_fwd: null operand");
  RP_REQUIRE(rp_aligned16(p->bias) && rp_aligned16(p->beta) && rp_aligned16(p->residual) && rp_aligned16(p->x_out) &&
                 rp_aligned16(p->h_out) && p->ldr % 4 == 0 && p->ldx_out % 4 == 0 && p->ldh % 8 == 0 &&
                 p->ldr >= 512 && p->ldx_out >= 512 && p->ldh >= 512,
             "rp_gemm_ln_fwd: output / residual alignment or leading dims");
  RP_REQUIRE(!d.drop_thresh || M * 512 < (int64_t)UINT32_MAX, "rp_gemm_ln_fwd: dropout index overflow");
  d.bias = p->bias; d.beta = p->beta; d.eps = p->eps;
  d.residual = p->residual; d.ldr = p->ldr;
  d.xo = p->x_out; d.ldxo = p->ldx_out;
  d.h = (bf16*)p->h_out; d.ldh = p->ldh;
  return RP_OK;
}

static int gemm_ln_bwd_prep(int64_t M, int64_t K, const rp_gemm_ln_args* p, GlnDev& d) {
  const int rc = gemm_ln_common("rp_gemm_ln_bwd", M, K, p, d);
  if (rc) return rc;
  RP_REQUIRE(p->ldw >= 512 && p->ldw % 8 == 0, "rp_gemm_ln_bwd: W must be [K][ldw >= 512]");
  RP_REQUIRE(p->x && p->dx, "rp_gemm_ln_bwd: null x / dx");
  RP_REQUIRE(rp_aligned16(p->x) && rp_aligned16(p->dx) && (!p->dres || rp_aligned16(p->dres)) &&
                 (!p->dx_lp || rp_aligned16(p->dx_lp)) && p->ldx % 4 == 0 && p->lddx % 4 == 0 &&
                 p->lddres % 4 == 0 && p->lddx_lp % 8 == 0 && p->ldx >= 512 && p->lddx >= 512 &&
                 (!p->dres || p->lddres >= 512) && (!p->dx_lp || p->lddx_lp >= 512),
             "rp_gemm_ln_bwd: alignment or leading dims");
  RP_REQUIRE(p->lp_dropout_p >= 0.f && p->lp_dropout_p < 1.f, "rp_gemm_ln_bwd: lp_dropout_p must be in [0, 1)");
  RP_REQUIRE(!p->dgamma_part || p->ld_part >= 512, "rp_gemm_ln_bwd: ld_part < 512");
  d.x = p->x; d.ldx = p->ldx; d.dres = p->dres; d.lddres = p->lddres;
  d.dx = p->dx; d.lddx = p->lddx;
  d.dx_lp = (bf16*)p->dx_lp; d.lddx_lp = p->lddx_lp;
  d.lp_thresh = rp_dropout_thresh(p->lp_dropout_p);
  d.lp_scale = p->lp_dropout_p > 0.f ? 1.f / (1.f - p->lp_dropout_p) : 1.f;
  d.lp_seed = p->lp_seed;
  d.dgamma_part = p->dgamma_part; d.dbeta_part = p->dbeta_part; d.ld_part = p->ld_part;
  return RP_OK;
}

extern "C" int rp_gemm_ln_fwd(int64_t M, int64_t K, const rp_gemm_ln_args* p, void* stream) {
  GlnDev d;
  const int rc = gemm_ln_fwd_prep(M, K, p, d);
  if (rc) return rc;
  if (M == 0) return RP_OK;
  if (p->xchg) return lx_dispatch(true, M, K, d, p->xchg, (hipStream_t)stream, -1, LX_TIMEOUT_S);
  hipLaunchKernelGGL(gemm_ln_fwd_kernel, dim3((unsigned)(M / GL_BM)), dim3(GL_NT), 0, (hipStream_t)stream, M, K, d);
  return rp_check_launch("rp_gemm_ln_fwd");
}

extern "C" int rp_gemm_ln_bwd(int64_t M, int64_t K, const rp_gemm_ln_args* p, void* stream) {
  GlnDev d;
  const int rc = gemm_ln_bwd_prep(M, K, p, d);
  if (rc) return rc;
  if (M == 0) return RP_OK;
  if (p->xchg) return lx_dispatch(false, M, K, d, p->xchg, (hipStream_t)stream, -1, LX_TIMEOUT_S);
  hipLaunchKernelGGL(gemm_ln_bwd_kernel, dim3((unsigned)(M / GL_BM)), dim3(GL_NT), 0, (hipStream_t)stream, M, K, d);
  return rp_check_launch("rp_gemm_ln_bwd");
}

// Test hooks (include/rp_api.h, "Debug"): an exchange launch with only the first `tiles` workgroups and
// its own give-up bound (a row block left without a partner must fail loudly, not hang or corrupt
// silently), and a kernel that holds CU slots for a while (a seam beside another stream's long kernel).
extern "C" int rp_debug_gemm_ln_partial(int fwd, int64_t M, int64_t K, const rp_gemm_ln_args* p, int64_t tiles,
                                        double timeout_s, void* stream) {
  GlnDev d;
  const int rc = fwd ? gemm_ln_fwd_prep(M, K, p, d) : gemm_ln_bwd_prep(M, K, p, d);
  if (rc) return rc;
  RP_REQUIRE(p->xchg && M > 0 && tiles >= 0 && timeout_s > 0.0 && timeout_s <= 60.0,
             "rp_debug_gemm_ln_partial: needs an exchange workspace, M > 0, tiles >= 0, 0 < timeout_s <= 60");
  return lx_dispatch(fwd != 0, M, K, d, p->xchg, (hipStream_t)stream, tiles, timeout_s);
}

extern "C" int rp_debug_set_lnx_rows(int rows) {
  RP_REQUIRE(rows == 0 || rows == 32 || rows == 64 || rows == 128, "rp_debug_set_lnx_rows: 0 (automatic), 32, 64 or 128");
  g_lnx_rows_forced = rows;
  return RP_OK;
}

__global__ __launch_bounds__(NT) void occupy_kernel(uint64_t ticks, float* sink) {
  __shared__ float lds[16384];  // 64 KiB: two such workgroups fill a CU's LDS with the seams' 69 KB tiles
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (sink && threadIdx.x == 0 && lds[(blockIdx.x * 7) & (NT - 1)] < 0.f) sink[blockIdx.x] = 1.f;
}

extern "C" int rp_debug_occupy(int blocks, int us, void* stream) {
  RP_REQUIRE(blocks > 0 && blocks <= 65536 && us > 0 && us <= 10000000, "rp_debug_occupy: 0 < blocks <= 65536, 0 < us <= 1e7");
  hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, (uint64_t)us * 100u,
                     (float*)nullptr);
  return rp_check_launch("rp_debug_occupy");
}

#ifdef RP_GEMM_PROBE
extern "C" int rp_debug_lnx_probe(uint64_t* host, int n) {
  if (n > RP_PROBE_MAX * 8) n = RP_PROBE_MAX * 8;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lnx_probe), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
extern "C" int rp_debug_gemm_probe(uint64_t* host, int n) {
  if (n > RP_PROBE_MAX * 4) n = RP_PROBE_MAX * 4;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_probe), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif
