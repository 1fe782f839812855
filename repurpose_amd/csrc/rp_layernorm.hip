// LayerNorm forward/backward with the Repurpose fusions (reference models/MMCTransformer.py:35,
// 58, 65, 72, 84 and encoder-layer norm1/norm2; PE add :127 / :20-22; feature_map ReLU+Dropout
// :63-68).  One wavefront per row, the row held in registers (D/64 contiguous elements per lane),
// biased variance and eps as torch.nn.LayerNorm.  HBM-bound: forward moves D*(in+out) bytes per
// row, backward D*(dy+x+dx[+dx_lp]) bytes per row.
#include "rp_common.h"

namespace {

constexpr int LN_WAVES = 4;            // forward: rows handled concurrently per block
constexpr int LNB_WAVES = 8;           // backward: waves per block
constexpr int LN_ROWS_PER_BLOCK = 32;  // backward: rows per block (partials granularity), 4 per wave

template <int VPT>
__device__ __forceinline__ void load_row(float (&v)[VPT], const void* base, int dtype, int64_t off) {
  if (dtype == RP_BF16) {
    const bf16* p = (const bf16*)base + off;
    if constexpr (VPT % 8 == 0) {
#pragma unroll
      for (int i = 0; i < VPT; i += 8) {
        uint4 q = *reinterpret_cast<const uint4*>(p + i);
        const bf16* e = reinterpret_cast<const bf16*>(&q);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i + j] = (float)e[j];
      }
    } else if constexpr (VPT % 4 == 0) {
#pragma unroll
      for (int i = 0; i < VPT; i += 4) {
        uint2 q = *reinterpret_cast<const uint2*>(p + i);
        const bf16* e = reinterpret_cast<const bf16*>(&q);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i + j] = (float)e[j];
      }
    } else {
#pragma unroll
      for (int i = 0; i < VPT; ++i) v[i] = (float)p[i];
    }
  } else {
    const float* p = (const float*)base + off;
    if constexpr (VPT % 4 == 0) {
#pragma unroll
      for (int i = 0; i < VPT; i += 4) {
        float4 q = *reinterpret_cast<const float4*>(p + i);
        v[i] = q.x; v[i + 1] = q.y; v[i + 2] = q.z; v[i + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < VPT; ++i) v[i] = p[i];
    }
  }
}

template <int VPT>
__device__ __forceinline__ void store_row(const float (&v)[VPT], void* base, int dtype, int64_t off) {
  if (dtype == RP_BF16) {
    bf16* p = (bf16*)base + off;
    if constexpr (VPT % 8 == 0) {
#pragma unroll
      for (int i = 0; i < VPT; i += 8) {
        uint4 q;
        bf16* e = reinterpret_cast<bf16*>(&q);
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = (bf16)v[i + j];
        *reinterpret_cast<uint4*>(p + i) = q;
      }
    } else if constexpr (VPT % 4 == 0) {
#pragma unroll
      for (int i = 0; i < VPT; i += 4) {
        uint2 q;
        bf16* e = reinterpret_cast<bf16*>(&q);
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = (bf16)v[i + j];
        *reinterpret_cast<uint2*>(p + i) = q;
      }
    } else {
#pragma unroll
      for (int i = 0; i < VPT; ++i) p[i] = (bf16)v[i];
    }
  } else {
    float* p = (float*)base + off;
    if constexpr (VPT % 4 == 0) {
#pragma unroll
      for (int i = 0; i < VPT; i += 4) *reinterpret_cast<float4*>(p + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    } else {
#pragma unroll
      for (int i = 0; i < VPT; ++i) p[i] = v[i];
    }
  }
}

struct LnFwdDev {
  const void* x; int x_dtype; int64_t ldx;
  const float* gamma; const float* beta; float eps;
  const float* pe; int64_t pe_period;
  int relu; uint32_t drop_thresh; float drop_scale; uint32_t drop_seed;
  const uint32_t* seed_base;  // graph-replayable dropout base word (the launch's seed_base argument), or null
  float* out_f32; int64_t ld_out_f32;
  void* out_lp; int out_lp_dtype; int64_t ld_out_lp;
  float* mean; float* rstd;
};

template <int VPT>
__global__ __launch_bounds__(64 * LN_WAVES) void ln_fwd_kernel(int64_t rows, LnFwdDev a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = VPT * 64;
  const int c0 = lane * VPT;
  float v[VPT], pe[VPT], gm[VPT], bt[VPT];
  load_row<VPT>(v, a.x, a.x_dtype, row * a.ldx + c0);
  // the row-independent operands are issued with the row load, not after the reductions
  if (a.pe) load_row<VPT>(pe, a.pe, RP_F32, (row % a.pe_period) * D + c0);
  load_row<VPT>(gm, a.gamma, RP_F32, c0);
  load_row<VPT>(bt, a.beta, RP_F32, c0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) s += v[i];
  const float mean = rp_wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    float d = v[i] - mean;
    q += d * d;
  }
  const float var = rp_wave_sum(q) * (1.f / D);
  const float rstd = rsqrtf(var + a.eps);
  const uint32_t kb = a.drop_thresh ? rp_keep_bits<VPT>(rp_seed_eff(a.seed_base, a.drop_seed), (uint32_t)(row * D + c0), a.drop_thresh) : 0u;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    float y = (v[i] - mean) * rstd * gm[i] + bt[i];
    if (a.pe) y += pe[i];
    if (a.relu) y = fmaxf(y, 0.f);
    if (a.drop_thresh) y = ((kb >> i) & 1u) ? y * a.drop_scale : 0.f;
    v[i] = y;
  }
  if (a.out_f32) store_row<VPT>(v, a.out_f32, RP_F32, row * a.ld_out_f32 + c0);
  if (a.out_lp) store_row<VPT>(v, a.out_lp, a.out_lp_dtype, row * a.ld_out_lp + c0);
  if (lane == 0) {
    if (a.mean) a.mean[row] = mean;
    if (a.rstd) a.rstd[row] = rstd;
  }
}

struct LnBwdDev {
  const void* dy; int dy_dtype; int64_t lddy;
  const void* x; int x_dtype; int64_t ldx;
  const float* mean; const float* rstd; const float* gamma;
  const void* y; int y_dtype; int64_t ldy;
  uint32_t drop_thresh; float drop_scale; uint32_t drop_seed;
  const float* dres; int64_t lddres;
  float* dx; int64_t lddx;
  void* dx_lp; int dx_lp_dtype; int64_t lddx_lp;
  uint32_t lp_thresh; float lp_scale; uint32_t lp_seed;
  const uint32_t* seed_base;  // graph-replayable dropout base word (the launch's seed_base argument), or null
  float* dgamma_part; float* dbeta_part; int64_t ld_part;
};

template <int VPT>
__global__ __launch_bounds__(64 * LNB_WAVES) void ln_bwd_kernel(int64_t rows, LnBwdDev a) {
  constexpr int D = VPT * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = lane * VPT;
  float pg[VPT], pb[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) pg[i] = pb[i] = 0.f;
  float gam[VPT];
  load_row<VPT>(gam, a.gamma, RP_F32, c0);
  const uint32_t dseed = a.drop_thresh ? rp_seed_eff(a.seed_base, a.drop_seed) : 0u;
  const uint32_t lseed = a.lp_thresh ? rp_seed_eff(a.seed_base, a.lp_seed) : 0u;

  const int64_t rbeg = (int64_t)blockIdx.x * LN_ROWS_PER_BLOCK;
  for (int rr = w; rr < LN_ROWS_PER_BLOCK; rr += LNB_WAVES) {
    const int64_t row = rbeg + rr;
    if (row >= rows) break;
    float g[VPT], x[VPT], r[VPT];
    load_row<VPT>(g, a.dy, a.dy_dtype, row * a.lddy + c0);
    load_row<VPT>(x, a.x, a.x_dtype, row * a.ldx + c0);
    if (a.dres) load_row<VPT>(r, a.dres, RP_F32, row * a.lddres + c0);  // issued with the other loads
    float yv[VPT];
    if (a.y) load_row<VPT>(yv, a.y, a.y_dtype, row * a.ldy + c0);
    if (a.drop_thresh) {
      const uint32_t kb = rp_keep_bits<VPT>(dseed, (uint32_t)(row * D + c0), a.drop_thresh);
#pragma unroll
      for (int i = 0; i < VPT; ++i) g[i] = ((kb >> i) & 1u) ? g[i] * a.drop_scale : 0.f;
    }
    if (a.y) {
#pragma unroll
      for (int i = 0; i < VPT; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
    }
    const float mu = a.mean[row], rs = a.rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      x[i] = (x[i] - mu) * rs;  // xhat
      float gg = g[i] * gam[i];
      s1 += gg;
      s2 += gg * x[i];
      pg[i] += g[i] * x[i];
      pb[i] += g[i];
    }
    s1 = rp_wave_sum(s1) * (1.f / D);
    s2 = rp_wave_sum(s2) * (1.f / D);
    float dx[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) dx[i] = rs * (g[i] * gam[i] - s1 - x[i] * s2);
    if (a.dres) {
#pragma unroll
      for (int i = 0; i < VPT; ++i) dx[i] += r[i];
    }
    if (a.dx) store_row<VPT>(dx, a.dx, RP_F32, row * a.lddx + c0);
    if (a.dx_lp) {
      if (a.lp_thresh) {
        const uint32_t kb = rp_keep_bits<VPT>(lseed, (uint32_t)(row * D + c0), a.lp_thresh);
#pragma unroll
        for (int i = 0; i < VPT; ++i) dx[i] = ((kb >> i) & 1u) ? dx[i] * a.lp_scale : 0.f;
      }
      store_row<VPT>(dx, a.dx_lp, a.dx_lp_dtype, row * a.lddx_lp + c0);
    }
  }
  // combine the waves' partial affine gradients through LDS, one partial row per block
  __shared__ float red[2][LNB_WAVES][D];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    red[0][w][c0 + i] = pg[i];
    red[1][w][c0 + i] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 64 * LNB_WAVES) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < LNB_WAVES; ++k) {
      sg += red[0][k][c];
      sb += red[1][k][c];
    }
    if (a.dgamma_part) a.dgamma_part[(int64_t)blockIdx.x * a.ld_part + c] = sg;
    if (a.dbeta_part) a.dbeta_part[(int64_t)blockIdx.x * a.ld_part + c] = sb;
  }
}

#define RP_LN_DISPATCH(KERNEL, D, grid, block, s, rows, a)                                     \
  do {                                                                                        \
    switch (D) {                                                                              \
      case 64: hipLaunchKernelGGL(KERNEL<1>, grid, block, 0, s, rows, a); break;              \
      case 128: hipLaunchKernelGGL(KERNEL<2>, grid, block, 0, s, rows, a); break;             \
      case 256: hipLaunchKernelGGL(KERNEL<4>, grid, block, 0, s, rows, a); break;             \
      case 512: hipLaunchKernelGGL(KERNEL<8>, grid, block, 0, s, rows, a); break;             \
      case 1024: hipLaunchKernelGGL(KERNEL<16>, grid, block, 0, s, rows, a); break;           \
      default:                                                                                \
        rp_set_error("layernorm: D=%lld unsupported (64,128,256,512,1024)", (long long)(D));  \
        return RP_ERR_ARG;                                                                    \
    }                                                                                         \
    return rp_check_launch("rp_layernorm");                                                   \
  } while (0)

}  // namespace

extern "C" int rp_layernorm_fwd(int64_t rows, int64_t D, const rp_ln_fwd_args* p, void* stream) {
  RP_REQUIRE(p && p->x && p->gamma && p->beta, "rp_layernorm_fwd: null argument");
  RP_REQUIRE(p->x_dtype == RP_F32 || p->x_dtype == RP_BF16, "rp_layernorm_fwd: bad x dtype");
  RP_REQUIRE(!p->pe || p->pe_period > 0, "rp_layernorm_fwd: pe_period must be > 0");
  if (rows <= 0) return RP_OK;
  RP_REQUIRE(!p->out_f32 || p->ld_out_f32 % 4 == 0, "rp_layernorm_fwd: ld_out_f32 %% 4");
  RP_REQUIRE(p->x_dtype != RP_F32 || p->ldx % 4 == 0, "rp_layernorm_fwd: ldx %% 4");
  LnFwdDev a{};
  a.x = p->x; a.x_dtype = p->x_dtype; a.ldx = p->ldx;
  a.gamma = p->gamma; a.beta = p->beta; a.eps = p->eps;
  a.pe = p->pe; a.pe_period = p->pe_period;
  a.relu = p->relu;
  RP_REQUIRE(p->dropout_p >= 0.f && p->dropout_p < 1.f, "rp_layernorm_fwd: dropout_p must be in [0, 1)");
  a.drop_thresh = rp_dropout_thresh(p->dropout_p);
  a.drop_scale = p->dropout_p > 0.f ? 1.f / (1.f - p->dropout_p) : 1.f;
  a.drop_seed = p->dropout_seed;
  a.seed_base = a.drop_thresh ? p->seed_base : nullptr;
  a.out_f32 = p->out_f32; a.ld_out_f32 = p->ld_out_f32;
  a.out_lp = p->out_lp; a.out_lp_dtype = p->out_lp_dtype; a.ld_out_lp = p->ld_out_lp;
  a.mean = p->mean; a.rstd = p->rstd;
  dim3 grid((unsigned)((rows + LN_WAVES - 1) / LN_WAVES)), block(64 * LN_WAVES);
  RP_LN_DISPATCH(ln_fwd_kernel, D, grid, block, (hipStream_t)stream, rows, a);
}

extern "C" int64_t rp_layernorm_bwd_blocks(int64_t rows) {
  return (rows + LN_ROWS_PER_BLOCK - 1) / LN_ROWS_PER_BLOCK;
}

extern "C" int rp_layernorm_bwd(int64_t rows, int64_t D, const rp_ln_bwd_args* p, void* stream) {
  RP_REQUIRE(p && p->dy && p->x && p->mean && p->rstd && p->gamma, "rp_layernorm_bwd: null argument");
  if (rows <= 0) return RP_OK;
  LnBwdDev a{};
  a.dy = p->dy; a.dy_dtype = p->dy_dtype; a.lddy = p->lddy;
  a.x = p->x; a.x_dtype = p->x_dtype; a.ldx = p->ldx;
  a.mean = p->mean; a.rstd = p->rstd; a.gamma = p->gamma;
  a.y = p->y; a.y_dtype = p->y_dtype; a.ldy = p->ldy;
  RP_REQUIRE(p->dropout_p >= 0.f && p->dropout_p < 1.f && p->dx_lp_dropout_p >= 0.f && p->dx_lp_dropout_p < 1.f,
             "rp_layernorm_bwd: dropout_p must be in [0, 1)");
  a.drop_thresh = rp_dropout_thresh(p->dropout_p);
  a.drop_scale = p->dropout_p > 0.f ? 1.f / (1.f - p->dropout_p) : 1.f;
  a.drop_seed = p->dropout_seed;
  a.dres = p->dres; a.lddres = p->lddres;
  a.dx = p->dx_f32; a.lddx = p->lddx;
  a.dx_lp = p->dx_lp; a.dx_lp_dtype = p->dx_lp_dtype; a.lddx_lp = p->lddx_lp;
  a.lp_thresh = rp_dropout_thresh(p->dx_lp_dropout_p);
  a.lp_scale = p->dx_lp_dropout_p > 0.f ? 1.f / (1.f - p->dx_lp_dropout_p) : 1.f;
  a.lp_seed = p->dx_lp_seed;
  a.seed_base = (a.drop_thresh || a.lp_thresh) ? p->seed_base : nullptr;
  a.dgamma_part = p->dgamma_part; a.dbeta_part = p->dbeta_part;
  a.ld_part = p->ld_part ? p->ld_part : D;
  RP_REQUIRE(a.ld_part >= D, "rp_layernorm_bwd: ld_part < D");
  dim3 grid((unsigned)rp_layernorm_bwd_blocks(rows)), block(64 * LNB_WAVES);
  RP_LN_DISPATCH(ln_bwd_kernel, D, grid, block, (hipStream_t)stream, rows, a);
}
