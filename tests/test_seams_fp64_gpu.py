"""The bf16 kernels that ship at the metric shape (M = B*T = 16384 tokens) against an fp64 torch
restatement of the op they compute — not only against the unfused HIP kernels they replace:

* the exchange GEMM + LayerNorm seams (rp_gemm_ln_fwd / rp_gemm_ln_bwd on 128 x 128 tiles, and forced
  onto the 64- and 32-row exchange tiles): ``y = dropout(x W^T + b) + residual``, ``h = LayerNorm(y)``
  (reference: nn.TransformerEncoderLayer's out_proj / linear2 + dropout + residual + norm,
  /root/reference/models/MMCTransformer.py:41-55), and the backward's dh = dY W, LayerNorm backward,
  residual-gradient add, masked bf16 copy and gamma / beta gradients;
* the d_ff = 2048 GEMMs on the 256-row phased kernel (linear1 forward with ReLU + dropout, linear2
  dgrad gated by the saved activation);
* the out_proj dgrad with the attention delta in its epilogue (rp_gemm_attn_dout_delta).

Dropout masks come from the torch restatement of the element stream (test_kernels_gpu.keep_mask).
Tolerances: fp32 accumulation against fp64 (1e-4-scale absolute), one bf16 rounding step on bf16
outputs, fp32 summation order on the column sums."""
import math

import pytest
import torch

from repurpose_amd import _native as N
from repurpose_amd import kernels as K

from .test_kernels_gpu import close, keep_mask, rnd

pytestmark = pytest.mark.gpu
D = 512
M = 16384


@pytest.fixture(params=[(0, 16384), (64, 16384), (32, 16384), (0, 8192), (0, 4096)],
                ids=["auto-16384", "64rows-16384", "32rows-16384", "auto-8192", "auto-4096"])
def rows(request):
    """(tile rows, M): 0 = the host's own choice — 128-row exchange tiles at the metric shape
    (M = 16384), 64-row at config 2 (M = 8192), 32-row at config 4 (M = 4096); 64 / 32 forced at the
    metric shape."""
    N.call("rp_debug_set_lnx_rows", int(request.param[0]))
    yield request.param
    N.call("rp_debug_set_lnx_rows", 0)


def _bf16_close(got, ref, what, extra=0.0):
    """got (bf16) is ref (fp64) rounded once to bf16, up to one more bf16 step and ``extra`` absolute."""
    g, r = got.double(), ref.double()
    lim = r.abs() * 2.0 ** -8 + 1e-6 + extra
    bad = int(((g - r).abs() > lim).sum().item())
    assert bad == 0, f"{what}: {bad} elements off, max err {(g - r).abs().max().item():.3e}"


def _drop(z, seed, p):
    if not p:
        return z
    idx = torch.arange(z.numel(), device=z.device, dtype=torch.int64).view(z.shape)
    return torch.where(keep_mask(seed, idx, p), z / (1.0 - p), torch.zeros_like(z))


@pytest.mark.parametrize("Kd,p", [(512, 0.1), (2048, 0.1), (2048, 0.0)])
def test_seam_fwd_against_fp64(dev, rows, Kd, p):
    M = rows[1]
    x = rnd(M, Kd, dev=dev, seed=Kd + 1).to(torch.bfloat16)
    W = rnd(D, Kd, dev=dev, seed=Kd + 2, scale=0.03).to(torch.bfloat16)
    b = rnd(D, dev=dev, seed=Kd + 3, scale=0.1)
    res = rnd(M, D, dev=dev, seed=Kd + 4) + 1.0
    gm = 1.0 + rnd(D, dev=dev, seed=Kd + 5, scale=0.1)
    bt = rnd(D, dev=dev, seed=Kd + 6, scale=0.1)
    y, h, mu, rs = K.linear_ln_fwd(x, W, b, res, gm, bt, dropout_p=p, seed=77)
    torch.cuda.synchronize()
    y_ref = _drop(x.double() @ W.double().T + b.double(), 77, p) + res.double()
    close(y, y_ref, atol=2e-4 * math.sqrt(Kd / 512), what="x_out")
    # the LayerNorm of the kernel's own x_out, in fp64
    yd = y.double()
    mu_ref = yd.mean(1)
    rs_ref = 1.0 / torch.sqrt(((yd - mu_ref[:, None]) ** 2).mean(1) + 1e-5)
    close(mu, mu_ref, atol=1e-6, rtol=1e-5, what="mean")
    close(rs, rs_ref, atol=0, rtol=1e-5, what="rstd")
    h_ref = (yd - mu_ref[:, None]) * rs_ref[:, None] * gm.double() + bt.double()
    _bf16_close(h, h_ref, "h")


@pytest.mark.parametrize("Kd,lp", [(2048, 0.1), (1536, 0.1), (1536, 0.0)])
def test_seam_bwd_against_fp64(dev, rows, Kd, lp):
    M = rows[1]
    dy = rnd(M, Kd, dev=dev, seed=3 * Kd + 1).to(torch.bfloat16)
    W = rnd(Kd, D, dev=dev, seed=3 * Kd + 2, scale=0.03).to(torch.bfloat16)
    x = rnd(M, D, dev=dev, seed=3 * Kd + 3) + 0.5
    gm = 1.0 + rnd(D, dev=dev, seed=3 * Kd + 4, scale=0.1)
    _, _, mu, rs = K.layernorm_fwd(x, gm, torch.zeros(D, device=dev), out_f32=False, lp_dtype=torch.bfloat16)
    dres = rnd(M, D, dev=dev, seed=3 * Kd + 5)
    flat = torch.zeros(2 * D, device=dev)  # gamma | beta gradients, adjacent as in the flat gradient buffer
    dx, dxl = K.linear_ln_bwd(dy, W, x, mu, rs, gm, dres=dres, lp_dtype=torch.bfloat16, lp_dropout_p=lp, lp_seed=5,
                              dgamma=flat[:D], dbeta=flat[D:])
    torch.cuda.synchronize()
    dh = dy.double() @ W.double()
    xh = (x.double() - mu.double()[:, None]) * rs.double()[:, None]
    g = dh * gm.double()
    dx_ref = rs.double()[:, None] * (g - g.mean(1, keepdim=True) - xh * (g * xh).mean(1, keepdim=True)) + dres.double()
    close(dx, dx_ref, atol=2e-4 * math.sqrt(Kd / 512), what="dx")
    _bf16_close(dxl, _drop(dx.double(), 5, lp), "dx_lp")
    dgam, dbet = (dh * xh).sum(0), dh.sum(0)
    close(flat[:D], dgam, atol=2e-5 * dgam.abs().max().item() + 2e-3, what="dgamma")
    close(flat[D:], dbet, atol=2e-5 * dbet.abs().max().item() + 2e-3, what="dbeta")


@pytest.mark.parametrize("M", [16384, 4096])
def test_dff_gemms_against_fp64(dev, M):
    """linear1 forward (ReLU + dropout, bf16 out) and linear2 dgrad through the saved activation's
    gate (bf16 out): the 256-row phased kernel at the metric shape; at config 4 (M = 4096) the
    gate-batched 32 / 64-row tiles."""
    Kd, F, p = 512, 2048, 0.1
    x = rnd(M, Kd, dev=dev, seed=21).to(torch.bfloat16)
    W1 = rnd(F, Kd, dev=dev, seed=22, scale=0.05).to(torch.bfloat16)
    b1 = rnd(F, dev=dev, seed=23, scale=0.1)
    h = K.linear_fwd(x, W1, b1, out_dtype=torch.bfloat16, relu=True, dropout_p=p, seed=99)
    torch.cuda.synchronize()
    h_ref = _drop(torch.relu(x.double() @ W1.double().T + b1.double()), 99, p)
    _bf16_close(h, h_ref, "linear1 forward", extra=2e-5)
    frac = (h == 0).float().mean().item()
    assert 0.5 < frac < 0.6, frac  # ReLU zeros half, dropout another tenth of the rest
    W2 = rnd(D, F, dev=dev, seed=24, scale=0.03).to(torch.bfloat16)
    g2 = rnd(M, D, dev=dev, seed=25).to(torch.bfloat16)
    dh = K.linear_dgrad(g2, W2, out_dtype=torch.bfloat16, gate=h, gate_scale=1.0 / (1.0 - p))
    torch.cuda.synchronize()
    dh_ref = (g2.double() @ W2.double()) * (h.double() > 0) / (1.0 - p)
    _bf16_close(dh, dh_ref, "linear2 dgrad (gated)", extra=2e-5)


@pytest.mark.parametrize("p", [0.1, 0.0])
@pytest.mark.parametrize("B,T", [(8, 2048), (8, 1024), (1, 4096)])
def test_dout_delta_against_fp64(dev, p, B, T):
    """dO = g1 W (bf16) and the three delta planes, from the stored bf16 dO and the attention output
    hi + lo, against fp64 — at the metric shape (128-row tiles) and configs 2 / 4 (64- / 32-row)."""
    H = 8
    M = B * T
    g1 = rnd(M, D, dev=dev, seed=31).to(torch.bfloat16)
    W = rnd(D, D, dev=dev, seed=32, scale=0.05).to(torch.bfloat16)
    o = rnd(M, D, dev=dev, seed=33).to(torch.bfloat16)
    olo = (rnd(M, D, dev=dev, seed=34) * 2.0 ** -9).to(torch.bfloat16)
    lse = rnd(B, H, T, dev=dev, seed=35)
    dO, delta = K.attn_dout_delta(g1, W, o, olo, lse, B, T, H, p)
    torch.cuda.synchronize()
    _bf16_close(dO, g1.double() @ W.double(), "dO", extra=2e-5)
    dd = (dO.double() * (o.double() + olo.double())).view(B, T, H, 64).sum(-1).permute(0, 2, 1)  # [B, H, T]
    ds = 1.0 / (1.0 - p)
    close(delta[0], dd, atol=1e-4, rtol=1e-5, what="delta")
    close(delta[1], -dd / ds, atol=1e-4, rtol=1e-5, what="-delta / ds")
    close(delta[2], -(lse.double() * math.log2(math.e) - math.log2(ds)), atol=1e-5, rtol=1e-6, what="lse plane")


def test_qkv_forward_against_fp64(dev):
    """The QKV projection as the step launches it (bf16 out, the Q columns prescaled by
    scale * log2(e) after the bias — the attention kernels' RP_ATTN_Q_PRESCALED input) at the metric
    shape: 1,536 tiles of 128 x 128 on the one-stage LDS configuration."""
    x = rnd(M, D, dev=dev, seed=41).to(torch.bfloat16)
    W = rnd(3 * D, D, dev=dev, seed=42, scale=0.05).to(torch.bfloat16)
    b = rnd(3 * D, dev=dev, seed=43, scale=0.1)
    c = 0.125 * math.log2(math.e)
    y = K.linear_fwd(x, W, b, out_dtype=torch.bfloat16, col_scale_n=D, col_scale=c)
    torch.cuda.synchronize()
    ref = x.double() @ W.double().T + b.double()
    ref[:, :D] *= c
    _bf16_close(y, ref, "qkv", extra=2e-5)

