"""The fused GEMM + LayerNorm seams (rp_gemm_ln_fwd / rp_gemm_ln_bwd) against the unfused pair of
launches they replace, bit for bit: linear_fwd(residual, dropout) -> layernorm_fwd and
linear_dgrad(fp32) -> layernorm_bwd (reference seams: the pre-LN encoder layer of
models/MMCTransformer.py:41-55, x1 = x + drop1(out_proj(.)), norm2(x1), and their autograd).  Shapes
are the encoder's: K = 512 (out_proj) and 2048 (linear2) forward, K = 2048 (linear1) and 1536
(in_proj) backward, plus the bench's row count."""
import pytest
import torch

from repurpose_amd import kernels as K

pytestmark = pytest.mark.gpu

D = 512


def _r(g, *s, dev, dt=torch.bfloat16, sc=1.0):
    return (torch.randn(*s, generator=g) * sc).to(dev, dt)


@pytest.mark.parametrize("M,Kd,p", [(1024, 512, 0.0), (1024, 2048, 0.1), (16384, 512, 0.1), (64, 1536, 0.1)])
def test_linear_ln_fwd_bitwise(dev, M, Kd, p):
    g = torch.Generator().manual_seed(M + Kd)
    x, W = _r(g, M, Kd, dev=dev), _r(g, D, Kd, dev=dev, sc=0.03)
    b = _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    res = _r(g, M, D, dev=dev, dt=torch.float32)
    gm, bt = 1.0 + _r(g, D, dev=dev, dt=torch.float32, sc=0.1), _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    y0 = K.linear_fwd(x, W, b, out_dtype=torch.float32, dropout_p=p, seed=77, residual=res)
    _, h0, mu0, rs0 = K.layernorm_fwd(y0, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
    y1, h1, mu1, rs1 = K.linear_ln_fwd(x, W, b, res, gm, bt, dropout_p=p, seed=77)
    torch.cuda.synchronize()
    for n, u, v in (("y", y0, y1), ("h", h0, h1), ("mean", mu0, mu1), ("rstd", rs0, rs1)):
        assert torch.equal(u, v), f"{n}: max diff {(u.float() - v.float()).abs().max().item():.3e}"


@pytest.mark.parametrize("M,Kd,lp", [(1024, 2048, 0.1), (1024, 1536, 0.0), (16384, 2048, 0.1), (64, 512, 0.1)])
@pytest.mark.parametrize("with_lp", [True, False])
def test_linear_ln_bwd_bitwise(dev, M, Kd, lp, with_lp):
    g = torch.Generator().manual_seed(3 * M + Kd)
    dy, W = _r(g, M, Kd, dev=dev), _r(g, Kd, D, dev=dev, sc=0.03)
    x = _r(g, M, D, dev=dev, dt=torch.float32)
    gm = 1.0 + _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    _, _, mu, rs = K.layernorm_fwd(x, gm, torch.zeros(D, device=dev), out_f32=False, lp_dtype=torch.bfloat16)
    dres = _r(g, M, D, dev=dev, dt=torch.float32)
    lpd = torch.bfloat16 if with_lp else None
    flat0 = torch.zeros(2 * D, device=dev)  # gamma | beta adjacent, as in the flat gradient buffer
    flat1 = torch.zeros(2 * D, device=dev)
    dh = K.linear_dgrad(dy, W, out_dtype=torch.float32)
    dx0, dl0 = K.layernorm_bwd(dh, x, mu, rs, gm, dres=dres, lp_dtype=lpd, lp_dropout_p=lp, lp_seed=5,
                               dgamma=flat0[:D], dbeta=flat0[D:])
    dx1, dl1 = K.linear_ln_bwd(dy, W, x, mu, rs, gm, dres=dres, lp_dtype=lpd, lp_dropout_p=lp, lp_seed=5,
                               dgamma=flat1[:D], dbeta=flat1[D:])
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1), f"dx: {(dx0 - dx1).abs().max().item():.3e}"
    if with_lp:
        assert torch.equal(dl0, dl1)
    else:
        assert dl0 is None and dl1 is None
    assert torch.equal(flat0, flat1), f"dgamma/dbeta: {(flat0 - flat1).abs().max().item():.3e}"


def test_linear_ln_rejects_bad_shapes(dev):
    x = torch.zeros(100, 512, device=dev, dtype=torch.bfloat16)  # M not a multiple of 64
    W = torch.zeros(512, 512, device=dev, dtype=torch.bfloat16)
    v = torch.zeros(512, device=dev)
    with pytest.raises(RuntimeError, match="multiple of 64"):
        K.linear_ln_fwd(x, W, v, torch.zeros(100, 512, device=dev), v, v)


def test_model_fused_seams_bitwise(dev, monkeypatch):
    """A bf16 training step (dropout on) with the fused seams equals the unfused step bit for bit:
    loss, logits and every gradient (L = 2 tri-modal, ragged lengths)."""
    from repurpose_amd.MMCTransformer import MMCTransformer

    from .test_model_gpu import TRI, make_batch, to_dev

    b = to_dev(make_batch(TRI, 2, 256, [256, 190], seed=4), dev)

    def run(flag):
        monkeypatch.setenv("RP_GEMM_LN", flag)
        torch.manual_seed(11)
        m = MMCTransformer(**TRI, compute_dtype="bf16").to(dev).train()
        out = m(b)
        loss = m.losses(*out)["cls_loss"]
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach(), out[1].detach().clone(), m.flat_grads()[:m.trainable_numel()].clone()

    l0, o0, g0 = run("0")
    l1, o1, g1 = run("1")  # opt-in path
    assert torch.equal(o0, o1)
    assert torch.equal(l0, l1)
    assert torch.equal(g0, g1), f"grads: {(g0 - g1).abs().max().item():.3e}"
