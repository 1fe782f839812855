"""The fused GEMM + LayerNorm seams (rp_gemm_ln_fwd / rp_gemm_ln_bwd) against the unfused pair of
launches they replace: linear_fwd(residual, dropout) -> layernorm_fwd and linear_dgrad(fp32) ->
layernorm_bwd (reference seams: the pre-LN encoder layer of models/MMCTransformer.py:41-55, x1 = x +
drop1(out_proj(.)), norm2(x1), and their autograd).  The 64-row full-row kernels (RP_GEMM_LNX=0) bit
for bit; the 128 x 128 kernels whose column tiles exchange the row statistics with x_out bitwise and the
LayerNorm outputs to fp32 rounding of the row sums, the exchange workspace left zeroed, no wait given up.
Shapes are the encoder's: K = 512 (out_proj) and 2048 (linear2) forward, K = 2048 (linear1) and 1536
(in_proj) backward, plus the bench's row count."""
import ctypes

import pytest
import torch

from repurpose_amd import _native as N
from repurpose_amd import kernels as K


@pytest.fixture
def rows64(monkeypatch):
    monkeypatch.setenv("RP_GEMM_LNX", "0")

pytestmark = pytest.mark.gpu

D = 512


def _r(g, *s, dev, dt=torch.bfloat16, sc=1.0):
    return (torch.randn(*s, generator=g) * sc).to(dev, dt)


@pytest.mark.parametrize("M,Kd,p", [(1024, 512, 0.0), (1024, 2048, 0.1), (16384, 512, 0.1), (64, 1536, 0.1)])
def test_linear_ln_fwd_bitwise(dev, rows64, M, Kd, p):
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
def test_linear_ln_bwd_bitwise(dev, rows64, M, Kd, lp, with_lp):
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

    monkeypatch.setenv("RP_GEMM_LNX", "0")
    l0, o0, g0 = run("0")
    l1, o1, g1 = run("1")  # the 64-row full-row kernels
    assert torch.equal(o0, o1)
    assert torch.equal(l0, l1)
    assert torch.equal(g0, g1), f"grads: {(g0 - g1).abs().max().item():.3e}"


def _force_rows(rows):
    N.call("rp_debug_set_lnx_rows", int(rows))


@pytest.fixture(params=["32", "64", "128"])
def lnx_rows(request):
    """The exchange tile height: 32 x 128 or 64 x 128 tiles (the host's choices where taller tiles would
    leave CUs idle) or 128 x 128 ones (M % 128 == 0, else 64), forced by the rp_debug_set_lnx_rows hook."""
    _force_rows(request.param)
    yield request.param
    _force_rows(0)


def _ws_clean(dev, M):
    """The error word and the arrive / done counters of every row block are zero again (the partial
    pairs after them are data)."""
    ws = K._lnx_ws(torch.device(dev), M)
    assert ws is not None
    torch.cuda.synchronize()
    assert int(ws[:4].count_nonzero().item()) == 0, "an exchange wait gave up"
    rec = 256 + 4 * 128 * 8  # one 128-row record: four counter pairs (32 of 256 bytes), then its partial pairs
    nr = (M + 127) // 128
    head = ws[256:256 + nr * rec].view(nr, rec)[:, :32]
    assert int(head.count_nonzero().item()) == 0, "exchange counters not left zeroed"


def _close_bf16(u, v):
    """bf16 outputs of row statistics that differ in the last fp32 bits: at most one bf16 step apart."""
    u, v = u.float(), v.float()
    tol = u.abs() * 2.0 ** -7 + 1e-6
    assert bool(((u - v).abs() <= tol).all()), f"max diff {(u - v).abs().max().item():.3e}"
    assert (u != v).float().mean().item() < 0.01


@pytest.mark.parametrize("M,Kd,p", [(1024, 512, 0.0), (1024, 2048, 0.1), (16384, 512, 0.1), (16384, 2048, 0.1),
                                    (128, 1536, 0.1), (4096, 512, 0.1), (192, 2048, 0.1)])
def test_linear_ln_fwd_exchange(dev, lnx_rows, M, Kd, p):
    g = torch.Generator().manual_seed(M + Kd + 1)
    x, W = _r(g, M, Kd, dev=dev), _r(g, D, Kd, dev=dev, sc=0.03)
    b = _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    res = _r(g, M, D, dev=dev, dt=torch.float32) + 3.0  # a row mean far from 0: the parallel variance
    gm, bt = 1.0 + _r(g, D, dev=dev, dt=torch.float32, sc=0.1), _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    y0 = K.linear_fwd(x, W, b, out_dtype=torch.float32, dropout_p=p, seed=77, residual=res)
    _, h0, mu0, rs0 = K.layernorm_fwd(y0, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
    outs = [K.linear_ln_fwd(x, W, b, res, gm, bt, dropout_p=p, seed=77) for _ in range(3)]
    torch.cuda.synchronize()
    y1, h1, mu1, rs1 = outs[0]
    assert torch.equal(y0, y1), f"x_out: {(y0 - y1).abs().max().item():.3e}"
    torch.testing.assert_close(mu1, mu0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rs1, rs0, rtol=1e-5, atol=0)
    _close_bf16(h0, h1)
    for o in outs[1:]:  # deterministic launch to launch: the counters come back to zero
        assert all(torch.equal(u, v) for u, v in zip(outs[0], o))
    _ws_clean(dev, M)


@pytest.mark.parametrize("M,Kd,lp", [(1024, 2048, 0.1), (1024, 1536, 0.0), (16384, 2048, 0.1), (16384, 1536, 0.1),
                                     (128, 512, 0.1), (4096, 2048, 0.1), (192, 512, 0.0)])
@pytest.mark.parametrize("with_lp", [True, False])
def test_linear_ln_bwd_exchange(dev, lnx_rows, M, Kd, lp, with_lp):
    g = torch.Generator().manual_seed(3 * M + Kd + 1)
    dy, W = _r(g, M, Kd, dev=dev), _r(g, Kd, D, dev=dev, sc=0.03)
    x = _r(g, M, D, dev=dev, dt=torch.float32)
    gm = 1.0 + _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    _, _, mu, rs = K.layernorm_fwd(x, gm, torch.zeros(D, device=dev), out_f32=False, lp_dtype=torch.bfloat16)
    dres = _r(g, M, D, dev=dev, dt=torch.float32)
    lpd = torch.bfloat16 if with_lp else None
    flat0 = torch.zeros(2 * D, device=dev)
    dh = K.linear_dgrad(dy, W, out_dtype=torch.float32)
    dx0, dl0 = K.layernorm_bwd(dh, x, mu, rs, gm, dres=dres, lp_dtype=lpd, lp_dropout_p=lp, lp_seed=5,
                               dgamma=flat0[:D], dbeta=flat0[D:])
    runs = []
    for _ in range(2):
        flat1 = torch.zeros(2 * D, device=dev)
        dx1, dl1 = K.linear_ln_bwd(dy, W, x, mu, rs, gm, dres=dres, lp_dtype=lpd, lp_dropout_p=lp, lp_seed=5,
                                   dgamma=flat1[:D], dbeta=flat1[D:])
        runs.append((dx1, dl1, flat1))
    torch.cuda.synchronize()
    dx1, dl1, flat1 = runs[0]
    scale = dx0.abs().max().item()
    assert (dx1 - dx0).abs().max().item() <= 2e-6 * scale, f"dx: {(dx1 - dx0).abs().max().item():.3e} of {scale:.3e}"
    if with_lp:
        _close_bf16(dl0, dl1)
    else:
        assert dl0 is None and dl1 is None
    torch.testing.assert_close(flat1, flat0, rtol=1e-4, atol=1e-4 * flat0.abs().max().item())
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][2], runs[1][2])
    _ws_clean(dev, M)


def test_model_fused_seams_exchange(dev, lnx_rows, monkeypatch):
    """A bf16 training step with every seam on the exchange kernels: against the unfused bf16 step the
    loss and logits agree to bf16 rounding; against the fp32 step (dropout off) its gradients are as close
    as the unfused bf16 step's (within 1.25x: the two bf16 steps differ from each other by about as much
    as either differs from fp32, 4 % at this small shape)."""
    from repurpose_amd.MMCTransformer import MMCTransformer

    from .test_model_gpu import TRI, make_batch, to_dev

    b = to_dev(make_batch(TRI, 2, 256, [256, 190], seed=4), dev)

    def run(flag, dtype, p):
        monkeypatch.setenv("RP_GEMM_LN", flag)
        torch.manual_seed(11)
        m = MMCTransformer(**TRI, compute_dtype=dtype).to(dev).train()
        if p is not None:
            m.DROPOUT = p
        out = m(b)
        loss = m.losses(*out)["cls_loss"]
        loss.backward()
        torch.cuda.synchronize()
        assert torch.isfinite(loss).item()
        return loss.detach(), out[1].detach().float().clone(), m.flat_grads()[:m.trainable_numel()].double().clone()

    l0, o0, _ = run("0", "bf16", None)  # dropout on
    l1, o1, _ = run("1", "bf16", None)
    assert abs(l1.item() - l0.item()) <= 1e-3 * abs(l0.item())
    assert (o1 - o0).abs().max().item() <= 3e-2 * o0.abs().max().item()
    _, _, g32 = run("0", "fp32", 0.0)
    _, _, g0 = run("0", "bf16", 0.0)
    _, _, g1 = run("1", "bf16", 0.0)
    e0 = ((g0 - g32).norm() / g32.norm()).item()
    e1 = ((g1 - g32).norm() / g32.norm()).item()
    print(f"step gradients vs fp32: unfused bf16 {e0:.3e}, exchange seams {e1:.3e}")
    assert e1 <= 1.25 * e0 + 1e-3, (e0, e1)
    _ws_clean(dev, 512)


def test_linear_ln_exchange_mixed_rows(dev):
    """One workspace shared by launches of different row counts and tile heights (the record of a row
    block does not move with M or the kernel): each launch agrees with the unfused pair and leaves the
    counters zeroed."""
    try:
        _mixed_rows(dev)
    finally:
        _force_rows(0)


def _mixed_rows(dev):
    for M, rows in ((4096, "128"), (8192, "64"), (16384, "128"), (1024, "64"), (8192, "128"), (384, "64"),
                    (4096, "32"), (320, "128"), (8192, "32"), (4096, "64"), (192, "32")):
        _force_rows(rows)
        g = torch.Generator().manual_seed(M)
        x, W = _r(g, M, 512, dev=dev), _r(g, D, 512, dev=dev, sc=0.03)
        b, res = _r(g, D, dev=dev, dt=torch.float32, sc=0.1), _r(g, M, D, dev=dev, dt=torch.float32)
        gm, bt = 1.0 + _r(g, D, dev=dev, dt=torch.float32, sc=0.1), _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
        y0 = K.linear_fwd(x, W, b, out_dtype=torch.float32, residual=res)
        _, h0, mu0, rs0 = K.layernorm_fwd(y0, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
        _, h1, mu1, rs1 = K.linear_ln_fwd(x, W, b, res, gm, bt)
        torch.testing.assert_close(mu1, mu0, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rs1, rs0, rtol=1e-5, atol=0)
        _close_bf16(h0, h1)
        _ws_clean(dev, M)


# ------------------------------------------------------------------ exchange progress and fault reporting
def _fwd_case(dev, M, Kd, seed):
    g = torch.Generator().manual_seed(seed)
    x, W = _r(g, M, Kd, dev=dev), _r(g, D, Kd, dev=dev, sc=0.03)
    b, res = _r(g, D, dev=dev, dt=torch.float32, sc=0.1), _r(g, M, D, dev=dev, dt=torch.float32)
    gm, bt = 1.0 + _r(g, D, dev=dev, dt=torch.float32, sc=0.1), _r(g, D, dev=dev, dt=torch.float32, sc=0.1)
    return x, W, b, res, gm, bt


def _fwd_check(x, W, b, res, gm, bt, p=0.1):
    y0 = K.linear_fwd(x, W, b, out_dtype=torch.float32, dropout_p=p, seed=9, residual=res)
    _, h0, mu0, rs0 = K.layernorm_fwd(y0, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
    y1, h1, mu1, rs1 = K.linear_ln_fwd(x, W, b, res, gm, bt, dropout_p=p, seed=9)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    torch.testing.assert_close(mu1, mu0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rs1, rs0, rtol=1e-5, atol=0)
    _close_bf16(h0, h1)


@pytest.mark.parametrize("fwd", [True, False])
def test_exchange_missing_partner_fails_loudly(dev, fwd):
    """A launch whose last row block lacks a partner tile (the test hook launches one workgroup fewer than
    the grid) gives up after its bound and sets the library's fault word: rp_gemm_ln_status and the next
    seam call raise RuntimeError (never a silent result), the workspace is reset, and the seams that follow
    agree with the unfused pair again with the counters left zeroed."""
    M, Kd = 4096, 512
    x, W, b, res, gm, bt = _fwd_case(dev, M, Kd, 21)
    assert N.load().rp_gemm_ln_status() == N.RP_OK
    if fwd:
        a, outs = K.ln_fwd_args(x, W, b, res, gm, bt)
    else:
        _, _, mu, rs = K.layernorm_fwd(res, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
        a, outs = K.ln_bwd_args(x, W.t().contiguous(), res, mu, rs, gm, dres=res, lp_dtype=torch.bfloat16)
    tiles = 127  # the first 127 workgroups: every row block of the first four 32-block chunks but the last is whole
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    N.call("rp_debug_gemm_ln_partial", int(fwd), M, Kd, ctypes.byref(a), tiles, 0.05, st)
    torch.cuda.synchronize()
    assert N.load().rp_gemm_ln_status() == N.RP_ERR_LAUNCH
    assert "gave up" in N.last_error()
    with pytest.raises(RuntimeError, match="gave up"):  # the next seam call refuses to run
        K.linear_ln_fwd(x, W, b, res, gm, bt)
    assert N.load().rp_gemm_ln_status() == N.RP_OK  # reset by the failing call's handler
    _ws_clean(dev, M)
    _fwd_check(x, W, b, res, gm, bt)
    _ws_clean(dev, M)
    # the same through the status check a captured step's replay runs
    N.call("rp_debug_gemm_ln_partial", int(fwd), M, Kd, ctypes.byref(a), tiles, 0.05, st)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="gave up"):
        K.lnx_status()
    K.lnx_status()
    _ws_clean(dev, M)


def test_exchange_beside_long_kernel(dev):
    """A seam launched while another stream's long kernel holds CU slots (384 workgroups with 64 KiB of LDS
    each for 150 ms: half the CUs cannot take a seam workgroup until it retires): forward and backward
    still equal the unfused pair, no wait gives up, the counters come back to zero."""
    M = 16384
    x, W, b, res, gm, bt = _fwd_case(dev, M, 512, 22)
    dy = _r(torch.Generator().manual_seed(5), M, 2048, dev=dev)
    W2 = _r(torch.Generator().manual_seed(6), 2048, D, dev=dev, sc=0.03)
    _, _, mu, rs = K.layernorm_fwd(res, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
    dh = K.linear_dgrad(dy, W2, out_dtype=torch.float32)
    dx0, dl0 = K.layernorm_bwd(dh, res, mu, rs, gm, dres=res, lp_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(dev)
    for _ in range(2):
        N.call("rp_debug_occupy", 384, 150000, ctypes.c_void_p(side.cuda_stream))
        _fwd_check(x, W, b, res, gm, bt)
        N.call("rp_debug_occupy", 384, 150000, ctypes.c_void_p(side.cuda_stream))
        dx1, dl1 = K.linear_ln_bwd(dy, W2, res, mu, rs, gm, dres=res, lp_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        assert (dx1 - dx0).abs().max().item() <= 2e-6 * dx0.abs().max().item()
        _close_bf16(dl0, dl1)
    K.lnx_status()
    _ws_clean(dev, M)


@pytest.mark.parametrize("rows", ["128", "32"])
def test_exchange_launches_split_at_capacity(dev, rows):
    """Row counts whose exchange grid exceeds the co-resident capacity (CUs x 2) are issued as several
    launches of whole row blocks: M = 32,768 on 128-row tiles (two launches on 256 CUs) and M = 16,384 on
    forced 32-row tiles (four).  Results equal the unfused pair (dropout indices are the seam's global
    rows), the counters return to zero."""
    _force_rows(rows)
    try:
        M = 32768 if rows == "128" else 16384
        _fwd_check(*_fwd_case(dev, M, 512, 23))
        _ws_clean(dev, M)
    finally:
        _force_rows(0)
