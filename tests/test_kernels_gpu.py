"""Per-kernel numerics on the GPU, each HIP kernel against a plain PyTorch fp32/fp64 reference of
the same op (dropout masks reproduced by a torch restatement of the counter hash)."""
import math

import numpy as np
import pytest
import torch

from repurpose_amd import kernels as K

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF


def rp_hash(seed, idx):
    h = (idx * 0x9E3779B1 + seed) & M32
    h = h ^ (h >> 16)
    h = (h * 0x7FEB352D) & M32
    h = h ^ (h >> 15)
    h = (h * 0x846CA68B) & M32
    h = h ^ (h >> 16)
    return h


def keep_mask(seed, idx, p):
    """GEMM / LayerNorm element dropout (csrc/rp_common.h rp_keep8): per aligned group of 8
    elements one rp_hash word w0, then three MWC64X words (x ^ c) from x = w0, c = w0 >> 1; 16-bit
    halves read as int16."""
    thr = int(p * 65536 + 0.5)
    w0 = rp_hash(seed, idx >> 3)
    words = [w0]
    x, c = w0, w0 >> 1
    for _ in range(3):
        x, c = mwc_step(x, c)
        words.append(x ^ c)
    W = torch.stack(words, -1)
    e = idx & 7
    w = torch.gather(W, -1, (e >> 1).unsqueeze(-1)).squeeze(-1)
    half = torch.where((e & 1) == 1, w >> 16, w & 0xFFFF)
    sgn = torch.where(half >= 32768, half - 65536, half)
    return sgn >= thr - 32768


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev)


def close_per_seq(a, b, B, atol, rtol=0.0, what=""):
    """close() with the absolute tolerance taken relative to each sequence's gradient magnitude
    (rows [B*T, cols], sequence s = rows s*T..): a sequence with one or two valid keys collects every
    query's probability mass on them, so its dV is a sum of ~T dO rows (|dV| ~ 100 at T = 1030) and
    an absolute bound sized for |dV| ~ 1 would demand 5 significant digits from bf16."""
    a = a.double().cpu()
    b = b.double().cpu()
    T = a.shape[0] // B
    lim = torch.empty_like(b)
    for s_ in range(B):
        rows = slice(s_ * T, (s_ + 1) * T)
        lim[rows] = atol * max(1.0, b[rows].abs().max().item()) + rtol * b[rows].abs()
    err = (a - b).abs()
    bad = (err > lim).sum().item()
    assert bad == 0, f"{what}: {bad} elements off, max err {err.max().item():.3e}"


def close(a, b, atol, rtol=0.0, what=""):
    a = a.double().cpu()
    b = b.double().cpu()
    err = (a - b).abs()
    lim = atol + rtol * b.abs()
    bad = (err > lim).sum().item()
    assert bad == 0, f"{what}: {bad} elements off, max err {err.max().item():.3e}"


# ----------------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,Kd", [(256, 128, 64), (300, 136, 200), (17, 520, 2944), (1000, 1536, 512), (333, 200, 128)])
def test_gemm_three_layouts(dev, dtype, M, N, Kd):
    x = rnd(M, Kd, dev=dev, seed=1).to(dtype)
    w = rnd(N, Kd, dev=dev, seed=2, scale=0.05).to(dtype)
    b = rnd(N, dev=dev, seed=3)
    tol = 2e-4 if dtype == torch.float32 else 2e-3
    xd, wd = x.double(), w.double()
    y = K.linear_fwd(x, w, b, out_dtype=torch.float32)
    close(y, xd @ wd.T + b.double(), atol=tol * math.sqrt(Kd), what="fwd")
    dy = rnd(M, N, dev=dev, seed=4).to(dtype)
    dx = K.linear_dgrad(dy, w, out_dtype=torch.float32)
    close(dx, dy.double() @ wd, atol=tol * math.sqrt(N), what="dgrad")
    dW = torch.full((N, Kd), 0.5, device=dev)
    K.linear_wgrad(dy, x, dW, accumulate=True)
    close(dW, dy.double().T @ xd + 0.5, atol=tol * math.sqrt(M) * 2, what="wgrad")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dev, dtype):
    M, N, Kd = 384, 256, 128
    x = rnd(M, Kd, dev=dev, seed=5).to(dtype)
    w = rnd(N, Kd, dev=dev, seed=6, scale=0.1).to(dtype)
    b = rnd(N, dev=dev, seed=7)
    res = rnd(M, N, dev=dev, seed=8)
    p, seed = 0.1, 12345
    y = K.linear_fwd(x, w, b, out_dtype=torch.float32, relu=True, dropout_p=p, seed=seed, residual=res)
    z = torch.relu(x.double() @ w.double().T + b.double())
    idx = torch.arange(M * N, device=dev, dtype=torch.int64).view(M, N)
    keep = keep_mask(seed, idx, p)
    ref = torch.where(keep, z / (1 - p), torch.zeros_like(z)) + res.double()
    tol = 1e-4 if dtype == torch.float32 else 2e-3
    close(y, ref, atol=tol * 20, what="relu+dropout+residual")
    frac = 1 - keep.float().mean().item()
    assert abs(frac - 0.1) < 0.01
    # gate (relu/dropout backward) with bf16 output
    gate = rnd(M, N, dev=dev, seed=9).to(dtype)
    dy = rnd(M, Kd, dev=dev, seed=10).to(dtype)
    dx = K.linear_dgrad(dy, w.t().contiguous(), out_dtype=dtype, gate=gate, gate_scale=1.25)
    ref = (dy.double() @ w.double().T) * 1.25 * (gate.double() > 0)
    close(dx, ref, atol=(1e-4 if dtype == torch.float32 else 3e-2), rtol=(0 if dtype == torch.float32 else 1e-2),
          what="gate")


def test_gemm_identity_asymmetric(dev):
    # A = I with an asymmetric B catches a transposed C write (guide §3)
    n = 128
    eye = torch.eye(n, device=dev, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=dev).view(n, n) % 251).to(torch.bfloat16)
    y = K.linear_fwd(eye, B, None, out_dtype=torch.float32)
    assert torch.equal(y, B.float().T)


# ----------------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [256, 512])
def test_layernorm_fwd_bwd(dev, D):
    rows = 333
    x = rnd(rows, D, dev=dev, seed=1, scale=3.0) + 0.5
    gam = rnd(D, dev=dev, seed=2) * 0.2 + 1
    bet = rnd(D, dev=dev, seed=3) * 0.1
    T = 37
    pe = rnd(1, 64, D, dev=dev, seed=4)
    of, ol, mu, rs = K.layernorm_fwd(x, gam, bet, pe=pe, pe_period=T, lp_dtype=torch.bfloat16)
    xr = x.double().requires_grad_(True)
    ln = torch.nn.functional.layer_norm(xr, (D,), gam.double(), bet.double(), 1e-5)
    ref = ln + pe[0].double()[torch.arange(rows, device=dev) % T]
    close(of, ref.detach(), atol=2e-5, what="ln fwd")
    close(ol, ref.detach(), atol=3e-2, rtol=1e-2, what="ln fwd bf16")
    dy = rnd(rows, D, dev=dev, seed=5)
    dres = rnd(rows, D, dev=dev, seed=6)
    dg = torch.zeros(D, device=dev)
    db = torch.zeros(D, device=dev)
    dx, _ = K.layernorm_bwd(dy, x, mu, rs, gam, dres=dres, dgamma=dg, dbeta=db)
    gr = torch.autograd.grad(ln, xr, dy.double())[0] + dres.double()
    close(dx, gr, atol=2e-4, what="ln bwd dx")
    xhat = (x.double() - x.double().mean(1, keepdim=True)) / torch.sqrt(x.double().var(1, unbiased=False, keepdim=True) + 1e-5)
    close(dg, (dy.double() * xhat).sum(0), atol=5e-3, what="dgamma")
    close(db, dy.double().sum(0), atol=5e-3, what="dbeta")


def test_layernorm_relu_dropout(dev):
    rows, D, p, seed = 200, 512, 0.1, 777
    x = rnd(rows, D, dev=dev, seed=11)
    gam = torch.ones(D, device=dev)
    bet = rnd(D, dev=dev, seed=12) * 0.3
    of, _, mu, rs = K.layernorm_fwd(x, gam, bet, relu=True, dropout_p=p, seed=seed)
    xr = x.double().requires_grad_(True)
    z = torch.relu(torch.nn.functional.layer_norm(xr, (D,), gam.double(), bet.double(), 1e-5))
    keep = keep_mask(seed, torch.arange(rows * D, device=dev).view(rows, D), p)
    ref = torch.where(keep, z / (1 - p), torch.zeros_like(z))
    close(of, ref.detach(), atol=5e-5, what="ln relu dropout")
    dy = rnd(rows, D, dev=dev, seed=13)
    dx, dxl = K.layernorm_bwd(dy, x, mu, rs, gam, y=of, dropout_p=p, seed=seed, lp_dtype=torch.bfloat16,
                              lp_dropout_p=p, lp_seed=99)
    gr = torch.autograd.grad(ref, xr, dy.double())[0]
    close(dx, gr, atol=3e-4, what="ln relu dropout bwd")
    k2 = keep_mask(99, torch.arange(rows * D, device=dev).view(rows, D), p)
    close(dxl, torch.where(k2, gr / (1 - p), torch.zeros_like(gr)), atol=3e-2, rtol=1e-2, what="masked lp dx")


# ----------------------------------------------------------------------------------- attention
MWC_A_COMPL = (1 << 32) - 4294883355  # csrc/rp_attention.hip MWC_A = 2^32 - 83941


def mwc_step(x, c):
    """One MWC64X step, t = A x + c = x 2^32 + (c - 83941 x), in exact int64 arithmetic: returns
    (lo(t), hi(t))."""
    d = c - MWC_A_COMPL * x
    lo = torch.remainder(d, 1 << 32)
    return lo, x + torch.div(d - lo, 1 << 32, rounding_mode="floor")


def attn_keep(B, H, T, p, seed, dev, Tk=None):
    """torch restatement of the attention dropout bits (include/rp_api.h, rp_attn_fwd): per (query,
    lane group g) one MWC64X stream seeded x = rp_hash(seed_bh, q*4 + g), c = rp_hash(x, 0x6A09E667)
    >> 1; eight output words (x ^ c after each step) per 64-key tile in tile order; 16-bit halves
    read as int16.  Tk (cross attention): T queries x Tk keys."""
    Tk = T if Tk is None else Tk
    KT = (Tk + 63) // 64
    bh = torch.arange(B * H, device=dev, dtype=torch.int64)
    sbh = rp_hash(seed, bh).view(B * H, 1, 1)
    q = torch.arange(T, device=dev, dtype=torch.int64).view(1, T, 1)
    g = torch.arange(4, device=dev, dtype=torch.int64).view(1, 1, 4)
    x = rp_hash(sbh, q * 4 + g)                                 # [BH, T, 4]
    c = rp_hash(x, 0x6A09E667) >> 1
    tiles = []
    for _ in range(KT):
        words = []
        for _ in range(8):
            x, c = mwc_step(x, c)
            words.append(x ^ c)
        tiles.append(torch.stack(words, -1))                    # [BH, T, g, j]
    w = torch.stack(tiles, 2)                                   # [BH, T, KT, g, j]
    half = torch.stack([w & 0xFFFF, w >> 16], -1)               # [BH, T, KT, g, j, lo/hi]
    sgn = torch.where(half >= 32768, half - 65536, half)
    keep = sgn >= int(p * 65536 + 0.5) - 32768
    keep = keep.view(B * H, T, KT, 4, 4, 2, 2)                  # [.., g, kt, r>>1, r&1]
    keep = keep.permute(0, 1, 2, 4, 3, 5, 6).reshape(B * H, T, KT * 64)[:, :, :Tk]
    return keep.reshape(B, H, T, Tk)


def test_mwc_restatement_matches_the_full_product():
    """the int64 MWC step equals the 64-bit product A x + c computed with Python integers"""
    import random
    rng = random.Random(5)
    xs = [rng.randrange(1 << 32) for _ in range(256)] + [0, 1, M32]
    cs = [rng.randrange(1 << 31) for _ in range(256)] + [0, (1 << 31) - 1, 4294883354]
    x = torch.tensor(xs, dtype=torch.int64)
    c = torch.tensor(cs, dtype=torch.int64)
    lo, hi = mwc_step(x, c)
    for xi, ci, l, h in zip(xs, cs, lo.tolist(), hi.tolist()):
        t = 4294883355 * xi + ci
        assert (l, h) == (t & M32, t >> 32)


def attn_ref(qkv, kv, B, T, H, p=0.0, seed=0):
    dk = qkv.shape[1] // (3 * H)
    q, k, v = qkv.view(B, T, 3, H, dk).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dk)
    s = s.masked_fill(~kv.bool().view(B, 1, 1, T), float("-inf"))
    P = torch.softmax(s, -1)
    if p > 0:
        keep = attn_keep(B, H, T, p, seed, qkv.device)
        P = torch.where(keep, P / (1 - p), torch.zeros_like(P))
    o = P @ v
    return o.permute(0, 2, 1, 3).reshape(B * T, H * dk)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T,p", [(64, 0.0), (100, 0.0), (200, 0.1), (256, 0.0), (333, 0.1)])
def test_attention_fwd_bwd(dev, dtype, T, p):
    B, H = 2, 8
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=T).to(dtype)
    lens = torch.tensor([T, max(1, T - 37)], device=dev)
    kv = (torch.arange(T, device=dev)[None] < lens[:, None]).to(torch.uint8)
    seed = 4242
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, seed)
    ref_in = qkv.double().requires_grad_(True)
    ref = attn_ref(ref_in, kv, B, T, H, p, seed)
    ftol = 2e-5 if dtype == torch.float32 else 2e-2
    close(o, ref.detach(), atol=ftol, rtol=ftol, what="attn fwd")
    if p > 0:  # the stored keep bits are exactly the restated ones
        KT, ldm = (T + 63) // 64, (T + 127) // 128 * 128
        words = mask.view(B * H, KT, 4, ldm)[..., :T].to(torch.int64) & 0xFFFF  # [bh, tile, g, q]
        bits = (words.unsqueeze(-1) >> torch.arange(16, device=dev)) & 1       # [bh, tile, g, q, kt*4+r]
        bits = bits.view(B * H, KT, 4, T, 4, 4)                                  # [bh, tile, g, q, kt, r]
        got = bits.permute(0, 3, 1, 4, 2, 5).reshape(B * H, T, KT * 64)[:, :, :T].bool()
        assert torch.equal(got, attn_keep(B, H, T, p, seed, dev).view(B * H, T, T))
    do = rnd(B * T, H * 64, dev=dev, seed=T + 1).to(dtype)
    dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask)
    gref = torch.autograd.grad(ref, ref_in, do.double())[0]
    btol = 1e-4 if dtype == torch.float32 else 6e-2
    close(dqkv, gref, atol=btol, rtol=btol, what="attn bwd")


def mha_ref(q, k, v, kv, B, Tq, Tk, H, scale, keep=None, p=0.0):
    """torch restatement of the general attention core (fp64): softmax(scale*QK^T + key mask) V, with
    the stored dropout bits `keep` [B, H, Tq, Tk] applied as (keep / (1 - p)) when given."""
    dk = 64
    qh = q[:, :H * dk].reshape(B, Tq, H, dk).permute(0, 2, 1, 3)
    kh = k[:, :H * dk].reshape(B, Tk, H, dk).permute(0, 2, 1, 3)
    vh = v[:, :H * dk].reshape(B, Tk, H, dk).permute(0, 2, 1, 3)
    s = (qh @ kh.transpose(-1, -2)) * scale
    s = s.masked_fill(~kv.bool().view(B, 1, 1, Tk), float("-inf"))
    P = torch.softmax(s, -1)
    if keep is not None:
        P = torch.where(keep, P / (1 - p), torch.zeros_like(P))
    o = P @ vh
    return o.permute(0, 2, 1, 3).reshape(B * Tq, H * dk)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Tq,Tk", [(100, 37), (64, 256), (130, 129)])
def test_mha_cross_strided(dev, dtype, Tq, Tk):
    """Cross attention (Tq != Tk) on strided row views (q from a wider buffer, k/v interleaved
    columns of one [B*Tk, 2*H*dk] buffer), key padding on the context."""
    B, H, dk = 2, 4, 64
    qbuf = rnd(B * Tq, H * dk + 64, dev=dev, seed=Tq).to(dtype)
    kvbuf = rnd(B * Tk, 2 * H * dk, dev=dev, seed=Tk + 7).to(dtype)
    q, k, v = qbuf[:, 32:32 + H * dk], kvbuf[:, :H * dk], kvbuf[:, H * dk:]
    lens = torch.tensor([Tk, max(1, Tk // 3)], device=dev)
    kv = (torch.arange(Tk, device=dev)[None] < lens[:, None]).to(torch.uint8)
    scale = 0.125
    o, lse, _ = K.mha_fwd(q, k, v, kv, B, Tq, Tk, H, scale)
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
    ref = mha_ref(qd, kd, vd, kv, B, Tq, Tk, H, scale)
    ftol = 2e-5 if dtype == torch.float32 else 2e-2
    close(o, ref.detach(), atol=ftol, rtol=ftol, what="mha fwd")
    do = rnd(B * Tq, H * dk, dev=dev, seed=Tq + Tk).to(dtype)
    dq, dkk, dv = K.mha_bwd(q, k, v, o, do, lse, kv, B, Tq, Tk, H, scale)
    gq, gk, gv = torch.autograd.grad(ref, (qd, kd, vd), do.double())
    btol = 1e-4 if dtype == torch.float32 else 6e-2
    close(dq, gq, atol=btol, rtol=btol, what="mha dq")
    close(dkk, gk, atol=btol, rtol=btol, what="mha dk")
    close(dv, gv, atol=btol, rtol=btol, what="mha dv")


def prescale_q(qkv, H, scale):
    """The model's QKV GEMM epilogue (col_scale): Q columns -> bf16(Q * scale * log2 e).  Returns the
    kernel operand and the fp64 Q it stands for (Q' / c), which the reference then uses."""
    c = scale * K.LOG2E
    qp = qkv.clone()
    qp[:, :H * 64] = (qkv[:, :H * 64].float() * c).to(qkv.dtype)
    eff = qp.double()
    eff[:, :H * 64] /= c
    return qp, eff


@pytest.mark.gpu
@pytest.mark.parametrize("q_prescaled", [False, True])
def test_attention_128_blocks_ragged_dropout(dev, q_prescaled, p=0.1):
    """Self attention on the 128-row block path (B*H*ceil(T/128) >= 512 workgroups; the smaller test
    shapes above take the 64-row path), ragged T and key padding down to one and two valid keys,
    dropout keep bits vs the restatement, fwd and bwd vs fp64.  A sequence with one valid key puts
    every query's whole mass on it, so its dV sums ~1000 recomputed probabilities: this pins that the
    backward recomputes exactly the forward's P (same bf16-rounded Q * scale * log2 e in all three
    kernels, with the prescale done by the kernels or by the producer), and that delta = rowsum(dO * O)
    is taken from the unrounded output (out_lo), without which that key's dK (exactly 0) would collect
    ~1000 rounding residuals of O."""
    B, H, T = 8, 8, 1030
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=T).to(torch.bfloat16)
    lens = torch.tensor([T, T - 1, 1000, 777, 640, 129, 2, 1], device=dev)
    kv = (torch.arange(T, device=dev)[None] < lens[:, None]).to(torch.uint8)
    seed = 99
    if q_prescaled:
        qkv, eff = prescale_q(qkv, H, 0.125)
    else:
        eff = qkv.double()
    olo = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, seed, q_prescaled=q_prescaled, out_lo=olo)
    ref_in = eff.requires_grad_(True)
    ref = attn_ref(ref_in, kv, B, T, H, p, seed)
    close(o, ref.detach(), atol=2e-2, rtol=2e-2, what="attn fwd (128 blocks)")
    # hi + lo carries the output to ~2^-17
    close(o.double() + olo.double(), ref.detach(), atol=2e-2, rtol=2e-2, what="attn fwd hi+lo")
    if p > 0:
        KT, ldm = (T + 63) // 64, (T + 127) // 128 * 128
        words = mask.view(B * H, KT, 4, ldm)[..., :T].to(torch.int64) & 0xFFFF
        bits = ((words.unsqueeze(-1) >> torch.arange(16, device=dev)) & 1).view(B * H, KT, 4, T, 4, 4)
        got = bits.permute(0, 3, 1, 4, 2, 5).reshape(B * H, T, KT * 64)[:, :, :T].bool()
        assert torch.equal(got, attn_keep(B, H, T, p, seed, dev).view(B * H, T, T))
    do = rnd(B * T, H * 64, dev=dev, seed=T + 1).to(torch.bfloat16)
    dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=q_prescaled, out_lo=olo)
    gref = torch.autograd.grad(ref, ref_in, do.double())[0]
    for part, name in enumerate("qkv"):
        cols = slice(part * H * 64, (part + 1) * H * 64)
        close_per_seq(dqkv[:, cols], gref[:, cols], B, atol=6e-2, rtol=6e-2, what=f"attn d{name} (128 blocks)")
    # the one-key sequence (dK = 0: its scores never matter; dV = the kept dO mass of all queries):
    # the recomputed P is the forward's, so dV is within bf16 rounding of the exact sum
    rows = slice(7 * T, 7 * T + 1)
    dv1, rv1 = dqkv[rows, 2 * H * 64:].double().cpu(), gref[rows, 2 * H * 64:].cpu()
    assert ((dv1 - rv1).abs().max() / rv1.abs().max()).item() < 1e-2
    assert dqkv[rows, H * 64:2 * H * 64].abs().max().item() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("split", ["1", "3"])
@pytest.mark.parametrize("p", [0.1, 0.0])
def test_attention_split_workgroups(dev, monkeypatch, p, split):
    """RP_ATTN_SPLIT=1 forces the split 8-wave kernels (SPL = 2: the reduced sequence range in two halves,
    partials merged through LDS; auto-selected when the 128-row grid fills the CUs only once, config 4),
    =3 the three-part 12-wave forward (auto-selected for a grid's last partial round) on the ragged
    test: T = 1030 is 17 key / query tiles (halves 9 + 8, thirds 6 + 6 + 5: the short part idles through
    its last ring step), the two shortest sequences have no valid key past the first part (empty parts
    in the merge), the dropout keep bits bit for bit against the restatement (the later parts' MWC
    streams start from the skip-ahead multiplier), fwd and every gradient vs fp64."""
    monkeypatch.setenv("RP_ATTN_SPLIT", split)
    monkeypatch.setenv("RP_ATTN_ROLES", "0")  # the backward's own split kernels, not the two-role launch
    test_attention_128_blocks_ragged_dropout(dev, True, p=p)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [200, 130])
def test_attention_split3_short_ranges(dev, monkeypatch, T):
    """The three-part forward when a part gets no key tile (T = 200: 4 tiles -> 2 + 2 + 0; T = 130:
    3 tiles -> 1 + 1 + 1), on the 128-row LDS-DMA path (B = 16: 256 blocks): keep bits bitwise and
    outputs within bf16 rounding of the unsplit kernel."""
    B, H, p, seed = 16, 8, 0.1, 5
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=T).to(torch.bfloat16)
    kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
    kv[1, T - 37:] = 0
    kv[2, 64:] = 0  # no valid key past the first tile: the later parts are empty in the merge
    res = {}
    for flag in ("3", "0"):
        monkeypatch.setenv("RP_ATTN_SPLIT", flag)
        res[flag] = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, seed)
    (o3, l3, m3), (o0, l0, m0) = res["3"], res["0"]
    KT, ldm = (T + 63) // 64, (T + 127) // 128 * 128
    valid = lambda m: m.view(B * H, KT, 4, ldm)[..., :T]  # noqa: E731 (rows past T are never written)
    assert torch.equal(valid(m3), valid(m0))
    close(o3, o0.double(), atol=1e-2, rtol=1e-2, what=f"split3 vs unsplit T={T}")
    assert (l3 - l0).abs().max().item() < 5e-3


@pytest.mark.gpu
def test_mha_cross_128_blocks(dev):
    """Cross attention (Tq != Tk, both ragged) on the 128-row block path of all three kernels."""
    B, H, Tq, Tk, dk = 8, 8, 1100, 1000, 64
    q = rnd(B * Tq, H * dk, dev=dev, seed=5).to(torch.bfloat16)
    kvbuf = rnd(B * Tk, 2 * H * dk, dev=dev, seed=6).to(torch.bfloat16)
    k, v = kvbuf[:, :H * dk], kvbuf[:, H * dk:]
    lens = torch.tensor([Tk, 999, 900, 513, 500, 128, 2, 1], device=dev)  # one / two valid keys: see above
    kv = (torch.arange(Tk, device=dev)[None] < lens[:, None]).to(torch.uint8)
    o, lse, _ = K.mha_fwd(q, k, v, kv, B, Tq, Tk, H, 0.125)
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
    ref = mha_ref(qd, kd, vd, kv, B, Tq, Tk, H, 0.125)
    close(o, ref.detach(), atol=2e-2, rtol=2e-2, what="mha fwd (128 blocks)")
    do = rnd(B * Tq, H * dk, dev=dev, seed=7).to(torch.bfloat16)
    dq, dkk, dv = K.mha_bwd(q, k, v, o, do, lse, kv, B, Tq, Tk, H, 0.125)
    gq, gk, gv = torch.autograd.grad(ref, (qd, kd, vd), do.double())
    close_per_seq(dq, gq, B, atol=6e-2, rtol=6e-2, what="mha dq (128 blocks)")
    close_per_seq(dkk, gk, B, atol=6e-2, rtol=6e-2, what="mha dk (128 blocks)")
    close_per_seq(dv, gv, B, atol=6e-2, rtol=6e-2, what="mha dv (128 blocks)")


@pytest.mark.gpu
@pytest.mark.parametrize("split", ["1", "0"])
def test_mha_cross_dropout_prescaled(dev, monkeypatch, split):
    """Cross attention (Tq = 1100, Tk = 1000, ragged keys) with dropout 0.1 and the producer's Q prescale,
    so all three phases run the LDS-DMA kernels: forced split 8-wave workgroups (RP_ATTN_SPLIT=1: the
    forward / dQ split 16 key tiles 8 + 8, dK/dV 18 query tiles 9 + 9) and unsplit.  Keep bits bit for bit
    against the restatement (Tq x Tk streams), forward and every gradient vs fp64."""
    monkeypatch.setenv("RP_ATTN_SPLIT", split)
    monkeypatch.setenv("RP_ATTN_ROLES", "0")  # the per-phase kernels (the two-role launch: test above)
    B, H, Tq, Tk, p, seed = 8, 8, 1100, 1000, 0.1, 31
    c = 0.125 * K.LOG2E
    q = rnd(B * Tq, H * 64, dev=dev, seed=15).to(torch.bfloat16)
    qp = (q.float() * c).to(torch.bfloat16)
    kvbuf = rnd(B * Tk, 2 * H * 64, dev=dev, seed=16).to(torch.bfloat16)
    k, v = kvbuf[:, :H * 64], kvbuf[:, H * 64:]
    lens = torch.tensor([Tk, 999, 900, 513, 500, 128, 64, 700], device=dev)
    kv = (torch.arange(Tk, device=dev)[None] < lens[:, None]).to(torch.uint8)
    o, lse, mask = K.mha_fwd(qp, k, v, kv, B, Tq, Tk, H, 0.125, dropout_p=p, seed=seed, q_prescaled=True)
    KT, ldm = (Tk + 63) // 64, (Tq + 127) // 128 * 128
    words = mask.view(B * H, KT, 4, ldm)[..., :Tq].to(torch.int64) & 0xFFFF
    bits = ((words.unsqueeze(-1) >> torch.arange(16, device=dev)) & 1).view(B * H, KT, 4, Tq, 4, 4)
    got = bits.permute(0, 3, 1, 4, 2, 5).reshape(B * H, Tq, KT * 64)[:, :, :Tk].bool()
    keep = attn_keep(B, H, Tq, p, seed, dev, Tk=Tk)
    assert torch.equal(got, keep.view(B * H, Tq, Tk))
    qd = (qp.double() / c).requires_grad_(True)
    kd, vd = (t.double().requires_grad_(True) for t in (k, v))
    ref = mha_ref(qd, kd, vd, kv, B, Tq, Tk, H, 0.125, keep=keep, p=p)
    close(o, ref.detach(), atol=2e-2, rtol=2e-2, what="mha fwd dropout")
    do = rnd(B * Tq, H * 64, dev=dev, seed=17).to(torch.bfloat16)
    dq, dkk, dv = K.mha_bwd(qp, k, v, o, do, lse, kv, B, Tq, Tk, H, 0.125, dropout_p=p, dropmask=mask,
                            q_prescaled=True)
    gq, gk, gv = torch.autograd.grad(ref, (qd, kd, vd), do.double())
    close_per_seq(dq, gq, B, atol=6e-2, rtol=6e-2, what="mha dq dropout")
    close_per_seq(dkk, gk, B, atol=6e-2, rtol=6e-2, what="mha dk dropout")
    close_per_seq(dv, gv, B, atol=6e-2, rtol=6e-2, what="mha dv dropout")


def test_attention_lse(dev):
    B, H, T = 1, 8, 96
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=3)
    kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
    _, lse, _ = K.attn_fwd(qkv, kv, B, T, H, 0.125)
    q, k, _ = qkv.double().view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = torch.logsumexp((q @ k.transpose(-1, -2)) * 0.125, -1)
    close(lse, ref, atol=1e-5, what="lse")


# ----------------------------------------------------------------------------------- small ops
def test_focal_fused(dev):
    n = 5000
    x = rnd(n, dev=dev, seed=1, scale=4)
    t = (rnd(n, dev=dev, seed=2) > 0).float()
    m = (rnd(n, dev=dev, seed=3) > -0.5).to(torch.uint8)
    xr = x.double().requires_grad_(True)
    pr = torch.sigmoid(xr)
    ce = torch.nn.functional.binary_cross_entropy_with_logits(xr, t.double(), reduction="none")
    pt = pr * t + (1 - pr) * (1 - t)
    fl = (0.7 * t + 0.3 * (1 - t)) * ce * (1 - pt) ** 2
    ref = (fl * m).sum()
    s = K.focal_fwd_sum(x, t, m)  # many workgroups (rp_focal_fwd_sum_ws): 5000 frames = ten chunks
    close(s, ref.detach(), atol=1e-3, rtol=1e-5, what="focal sum")
    assert torch.equal(s, K.focal_fwd_sum(x, t, m))  # deterministic
    one = torch.empty((), device=dev)  # the single-workgroup entry point
    from repurpose_amd import _native as N
    N.call("rp_focal_fwd_sum", K._p(x), K._p(t), K._p(m), n, 0.7, 2.0, K._p(one), K._stream(x))
    close(one, ref.detach(), atol=1e-3, rtol=1e-5, what="focal sum (one workgroup)")
    assert K.focal_fwd_sum(x[:0], t[:0]).item() == 0.0
    g = torch.tensor(1.7, device=dev)
    dx = K.focal_bwd(x, t, m, g.view(1))
    gr = torch.autograd.grad(ref * 1.7, xr)[0]
    close(dx, gr, atol=1e-6, rtol=1e-4, what="focal grad")
    close(K.focal_elementwise(x, t), fl.detach(), atol=1e-6, rtol=1e-5, what="focal elementwise")


def test_rowdot_colsum_concat_cast(dev):
    rows, Kd = 777, 256
    X = rnd(rows, Kd, dev=dev, seed=1)
    W = rnd(2, Kd, dev=dev, seed=2) * 0.1
    b = rnd(2, dev=dev, seed=3)
    out = K.rowdot_fwd(X, W, b, relu=True)
    close(out, torch.relu(X.double() @ W.double().T + b.double()), atol=1e-5, what="rowdot")
    # bf16 rows: the eight-lanes-per-row kernel (K % 8 == 0) and the one-wave-per-row fallback (K = 100)
    for kk, nn in ((256, 1), (256, 4), (200, 3), (100, 2)):
        Xb = rnd(rows, kk, dev=dev, seed=kk + nn).to(torch.bfloat16)
        Wb = rnd(nn, kk, dev=dev, seed=kk - nn) * 0.1
        bb = rnd(nn, dev=dev, seed=nn)
        close(K.rowdot_fwd(Xb, Wb, bb), Xb.double() @ Wb.double().T + bb.double(), atol=1e-5, what=f"rowdot bf16 {kk}")
    dout = rnd(rows, 2, dev=dev, seed=4)
    G = rnd(rows, Kd, dev=dev, seed=5)
    dX = K.rowdot_bwd_dx(dout, W, gate=G, gate_scale=2.0)
    close(dX, (dout.double() @ W.double()) * 2 * (G > 0), atol=1e-5, what="rowdot bwd")
    w = rnd(rows, dev=dev, seed=6)
    cs = K.colsum(X, w=w)
    close(cs, (X.double() * w.double()[:, None]).sum(0), atol=1e-3, what="colsum")
    Xb = X.to(torch.bfloat16)
    close(K.colsum(Xb), Xb.double().sum(0), atol=1e-3, what="colsum bf16")
    for r, c in ((5000, 96), (300, 250)):  # two-pass path; ragged last column chunk
        Y = rnd(r, c, dev=dev, seed=r)
        acc = rnd(c, dev=dev, seed=c)
        close(K.colsum(Y, out=acc.clone(), accumulate=True), acc.double() + Y.double().sum(0), atol=2e-3,
              what=f"colsum {r}x{c}")
    v = rnd(3, 5, 8, dev=dev, seed=7)
    a = rnd(3, 5, 16, dev=dev, seed=8)
    t = rnd(3, 5, 4, dev=dev, seed=9)
    cat = K.concat_rows(v, a, t, torch.float32)
    assert torch.equal(cat, torch.cat([v, a, t], -1).view(15, 28))
    catb = K.concat_rows(v, a, t, torch.bfloat16)
    assert torch.equal(catb, torch.cat([v, a, t], -1).view(15, 28).to(torch.bfloat16))
    dst = torch.empty(15 * 28, dtype=torch.bfloat16, device=dev)
    K.cast_bf16(cat.view(-1), dst)
    assert torch.equal(dst, cat.view(-1).to(torch.bfloat16))


def test_adam_matches_torch(dev):
    n = 10_000
    p0 = rnd(n, dev=dev, seed=1)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=1e-3, weight_decay=1e-4)
    p = p0.clone()
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    plp = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in range(1, 4):
        g = rnd(n, dev=dev, seed=10 + step)
        p_ref.grad = g.clone()
        opt.step()
        K.adam_step(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-4, step, p_lp=plp)
    close(p, p_ref.detach(), atol=1e-6, what="adam")
    assert torch.equal(plp, p.to(torch.bfloat16))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T,Nn,Kd", [(16384, 512, 512), (771, 2048, 512), (100, 256, 2944), (5000, 1536, 512),
                                        (4096, 200, 136), (1024, 2048, 512)])
def test_wgrad_splitk_with_bias(dev, dtype, T, Nn, Kd):
    dy = rnd(T, Nn, dev=dev, seed=1).to(dtype)
    x = rnd(T, Kd, dev=dev, seed=2).to(dtype)
    dW = torch.full((Nn, Kd), 0.25, device=dev)
    db = torch.full((Nn,), -1.0, device=dev)
    K.linear_wgrad(dy, x, dW, db=db, accumulate=True)
    ref = dy.double().T @ x.double() + 0.25
    tol = (1e-4 if dtype == torch.float32 else 1e-3) * math.sqrt(T)
    close(dW, ref, atol=tol, what="wgrad")
    close(db, dy.double().sum(0) - 1.0, atol=tol, what="bias grad")
    # overwrite mode and determinism
    dW2 = torch.empty_like(dW)
    K.linear_wgrad(dy, x, dW2, accumulate=False)
    dW3 = torch.empty_like(dW)
    K.linear_wgrad(dy, x, dW3, accumulate=False)
    assert torch.equal(dW2, dW3)
    close(dW2, ref - 0.25, atol=tol, what="wgrad overwrite")


def test_colsum_batched_equals_per_item(dev):
    """rp_colsum_batched (every LayerNorm's gamma / beta partials of a backward in one launch) gives
    bitwise the per-item rp_colsum results, accumulate and overwrite, ragged shapes, 70 items
    (two launches), strided rows."""
    items = []
    for i in range(70):
        rows, cols = [(512, 1024), (7, 512), (33, 12), (1, 4), (300, 260)][i % 5]
        X = rnd(rows, cols + 4, dev=dev, seed=100 + i)[:, 2:2 + cols] if i % 3 == 0 else rnd(rows, cols, dev=dev, seed=100 + i)
        items.append((X, rnd(cols, dev=dev, seed=300 + i)))
    want = [o.clone() for _, o in items]
    for (X, _), w in zip(items, want):
        K.colsum(X, out=w, accumulate=True)
    K.colsum_batched(items, accumulate=True)
    for (_, o), w in zip(items, want):
        assert torch.equal(o, w)
    K.colsum_batched(items, accumulate=False)
    for (X, o) in items:
        assert torch.equal(o, K.colsum(X))


def test_wgrad_grouped_whole_k(dev):
    """rp_gemm_wgrad_grouped: several (dY, X) pairs of different shapes over one token range in one
    launch (whole-K tiles, bias from the staged dY tiles), strided dY views, items without a bias,
    accumulate and overwrite modes, deterministic; 70 items -> two launches (64 per launch)."""
    T = 1216  # a multiple of 64, not of 128
    shapes = [(512, 2048), (2048, 512), (512, 512), (1536, 512), (256, 136), (8, 64)]
    items, refs = [], []
    big = rnd(T, 1536 + 64, dev=dev, seed=40).to(torch.bfloat16)
    for i, (n_out, n_in) in enumerate(shapes):
        dy = big[:, 8:8 + n_out] if n_out <= 1536 else rnd(T, n_out, dev=dev, seed=41 + i).to(torch.bfloat16)
        x = rnd(T, n_in, dev=dev, seed=60 + i).to(torch.bfloat16)
        dW = torch.full((n_out, n_in), 0.5, device=dev)
        db = torch.full((n_out,), -2.0, device=dev) if i != 2 else None
        items.append((dy, x, dW, db))
        refs.append((dy.double().T @ x.double() + 0.5, (dy.double().sum(0) - 2.0) if db is not None else None))
    K.linear_wgrad_grouped(items, accumulate=True)
    tol = 1e-3 * math.sqrt(T)
    for (dy, x, dW, db), (rw, rb) in zip(items, refs):
        close(dW, rw, atol=tol, what=f"grouped wgrad {tuple(dW.shape)}")
        if db is not None:
            close(db, rb, atol=tol, what=f"grouped bias {tuple(db.shape)}")
    outs = []
    for _ in range(2):
        its = [(dy, x, torch.empty_like(dW), None) for dy, x, dW, _ in items] * 12  # 72 items
        its = its[:70]
        K.linear_wgrad_grouped(its, accumulate=False)
        outs.append([w for _, _, w, _ in its])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    for (dy, x, dW, _), w in zip(its, outs[0]):
        close(w, dy.double().T @ x.double(), atol=tol, what="grouped wgrad overwrite")


def test_wgrad_grouped_metric_shape(dev):
    """The grouped weight gradients as the step launches them at the metric shape: one encoder layer's
    four items (linear2, linear1, out_proj, in_proj) over T = 16,384 tokens on the 256 x 256 whole-K
    tiles, with their biases, against fp64."""
    T = 16384
    shapes = [(512, 2048), (2048, 512), (512, 512), (1536, 512)]
    items, refs = [], []
    for i, (n_out, n_in) in enumerate(shapes):
        dy = rnd(T, n_out, dev=dev, seed=70 + i).to(torch.bfloat16)
        x = rnd(T, n_in, dev=dev, seed=80 + i).to(torch.bfloat16)
        items.append((dy, x, torch.empty(n_out, n_in, device=dev), torch.empty(n_out, device=dev)))
        refs.append((dy.double().T @ x.double(), dy.double().sum(0)))
    K.linear_wgrad_grouped(items, accumulate=False)
    tol = 2e-4 * math.sqrt(T)
    for (dy, x, dW, db), (rw, rb) in zip(items, refs):
        close(dW, rw, atol=tol, what=f"grouped wgrad {tuple(dW.shape)}")
        close(db, rb, atol=tol, what=f"grouped bias {tuple(db.shape)}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("qpre", [False, True])
def test_attention_bwd_fused_delta_matches_unfused(dev, dtype, p, qpre):
    """rp_attn_bwd_dq_delta (delta formed inside the dQ kernel, dQ before dK/dV) against the unfused
    sequence rp_attn_bwd_delta -> rp_attn_bwd_dkdv -> rp_attn_bwd_dq on the same inputs; with the
    Q-prescaled flag in bf16 the dK/dV step is the LDS-DMA kernel, which reads the row constants either
    delta producer writes (workspace planes 1, 2)."""
    from repurpose_amd import _native as N
    B, H, T = 2, 8, 200
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=5).to(dtype)
    kv = (torch.arange(T, device=dev)[None] < torch.tensor([T, 150], device=dev)[:, None]).to(torch.uint8)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 77, q_prescaled=qpre)
    do = rnd(B * T, H * 64, dev=dev, seed=6).to(dtype)
    dt = (N.RP_BF16 if dtype == torch.bfloat16 else N.RP_F32) | (K.RP_ATTN_Q_PRESCALED if qpre else 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    P = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    outs = []
    for fused in (True, False):
        dqkv = torch.full_like(qkv, float("nan"))
        delta = torch.full((3, B, H, T), float("nan"), device=dev)
        args = (P(qkv), P(do), P(lse), P(delta), P(kv), B, T, H, 64, 0.125, p, P(mask), P(dqkv), st)
        if fused:
            N.call("rp_attn_bwd_dq_delta", dt, P(qkv), P(o), P(None), P(do), P(lse), P(delta), P(kv), B, T, H, 64, 0.125, p,
                   P(mask), P(dqkv), st)
            N.call("rp_attn_bwd_dkdv", dt, *args)
        else:
            N.call("rp_attn_bwd_delta", dt, P(o), P(None), P(do), P(lse), B, T, H, 64, p, P(delta), st)
            N.call("rp_attn_bwd_dkdv", dt, *args)
            N.call("rp_attn_bwd_dq", dt, *args)
        outs.append((dqkv, delta))
    torch.cuda.synchronize()
    dref = (do.double() * o.double()).view(B, T, H, 64).sum(-1).permute(0, 2, 1)
    for dqkv, delta in outs:
        close(delta[0], dref, atol=1e-4, rtol=1e-4, what="delta")
        assert torch.isfinite(dqkv).all()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(outs[0][0], outs[1][0].double(), atol=tol, rtol=tol, what="fused vs unfused dqkv")


# ------------------------------------------------------------------- metric-shape (full size) checks
def test_gemm_metric_shapes_bf16(dev):
    """Every Linear of an encoder layer at the bench shape (M = B*T = 16384 tokens): fwd, dgrad and
    the split-K wgrad against an fp64 torch product of the same bf16 operands."""
    M = 16384
    for (n, k) in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]:
        x = rnd(M, k, dev=dev, seed=n + k).to(torch.bfloat16)
        w = rnd(n, k, dev=dev, seed=n * k, scale=0.05).to(torch.bfloat16)
        b = rnd(n, dev=dev, seed=3)
        y = K.linear_fwd(x, w, b, out_dtype=torch.float32)
        close(y, x.double() @ w.double().T + b.double(), atol=2e-3 * math.sqrt(k), what=f"fwd {n}x{k}")
        dy = rnd(M, n, dev=dev, seed=n - k).to(torch.bfloat16)
        close(K.linear_dgrad(dy, w, out_dtype=torch.float32), dy.double() @ w.double(), atol=2e-3 * math.sqrt(n),
              what=f"dgrad {n}x{k}")
        dW = torch.zeros(n, k, device=dev)
        db = torch.zeros(n, device=dev)
        K.linear_wgrad(dy, x, dW, db=db)
        close(dW, dy.double().T @ x.double(), atol=4e-3 * math.sqrt(M), what=f"wgrad {n}x{k}")
        close(db, dy.double().sum(0), atol=1e-3 * math.sqrt(M), what=f"bias grad {n}")


@pytest.mark.parametrize("M", [4096, 4000])
def test_gemm_64_row_tiles_bitwise(dev, monkeypatch, M):
    """The 64 x 128 tile variant (auto-selected where the 128 x 128 grid leaves CUs idle: config 4's
    d_model = 512 GEMMs at M = 4096) runs every output element's MFMA chain in the same K order as the
    128 x 128 kernel: forward with bias + dropout + residual (fp32), the bf16 forward, the fp32 and the
    gated bf16 dgrad are bitwise the 128-row kernel's (RP_GEMM_BM64=1 vs 0), ragged M included, and
    match fp64."""
    outs = {}
    # "32": 32 x 128 tiles
    for flag in ("1", "0", "32"):
        monkeypatch.setenv("RP_GEMM_BM64", "1" if flag == "32" else flag)
        monkeypatch.setenv("RP_GEMM_BM32", "1" if flag == "32" else "0")
        res = []
        for (n, k) in [(512, 512), (512, 2048)]:
            x = rnd(M, k, dev=dev, seed=n + k).to(torch.bfloat16)
            w = rnd(n, k, dev=dev, seed=n * k, scale=0.05).to(torch.bfloat16)
            b = rnd(n, dev=dev, seed=3)
            r = rnd(M, n, dev=dev, seed=5)
            res.append(K.linear_fwd(x, w, b, out_dtype=torch.float32, dropout_p=0.1, seed=11, residual=r))
            res.append(K.linear_fwd(x, w, b))
            dy = rnd(M, n, dev=dev, seed=n - k).to(torch.bfloat16)
            res.append(K.linear_dgrad(dy, w, out_dtype=torch.float32))
            gate = rnd(M, k, dev=dev, seed=7).to(torch.bfloat16)
            res.append(K.linear_dgrad(dy, w, out_dtype=torch.bfloat16, gate=gate, gate_scale=1.25))
            if flag == "1":
                close(res[-2], dy.double() @ w.double(), atol=2e-3 * math.sqrt(n), what=f"dgrad {n}x{k} M={M}")
                close(res[-3], x.double() @ w.double().T + b.double(), atol=2e-2, rtol=1e-2, what=f"fwd {n}x{k}")
        outs[flag] = res
    for a, c, e in zip(outs["1"], outs["0"], outs["32"]):
        assert torch.equal(a, c) and torch.equal(a, e)


@pytest.mark.parametrize("M", [384, 4096, 8192])
@pytest.mark.parametrize("tiles", ["128", "64", "32"])
def test_gemm_gate_batched_bitwise(dev, monkeypatch, M, tiles):
    """The gated bf16 dgrad (d_ff backward through ReLU + dropout) with the pass's gate chunks loaded
    before its stores (the default) is bitwise the per-chunk epilogue (RP_GEMM_GATEB=0) on 128-, 64- and
    32-row tiles (all three staging forms), ragged M included, and matches fp64."""
    monkeypatch.setenv("RP_GEMM_BM64", "0" if tiles == "128" else "1")
    monkeypatch.setenv("RP_GEMM_BM32", "1" if tiles == "32" else "0")
    monkeypatch.setenv("RP_GEMM8", "0")
    n, k = 512, 2048
    dy = rnd(M, n, dev=dev, seed=M + 1).to(torch.bfloat16)
    w = rnd(n, k, dev=dev, seed=M + 2, scale=0.05).to(torch.bfloat16)
    gate = rnd(M, k, dev=dev, seed=M + 3).to(torch.bfloat16)
    outs = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("RP_GEMM_GATEB", flag)
        outs[flag] = K.linear_dgrad(dy, w, out_dtype=torch.bfloat16, gate=gate, gate_scale=1.25)
    torch.cuda.synchronize()
    assert torch.equal(outs["0"], outs["1"])
    ref = (dy.double() @ w.double()) * 1.25 * (gate.double() > 0)
    close(outs["1"], ref, atol=2e-3 * math.sqrt(n), rtol=1e-2, what=f"gated dgrad M={M}")


@pytest.mark.parametrize("B,T,qpre,roles", [(8, 2048, False, "1"), (8, 2048, True, "1"), (8, 2048, True, "0"),
                                            (1, 4096, True, "1")])
def test_attention_metric_shape_bf16_dropout(dev, monkeypatch, B, T, qpre, roles):
    """Attention at the bench shape (B = 8, T = 2048, H = 8, dk = 64) and at config 4's (B = 1, T = 4096)
    with dropout 0.1 and ragged key padding: forward output and all three gradients against an fp64
    torch restatement (same bf16 inputs, the restated keep bits) on a sample of (batch, head) pairs.
    With the producer's Q prescale (qpre, what the model runs) the shipping LDS-DMA kernels run: the
    delta pass and the two-role launch (attn_bwd_roles_kernel) at both shapes — asserted — and with
    RP_ATTN_ROLES=0 the fused-delta dQ kernel then the 128-key dK/dV kernel (the per-phase form)."""
    monkeypatch.setenv("RP_ATTN_ROLES", roles)
    H = 8
    qkv0 = rnd(B * T, 3 * H * 64, dev=dev, seed=21).to(torch.bfloat16)
    if qpre:
        qkv, eff = prescale_q(qkv0, H, 0.125)
    else:
        qkv, eff = qkv0, qkv0.double()
    lens = torch.tensor([T, T - 1, 1900, 1537, T, 1024, 2047, 64][:B] if B > 1 else [T - 301], device=dev)
    kv = (torch.arange(T, device=dev)[None] < lens[:, None]).to(torch.uint8)
    p, seed = 0.1, 777
    olo = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, seed, q_prescaled=qpre, out_lo=olo)
    do = rnd(B * T, H * 64, dev=dev, seed=22).to(torch.bfloat16)
    assert K.attn_bwd_uses_roles(qkv, B, T, H, q_prescaled=qpre) == (qpre and roles == "1")
    dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=qpre, out_lo=olo)
    keep_all = attn_keep(B, H, T, p, seed, dev)                       # [B, H, T, T]
    q, k, v = eff.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)        # [B, H, T, 64]
    dq, dk, dv = dqkv.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    og = o.view(B, T, H, 64).permute(0, 2, 1, 3)
    dog = do.view(B, T, H, 64).permute(0, 2, 1, 3)
    for (bb, hh) in ([(3, 5), (6, 0)] if B > 1 else [(0, 2), (0, 7)]):
        qd, kd, vd = (t[bb, hh].double().requires_grad_(True) for t in (q, k, v))
        s = (qd @ kd.T) * 0.125
        s = s.masked_fill(~kv[bb].bool()[None, :], float("-inf"))
        P = torch.softmax(s, -1)
        P = torch.where(keep_all[bb, hh], P / (1 - p), torch.zeros_like(P))
        ref = P @ vd
        close(og[bb, hh], ref.detach(), atol=2e-2, rtol=2e-2, what=f"fwd b{bb} h{hh}")
        gq, gk, gv = torch.autograd.grad(ref, (qd, kd, vd), dog[bb, hh].double())
        valid = kv[bb].bool()
        close(dq[bb, hh], gq, atol=6e-2, rtol=6e-2, what=f"dq b{bb} h{hh}")
        close(dk[bb, hh][valid], gk[valid], atol=6e-2, rtol=6e-2, what=f"dk b{bb} h{hh}")
        close(dv[bb, hh][valid], gv[valid], atol=6e-2, rtol=6e-2, what=f"dv b{bb} h{hh}")
        assert torch.count_nonzero(dk[bb, hh][~valid]) == 0 and torch.count_nonzero(dv[bb, hh][~valid]) == 0


@pytest.mark.parametrize("B,T,p", [(1, 4096, 0.1), (1, 4096, 0.0), (2, 2048, 0.1), (1, 4000, 0.1)])
def test_attention_bwd_roles_matches_two_kernels(dev, monkeypatch, B, T, p):
    """The two-role backward (one launch: dK/dV blocks and dQ blocks side by side, delta formed by its
    own pass; chosen where each grid alone fills the CUs once but not twice — config 4) against the
    two-kernel form (RP_ATTN_ROLES=0: fused-delta dQ, then dK/dV, as eight-wave split workgroups), Q
    prescaled, ragged keys: equal up to delta's rounding, and bitwise repeatable.  Also the key-padded
    T = 4000 (a partial last 128-block on both sides) and B = 2, T = 2048 (grids of 256 too)."""
    H = 8
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=41).to(torch.bfloat16)
    qkv[:, :H * 64] = (qkv[:, :H * 64].float() * (0.125 * K.LOG2E)).to(torch.bfloat16)
    lens = torch.tensor([T, T - 77][:B], device=dev)
    kv = (torch.arange(T, device=dev)[None] < lens[:, None]).to(torch.uint8)
    olo = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 93, q_prescaled=True, out_lo=olo)
    do = rnd(B * T, H * 64, dev=dev, seed=42).to(torch.bfloat16)
    outs = {}
    for flag in ("0", "1", "1"):
        monkeypatch.setenv("RP_ATTN_ROLES", flag)
        r = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask if p else None, q_prescaled=True,
                       out_lo=olo)
        torch.cuda.synchronize()
        if flag in outs:
            assert torch.equal(r, outs[flag]), "two-role backward not repeatable"
        outs[flag] = r
    assert torch.isfinite(outs["1"]).all()
    close(outs["1"].float(), outs["0"].double(), atol=2e-2, rtol=2e-2, what="two-role vs two-kernel dqkv")
    dkv = outs["1"].view(B, T, 3, H * 64)[:, :, 1:]
    for bb in range(B):
        assert torch.count_nonzero(dkv[bb, int(lens[bb]):]) == 0  # padded keys: no gradient


@pytest.mark.parametrize("T", [128, 192, 4096])
def test_wgrad_grouped_repeat_bitwise(dev, T):
    """Race guard for the 256-row kernel's LDS-DMA pipeline: the grouped weight gradients of the
    encoder's four shapes, relaunched eight times, are bitwise identical every time and every launch
    matches fp64 (a K-tile read before its fills land gives O(1) errors).  Short token ranges (two and
    three K-tiles, the DDP test's T = 128) leave the fills the least time to land."""
    shapes = [(512, 2048), (2048, 512), (512, 512), (1536, 512)] * 2
    items = []
    for i, (n_out, n_in) in enumerate(shapes):
        dy = rnd(T, n_out, dev=dev, seed=300 + i).to(torch.bfloat16)
        x = rnd(T, n_in, dev=dev, seed=400 + i).to(torch.bfloat16)
        items.append((dy, x, torch.empty(n_out, n_in, device=dev), torch.empty(n_out, device=dev)))
    refs = [(dy.double().T @ x.double(), dy.double().sum(0)) for dy, x, _, _ in items]
    first = None
    for _ in range(8):
        K.linear_wgrad_grouped(items, accumulate=False)
        got = [torch.cat([w.reshape(-1), b]) for _, _, w, b in items]
        for (_, _, w, b), (rw, rb) in zip(items, refs):
            close(w, rw, atol=1e-3 * math.sqrt(T), what=f"grouped wgrad T={T}")
            close(b, rb, atol=1e-3 * math.sqrt(T), what=f"grouped bias T={T}")
        if first is None:
            first = got
        else:
            for a, c in zip(first, got):
                assert torch.equal(a, c)


@pytest.mark.parametrize("Kr", [128, 192, 512])
def test_gemm8_dgrad_gate_prefetch_repeat_bitwise(dev, Kr):
    """Race guard for the 256-row kernel's gated dgrad (the linear2 dgrad of the encoder: bf16 ReLU /
    dropout gate touched one K-tile before the epilogue, two loads left in flight by the counted
    waits of the last two K-tiles): relaunched eight times at short reduction depths, every launch
    matches fp64 and is bitwise the first."""
    M, Nout = 16384, 2048
    dy = rnd(M, Kr, dev=dev, seed=500 + Kr).to(torch.bfloat16)
    w = rnd(Kr, Nout, dev=dev, seed=600 + Kr, scale=0.05).to(torch.bfloat16)
    gate = rnd(M, Nout, dev=dev, seed=700 + Kr).to(torch.bfloat16)
    ref = (dy.double() @ w.double()) * (gate.double() > 0) * (1 / 0.9)
    first = None
    for _ in range(8):
        got = K.linear_dgrad(dy, w, out_dtype=torch.bfloat16, gate=gate, gate_scale=1 / 0.9)
        close(got, ref, atol=2e-2 + 4e-3 * math.sqrt(Kr), rtol=1e-2, what=f"gated dgrad K={Kr}")
        if first is None:
            first = got.clone()
        else:
            assert torch.equal(first, got)


def test_gemm8_forward_dropout_bits(dev, monkeypatch):
    """The 256-row kernel's bf16 forward with ReLU + element dropout (the encoder's linear1 at the bench
    shape) drops exactly the elements the 128 x 128 kernel drops (the stream is a function of the element index; bias large enough that ReLU clips nothing),
    keeps the rest within bf16 rounding of each other, and repeats bitwise."""
    M, Nout, Kd = 16384, 2048, 512
    x = rnd(M, Kd, dev=dev, seed=31).to(torch.bfloat16)
    w = rnd(Nout, Kd, dev=dev, seed=32, scale=0.02).to(torch.bfloat16)
    b = torch.full((Nout,), 8.0, device=dev)
    y8 = K.linear_fwd(x, w, b, relu=True, dropout_p=0.1, seed=1234)
    y8b = K.linear_fwd(x, w, b, relu=True, dropout_p=0.1, seed=1234)
    monkeypatch.setenv("RP_GEMM8", "0")
    y1 = K.linear_fwd(x, w, b, relu=True, dropout_p=0.1, seed=1234)
    torch.cuda.synchronize()
    assert torch.equal(y8, y8b)
    assert torch.equal(y8 == 0, y1 == 0)
    frac = (y8 == 0).float().mean().item()
    assert abs(frac - 0.1) < 0.002, frac
    close(y8.float(), y1.double(), atol=0.1, rtol=1e-2, what="gemm8 vs 128-tile dropout forward")


@pytest.mark.parametrize("B,T,p", [(8, 2048, 0.1), (2, 384, 0.0), (4, 2048, 0.1), (1, 4096, 0.1)])
def test_attn_dout_delta_fused_bitwise(dev, B, T, p):
    """rp_gemm_attn_dout_delta (the out_proj dgrad with the attention delta pre-pass in its epilogue)
    against the two launches it replaces: dO bitwise the plain dgrad GEMM's, the three delta planes
    bitwise rp_attn_bwd_delta's on that dO, and the attention backward fed those planes bitwise the
    backward that forms them itself (two-role launch at the metric shape).  Tile heights: 128 rows at
    the metric shape, 64 at M = 8192, 32 at config 4 (M = 4096) and M = 768."""
    H, d = 8, 512
    M = B * T
    g1 = rnd(M, d, dev=dev, seed=51).to(torch.bfloat16)
    W = rnd(d, d, dev=dev, seed=52, scale=0.05).to(torch.bfloat16)
    qkv = rnd(M, 3 * d, dev=dev, seed=53).to(torch.bfloat16)
    qkv, _ = prescale_q(qkv, H, 0.125)
    kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
    kv[-1, T // 3:] = 0
    olo = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 7, q_prescaled=True, out_lo=olo)
    do_ref = K.linear_dgrad(g1, W, out_dtype=torch.bfloat16)
    do, delta = K.attn_dout_delta(g1, W, o, olo, lse, B, T, H, p)
    assert torch.equal(do, do_ref)
    delta_ref = K.attn_delta(o, olo, do_ref, lse, B, T, H, p)
    assert torch.equal(delta, delta_ref)
    ref = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo)
    got = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo, delta=delta)
    if K.attn_bwd_uses_roles(qkv, B, T, H, q_prescaled=True):
        assert torch.equal(got, ref)  # the same delta planes into the same launch
    else:  # the small-grid dQ kernel forms delta itself when not given it: same value, another sum order
        close(got, ref.double(), atol=2e-2, rtol=2e-2, what="given-delta vs fused-delta backward")
