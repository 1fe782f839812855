"""repurpose_amd.transformer (drop-in for models/transformer.py) against the CPU restatement in
oracle/transformer_oracle.py: structure on CPU; forward and gradients on the GPU (fp32)."""
import pytest
import torch

from oracle import transformer_oracle as O
from repurpose_amd import kernels as K
from repurpose_amd import transformer as R

D, H, DFF = 128, 2, 256  # head dim 64, as the kernels implement

CASES = {
    "MultiHeadAttention": lambda m: m.MultiHeadAttention(D, H),
    "MLP": lambda m: m.MLP(96, DFF, D),
    "EncoderLayer": lambda m: m.EncoderLayer(D, H, DFF),
    "CrossAttentionEncoderLayer": lambda m: m.CrossAttentionEncoderLayer(D, H, DFF),
    "CrossSelfEncoderLayer": lambda m: m.CrossSelfEncoderLayer(D, H, DFF),
    "UniModalEncoder": lambda m: m.UniModalEncoder(96, D, 2, H, DFF),
}


def build(name, seed=0):
    torch.manual_seed(seed)
    ref = CASES[name](O)
    torch.manual_seed(seed)
    ours = CASES[name](R)
    return ref, ours


@pytest.mark.parametrize("name", list(CASES))
def test_state_dict_and_init_match(name):
    ref, ours = build(name)
    a, b = ref.state_dict(), ours.state_dict()
    assert list(a) == list(b)
    for k in a:
        assert a[k].shape == b[k].shape, k
        assert torch.equal(a[k], b[k]), k  # same construction order -> same seeded init


def test_positional_encoding_keeps_batch_index_quirk():
    pe = R.PositionalEncoding(16, max_len=50)
    x = torch.zeros(3, 7, 16)
    y = pe(x)
    for b in range(3):  # sample b gets pe[b] at every timestep (seq-first table on batch-first input)
        assert torch.equal(y[b], pe.pe[b].expand(7, 16))


def _inputs(name, dev, B=2, T=70, Tc=45):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, T, 96 if name in ("MLP", "UniModalEncoder") else D, generator=g)
    ctx = torch.randn(B, T if name == "CrossSelfEncoderLayer" else Tc, D, generator=g)
    lens = torch.tensor([T, T - 23])
    mask = (torch.arange(T)[None] < lens[:, None]).unsqueeze(1)          # [B, 1, T]
    clens = torch.tensor([ctx.shape[1], ctx.shape[1] - 11])
    cmask = (torch.arange(ctx.shape[1])[None] < clens[:, None]).unsqueeze(1)
    return x, ctx, mask, cmask


def _call(name, m, x, ctx, mask, cmask):
    if name == "MultiHeadAttention":
        return m(x, ctx, ctx * 0.5 + 1.0, cmask)  # distinct q, k, v sources
    if name == "MLP":
        return m(x)
    if name == "EncoderLayer":
        return m(x, mask)
    if name == "CrossAttentionEncoderLayer":
        return m(x, ctx, cmask)
    if name == "CrossSelfEncoderLayer":
        return m(x, ctx, mask)
    return m(x, mask)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_forward_backward_parity(dev, name):
    ref, ours = build(name)
    ours = ours.to(dev)
    x, ctx, mask, cmask = _inputs(name, dev)
    xr, cr = x.clone().requires_grad_(True), ctx.clone().requires_grad_(True)
    yr = _call(name, ref, xr, cr, mask, cmask)
    xo, co = x.to(dev).requires_grad_(True), ctx.to(dev).requires_grad_(True)
    yo = _call(name, ours, xo, co, mask.to(dev), cmask.to(dev))
    err = (yo.detach().cpu() - yr.detach()).abs().max().item()
    assert err < 1e-3 * max(1.0, yr.abs().max().item()), f"{name} forward max|err| {err:.3e}"
    w = torch.randn(yr.shape, generator=torch.Generator().manual_seed(9))
    (yr * w).sum().backward()
    (yo * w.to(dev)).sum().backward()
    pairs = [("x", xr.grad, xo.grad)]
    if name in ("MultiHeadAttention", "CrossAttentionEncoderLayer", "CrossSelfEncoderLayer"):
        pairs.append(("context", cr.grad, co.grad))
    pairs += [(n, p.grad, q.grad) for (n, p), q in zip(ref.named_parameters(), ours.parameters())]
    # denominators floored at 1% of the largest reference gradient: some gradients are exactly zero in
    # exact arithmetic (e.g. the key-projection bias: softmax is shift-invariant) and only rounding noise
    gmax = max(a.abs().max().item() for _, a, _ in pairs)
    for n, a, b in pairs:
        assert b is not None, n
        rel = (b.cpu() - a).abs().max().item() / max(a.abs().max().item(), 1e-2 * gmax)
        assert rel < 2e-3, f"{name} grad {n}: rel err {rel:.3e}"


def _mha_case(dev, d_model, heads, cmask_lens, seed=0, mask_fn=None):
    """MultiHeadAttention fwd + every gradient vs the oracle (masked_fill(-1e9) reference semantics)."""
    torch.manual_seed(seed)
    ref = O.MultiHeadAttention(d_model, heads)
    torch.manual_seed(seed)
    ours = R.MultiHeadAttention(d_model, heads).to(dev)
    g = torch.Generator().manual_seed(3)
    B, T, Tc = len(cmask_lens), 40, 33
    x = torch.randn(B, T, d_model, generator=g)
    c = torch.randn(B, Tc, d_model, generator=g)
    mask = (torch.arange(Tc)[None] < torch.tensor(cmask_lens)[:, None]).unsqueeze(1)  # [B, 1, Tc]
    if mask_fn is not None:
        mask = mask_fn(mask, T)
    xr, cr = x.clone().requires_grad_(True), c.clone().requires_grad_(True)
    yr = ref(xr, cr, cr, mask)
    xo, co = x.to(dev).requires_grad_(True), c.to(dev).requires_grad_(True)
    yo = ours(xo, co, co, mask.to(dev))
    err = (yo.detach().cpu() - yr.detach()).abs().max().item()
    assert err < 1e-3 * max(1.0, yr.abs().max().item()), f"forward max|err| {err:.3e}"
    w = torch.randn(yr.shape, generator=torch.Generator().manual_seed(9))
    (yr * w).sum().backward()
    (yo * w.to(dev)).sum().backward()
    pairs = [("x", xr.grad, xo.grad), ("context", cr.grad, co.grad)]
    pairs += [(n, p.grad, q.grad) for (n, p), q in zip(ref.named_parameters(), ours.parameters())]
    gmax = max(a.abs().max().item() for _, a, _ in pairs)
    for n, a, b in pairs:
        rel = (b.cpu() - a).abs().max().item() / max(a.abs().max().item(), 1e-2 * gmax)
        assert rel < 2e-3, f"grad {n}: rel err {rel:.3e}"


@pytest.mark.gpu
def test_sequence_without_valid_keys_averages_all_values(dev):
    """models/transformer.py:69-73: a context with no valid key gets masked_fill(-1e9) on every score,
    so softmax is uniform over ALL keys (padded ones included) and q / k get no gradient."""
    _mha_case(dev, D, H, [33, 0])


@pytest.mark.gpu
@pytest.mark.parametrize("d_model,heads", [(128, 4), (96, 6), (64, 1)])
def test_head_dims_below_64(dev, d_model, heads):
    """d_k = d_model / num_heads of 32, 16 and 64 (the reference takes any, :42)."""
    _mha_case(dev, d_model, heads, [33, 20])


@pytest.mark.gpu
def test_per_query_masks(dev):
    """[B, Tq, Tk] masks whose rows agree for every query (flash path), and masks that differ between
    queries — random, with fully masked rows among them (the general core, -1e9 semantics)."""
    _mha_case(dev, D, H, [33, 20], mask_fn=lambda m, T: m.expand(m.shape[0], T, m.shape[2]).contiguous())
    g = torch.Generator().manual_seed(17)

    def varying(m, T):
        r = (torch.rand(m.shape[0], T, m.shape[2], generator=g) > 0.4) & m
        r[0, 5] = False  # a query with no valid key: uniform over all keys
        return r

    _mha_case(dev, D, H, [33, 20], mask_fn=varying)


@pytest.mark.gpu
def test_causal_self_attention(dev):
    """A causal (lower-triangular) mask on self attention, as a user of the reference module would pass."""
    torch.manual_seed(0)
    ref = O.MultiHeadAttention(D, H)
    torch.manual_seed(0)
    ours = R.MultiHeadAttention(D, H).to(dev)
    x = torch.randn(2, 37, D, generator=torch.Generator().manual_seed(1))
    causal = torch.tril(torch.ones(37, 37, dtype=torch.bool)).expand(2, 37, 37)
    xr, xo = x.clone().requires_grad_(True), x.to(dev).requires_grad_(True)
    yr, yo = ref(xr, xr, xr, causal), ours(xo, xo, xo, causal.to(dev))
    assert (yo.detach().cpu() - yr.detach()).abs().max().item() < 1e-3 * max(1.0, yr.abs().max().item())
    w = torch.randn(yr.shape, generator=torch.Generator().manual_seed(2))
    (yr * w).sum().backward()
    (yo * w.to(dev)).sum().backward()
    rel = (xo.grad.cpu() - xr.grad).abs().max().item() / xr.grad.abs().max().item()
    assert rel < 2e-3, rel


@pytest.mark.gpu
@pytest.mark.parametrize("d_model,heads", [(256, 2), (192, 2), (320, 4)])
def test_head_dims_above_64(dev, d_model, heads):
    """d_k = 128, 96 and 80 (the reference takes any, :42): the general core."""
    _mha_case(dev, d_model, heads, [33, 20])


@pytest.mark.gpu
def test_batch_key_mask_broadcasts_like_the_reference(dev):
    """A [B, Tk] mask: the reference's unsqueeze(1) makes it [B, 1, Tk], which broadcasts against the
    scores [B, H, Tq, Tk] as [1, B, 1, Tk] — per HEAD when B == H, an error otherwise."""
    torch.manual_seed(0)
    ref = O.MultiHeadAttention(D, H)
    torch.manual_seed(0)
    ours = R.MultiHeadAttention(D, H).to(dev)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(H, 12, D, generator=g)  # B == H
    m = torch.rand(H, 12, generator=g) > 0.3
    yr = ref(x, x, x, m)
    yo = ours(x.to(dev), x.to(dev), x.to(dev), m.to(dev))
    assert (yo.detach().cpu() - yr.detach()).abs().max().item() < 1e-3 * max(1.0, yr.abs().max().item())
    x3 = torch.randn(3, 12, D, generator=g)  # B = 3 is neither 1 nor H: the reference raises
    m3 = torch.ones(3, 12, dtype=torch.bool)
    with pytest.raises(RuntimeError):
        ref(x3, x3, x3, m3)
    with pytest.raises(RuntimeError):
        ours(x3.to(dev), x3.to(dev), x3.to(dev), m3.to(dev))


def test_indivisible_model_width_is_refused():
    with pytest.raises(ValueError):
        R.MultiHeadAttention(250, 4)


@pytest.mark.gpu
def test_general_core_without_queries_gives_zero_key_value_gradients(dev):
    """Tq = 0 on the general attention core (any d_k): dK = dV = 0 as the reference's autograd gives,
    never uninitialised memory."""
    B, Tk, H, dk = 2, 9, 2, 128
    g = torch.Generator().manual_seed(6)
    k = torch.randn(B * Tk, H * dk, generator=g).to(dev)
    v = torch.randn(B * Tk, H * dk, generator=g).to(dev)
    q = torch.empty(0, H * dk, device=dev)
    out, probs = K.mha_general_fwd(q, k, v, None, B, 0, Tk, H, dk, 0.1)
    assert out.shape[0] == 0
    dq, dkk, dv = K.mha_general_bwd(q, k, v, torch.empty(0, H * dk, device=dev), probs, None, B, 0, Tk, H, dk, 0.1)
    assert dq.shape[0] == 0
    assert torch.equal(dkk, torch.zeros_like(dkk)) and torch.equal(dv, torch.zeros_like(dv))
