"""Gradient-norm logging (reference main.py:345-367) through rp_sumsq_batched: the same keys in the
same order as the reference's loop, values equal to torch's norms (fp64 here, fp32 there)."""
import math

import pytest
import torch

from repurpose_amd import kernels as K
from repurpose_amd.gradnorm import grad_norms
from repurpose_amd.MMCTransformer import MMCTransformer

pytestmark = pytest.mark.gpu


def reference_loop(model):
    """main.py:345-367 as written (torch norms, one .item() per tensor)."""
    m = model.module if hasattr(model, "module") else model
    out = {}
    for name, module in m.named_modules():
        if isinstance(module, torch.nn.Linear):
            if module.weight.grad is not None:
                out[f"grad_norm/{name}_weight"] = module.weight.grad.norm().item()
            if module.bias is not None and module.bias.grad is not None:
                out[f"grad_norm/{name}_bias"] = module.bias.grad.norm().item()
    total = 0
    for p in m.parameters():
        if p.grad is not None:
            total += p.grad.data.norm(2).item() ** 2
    out["grad_norm/total"] = total ** 0.5
    return out


def test_sumsq_batched_sizes_offsets_and_chunks(dev):
    g = torch.Generator().manual_seed(3)
    base = torch.randn(300000, generator=g).to(dev)
    # odd lengths, 4-byte (not 16-byte) aligned starts, an empty tensor, 70 items -> two launches
    ts = [base[o:o + n] for o, n in [(0, 1), (1, 7), (3, 1000), (5, 65537), (0, 0), (9, 4), (2, 3)]]
    ts += [torch.randn(int(n), generator=g).to(dev) for n in torch.randint(1, 5000, (63,), generator=g)]
    got = K.sumsq_batched(ts).cpu()
    want = torch.tensor([float((t.double() ** 2).sum()) for t in ts], dtype=torch.float64)
    torch.testing.assert_close(got, want, rtol=1e-12, atol=0)
    again = K.sumsq_batched(ts).cpu()
    assert torch.equal(got, again)  # fixed summation order


def test_sumsq_batched_rejects_non_fp32(dev):
    with pytest.raises(ValueError):
        K.sumsq_batched([torch.ones(4, device=dev, dtype=torch.bfloat16)])


def test_grad_norms_match_reference_loop(dev):
    cfg = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=2, text_num_layers=3,
               cross_num_layers=3, num_heads=8)
    torch.manual_seed(0)
    m = MMCTransformer(**cfg, compute_dtype="fp32").to(dev).train()
    g = torch.Generator().manual_seed(1)
    B, T = 2, 128
    batch = {"visual_feats": torch.randn(B, T, 512, generator=g), "audio_feats": torch.randn(B, T, 2048, generator=g),
             "text_feats": torch.randn(B, T, 384, generator=g),
             "masks": (torch.arange(T)[None] < torch.tensor([128, 90])[:, None]).unsqueeze(1),
             "labels": (torch.rand(B, T, generator=g) < 0.35).float(), "segments": torch.rand(B, T, 2, generator=g)}
    batch = {k: v.to(dev) for k, v in batch.items()}
    out = m(batch)
    m.losses(*out)["cls_loss"].backward()
    got = grad_norms(m)
    ref = reference_loop(m)
    assert list(got) == list(ref)  # same keys, same order (reg_head has no gradient in either)
    assert not any(k.startswith("grad_norm/reg_head") for k in got)
    for k in ref:
        assert math.isclose(got[k], ref[k], rel_tol=2e-6, abs_tol=1e-12), (k, got[k], ref[k])
    # the wrapper's .module is unwrapped as in the reference
    wrapped = type("W", (), {"module": m})()
    assert grad_norms(wrapped) == got
