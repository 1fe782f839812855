"""BASELINE.json configurations at the depth and lengths that ship (configs/Repurpose.yaml:22-32:
L = 16 tri-modal, d 512, 8 heads, d_ff 2048), HIP path vs the CPU oracle restatement of
models/MMCTransformer.py.

  * fp32 parity gate: per-frame logits and offsets within 1e-3 of the oracle, loss within
    1e-3 relative, at L = 16, T = 1024, ragged lengths (north star: "1e-3 fp32 on per-frame scores");
  * config 2 (L = 16, T = 1024, B = 8, bf16): all 8 sequences' logits within 5e-2 of the fp32 oracle
    (reported mode, not the parity gate) and one training step's gradients within the L = 16 bf16-vs-fp32
    gradient tolerances of the fp32 GPU gradients;
  * config 4 (T = 4096, B = 1): the fp32 L = 16 forward against the oracle, the bf16 model as config 2
    (its split attention and 64-row GEMM kernels), and the bf16 attention kernels (dropout on, keep bits
    stored) against an fp64 restatement and the unsplit kernels at that length;
  * config 5 (inference, 64 videos): scripts/val_atiou.py at L = 16 — identical proposals and AtIoU
    against the CPU restatement of inference_ + calculate_tiou.
"""
import math
import os
import sys

import pytest
import torch

from oracle.mmct_oracle import MMCTransformer as Oracle
from repurpose_amd import kernels as K
from repurpose_amd.MMCTransformer import MMCTransformer

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L16 = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=16, text_num_layers=3,
           cross_num_layers=3, num_heads=8)


def _threads():
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1))


def batch(B, T, lens, seed):
    """SURVEY §8d input statistics (unit-norm CLIP rows, non-negative PANNs, unit-norm text with silent
    seconds zeroed), ragged lengths, zero padding as collate_fn writes it."""
    g = torch.Generator().manual_seed(seed)
    v = torch.randn(B, T, 512, generator=g)
    v = v / v.norm(dim=-1, keepdim=True)
    a = torch.relu(torch.randn(B, T, 2048, generator=g))
    t = torch.randn(B, T, 384, generator=g)
    t = t / t.norm(dim=-1, keepdim=True) * (torch.rand(B, T, 1, generator=g) > 0.3)
    mask = (torch.arange(T)[None] < torch.tensor(lens)[:, None]).unsqueeze(1)
    m3 = mask.transpose(1, 2)
    return {"visual_feats": v * m3, "audio_feats": a * m3, "text_feats": t * m3, "masks": mask,
            "labels": (torch.rand(B, T, generator=g) < 0.35).float() * m3[..., 0],
            "segments": torch.rand(B, T, 2, generator=g) * 30}


def to_dev(b, dev):
    return {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in b.items()}


def models(dtype, seed=1234):
    torch.manual_seed(seed)
    ref = Oracle(**L16).eval()
    m = MMCTransformer(**L16, compute_dtype=dtype)
    m.load_state_dict(ref.state_dict())
    return ref, m


def fp32_gate(dev, B, T, lens, seed):
    _threads()
    ref, m = models("fp32")
    m.to(dev).eval()
    b = batch(B, T, lens, seed)
    with torch.no_grad():
        r = ref(b)
        out = m(to_dev(b, dev))
    valid = b["masks"][:, 0, :]
    e_log = (out[1].cpu() - r[1])[valid].abs().max().item()
    e_off = (out[2].cpu() - r[2])[valid].abs().max().item()
    lr = ref.losses(*r)["cls_loss"].item()
    lm = m.losses(*out)["cls_loss"].item()
    print(f"L16 fp32 T={T}: logits max err {e_log:.2e}, offsets {e_off:.2e}, loss {lm:.6f} vs {lr:.6f}")
    assert e_log < 1e-3, f"logits max err {e_log}"
    assert e_off < 1e-3, f"offsets max err {e_off}"
    assert abs(lm - lr) <= 1e-3 * max(1.0, abs(lr)), (lm, lr)


@pytest.mark.timeout(300)
def test_fp32_gate_L16_T1024_ragged(dev):
    fp32_gate(dev, 2, 1024, [1024, 700], seed=21)


@pytest.mark.timeout(300)
def test_config4_fp32_gate_L16_T4096(dev):
    fp32_gate(dev, 1, 4096, [4096], seed=44)


@pytest.mark.timeout(600)
def test_config2_bf16_L16_T1024_B8(dev):
    """Config 2 over the WHOLE batch: all 8 sequences of the bf16 forward (ragged lengths) against the
    fp32 oracle (run two sequences at a time on the CPU: attention is per sequence, every other op per
    row, so the sub-batches see the padded batch's computation), and one bf16 training step's gradients
    at that shape against the fp32 GPU gradients of the same model and batch (dropout off), with the
    tolerances of the L = 16 grouped-gradient gate (tests/test_depth_gpu.py): per tensor
    ||g_bf16 - g_fp32|| <= 0.10 ||g_fp32||, flat <= 0.03.  At M = 8192 the d_model GEMMs run on the
    64 x 128 tiles."""
    bf16_whole_batch(dev, 8, 1024, [1024, 1024, 1000, 900, 800, 777, 512, 300], seed=22, tag="config 2")


@pytest.mark.timeout(600)
def test_config4_bf16_L16_T4096_B1(dev):
    """Config 4 (T = 4096, B = 1) in bf16 through the kernels only that shape selects — the three-part
    split attention forward, the delta pass + two-role backward launch (attn_bwd_roles_kernel: dK/dV and
    dQ workgroups side by side), 64- and 32-row GEMM tiles — checked as config 2: logits against the fp32
    oracle, one step's gradients (dropout off) against the fp32 GPU gradients.  The roles kernel with
    dropout is checked against fp64 in test_config4_bf16_attention_T4096_dropout."""
    bf16_whole_batch(dev, 1, 4096, [4000], seed=45, tag="config 4", sub=1)


def bf16_whole_batch(dev, B, T, lens, seed, tag, sub=2):
    _threads()
    ref, m = models("bf16")
    m.to(dev).eval()
    b = batch(B, T, lens, seed=seed)
    errs = []
    with torch.no_grad():
        out = m(to_dev(b, dev))
        for s0 in range(0, B, sub):
            sb = {k: v[s0:s0 + sub] for k, v in b.items()}
            r = ref(sb)
            valid = sb["masks"][:, 0, :]
            for j in range(sub):
                errs.append((out[1][s0 + j].float().cpu() - r[1][j])[valid[j]].abs().max().item())
    print(f"{tag} bf16 L16: per-sequence logits max err vs fp32 oracle {[f'{e:.2e}' for e in errs]}")
    assert len(errs) == B and max(errs) < 5e-2, errs
    del ref

    # one training step of the configuration's shape, bf16 against the fp32 GPU gradients
    dev_b = to_dev(b, dev)

    def grads(dtype):
        _, mm = models(dtype)
        mm.to(dev).train()
        mm.DROPOUT = 0.0
        loss = mm.losses(*mm(dev_b))["cls_loss"] / B
        loss.backward()
        torch.cuda.synchronize()
        assert torch.isfinite(loss).item()
        g = {n: p.grad.detach().double() for n, p in mm.named_parameters() if p.grad is not None}
        return g, mm.flat_grads()[:mm.trainable_numel()].double().clone()

    g32, f32 = grads("fp32")
    g16, f16 = grads("bf16")
    assert g32.keys() == g16.keys() and len(g32) == 16 * 12 + 18
    worst = (0.0, "")
    for n in g32:
        rel = ((g16[n] - g32[n]).norm() / (g32[n].norm() + 1e-12)).item()
        worst = max(worst, (rel, n))
        assert g16[n].abs().max().item() > 0, n
        assert rel <= 0.10, f"{n}: ||bf16 - fp32|| / ||fp32|| = {rel:.3e}"
    flat = ((f16 - f32).norm() / f32.norm()).item()
    print(f"{tag} step gradients bf16 vs fp32: flat rel {flat:.3e}, worst tensor {worst[0]:.3e} ({worst[1]})")
    assert torch.isfinite(f16).all().item() and flat <= 0.03


def attn_ref64(qkv, kv, B, T, H, p, seed, dev):
    from tests.test_kernels_gpu import attn_ref
    return attn_ref(qkv, kv, B, T, H, p, seed)


@pytest.mark.timeout(300)
def test_config4_bf16_attention_T4096_dropout(dev, monkeypatch):
    """rp_attn fwd/bwd at T = 4096, B = 1 (8 heads: 256 blocks of 128 rows -> the three-part split
    forward and the two-role backward launch, asserted), dropout 0.1 with the stored keep bits, the Q
    columns prescaled as the model's QKV GEMM writes them; fwd and every gradient (dQ, dK, dV of all 8
    heads) vs fp64, and against the unsplit 4-wave kernels (RP_ATTN_SPLIT=0 and RP_ATTN_ROLES=0): keep bits bit for bit (the later key parts' streams are advanced by the skip-ahead
    multiplier), outputs and gradients within bf16 rounding."""
    from tests.test_kernels_gpu import close, close_per_seq, prescale_q, rnd
    B, H, T, p, seed = 1, 8, 4096, 0.1, 7
    qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=3).to(torch.bfloat16)
    kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
    kv[:, 3900:] = 0
    qkv, eff = prescale_q(qkv, H, 0.125)
    olo = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, seed, q_prescaled=True, out_lo=olo)
    ref_in = eff.requires_grad_(True)
    ref = attn_ref64(ref_in, kv, B, T, H, p, seed, dev)
    close(o, ref.detach(), atol=2e-2, rtol=2e-2, what="attn fwd T=4096")
    do = rnd(B * T, H * 64, dev=dev, seed=4).to(torch.bfloat16)
    assert K.attn_bwd_uses_roles(qkv, B, T, H, q_prescaled=True)
    dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo)
    gref = torch.autograd.grad(ref, ref_in, do.double())[0]
    for part, name in enumerate("qkv"):
        cols = slice(part * H * 64, (part + 1) * H * 64)
        close_per_seq(dqkv[:, cols], gref[:, cols], B, atol=6e-2, rtol=6e-2, what=f"attn d{name} T=4096")
    monkeypatch.setenv("RP_ATTN_SPLIT", "0")
    monkeypatch.setenv("RP_ATTN_ROLES", "0")
    assert not K.attn_bwd_uses_roles(qkv, B, T, H, q_prescaled=True)
    o0, lse0, mask0 = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, seed, q_prescaled=True, out_lo=olo.clone())
    assert torch.equal(mask0, mask)
    close(o, o0.double(), atol=1e-2, rtol=1e-2, what="split vs unsplit fwd")
    # with dropout the row sums come off the MFMA over the bf16-rounded P (relative to each half's own
    # running reference), so lse moves by up to ~ln(1 + 2^-8) between the two forms
    assert (lse - lse0).abs().max().item() < 5e-3
    dqkv0 = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo)
    close(dqkv, dqkv0.double(), atol=2e-2, rtol=2e-2, what="split vs unsplit bwd")


@pytest.mark.timeout(600)
def test_config5_val_split_atiou_64_videos_L16(dev):
    """North star: val-split AtIoU within +-0.1 of the CPU reference — here identical, on the first 64
    videos of the reference's data/val.json (real durations and segments; synthetic features)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import val_atiou
    r = val_atiou.run(videos=64, layers=16)
    print(r)
    assert r["videos"] == 64 and r["layers"] == 16
    assert r["identical_proposals"], r
    assert r["abs_diff"] < 1e-12 and r["within_0.1"], r
    assert r["proposals_gpu"] > 0
