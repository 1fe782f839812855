"""Gradient gates at the depth that ships: the reference trains 16 encoder layers
(configs/Repurpose.yaml:28; backward at main.py:339).

* fp32 (parity mode): every trainable gradient of the L = 16 tri-modal model against torch autograd
  through the CPU oracle in float64 (stock nn.TransformerEncoderLayer modules, the reference's
  construction order), ragged lengths, dropout off: the whole gradient no farther from the fp64
  gradient (norm) than 4x the reference's own fp32 arithmetic (the oracle in float32), and every tensor
  within a coarse bound that single ReLU-gate flips stay inside;
* bf16 (bench mode) with the deferred grouped weight gradients active — the single 16-layer
  rp_gemm_wgrad_grouped launch the bench runs — against the fp32 GPU gradients of the same model on
  the same batch: per tensor ||g_bf16 - g_fp32||_2 <= 0.10 ||g_fp32||_2 (bf16 operands carry 2^-9
  relative rounding per MFMA input through 16 layers of backward), and <= 0.03 over the flat buffer;
* the L = 16 bf16-vs-fp32 training trajectory (the round-2 40-step script, shortened): 10 FusedAdam
  steps at T = 512, dropout off, losses within 2 % per step and 0.6 % on average.
"""
import numpy as np
import pytest
import torch

from oracle.mmct_oracle import MMCTransformer as Oracle
from repurpose_amd.MMCTransformer import MMCTransformer
from repurpose_amd.optim import FusedAdam

from .test_model_gpu import TRI, make_batch, to_dev

pytestmark = pytest.mark.gpu

L16 = dict(TRI, self_num_layers=16)


def _grads(m):
    return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters() if p.grad is not None}


def test_backward_fp32_parity_L16(dev):
    """The exact gradient is the oracle in float64.  At 16 layers fp32 arithmetic itself (the CPU oracle
    in float32 included) lands up to 1.5e-2 (max-abs) / 1.5e-3 (norm) from it on single tensors (ReLU
    gates of linear1 flip on pre-activations within fp32 rounding of zero), so a fixed per-tensor
    max-abs gate against the fp32 oracle measures rounding, not the kernels.  Gates: the GPU fp32
    gradient of the whole model within 1e-3 (or 4x the fp32 reference's own distance) in norm, the
    median tensor within 2e-4 (a systematic error moves every tensor; a flip moves one or two), and per
    tensor a coarse bound (norm 5e-3, max-abs 2.5e-2) that single flips stay inside and a broken kernel
    or layer (O(1) off) does not."""
    torch.manual_seed(3)
    ref = Oracle(**L16).eval()  # dropout off; autograd runs the training path of the encoder layers
    torch.manual_seed(3)
    m = MMCTransformer(**L16, compute_dtype="fp32").to(dev).train()
    m.DROPOUT = 0.0
    b = make_batch(L16, 2, 256, [256, 173], seed=8)
    lr = ref.losses(*ref(b))["cls_loss"]
    lr.backward()
    g32 = {n: q.grad.detach().double().clone() for n, q in ref.named_parameters() if q.grad is not None}
    ref64 = ref.double()
    ref64.zero_grad()
    b64 = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in b.items()}
    l64 = ref64.losses(*ref64(b64))["cls_loss"]
    l64.backward()
    lm = m.losses(*m(to_dev(b, dev)))["cls_loss"]
    lm.backward()
    torch.cuda.synchronize()
    assert abs(lm.item() - l64.item()) < 1e-3 * max(1.0, abs(l64.item()))
    rows = []
    for (n, p), (n2, q) in zip(m.named_parameters(), ref64.named_parameters()):
        assert n == n2
        if n.startswith("reg_head."):
            assert p.grad is None and q.grad is None
            continue
        g, gx, gr = p.grad.cpu().double(), q.grad.double(), g32[n]
        rows.append((n, (g - gx).abs().max().item() / (gx.abs().max().item() + 1e-30),
                     (gr - gx).abs().max().item() / (gx.abs().max().item() + 1e-30),
                     (g - gx).norm().item() / (gx.norm().item() + 1e-30),
                     (gr - gx).norm().item() / (gx.norm().item() + 1e-30)))
    # A ReLU gate of linear1 whose pre-activation lies within rounding of zero flips between fp32
    # implementations and moves single gradient elements: measured on layer 8's linear1.weight, max-abs
    # 1.5e-2 / norm 1.5e-3 from fp64 for this container's CPU fp32 AND for the GPU fp32 path, 2.8e-5 for
    # the GPU box's CPU fp32 (another BLAS build).  So per tensor only a coarse bound (a broken kernel or
    # layer is off by O(1)), and the tight gate on the whole gradient, where a flip is diluted.
    n_checked = 0
    for n, e_max, r_max, e_nrm, r_nrm in rows:
        n_checked += 1
        assert e_max <= 2.5e-2, f"{n}: max-abs rel {e_max:.2e} (fp32 reference {r_max:.2e})"
        assert e_nrm <= 5e-3, f"{n}: norm rel {e_nrm:.2e} (fp32 reference {r_nrm:.2e})"
    gm = torch.cat([p.grad.cpu().double().flatten() for n, p in m.named_parameters() if p.grad is not None])
    gx = torch.cat([q.grad.double().flatten() for n, q in ref64.named_parameters() if q.grad is not None])
    gr = torch.cat([g32[n].flatten() for n, q in ref64.named_parameters() if q.grad is not None])
    e_flat = ((gm - gx).norm() / gx.norm()).item()
    r_flat = ((gr - gx).norm() / gx.norm()).item()
    med = sorted(r[3] for r in rows)[len(rows) // 2]
    r_med = sorted(r[4] for r in rows)[len(rows) // 2]
    print(f"L=16 fp32 vs fp64: flat norm error {e_flat:.2e} (fp32 reference {r_flat:.2e}); median tensor "
          f"{med:.2e} (reference {r_med:.2e}); worst tensor {max(rows, key=lambda r: r[3])[0]} norm "
          f"{max(r[3] for r in rows):.2e}")
    # one flipped gate moved the flat norm to 3.2e-4 on one box (layer 8 linear1.weight 1.5e-3)
    assert e_flat <= max(1e-3, 4 * r_flat), (e_flat, r_flat)
    assert med <= 2e-4, (med, r_med)
    assert n_checked == 16 * 12 + 18  # every encoder tensor + input projection/norm, encoder norm, feature map, cls head


def test_bf16_grouped_gradients_track_fp32_L16(dev, monkeypatch):
    monkeypatch.setenv("RP_WGRAD_GROUPED", "1")
    b = to_dev(make_batch(L16, 2, 256, [256, 200], seed=12), dev)

    def grads(dtype):
        torch.manual_seed(7)
        m = MMCTransformer(**L16, compute_dtype=dtype).to(dev).train()
        m.DROPOUT = 0.0
        (m.losses(*m(b))["cls_loss"] / 2).backward()
        torch.cuda.synchronize()
        return _grads(m), m.flat_grads()[:m.trainable_numel()].double()

    g32, f32 = grads("fp32")
    g16, f16 = grads("bf16")
    assert g32.keys() == g16.keys()
    worst = (0.0, "")
    for n in g32:
        rel = ((g16[n] - g32[n]).norm() / (g32[n].norm() + 1e-12)).item()
        worst = max(worst, (rel, n))
        assert rel <= 0.10, f"{n}: ||bf16 - fp32|| / ||fp32|| = {rel:.3e}"
    flat = ((f16 - f32).norm() / f32.norm()).item()
    print(f"L=16 bf16 (grouped wgrad) vs fp32: flat rel {flat:.3e}, worst tensor {worst[0]:.3e} ({worst[1]})")
    assert flat <= 0.03


def test_bf16_training_tracks_fp32_L16(dev):
    batches = [to_dev(make_batch(L16, 2, 512, [512, 400], seed=90 + i), dev) for i in range(3)]

    def run(dtype):
        torch.manual_seed(1234)
        m = MMCTransformer(**L16, compute_dtype=dtype).to(dev).train()
        m.DROPOUT = 0.0
        opt = FusedAdam(m, lr=1e-4, weight_decay=1e-4)
        out = []
        for s in range(10):
            opt.zero_grad()
            loss = m.losses(*m(batches[s % 3]))["cls_loss"] / 2
            loss.backward()
            opt.step()
            out.append(loss.item())
        return out

    f32, b16 = run("fp32"), run("bf16")
    assert all(np.isfinite(f32)) and all(np.isfinite(b16))
    rel = [abs(a - b) / abs(a) for a, b in zip(f32, b16)]
    print("L=16 T=512 loss rel dev per step", [f"{r:.1e}" for r in rel])
    # measured on MI355X (round 3): per step 4e-4 .. 1.0e-2, mean 3.6e-3; the largest deviation is the
    # step after the lr-1e-4 loss spike (step 2: loss x5), where bf16 rounding of the Adam-updated
    # weights moves the trajectory most.  Gate: every step within 2 %, the mean within 0.6 %.
    assert max(rel) <= 2e-2 and float(np.mean(rel)) <= 6e-3, (f32, b16)
