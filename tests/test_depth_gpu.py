"""Gradient gates at the depth that ships: the reference trains 16 encoder layers
(configs/Repurpose.yaml:28; backward at main.py:339).

* fp32 (parity mode): every trainable gradient of the L = 16 tri-modal model against torch autograd
  through the CPU oracle in float64 (stock nn.TransformerEncoderLayer modules, the reference's
  construction order), ragged lengths, dropout off.  With every ReLU's on/off pattern pinned to the GPU
  forward's, each tensor within 5x the oracle-in-fp32's own distance to fp64; unpinned, a coarse bound
  per tensor that single ReLU switches (pre-activations within rounding of zero) stay inside;
* bf16 (bench mode) with the deferred grouped weight gradients active — the single 16-layer
  rp_gemm_wgrad_grouped launch the bench runs — against the fp32 GPU gradients of the same model on
  the same batch: per tensor ||g_bf16 - g_fp32||_2 <= 0.10 ||g_fp32||_2 (bf16 operands carry 2^-9
  relative rounding per MFMA input through 16 layers of backward), and <= 0.03 over the flat buffer;
* the L = 16 bf16-vs-fp32 training trajectory (the round-2 40-step script, shortened): 10 FusedAdam
  steps at T = 512, dropout off, losses within 2 % per step and 0.6 % on average.
"""
import copy

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


class _Gate(torch.nn.Module):
    """A ReLU whose on/off pattern is given (the GPU forward's): z * gate, gradient gate."""

    def __init__(self, gate):
        super().__init__()
        self.gate = gate

    def forward(self, z):
        return z * self.gate.to(z.dtype)


def _pin_relus(oracle, gates, B, T):
    """Every ReLU of the oracle's trained path follows the GPU forward's decisions."""
    for l, layer in enumerate(oracle.multimodal_encoder.layers):
        layer.activation = _Gate(gates["layers"][l].view(B, T, -1))
    oracle.feature_map[2] = _Gate(gates["feats"].view(B, T, -1))
    oracle.cls_head[2] = _Gate(gates["c1"].view(B, T, -1))
    oracle.cls_head[5] = _Gate(gates["c2"].view(B, T, -1))


def _grads_of(oracle, b, dtype):
    o = copy.deepcopy(oracle).to(dtype)
    o.zero_grad()
    bb = {k: (v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in b.items()}
    o.losses(*o(bb))["cls_loss"].backward()
    return {n: q.grad.detach().double().clone() for n, q in o.named_parameters() if q.grad is not None}


def test_backward_fp32_parity_L16(dev):
    """fp32 gradients at the shipped depth against the exact (fp64) gradient.

    A ReLU whose pre-activation lies within rounding of zero switches between fp32 implementations, and
    one switched unit of a linear1 moves that layer's weight gradient by ~1e-3 and every layer below it
    by ~1e-4 (measured: the GPU fp32 path and this container's CPU fp32 oracle each carry one or two such
    switches at L = 16, on different layers).  So the tight gate runs with the gates pinned: the fp64
    oracle (and the CPU fp32 oracle, for the rounding scale) take every ReLU's on/off pattern from the
    GPU forward, and the GPU gradient must then be as close to fp64 as fp32 arithmetic is — per tensor
    within 5x the CPU fp32 oracle's distance (floor 2e-6), flat within 4x (measured: flat 5.0e-7 vs the
    CPU's 2.4e-7, worst tensor 2.7x).  Unpinned, every tensor stays
    within a coarse bound (norm 5e-3, max-abs 2.5e-2) that switches stay inside and a broken kernel or
    layer (O(1) off) does not."""
    torch.manual_seed(3)
    ref = Oracle(**L16).eval()  # dropout off; autograd runs the training path of the encoder layers
    torch.manual_seed(3)
    m = MMCTransformer(**L16, compute_dtype="fp32").to(dev).train()
    m.DROPOUT = 0.0
    B, T = 2, 256
    b = make_batch(L16, B, T, [256, 173], seed=8)
    out = m(to_dev(b, dev))
    S = out[1].grad_fn.run.saved  # the engine's saved forward activations (post-ReLU outputs)
    gates = {"layers": [(lay[13] > 0).cpu() for lay in S["layers"]], "feats": (S["feats"] > 0).cpu(),
             "c1": (S["c1"] > 0).cpu(), "c2": (S["c2"] > 0).cpu()}
    lm = m.losses(*out)["cls_loss"]
    lm.backward()
    torch.cuda.synchronize()
    g64 = _grads_of(ref, b, torch.float64)
    _pin_relus(ref, gates, B, T)
    p64 = _grads_of(ref, b, torch.float64)
    p32 = _grads_of(ref, b, torch.float32)
    rows = []
    for n, p in m.named_parameters():
        if n.startswith("reg_head."):
            assert p.grad is None and n not in g64
            continue
        g = p.grad.cpu().double()
        nrm = lambda a, x: ((a - x).norm() / (x.norm() + 1e-30)).item()  # noqa: E731
        rows.append((n, (g - g64[n]).abs().max().item() / (g64[n].abs().max().item() + 1e-30), nrm(g, g64[n]),
                     nrm(g, p64[n]), nrm(p32[n], p64[n])))
    assert len(rows) == 16 * 12 + 18  # every encoder tensor + input projection/norm, encoder norm, feature map, cls head
    for n, e_max, e_nrm, pe, pr in rows:  # unpinned: coarse
        assert e_max <= 2.5e-2, f"{n}: max-abs rel {e_max:.2e} (unpinned)"
        assert e_nrm <= 5e-3, f"{n}: norm rel {e_nrm:.2e} (unpinned)"
    flat = lambda gd: torch.cat([gd[n].flatten() for n, *_ in rows])  # noqa: E731
    gm = torch.cat([dict(m.named_parameters())[n].grad.cpu().double().flatten() for n, *_ in rows])
    e_flat = ((gm - flat(p64)).norm() / flat(p64).norm()).item()
    r_flat = ((flat(p32) - flat(p64)).norm() / flat(p64).norm()).item()
    worst = max(rows, key=lambda r: r[3] / max(2e-6, 5 * r[4]))
    print(f"L=16 fp32, gates pinned: flat {e_flat:.2e} (CPU fp32 {r_flat:.2e}); worst tensor {worst[0]} "
          f"{worst[3]:.2e} (CPU fp32 {worst[4]:.2e}); unpinned worst {max(r[2] for r in rows):.2e}")
    for n, e_max, e_nrm, pe, pr in rows:
        assert pe <= max(2e-6, 5 * pr), f"{n}: pinned norm rel {pe:.2e} (CPU fp32 {pr:.2e})"
    assert e_flat <= 4 * r_flat, (e_flat, r_flat)


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
