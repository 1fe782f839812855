"""GPU tIoU metric (rp_tiou_hits) and DIoU loss (rp_diou_*) against the CPU restatements in
oracle/metrics_oracle.py (utils/metrics.py:82-111, main.py:685-703) and oracle/focal_oracle.py
(models/losses.py:56-116)."""
import random

import pytest
import torch

from oracle import focal_oracle as FO
from oracle import metrics_oracle as MO
from repurpose_amd import losses as L
from repurpose_amd import metrics as M

pytestmark = pytest.mark.gpu
THR = (0.5, 0.6, 0.7, 0.8, 0.9)


def _videos(seed, V=40):
    rnd = random.Random(seed)
    gts, preds = [], []
    for v in range(V):
        ng = rnd.choice([0, 1, 3, 7])
        gts.append([[s, s + rnd.choice([5, 12.5, 30])] for s in (rnd.randint(0, 300) for _ in range(ng))])
        npd = rnd.choice([0, 1, 4, 20])
        p = []
        for _ in range(npd):
            s = rnd.uniform(0, 320)
            p.append([s, s + rnd.uniform(10.5, 89.5)])
        if gts[-1] and p:  # exact boundary cases: a copy of a reference, touching and nested segments
            g = gts[-1][0]
            p[0] = [float(g[0]), float(g[1])]
            if len(p) > 1:
                p[1] = [float(g[1]), float(g[1]) + 20.0]
        preds.append(torch.tensor(p, dtype=torch.float32).reshape(-1, 2))
    return gts, preds


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_tiou_matches_reference_exactly(dev, seed):
    gts, preds = _videos(seed)
    prec = M.tiou_precision_batched(gts, preds, THR).cpu()
    ref = [MO.calculate_tiou(g, p.tolist(), THR) for g, p in zip(gts, preds)]
    for v, d in enumerate(ref):
        for j, th in enumerate(THR):
            assert prec[v, j].item() == d[th], (v, th, prec[v, j].item(), d[th])
    tiou, at, n = M.evaluate_tiou(gts, preds, THR)
    rt, rat = MO.atiou(ref, THR)
    assert n == len(gts)
    for th in THR:
        assert abs(tiou[th] - rt[th]) < 1e-12
    assert abs(at - rat) < 1e-12


def test_tiou_no_references_and_no_predictions(dev):
    gts = [[], [[1.0, 2.0]], []]
    preds = [torch.tensor([[0.0, 5.0]]), torch.zeros(0, 2), torch.zeros(0, 2)]
    prec = M.tiou_precision_batched(gts, preds, THR).cpu()
    assert torch.equal(prec, torch.zeros(3, len(THR), dtype=torch.float64))


@pytest.mark.parametrize("reduction", ["none", "mean", "sum"])
def test_ctr_diou_fwd_bwd(dev, reduction):
    g = torch.Generator().manual_seed(3)
    a = torch.rand(4, 257, 2, generator=g) * 20
    t = torch.rand(4, 257, 2, generator=g) * 20
    a[0, :5] = t[0, :5]          # ties: min / max subgradients split
    a[1, :3, 0] = 0.0
    t[1, :3, 0] = 0.0            # zero-length-side cases
    ar, tr = a.clone().double().requires_grad_(True), t.clone().double().requires_grad_(True)
    ref = FO.ctr_diou_loss_1d(ar, tr, reduction=reduction)
    ad, td = a.to(dev).requires_grad_(True), t.to(dev).requires_grad_(True)
    out = L.ctr_diou_loss_1d(ad, td, reduction=reduction)
    assert (out.detach().cpu().double() - ref.detach()).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())
    w = torch.rand(ref.shape, generator=g, dtype=torch.float64) if reduction == "none" else torch.tensor(1.7, dtype=torch.float64)
    (ref * w).sum().backward()
    (out * w.to(dev).float()).sum().backward()
    for gr, go, n in ((ar.grad, ad.grad, "input"), (tr.grad, td.grad, "target")):
        err = (go.cpu().double() - gr).abs().max().item()
        assert err < 1e-4 * max(1.0, gr.abs().max().item()), f"{n} grad err {err:.3e}"


def test_ctr_diou_rejects_negative_offsets(dev):
    with pytest.raises(AssertionError):
        L.ctr_diou_loss_1d(-torch.ones(1, 4, 2, device=dev), torch.ones(1, 4, 2, device=dev))
