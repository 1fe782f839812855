"""TEST INFRASTRUCTURE ONLY — CPU restatement of ``models/losses.py``.

``sigmoid_focal_loss`` follows reference ``models/losses.py:4-53`` (alpha 0.7, gamma 2, fp32);
``ctr_diou_loss_1d`` follows ``:56-116`` (never called by the reference trainer).
"""
import torch
from torch.nn import functional as F


def sigmoid_focal_loss(inputs, targets, alpha: float = 0.7, gamma: float = 2.0,
                       reduction: str = "none"):
    x = inputs.float()
    t = targets.float()
    p = torch.sigmoid(x)
    ce = F.binary_cross_entropy_with_logits(x, t, reduction="none")
    pt = p * t + (1 - p) * (1 - t)
    loss = ce * ((1 - pt) ** gamma)
    if alpha >= 0:
        loss = (alpha * t + (1 - alpha) * (1 - t)) * loss
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def ctr_diou_loss_1d(input_offsets, target_offsets, reduction: str = "none", eps: float = 1e-8):
    a = input_offsets.float()
    g = target_offsets.float()
    assert (a >= 0.0).all(), "predicted offsets must be non-negative"
    assert (g >= 0.0).all(), "GT offsets must be non-negative"
    lp, rp = a[:, :, 0], a[:, :, 1]
    lg, rg = g[:, :, 0], g[:, :, 1]
    inter = torch.min(rp, rg) + torch.min(lp, lg)
    union = (lp + rp) + (lg + rg) - inter
    iou = inter / union.clamp(min=eps)
    enclose = torch.max(lp, lg) + torch.max(rp, rg)
    rho = 0.5 * (rp - lp - rg + lg)
    loss = 1.0 - iou + torch.square(rho / enclose.clamp(min=eps))
    if reduction == "mean":
        return loss.mean() if loss.numel() > 0 else 0.0 * loss.sum()
    if reduction == "sum":
        return loss.sum()
    return loss
