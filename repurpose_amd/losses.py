"""Drop-in ``models/losses.py`` on HIP kernels.

* ``sigmoid_focal_loss(inputs, targets, alpha=0.7, gamma=2.0, reduction="none")`` — reference
  ``models/losses.py:4-53`` (fvcore formulation), forward and backward on the GPU.
* ``focal_loss_masked_sum(logits, labels, masks)`` — the fused form used by
  ``MMCTransformer.losses`` (reference ``models/MMCTransformer.py:159-179``): one kernel computes
  ``sum(mask * focal)`` with a deterministic single-block reduction; the backward kernel writes
  ``dL/dlogit`` directly (no [B,T,1] intermediate).
* ``ctr_diou_loss_1d`` — reference ``:56-116``; never called by the reference trainer,
  kept for API completeness on torch tensor ops (rank-4 "next" item in SURVEY §8f).
"""
import torch

from . import kernels as K


class _FocalMaskedSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, mask, alpha, gamma):
        ctx.save_for_backward(logits, labels, mask)
        ctx.alpha, ctx.gamma = alpha, gamma
        return K.focal_fwd_sum(logits.reshape(-1), labels.reshape(-1), mask, alpha, gamma)

    @staticmethod
    def backward(ctx, g):
        logits, labels, mask = ctx.saved_tensors
        dx = K.focal_bwd(logits.reshape(-1), labels.reshape(-1), mask, g.reshape(1), ctx.alpha, ctx.gamma)
        return dx.view_as(logits), None, None, None, None


def focal_loss_masked_sum(out_cls_logits, gt_cls_labels, masks, alpha=0.7, gamma=2.0):
    """sum_{b,t} masks[b,0,t] * sigmoid_focal_loss(logits[b,t,0], labels[b,t])."""
    B = out_cls_logits.shape[0]
    T = out_cls_logits.shape[1]
    m = (masks.reshape(B, T) != 0).to(torch.uint8).reshape(-1)
    return _FocalMaskedSum.apply(out_cls_logits, gt_cls_labels.float(), m, alpha, gamma)


class _FocalElementwise(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, targets, alpha, gamma):
        ctx.save_for_backward(inputs, targets)
        ctx.alpha, ctx.gamma = alpha, gamma
        return K.focal_elementwise(inputs, targets, alpha, gamma).view(inputs.shape)

    @staticmethod
    def backward(ctx, g):
        x, t = ctx.saved_tensors
        dx = K.focal_bwd(x.reshape(-1), t.reshape(-1), None, g.reshape(-1), ctx.alpha, ctx.gamma, per_elem=True)
        return dx.view(x.shape), None, None, None


class _FocalSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, targets, alpha, gamma):
        ctx.save_for_backward(inputs, targets)
        ctx.alpha, ctx.gamma = alpha, gamma
        return K.focal_fwd_sum(inputs.reshape(-1), targets.reshape(-1), None, alpha, gamma)

    @staticmethod
    def backward(ctx, g):
        x, t = ctx.saved_tensors
        dx = K.focal_bwd(x.reshape(-1), t.reshape(-1), None, g.reshape(1), ctx.alpha, ctx.gamma)
        return dx.view(x.shape), None, None, None


def sigmoid_focal_loss(inputs, targets, alpha: float = 0.7, gamma: float = 2.0, reduction: str = "none"):
    """Reference ``models/losses.py:4-53`` (same defaults, same broadcasting-free contract:
    ``inputs`` and ``targets`` have the same shape)."""
    x = inputs.float()
    t = targets.float().expand_as(x)
    if reduction == "none":
        return _FocalElementwise.apply(x, t, alpha, gamma)
    s = _FocalSum.apply(x, t, alpha, gamma)
    if reduction == "sum":
        return s
    if reduction == "mean":
        return s / max(x.numel(), 1)
    raise ValueError(f"invalid reduction {reduction!r}")


def ctr_diou_loss_1d(input_offsets, target_offsets, reduction: str = "none", eps: float = 1e-8):
    """Reference ``models/losses.py:56-116`` (1-D distance-IoU on [B, T, 2] offsets)."""
    a = input_offsets.float()
    g = target_offsets.float()
    assert (a >= 0.0).all(), "predicted offsets must be non-negative"
    assert (g >= 0.0).all(), "GT offsets must be non-negative"
    lp, rp = a[:, :, 0], a[:, :, 1]
    lg, rg = g[:, :, 0], g[:, :, 1]
    inter = torch.min(lp, lg) + torch.min(rp, rg)
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
