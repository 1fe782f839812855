"""Drop-in ``models/losses.py`` on HIP kernels.

* ``sigmoid_focal_loss(inputs, targets, alpha=0.7, gamma=2.0, reduction="none")`` — reference
  ``models/losses.py:4-53`` (fvcore formulation), forward and backward on the GPU.
* ``focal_loss_masked_sum(logits, labels, masks)`` — the fused form used by
  ``MMCTransformer.losses`` (reference ``models/MMCTransformer.py:159-179``): one kernel computes
  ``sum(mask * focal)`` with a deterministic single-block reduction; the backward kernel writes
  ``dL/dlogit`` directly (no [B,T,1] intermediate).
* ``ctr_diou_loss_1d`` — reference ``:56-116``; never called by the reference trainer;
  fused forward / backward kernels rp_diou_fwd / rp_diou_bwd.
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
    if masks.dtype == torch.bool and masks.is_contiguous():
        m = masks.reshape(-1).view(torch.uint8)  # zero-copy: bool is stored as 0 / 1 bytes
    else:
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


class _CtrDiou(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, g, reduction, eps):
        shape = a.shape
        a2, g2 = a.reshape(-1, 2).contiguous(), g.reshape(-1, 2).contiguous()
        red = {"none": 0, "mean": 1, "sum": 2}[reduction]
        out = K.diou_fwd(a2, g2, eps, red)
        ctx.save_for_backward(a2, g2)
        ctx.red, ctx.eps, ctx.shape = red, eps, shape
        return out.view(shape[:-1]) if red == 0 else out

    @staticmethod
    def backward(ctx, gout):
        a2, g2 = ctx.saved_tensors
        n = a2.shape[0]
        per_elem = ctx.red == 0
        scale = (1.0 / n if n > 0 else 0.0) if ctx.red == 1 else 1.0
        go = gout.contiguous().float().reshape(-1) if per_elem else gout.float().reshape(1)
        dp, dg = K.diou_bwd(a2, g2, ctx.eps, go, per_elem, scale, want_pred=ctx.needs_input_grad[0],
                            want_gt=ctx.needs_input_grad[1])
        return (dp.view(ctx.shape) if dp is not None else None,
                dg.view(ctx.shape) if dg is not None else None, None, None)


def ctr_diou_loss_1d(input_offsets, target_offsets, reduction: str = "none", eps: float = 1e-8):
    """Reference ``models/losses.py:56-116`` (1-D distance-IoU on [..., 2] (left, right) offsets),
    forward and backward in the HIP kernels rp_diou_fwd / rp_diou_bwd.  Like the reference it asserts
    non-negative offsets (a device-to-host check)."""
    a = input_offsets.float()
    g = target_offsets.float()
    assert (a >= 0.0).all(), "predicted offsets must be non-negative"
    assert (g >= 0.0).all(), "GT offsets must be non-negative"
    if reduction not in ("none", "mean", "sum"):
        raise ValueError(f"ctr_diou_loss_1d: unknown reduction {reduction!r}")
    return _CtrDiou.apply(a, g, reduction, float(eps))
