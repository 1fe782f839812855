"""repurpose_amd — MI355X (gfx950) HIP implementation of the Repurpose tri-modal temporal
localisation hot path (MMCTransformer forward / focal loss / backward / DP gradient exchange /
inference + Soft-NMS), as drop-ins for the reference's modules:

    models.MMCTransformer.MMCTransformer   -> repurpose_amd.MMCTransformer.MMCTransformer
    models.losses.sigmoid_focal_loss       -> repurpose_amd.losses.sigmoid_focal_loss
    models.softnms.soft_nms_intervals_cpu  -> repurpose_amd.softnms.soft_nms_intervals_cpu
    utils.distributed.MultiGPUStrategy     -> repurpose_amd.distributed.MultiGPUStrategy
    utils.metrics.calculate_tiou           -> repurpose_amd.metrics.calculate_tiou

Kernels live in ``repurpose_amd/csrc`` behind the C ABI of ``include/rp_api.h``.
"""
from . import _native  # noqa: F401

__all__ = ["MMCTransformer", "sigmoid_focal_loss", "soft_nms_intervals_cpu"]


def __getattr__(name):
    if name == "MMCTransformer":
        from .MMCTransformer import MMCTransformer
        return MMCTransformer
    if name == "sigmoid_focal_loss":
        from .losses import sigmoid_focal_loss
        return sigmoid_focal_loss
    if name == "soft_nms_intervals_cpu":
        from .softnms import soft_nms_intervals_cpu
        return soft_nms_intervals_cpu
    raise AttributeError(name)
