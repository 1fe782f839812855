"""Drop-in ``models/softnms.py`` on the GPU (rp_softnms, one workgroup per video).

``soft_nms_intervals_cpu`` keeps the reference name and signature (``models/softnms.py:3``) and its
exact semantics, including the side effect of the reference on CPU score tensors: ``.cpu().numpy()``
aliases a CPU tensor, so the reference leaves the decayed, permuted scores in the caller's tensor
(SURVEY App. A-1).  When the caller passes a CPU tensor, the final score array computed on the GPU
is copied back into it; GPU tensors are left untouched (``.cpu()`` copies in the reference too).
The computation itself always runs on the GPU: there is no CPU fallback.  Any number of candidates
(the reference has no cap; inference_ passes at most pre_nms_topk = 1000).
"""
import numpy as np
import torch

from . import kernels as K

def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("repurpose_amd.softnms: a ROCm device is required (HIP kernel only)")
    return torch.device("cuda", torch.cuda.current_device())


def soft_nms_intervals_cpu(out_cls_logits, out_offsets, sigma=0.5, thresh=0.001, max_seg_num=20):
    src_scores = out_cls_logits
    scores = torch.as_tensor(out_cls_logits)
    segs = torch.as_tensor(out_offsets)
    n = int(segs.shape[0])
    dev = scores.device if scores.is_cuda else _device()
    s = scores.reshape(1, n).to(dev, torch.float32)
    g = segs.reshape(1, n, 2).to(dev, torch.float32)
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    ms = torch.tensor([int(max_seg_num)], dtype=torch.int32, device=dev)
    cpu_alias = isinstance(src_scores, torch.Tensor) and not src_scores.is_cuda
    keep, kc, final = K.softnms(s, g, cnt, float(sigma), float(thresh), ms, want_final_scores=cpu_alias)
    k = int(kc[0].item())
    out = keep[0, :k].cpu().numpy().astype(int)
    if cpu_alias and n > 0:
        with torch.no_grad():
            src_scores.view(-1).copy_(final[0, :n].to(src_scores.dtype).cpu())
    return out


def soft_nms_batched(scores, segs, counts, max_seg, sigma=0.5, thresh=0.001):
    """Batched GPU form: scores [B, cap], segs [B, cap, 2], counts / max_seg int [B]
    -> (keep [B, cap] int32 positions, keep_count [B] int32)."""
    keep, kc, _ = K.softnms(scores, segs, counts, float(sigma), float(thresh), max_seg)
    return keep, kc


def max_segments(duration, max_seg_per_min):
    """``int(np.ceil((vlen // 60) * max_seg_per_min))`` (reference ``MMCTransformer.py:255-257``)."""
    return int(np.ceil((duration // 60) * max_seg_per_min))
