"""Evaluation metric of the trainer (reference ``utils/metrics.py``).

``calculate_tiou`` (``:82-111``) is the "AtIoU" the trainer reports (``main.py:685-703``):
precision of predicted segments at each tIoU threshold, averaged over thresholds and videos.
The per-video host function keeps the reference's signature; ``evaluate_tiou`` scores a whole
batch of videos in one HIP launch (rp_tiou_hits, IoU in double like the reference's Python floats)
and, under torch.distributed, gathers every rank's per-video precisions so the full split is
scored (the reference scores only rank 0's shard).
``calculate_ap`` / ``calculate_recall`` (``:1-80``) are unused by the reference trainer and are
restated for API completeness.
"""
import torch
import torch.distributed as dist

from . import kernels as K

THRESHOLDS = (0.5, 0.6, 0.7, 0.8, 0.9)  # main.py:685


def _seg_iou(a, b):
    inter = max(0, min(a[1], b[1]) - max(a[0], b[0]))
    union = (a[1] - a[0]) + (b[1] - b[0]) - inter
    return inter / union if union != 0 else 0


def calculate_tiou(reference_segments, predicted_segments, tiou_thresholds=(0.5,)):
    best = [max((_seg_iou(p, r) for r in reference_segments), default=0) for p in predicted_segments]
    out = {}
    for th in tiou_thresholds:
        hits = sum(s >= th for s in best)
        out[th] = hits / len(predicted_segments) if len(predicted_segments) > 0 else 0
    return out


def _frame_hits(segments, n):
    hit = [0] * n
    for seg in segments:
        lo = int(seg[0]) if int(seg[0]) >= 0 else 0
        hi = int(seg[1]) if int(seg[1]) < n else n - 1
        for i in range(lo, hi + 1):
            hit[i] = 1
    return hit


def calculate_ap(segments, labels):
    pred = _frame_hits(segments, len(labels))
    npos = sum(labels)
    if npos == 0:
        return 0.0
    tp, acc = 0, 0.0
    for i, p in enumerate(pred):
        if p == 1 and labels[i] == 1:
            tp += 1
            acc += tp / (i + 1)
    return acc / npos


def calculate_recall(segments, labels):
    pred = _frame_hits(segments, len(labels))
    pos = sum(1 for l in labels if l == 1)
    if pos == 0:
        return 0.0
    return sum(1 for p, l in zip(pred, labels) if p == 1 and l == 1) / pos


def tiou_precision_batched(gt_segments, pred_segments, tiou_thresholds=THRESHOLDS, device=None):
    """Per-video calculate_tiou for a batch on the GPU.

    gt_segments: list (videos) of lists of (start, end); pred_segments: list of [P_v, 2] tensors or
    lists.  Returns a float64 tensor [V, n_thresholds] of precisions (0 for a video with no
    predictions), equal to calculate_tiou(gt, pred, thresholds)[th] for every video and threshold."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    V = len(gt_segments)
    preds = [torch.as_tensor(p, dtype=torch.float32).reshape(-1, 2) for p in pred_segments]
    P = max([p.shape[0] for p in preds] + [1])
    R = max([len(g) for g in gt_segments] + [1])
    pred = torch.zeros(V, P, 2, dtype=torch.float32)
    ref = torch.zeros(V, R, 2, dtype=torch.float64)
    npred = torch.tensor([p.shape[0] for p in preds], dtype=torch.int32)
    nref = torch.tensor([len(g) for g in gt_segments], dtype=torch.int32)
    for v in range(V):
        if preds[v].shape[0]:
            pred[v, :preds[v].shape[0]] = preds[v].cpu()
        if len(gt_segments[v]):
            ref[v, :len(gt_segments[v])] = torch.as_tensor(gt_segments[v], dtype=torch.float64).reshape(-1, 2)
    thr = torch.tensor(list(tiou_thresholds), dtype=torch.float64)
    hits = K.tiou_hits(pred.to(dev), npred.to(dev), ref.to(dev), nref.to(dev), thr.to(dev)).double()
    n = npred.to(dev).double().unsqueeze(1)
    return torch.where(n > 0, hits / n.clamp(min=1), torch.zeros_like(hits))


def gather_precisions(prec, video_ids=None, group=None):
    """All ranks' per-video precision rows [V_r, n_thr], concatenated in rank order.  The test
    loader's DistributedSampler (drop_last=False) pads the last shard by repeating videos, so with
    ``video_ids`` (one per row) each video is kept once, at its first occurrence — the mean is then
    over the split, not biased toward the repeated videos.  gloo gathers through host memory."""
    world = dist.get_world_size(group)
    host = dist.get_backend(group) == "gloo"
    src = prec.detach().double().cpu() if host else prec.detach().double()
    n = torch.tensor([src.shape[0]], device=src.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    cap = max(1, int(max(s.item() for s in sizes)))
    pad = torch.zeros(cap, src.shape[1], device=src.device, dtype=src.dtype)
    pad[:src.shape[0]] = src
    parts = [torch.zeros_like(pad) for _ in sizes]
    dist.all_gather(parts, pad, group=group)
    out = torch.cat([p[:int(s.item())] for p, s in zip(parts, sizes)], 0)
    if video_ids is not None:
        if len(video_ids) != prec.shape[0]:
            raise ValueError("gather_precisions: one video id per precision row")
        ids = [None] * world
        dist.all_gather_object(ids, list(video_ids), group=group)
        seen, keep = set(), []
        for i, v in enumerate(x for r in ids for x in r):
            if v not in seen:
                seen.add(v)
                keep.append(i)
        out = out[torch.tensor(keep, dtype=torch.long, device=out.device)]
    return out.to(prec.device)


def evaluate_tiou(gt_segments, pred_segments, tiou_thresholds=THRESHOLDS, gather=True, video_ids=None):
    """main.py:685-703 aggregation: tIoU[th] = mean over videos, AtIoU = mean over thresholds.
    With torch.distributed initialised (and gather=True) the per-video precisions of all ranks are
    gathered first (``gather_precisions``; pass ``video_ids`` to drop the sampler's padding
    repeats).  Returns (tIoU dict, AtIoU, number of videos scored)."""
    prec = tiou_precision_batched(gt_segments, pred_segments, tiou_thresholds)
    if gather and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        prec = gather_precisions(prec, video_ids)
    elif video_ids is not None:  # one process: drop repeats too
        seen, keep = set(), []
        for i, v in enumerate(video_ids):
            if v not in seen:
                seen.add(v)
                keep.append(i)
        prec = prec[torch.tensor(keep, dtype=torch.long, device=prec.device)]
    if prec.shape[0] == 0:
        raise ZeroDivisionError("evaluate_tiou: no videos (the reference divides by len(total_tIoU))")
    mean = prec.mean(0).cpu().tolist()
    tiou = {th: m for th, m in zip(tiou_thresholds, mean)}
    return tiou, sum(tiou.values()) / len(tiou), prec.shape[0]
