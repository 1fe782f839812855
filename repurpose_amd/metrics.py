"""Evaluation metric of the trainer (reference ``utils/metrics.py``), host side.

``calculate_tiou`` (``:82-111``) is the "AtIoU" the trainer reports (``main.py:685-703``):
precision of predicted segments at each tIoU threshold, averaged over thresholds and videos.
``calculate_ap`` / ``calculate_recall`` (``:1-80``) are unused by the reference trainer and are
restated for API completeness.  These are O(#pred x #gt) per video on tens of segments — host
work, off the hot path (SURVEY §8f rank 3 lists a GPU version as a later item).
"""


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
