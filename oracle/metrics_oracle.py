"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the reference's evaluation metric.

``calculate_tiou`` follows utils/metrics.py:82-111 (best IoU per prediction over the references,
``max(..., default=0)``; per-threshold precision = hits / #predictions, 0 without predictions);
``atiou`` follows the aggregation in main.py:685-703 (mean over videos per threshold, then mean
over thresholds).  Python floats (double) throughout, like the reference.
"""


def _iou(a, b):
    smax = max(a[0], b[0])
    emin = min(a[1], b[1])
    inter = max(0, emin - smax)
    union = (a[1] - a[0]) + (b[1] - b[0]) - inter
    return inter / union if union != 0 else 0


def calculate_tiou(reference_segments, predicted_segments, tiou_thresholds=(0.5,)):
    best = [max([_iou(p, r) for r in reference_segments], default=0) for p in predicted_segments]
    out = {}
    for th in tiou_thresholds:
        valid = sum(s >= th for s in best)
        out[th] = valid / len(predicted_segments) if len(predicted_segments) > 0 else 0
    return out


def atiou(per_video, thresholds):
    tiou = {th: sum(d[th] for d in per_video) / len(per_video) for th in thresholds}
    return tiou, sum(tiou.values()) / len(tiou)
