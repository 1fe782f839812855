"""TEST INFRASTRUCTURE ONLY — NumPy float32 restatement of ``models/softnms.py:3-38``.

Every behaviour-defining quirk of the reference is kept:

1. ``scores`` aliases the caller's CPU tensor (``.cpu().numpy()`` on a CPU tensor is a view),
   so the decayed / permuted scores leak back to the caller (``softnms.py:4``).
2. ``lengths = end - begin`` is computed once and never swapped (``:13``).
3. The selection test uses the *pre-swap* score of row i (``:18``).
4. ``argmax`` returns the first maximal index (``:22``).
5. The loop breaks *before* decaying once ``max_segments`` rows passed the threshold (``:26-29``).
6. All arithmetic is float32, decay ``w = exp(-(r*r)/sigma)`` with ``r = ov / tl`` (``:30-36``).
7. ``keep = O[s > thresh][:max_segments, 2]`` — original candidate ids (``:37``).
"""
import numpy as np


def _as_numpy(x):
    if hasattr(x, "cpu"):
        return x.cpu().numpy()
    return np.asarray(x)


def soft_nms_intervals_cpu(out_cls_logits, out_offsets, sigma=0.5, thresh=0.001, max_seg_num=20):
    s = _as_numpy(out_cls_logits)            # aliases a CPU torch tensor (quirk 1)
    segs = _as_numpy(out_offsets)
    n = segs.shape[0]
    rows = np.concatenate((segs, np.arange(0, n, dtype=np.float32).reshape(n, 1)), axis=1)
    begin = rows[:, 0]                        # views: follow the swaps below
    end = rows[:, 1]
    lengths = end - begin                     # computed once (quirk 2)
    limit = min(max_seg_num, n)
    picked = 0
    for i in range(n):
        t = s[i]                              # pre-swap copy (numpy scalar) (quirk 3)
        nxt = i + 1
        if i != n - 1:
            tail = s[nxt:]
            j = int(np.argmax(tail, axis=0)) + nxt
            if t < tail[j - nxt]:
                rows[[i, j]] = rows[[j, i]]
                s[i], s[j] = s[j].copy(), s[i].copy()
        if t > thresh:
            picked += 1
            if picked >= limit:
                break                         # quirk 5
        ov = np.clip(np.minimum(end[i], end[nxt:]) - np.maximum(begin[i], begin[nxt:]), a_min=0,
                     a_max=None)
        tl = lengths[i] + lengths[nxt:] - ov
        r = ov / tl
        s[nxt:] = np.exp(-(r * r) / sigma) * s[nxt:]
    return rows[s > thresh][:limit, 2].astype(int)
