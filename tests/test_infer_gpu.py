"""GPU inference post-processing (rp_infer_select, rp_softnms) against the NumPy/torch oracle:
identical proposal indices (SURVEY §8d parity gate) on hand-derived known answers, the committed
golden cases, random cases and the full inference_ path."""
import os

import numpy as np
import pytest
import torch

from oracle.mmct_oracle import postprocess, select_candidates
from oracle.softnms_oracle import soft_nms_intervals_cpu as nms_ref
from repurpose_amd import kernels as K
from repurpose_amd.softnms import soft_nms_intervals_cpu as nms_gpu

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
CFG = {"pre_nms_topk": 1000, "pre_nms_thresh": 0.5, "duration_thresh": 10, "duration_thresh_max": 90,
       "max_seg_per_min": 0.3, "nms_sigma": 0.5, "min_score": 0.01}


def _t(x):
    return torch.tensor(np.asarray(x, dtype=np.float32))


@pytest.mark.parametrize("scores,segs,thresh,ms,expect", [
    ([0.9, 0.8], [[0, 20], [30, 50]], 0.01, 0, []),
    ([0.9, 0.8, 0.7], [[0, 20], [30, 50], [60, 80]], 0.01, 20, [0, 1, 2]),
    ([0.5, 0.7, 0.7], [[0, 20], [30, 50], [60, 80]], 0.01, 20, [1, 2, 0]),
    ([0.9, 0.5, 0.8, 0.7], [[0, 10], [0, 100], [50, 60], [55, 65]], 0.1, 20, [0, 2, 3]),
    ([0.9, 0.8], [[0, 20], [0, 20]], 0.01, 1, [0]),
])
def test_softnms_known_answers(dev, scores, segs, thresh, ms, expect):
    keep = nms_gpu(_t(scores).to(dev), _t(segs).to(dev), 0.5, thresh, ms)
    assert keep.tolist() == expect


def test_softnms_cpu_alias_side_effect(dev):
    s = _t([0.9, 0.5, 0.8, 0.7])
    nms_gpu(s, _t([[0, 10], [0, 100], [50, 60], [55, 65]]), 0.5, 0.1, 20)
    np.testing.assert_allclose(s.numpy(), [0.9, 0.8, 0.69683, 0.065014], rtol=1e-4)


def test_softnms_golden_cases(dev):
    d = np.load(os.path.join(GOLD, "golden_softnms.npz"))
    for c in range(int(d["ncases"])):
        n = int(d[f"n{c}"])
        keep = nms_gpu(_t(d[f"scores{c}"][:n]).to(dev), _t(d[f"segs{c}"][:n]).to(dev), 0.5, float(d[f"thresh{c}"]),
                       int(d[f"maxseg{c}"]))
        assert keep.tolist() == d[f"keep{c}"].tolist(), f"case {c}"


def test_softnms_batched_random_vs_oracle(dev):
    rs = np.random.RandomState(0)
    B, cap = 16, 1000
    sc = np.zeros((B, cap), np.float32)
    sg = np.zeros((B, cap, 2), np.float32)
    cnt, ms = [], []
    for b in range(B):
        n = int(rs.randint(0, cap + 1))
        s = np.sort(rs.uniform(0.5, 1, n).astype(np.float32))[::-1]
        c = rs.uniform(0, 1800, n).astype(np.float32)
        sc[b, :n] = s
        sg[b, :n, 0] = c - rs.uniform(5.5, 45, n)
        sg[b, :n, 1] = c + rs.uniform(5.5, 45, n)
        cnt.append(n)
        ms.append(int(rs.randint(0, 40)))
    keep, kc, final = K.softnms(torch.from_numpy(sc).to(dev), torch.from_numpy(sg).to(dev),
                                torch.tensor(cnt, dtype=torch.int32, device=dev), 0.5, 0.01,
                                torch.tensor(ms, dtype=torch.int32, device=dev), want_final_scores=True)
    keep, kc = keep.cpu().numpy(), kc.cpu().numpy()
    for b in range(B):
        s = torch.from_numpy(sc[b, :cnt[b]].copy())
        ref = nms_ref(s, torch.from_numpy(sg[b, :cnt[b]]), 0.5, 0.01, ms[b])
        assert keep[b, :kc[b]].tolist() == ref.tolist(), f"video {b}"
        # every decayed score bit for bit: the kernel's exp is numpy's float32 exp algorithm
        np.testing.assert_array_equal(final[b, :cnt[b]].cpu().numpy(), s.numpy())


@pytest.mark.parametrize("n,ms", [(1500, 1500), (3000, 40), (6000, 6000), (6144, 300), (7000, 7000)])
def test_softnms_beyond_1024_candidates(dev, n, ms):
    """The reference function has no candidate cap (models/softnms.py:3-38): 1500 / 3000 candidates
    run from LDS (6000 / 6144: 117 / 120 KiB of dynamic LDS, above the 64 KiB default), 7000 from the
    global workspace path; indices and final scores match numpy."""
    rs = np.random.RandomState(n)
    s = np.sort(rs.uniform(0.0, 1, n).astype(np.float32))[::-1].copy()
    c = rs.uniform(0, 20000, n).astype(np.float32)
    g = np.stack([c - rs.uniform(5.5, 45, n), c + rs.uniform(5.5, 45, n)], 1).astype(np.float32)
    keep, kc, final = K.softnms(torch.from_numpy(s).view(1, n).to(dev), torch.from_numpy(g).view(1, n, 2).to(dev),
                                torch.tensor([n], dtype=torch.int32, device=dev), 0.5, 0.01,
                                torch.tensor([ms], dtype=torch.int32, device=dev), want_final_scores=True)
    st = torch.from_numpy(s.copy())
    ref = nms_ref(st, torch.from_numpy(g), 0.5, 0.01, ms)
    assert keep[0, :int(kc[0])].cpu().tolist() == ref.tolist()
    np.testing.assert_array_equal(final[0].cpu().numpy(), st.numpy())
    # and through the drop-in (CPU tensors in, the reference's in-place side effect out)
    st2 = torch.from_numpy(s.copy())
    k2 = nms_gpu(st2, torch.from_numpy(g), 0.5, 0.01, ms)
    assert k2.tolist() == ref.tolist()
    np.testing.assert_array_equal(st2.numpy(), st.numpy())


def test_select_matches_oracle(dev):
    g = torch.Generator().manual_seed(1)
    B, T = 4, 1801
    logits = torch.randn(B, T, generator=g) * 3
    offsets = torch.rand(B, T, 2, generator=g) * 60
    lens = [1801, 1500, 700, 90]
    mask = torch.arange(T)[None] < torch.tensor(lens)[:, None]
    count, idx, score, seg = K.infer_select(logits.to(dev), mask.to(dev), offsets.to(dev), 0.5, 1000, 10, 90)
    for b in range(B):
        ref = select_candidates(mask[b].unsqueeze(0), logits[b], offsets[b], CFG)
        n = int(count[b])
        assert n == len(ref["labels"])
        assert idx[b, :n].cpu().tolist() == ref["labels"].tolist()
        np.testing.assert_allclose(seg[b, :n].cpu().numpy(), ref["segments"].numpy(), rtol=0, atol=0)
        np.testing.assert_allclose(score[b, :n].cpu().numpy(), ref["scores"].numpy(), rtol=2e-7, atol=0)


def test_inference_end_to_end_matches_oracle_postprocess(dev):
    from repurpose_amd.MMCTransformer import MMCTransformer
    cfg = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=1, text_num_layers=3,
               cross_num_layers=3, num_heads=8)
    torch.manual_seed(0)
    m = MMCTransformer(**cfg, compute_dtype="fp32").to(dev).eval()
    g = torch.Generator().manual_seed(2)
    B, T = 3, 600
    lens = [600, 420, 250]
    batch = {"visual_feats": torch.randn(B, T, 512, generator=g), "audio_feats": torch.randn(B, T, 2048, generator=g),
             "text_feats": torch.randn(B, T, 384, generator=g),
             "masks": (torch.arange(T)[None] < torch.tensor(lens)[:, None]).unsqueeze(1),
             "labels": torch.zeros(B, T), "segments": torch.zeros(B, T, 2), "video_id": ["a", "b", "c"],
             "duration": lens}
    gb = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in batch.items()}
    res = m.inference_(gb, CFG)
    with torch.no_grad():
        masks, logits, offsets, _, _, _ = m(gb)
    ref = postprocess(masks.cpu(), logits.squeeze(-1).cpu(), offsets.cpu(), batch["video_id"], lens, CFG)
    for r, e in zip(res, ref):
        assert r["video_id"] == e["video_id"]
        assert r["labels"].cpu().tolist() == e["labels"].tolist()
        np.testing.assert_allclose(r["segments"].cpu().numpy(), e["segments"].numpy())


def test_val_split_atiou_matches_cpu_reference(dev):
    """North-star check on the reference's own validation labels (tests/golden/val_labels_64.json)
    with synthetic features: GPU inference_ + GPU tIoU vs the CPU restatement + calculate_tiou —
    identical proposals and AtIoU (the bar is +-0.1).  L = 2 keeps the CPU side fast; the L = 16
    run is scripts/val_atiou.py (profiles/)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import val_atiou
    r = val_atiou.run(videos=12, layers=2, threads=8)
    assert r["identical_proposals"], r
    assert r["abs_diff"] < 1e-12, r
    assert r["proposals_gpu"] > 0 and r["gt_segments"] > 0


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_length_buckets_give_the_padded_forward_proposals(dev, monkeypatch, dtype):
    """inference_ on a padded batch of ragged videos runs length buckets (RP_INFER_BUCKETS, default 4):
    every video's proposals are bit-identical to one padded forward (RP_INFER_BUCKETS=1)."""
    from repurpose_amd.MMCTransformer import MMCTransformer
    cfg = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=2, text_num_layers=3,
               cross_num_layers=3, num_heads=8)
    torch.manual_seed(0)
    m = MMCTransformer(**cfg, compute_dtype=dtype).to(dev).eval()
    sd = m.state_dict()
    with torch.no_grad():
        sd["cls_head.7.bias"].fill_(0.02)
        sd["reg_head.7.bias"].fill_(15.0)
    m.load_state_dict(sd)
    g = torch.Generator().manual_seed(5)
    lens = [900, 61, 333, 700, 128, 899, 64, 450, 17, 640]
    B, T = len(lens), max(lens)
    mask = (torch.arange(T)[None] < torch.tensor(lens)[:, None]).unsqueeze(1)
    batch = {"visual_feats": torch.randn(B, T, 512, generator=g), "audio_feats": torch.randn(B, T, 2048, generator=g),
             "text_feats": torch.randn(B, T, 384, generator=g), "masks": mask, "labels": torch.zeros(B, T),
             "segments": torch.zeros(B, T, 2)}
    batch = {k: v.to(dev) for k, v in batch.items()}
    batch["video_id"] = [f"v{i}" for i in range(B)]
    batch["duration"] = lens
    monkeypatch.setenv("RP_INFER_BUCKETS", "1")
    assert m._length_groups(batch["masks"]) == [(None, T)]
    ref = m.inference_(batch, CFG)
    monkeypatch.setenv("RP_INFER_BUCKETS", "4")
    groups = m._length_groups(batch["masks"])
    assert len(groups) == 4 and sorted(b for r, _ in groups for b in r) == list(range(B))
    assert all(tg < T for _, tg in groups[:-1])
    res = m.inference_(batch, CFG)
    assert sum(len(r["labels"]) for r in ref) > 0
    for r, e in zip(res, ref):
        assert r["video_id"] == e["video_id"] and r["duration"] == e["duration"]
        assert torch.equal(r["labels"], e["labels"])
        assert torch.equal(r["segments"], e["segments"])
        assert torch.equal(r["scores"], e["scores"])


def test_val_split_atiou_spread_heads_matches_cpu_reference(dev):
    """The same check with the heads spread (scripts/val_atiou.py heads='spread'): scores straddle
    the 0.5 threshold (about 4 % of the frames within 0.02 of it) and durations straddle the 10 s
    filter, so selection, duration filtering and Soft-NMS decide many near-boundary cases."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import val_atiou
    r = val_atiou.run(videos=24, layers=2, threads=8, heads="spread")
    assert r["identical_proposals"], r
    assert r["abs_diff"] < 1e-12, r
    assert r["proposals_gpu"] > 0
