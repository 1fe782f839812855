"""Batch collation (repurpose_amd.data) against the restatement of the reference's preprocessing /
collate_fn (oracle/data_oracle.py): host drop-ins on CPU, the device path (rp_pad_rows) on the GPU.
Items mimic the stored features: fp16 CLIP visual rows, fp32 PANNs audio rows, fp64 text rows
(possibly shorter than the visual length), int labels, (left, right) float offsets."""
import numpy as np
import pytest
import torch

from oracle import data_oracle as O
from repurpose_amd import data as D


def _batch(seed, lens=(37, 80, 5, 64)):
    rng = np.random.default_rng(seed)
    items = []
    for i, n in enumerate(lens):
        nt = max(0, n - 7) if i == 1 else n  # text shorter than the visual length for one video
        items.append({"video_id": f"vid{i}", "duration": n, "gt_segments": [[1.0, 9.0]],
                      "feats": {"visual": rng.standard_normal((n, 512)).astype(np.float16),
                                "audio": np.maximum(rng.standard_normal((n, 2048)), 0).astype(np.float32),
                                "text": rng.standard_normal((nt, 384))},
                      "labels": [int(x) for x in rng.integers(0, 2, n)],
                      "segments": [(float(a), float(b)) for a, b in rng.uniform(0, 30, (n, 2))]})
    return items


def _same(a, b):
    assert set(a) == set(b)
    for k in a:
        if torch.is_tensor(a[k]):
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
            assert torch.equal(a[k].cpu(), b[k].cpu()), k
        else:
            assert a[k] == b[k], k


@pytest.mark.parametrize("seed", [0, 1])
def test_collate_matches_reference(seed):
    batch = _batch(seed)
    _same(D.collate_fn(batch), O.collate_fn(batch))


def test_collate_errors():
    b = _batch(0, lens=(0, 0))
    with pytest.raises(ValueError):
        D.collate_fn(b)


def test_ragged_layout():
    batch = _batch(2)
    rb = D.collate_ragged(batch)
    assert rb.rows["visual"].dtype == np.float16 and rb.rows["text"].dtype == np.float64
    assert list(np.diff(rb.offsets["visual"])) == [37, 80, 5, 64]
    assert list(np.diff(rb.offsets["text"])) == [37, 73, 5, 64]
    r32 = D.collate_ragged(batch, f32=True)  # worker-side conversion: every row array fp32, same values
    assert all(v.dtype == np.float32 for v in r32.rows.values())
    assert np.array_equal(r32.rows["text"], rb.rows["text"].astype(np.float32))
    assert np.array_equal(r32.rows["visual"], rb.rows["visual"].astype(np.float32))
    assert all(np.array_equal(r32.offsets[k], rb.offsets[k]) for k in rb.offsets)


@pytest.mark.gpu
@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("seed", [0, 3])
def test_device_collate_matches_reference(dev, seed, f32):
    batch = _batch(seed)
    ref = O.collate_fn(batch)
    got = D.collate_ragged(batch, f32=f32).to_device(dev)
    _same(got, ref)
    got_t = D.collate_ragged(batch, test=True).to_device(dev)
    assert got_t["gt_segments"] == [it["gt_segments"] for it in batch]


@pytest.mark.gpu
@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("lens", [(37, 80, 5, 64), (64, 64, 64)])
def test_device_collate_in_place(dev, pinned, lens, f32):
    """to_device(out=...): the batch written into existing tensors (a captured step's static inputs, poisoned
    first) equals the reference collate bit for bit — ragged lengths (fp32 rows copied per sequence by DMA
    and their padding filled) and full lengths (one DMA copy per fp32 modality); pinned or pageable rows."""
    batch = _batch(5, lens)
    ref = O.collate_fn(batch)
    rb = D.collate_ragged(batch, f32=f32)
    if pinned:
        rb = rb.pin()
    T = max(lens)
    out = {k: torch.full_like(v, float("nan"), device=dev) if v.is_floating_point() else torch.ones_like(v, device=dev)
           for k, v in ref.items() if torch.is_tensor(v)}
    keep = {k: v.data_ptr() for k, v in out.items()}
    got = rb.to_device(dev, out=out)
    _same(got, ref)
    for k, v in out.items():  # written in place
        assert got[k].data_ptr() == keep[k], k
    assert got["visual_feats"].shape == (len(lens), T, 512)
    with pytest.raises(ValueError, match="contiguous fp32"):
        rb.to_device(dev, out=dict(out, audio_feats=out["audio_feats"][:, :-1]))
