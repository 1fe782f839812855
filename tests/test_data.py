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


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 3])
def test_device_collate_matches_reference(dev, seed):
    batch = _batch(seed)
    ref = O.collate_fn(batch)
    got = D.collate_ragged(batch).to_device(dev)
    _same(got, ref)
    got_t = D.collate_ragged(batch, test=True).to_device(dev)
    assert got_t["gt_segments"] == [it["gt_segments"] for it in batch]
