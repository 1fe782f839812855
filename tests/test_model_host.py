"""CPU tests of the drop-in host layer (no kernel launches): state_dict compatibility with the
reference layout, identical seeded initialisation, flat parameter storage, and the loud failure of
a CPU forward (the product has no CPU path)."""
import numpy as np
import pytest
import torch

from oracle.mmct_oracle import MMCTransformer as Oracle
from repurpose_amd.MMCTransformer import MMCTransformer

CFG = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=2, text_num_layers=3,
           cross_num_layers=3, num_heads=8)


def test_state_dict_keys_shapes_identical():
    a = Oracle(**CFG).state_dict()
    b = MMCTransformer(**CFG).state_dict()
    assert list(a.keys()) == list(b.keys())
    for k in a:
        assert a[k].shape == b[k].shape, k


def test_seeded_init_matches_reference_order():
    torch.manual_seed(1234)
    a = Oracle(**CFG).state_dict()
    torch.manual_seed(1234)
    b = MMCTransformer(**CFG).state_dict()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    # the RNG stream is left in the same state too
    torch.manual_seed(5)
    Oracle(**CFG)
    x = torch.rand(3)
    torch.manual_seed(5)
    MMCTransformer(**CFG)
    assert torch.equal(x, torch.rand(3))


def test_full_size_counts():
    m = MMCTransformer(**{**CFG, "self_num_layers": 16})
    assert sum(p.numel() for p in m.parameters()) == 52_608_771
    assert m.trainable_numel() >= 52_608_771 - 198_658


def test_flat_storage_views_and_checkpoint_roundtrip():
    m = MMCTransformer(**CFG)
    flat = m.flat_params()
    for n, p in m.named_parameters():
        o, shp = m._layout[n]
        assert p.data_ptr() == flat.data_ptr() + 4 * o and tuple(p.shape) == shp
        assert p.data_ptr() % 16 == 0
    ref = Oracle(**CFG)
    m.load_state_dict(ref.state_dict())
    assert m._flat_ok()
    for (n, p), (n2, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert n == n2 and torch.equal(p, q)
    # a checkpoint written by the drop-in loads into the reference layout
    ref.load_state_dict(m.state_dict())


def test_cpu_forward_fails_loudly():
    m = MMCTransformer(**{**CFG, "self_num_layers": 1})
    T = 8
    batch = {"visual_feats": torch.randn(1, T, 512), "audio_feats": torch.randn(1, T, 2048),
             "text_feats": torch.randn(1, T, 384), "masks": torch.ones(1, 1, T, dtype=torch.bool),
             "labels": torch.zeros(1, T), "segments": torch.zeros(1, T, 2)}
    with pytest.raises(RuntimeError, match="no CPU path"):
        m(batch)


def test_to_and_back_rebuilds_flat():
    m = MMCTransformer(**CFG)
    m.to(torch.float32)
    m.flat_params()
    assert m._flat_ok()
