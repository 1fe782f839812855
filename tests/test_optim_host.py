"""CPU tests of FusedAdam's drop-in surface (no kernel launches): the constructor forms the
reference trainer uses (``optim.Adam(model.parameters(), lr, weight_decay)``, main.py:190-191, also
through the wrap_model wrapper), and checkpoint compatibility of ``state_dict`` /
``load_state_dict`` with torch.optim.Adam's layout (main.py:222, :521, :729)."""
import pytest
import torch

from oracle.mmct_oracle import MMCTransformer as Oracle
from repurpose_amd.MMCTransformer import MMCTransformer, owner_of
from repurpose_amd.optim import FusedAdam

CFG = dict(vis_dim=64, aud_dim=32, text_dim=16, d_model=64, self_num_layers=2, text_num_layers=3,
           cross_num_layers=3, num_heads=1, d_ff=128)


class Wrapper(torch.nn.Module):  # what MultiGPUStrategy.wrap_model returns under DDP: .module
    def __init__(self, m):
        super().__init__()
        self.module = m


def test_constructor_forms():
    m = MMCTransformer(**CFG)
    assert owner_of(next(m.parameters())) is m
    for arg in (m, m.parameters(), Wrapper(m), Wrapper(m).parameters(), list(m.parameters())):
        opt = FusedAdam(arg, lr=1e-3, weight_decay=1e-4)
        assert opt.model is m
        assert len(opt.param_groups) == 1
        assert [id(p) for p in opt.param_groups[0]["params"]] == [id(p) for p in m.parameters()]
    with pytest.raises(ValueError):
        FusedAdam(torch.nn.Linear(2, 2).parameters())
    with pytest.raises(ValueError):
        FusedAdam(torch.nn.Linear(2, 2))
    with pytest.raises(ValueError):
        FusedAdam([{"params": list(m.parameters())}])


def _torch_adam_after_steps(ref, steps=3):
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        for n, p in ref.named_parameters():
            p.grad = None if n.startswith("reg_head.") else torch.randn(p.shape, generator=g)
        opt.step()
    return opt


def test_loads_reference_adam_checkpoint_and_saves_the_same_layout():
    torch.manual_seed(0)
    ref = Oracle(**CFG)
    topt = _torch_adam_after_steps(ref)
    sd = topt.state_dict()
    m = MMCTransformer(**CFG)
    m.load_state_dict(ref.state_dict())
    opt = FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-4)
    opt.load_state_dict(sd)
    assert opt._step == 3
    # the flat moment buffers hold the reference's per-parameter moments
    names = [n for n, _ in m.named_parameters()]
    for i, n in enumerate(names):
        if n.startswith("reg_head."):
            assert i not in sd["state"]
            continue
        o, _ = m._layout[n]
        k = sd["state"][i]["exp_avg"].numel()
        assert torch.equal(opt._m[o:o + k], sd["state"][i]["exp_avg"].reshape(-1)), n
        assert torch.equal(opt._v[o:o + k], sd["state"][i]["exp_avg_sq"].reshape(-1)), n
    # ...and state_dict() gives torch Adam's layout back: it loads into torch Adam unchanged
    out = opt.state_dict()
    assert sorted(out["state"]) == sorted(sd["state"])
    assert len(out["param_groups"][0]["params"]) == len(sd["param_groups"][0]["params"])
    topt2 = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    topt2.load_state_dict(out)
    for i, st in sd["state"].items():
        st2 = topt2.state_dict()["state"][i]
        assert float(st2["step"]) == float(st["step"])
        assert torch.equal(st2["exp_avg"], st["exp_avg"]) and torch.equal(st2["exp_avg_sq"], st["exp_avg_sq"])


def test_state_dict_resumes_in_torch_adam_through_a_checkpoint_file(tmp_path):
    """A FusedAdam checkpoint saved with torch.save and resumed by torch.optim.Adam (the reference
    trainer, main.py:222) steps every parameter from step 3 to 4 — no step tensor is shared — and does
    not alias FusedAdam's live moment buffers."""
    torch.manual_seed(0)
    ref = Oracle(**CFG)
    sd = _torch_adam_after_steps(ref).state_dict()
    m = MMCTransformer(**CFG)
    m.load_state_dict(ref.state_dict())
    opt = FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-4)
    opt.load_state_dict(sd)
    out = opt.state_dict()
    steps = [st["step"] for st in out["state"].values()]
    assert len({id(t) for t in steps}) == len(steps)
    f = tmp_path / "ckpt.pth"
    torch.save({"optimizer": out}, f)
    loaded = torch.load(f, weights_only=True)["optimizer"]
    topt2 = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    topt2.load_state_dict(loaded)
    for n, p in ref.named_parameters():
        p.grad = None if n.startswith("reg_head.") else torch.ones_like(p)
    before = opt._m.clone()
    topt2.step()
    for i, st in topt2.state_dict()["state"].items():
        assert float(st["step"]) == 4.0, i
    assert torch.equal(opt._m, before)  # the resumed torch Adam wrote its own copies
    # and the dict FusedAdam hands out is a snapshot, not a view of its flat buffers
    k = next(iter(out["state"]))
    out["state"][k]["exp_avg"].add_(1.0)
    assert torch.equal(opt._m, before)


def test_fresh_state_dict_matches_torch_adam_layout():
    m = MMCTransformer(**CFG)
    ref = Oracle(**CFG)
    a = FusedAdam(m, lr=2e-3, weight_decay=1e-4).state_dict()
    b = torch.optim.Adam(ref.parameters(), lr=2e-3, weight_decay=1e-4).state_dict()
    assert a["state"] == {} and b["state"] == {}
    assert a["param_groups"][0]["params"] == b["param_groups"][0]["params"]
    for k in ("lr", "betas", "eps", "weight_decay", "amsgrad", "maximize"):
        assert a["param_groups"][0][k] == b["param_groups"][0][k], k


def test_lowp_version_key_sees_parameter_updates():
    """In-place updates through the Parameters (torch Adam, load_state_dict's copy_) move only the
    Parameters' own version counters (p.data = view); the bf16 copy's key must see them."""
    m = MMCTransformer(**CFG)
    k0 = m._master_version()
    p = next(m.parameters())
    with torch.no_grad():
        p.add_(1.0)
    assert m._master_version() != k0
    k1 = m._master_version()
    m.load_state_dict(m.state_dict())
    assert m._master_version() != k1
