"""The captured training step (repurpose_amd/graph.py): a HIP-graph replay is the eager step.

* with dropout off, N replays give bitwise the parameters, moments and losses of N eager steps
  (same kernels; Adam reads the same coefficients from the device block), including new batches
  copied in with load() and an LR change between steps (LR schedulers keep working);
* with dropout on, every replay draws a fresh stream (device seed word rewritten per step), and two
  runners with the same seed reproduce each other bit for bit.
"""
import numpy as np
import pytest
import torch

from repurpose_amd.graph import CapturedTrainStep
from repurpose_amd.MMCTransformer import MMCTransformer
from repurpose_amd.optim import FusedAdam

from .test_model_gpu import TRI, make_batch, to_dev

pytestmark = pytest.mark.gpu


def _model(dev, dtype, dropout):
    torch.manual_seed(0)
    m = MMCTransformer(**TRI, compute_dtype=dtype).to(dev).train()
    m.DROPOUT = dropout
    return m, FusedAdam(m, lr=1e-3, weight_decay=1e-4)


def _batches(dev, n, B=2, T=192):
    return [{k: v for k, v in to_dev(make_batch(TRI, B, T, [T, 150], seed=20 + i), dev).items() if torch.is_tensor(v)}
            for i in range(n)]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_replay_equals_eager_without_dropout(dev, dtype):
    batches = _batches(dev, 5)
    me, oe = _model(dev, dtype, 0.0)
    eager_losses = []
    for i, b in enumerate(batches):
        if i == 3:
            oe.param_groups[0]["lr"] = 5e-4
        oe.zero_grad()
        out = me(b)
        loss = me.losses(*out)["cls_loss"] / 2
        loss.backward()
        oe.step()
        eager_losses.append(loss.item())

    mg, og = _model(dev, dtype, 0.0)
    static = {k: v.clone() for k, v in batches[0].items()}
    run = CapturedTrainStep(mg, og, static, warmup=1)
    graph_losses = []
    for i, b in enumerate(batches):
        if i == 3:
            og.param_groups[0]["lr"] = 5e-4
        run.load(b)
        graph_losses.append(run.step().item())
    torch.cuda.synchronize()
    assert run._graph is not None
    assert graph_losses == eager_losses
    n = me.trainable_numel()
    assert torch.equal(mg.flat_params()[:n], me.flat_params()[:n])
    assert torch.equal(og._m, oe._m) and torch.equal(og._v, oe._v)
    assert og._step == oe._step == 5
    if dtype == "bf16":
        assert torch.equal(mg._lp[:n], mg.flat_params()[:n].to(torch.bfloat16))
    # torch-Adam-layout state follows the replays
    assert float(og.state_dict()["state"][0]["step"]) == 5.0


def test_replays_draw_fresh_dropout_and_are_reproducible(dev):
    b = _batches(dev, 1)[0]

    def losses(seed, lr):
        m, o = _model(dev, "bf16", 0.1)
        o.param_groups[0]["lr"] = lr
        run = CapturedTrainStep(m, o, {k: v.clone() for k, v in b.items()}, warmup=1, seed=seed)
        out = [run.step().item() for _ in range(5)]
        torch.cuda.synchronize()
        return out, m.flat_params().clone()

    frozen, p0 = losses(7, 0.0)  # lr 0 (no weight decay effect: lr scales the whole update)
    # weights frozen: replays 2..5 differ only through their dropout streams
    assert len(set(frozen[1:])) == 4, frozen
    again, p1 = losses(7, 0.0)
    assert again == frozen and torch.equal(p0, p1)
    other, _ = losses(8, 0.0)
    assert other[1:] != frozen[1:]
    trained, _ = losses(7, 1e-3)
    assert all(np.isfinite(trained))


def test_eager_dropout_unaffected_by_a_live_capture(dev):
    """The graph-replayable dropout base is passed per launch (no process-wide library state): an
    eager model's dropout step gives bitwise the same loss and gradients whether or not another
    model's captured step exists in the process, including between that graph's replays."""
    b = _batches(dev, 1)[0]

    def eager(seed=123):
        m, _ = _model(dev, "bf16", 0.1)
        torch.manual_seed(seed)  # _Schedule draws its dropout base from the torch RNG
        out = m(b)
        loss = m.losses(*out)["cls_loss"] / 2
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), m.flat_grads().clone()

    l0, g0 = eager()
    mg, og = _model(dev, "bf16", 0.1)
    run = CapturedTrainStep(mg, og, {k: v.clone() for k, v in b.items()}, warmup=1, seed=5)
    run.step()
    run.step()  # captured and replayed: the graph's launches hold its device seed word
    assert run._graph is not None and mg._seed_base is None
    l1, g1 = eager()
    run.step()
    l2, g2 = eager()
    assert l1 == l0 and l2 == l0
    assert torch.equal(g1, g0) and torch.equal(g2, g0)
    # and a different torch seed does change the eager stream (the check has teeth)
    l3, _ = eager(seed=124)
    assert l3 != l0


def test_capture_requires_a_warmup_step(dev):
    m, o = _model(dev, "bf16", 0.0)
    with pytest.raises(ValueError, match="warmup"):
        CapturedTrainStep(m, o, _batches(dev, 1)[0], warmup=0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_captured_backward_writes_every_gradient(dev, dtype):
    """the captured step replaces zero_grad() by a backward that WRITES the gradients: poison every
    trained gradient view with NaN before the capture; the replays must still match eager steps
    bitwise (any gradient left to accumulate would carry the NaN into its parameters)"""
    batches = _batches(dev, 3)
    me, oe = _model(dev, dtype, 0.0)
    for b in batches:
        oe.zero_grad()
        out = me(b)
        (me.losses(*out)["cls_loss"] / 2).backward()
        oe.step()
    mg, og = _model(dev, dtype, 0.0)
    run = CapturedTrainStep(mg, og, {k: v.clone() for k, v in batches[0].items()}, warmup=1)
    run.load(batches[0])
    run.step()
    for p in mg.parameters():
        if p.grad is not None:
            p.grad.fill_(float("nan"))
    for b in batches[1:]:
        run.load(b)
        run.step()
    torch.cuda.synchronize()
    n = me.trainable_numel()
    assert torch.equal(mg.flat_params()[:n], me.flat_params()[:n])
    assert torch.equal(og._m, oe._m) and torch.equal(og._v, oe._v)
    assert not mg._grad_fresh


def test_replay_after_exchange_workspace_growth(dev, monkeypatch):
    """The seams on the exchange kernels (forced at this small shape) inside a captured step: after the
    capture a larger row count grows the device's exchange workspace (a new one is allocated; the one the
    graph holds stays alive) and an eager seam runs on the new one; the replays that follow still equal
    the eager steps bit for bit (a freed workspace under a live graph)."""
    from repurpose_amd import kernels as K

    monkeypatch.setenv("RP_GEMM_LN", "1")
    batches = _batches(dev, 4)
    me, oe = _model(dev, "bf16", 0.0)
    for b in batches:
        oe.zero_grad()
        out = me(b)
        (me.losses(*out)["cls_loss"] / 2).backward()
        oe.step()
    mg, og = _model(dev, "bf16", 0.0)
    run = CapturedTrainStep(mg, og, {k: v.clone() for k, v in batches[0].items()}, warmup=1)
    for i, b in enumerate(batches):
        run.load(b)
        run.step()
        if i == 1:
            held = K._LNX[dev][0].data_ptr()
            big = 2 * K._LNX[dev][1] + 64
            g = torch.Generator().manual_seed(3)
            x = torch.randn(big, 512, generator=g).to(dev, torch.bfloat16)
            W = (torch.randn(512, 512, generator=g) * 0.03).to(dev, torch.bfloat16)
            v = torch.zeros(512, device=dev)
            res = torch.randn(big, 512, generator=g).to(dev)
            K.linear_ln_fwd(x, W, v, res, v + 1.0, v)
            assert K._LNX[dev][0].data_ptr() != held
            assert any(w.data_ptr() == held for w in K._LNX_KEEP)
            del x, res
    torch.cuda.synchronize()
    n = me.trainable_numel()
    assert torch.equal(mg.flat_params()[:n], me.flat_params()[:n])
    K.lnx_status()


def test_two_input_sets_write_in_place_and_match_eager(dev):
    """CapturedTrainStep(input_sets=2): two graphs over two static input sets, alternating; each step's batch
    written into the free set through input_set(ahead=1) on a copy stream while the previous step runs
    (RaggedBatch.to_device(out=...), as bench.py's fresh-batch loop) — losses and parameters bitwise those
    of eager steps on the same batches (dropout off)."""
    from repurpose_amd import data as D

    from .test_data import _batch as items_batch

    cfg_items = [items_batch(30 + i, lens=(96, 96)) for i in range(5)]
    rbs = [D.collate_ragged(b).pin() for b in cfg_items]
    eager_batches = [{k: v for k, v in rb.to_device(dev).items() if torch.is_tensor(v)} for rb in rbs]
    torch.cuda.synchronize()
    me, oe = _model_items(dev)
    eager_losses = []
    for b in eager_batches:
        oe.zero_grad()
        out = me(b)
        loss = me.losses(*out)["cls_loss"] / 2
        loss.backward()
        oe.step()
        eager_losses.append(loss.item())

    mg, og = _model_items(dev)
    run = CapturedTrainStep(mg, og, {k: v.clone() for k, v in eager_batches[0].items()}, warmup=1, input_sets=2)
    copy = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)
    losses = []

    def stage(j, done):
        with torch.cuda.stream(copy):
            dst, used = run.input_set(ahead=j - done)
            if used is not None:
                copy.wait_event(used)
            rbs[j].to_device(dev, out=dst)
            ev = torch.cuda.Event()
            ev.record(copy)
        return ev

    ev = stage(0, 0)
    for j in range(len(rbs)):
        nxt = stage(j + 1, j) if j + 1 < len(rbs) else None
        main.wait_event(ev)
        losses.append(run.step().item())
        ev = nxt
    torch.cuda.synchronize()
    assert run._graphs[0] is not None and run._graphs[1] is not None
    assert losses == eager_losses
    n = me.trainable_numel()
    assert torch.equal(mg.flat_params()[:n], me.flat_params()[:n])


def _model_items(dev):
    torch.manual_seed(0)
    cfg = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=2, text_num_layers=3,
               cross_num_layers=3, num_heads=8)
    m = MMCTransformer(**cfg, compute_dtype="bf16").to(dev).train()
    m.DROPOUT = 0.0
    return m, FusedAdam(m, lr=1e-3, weight_decay=1e-4)
