"""World-size-2 gloo tests (CPU) of the distributed layer: MultiGPUStrategy API semantics and the
bucketed, range-driven gradient all-reducer used by the HIP backward."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeModel:
    """Exposes the flat-gradient interface of MMCTransformer."""

    def __init__(self, n, trainable):
        self.g = torch.zeros(n)
        self.n = trainable
        self._grad_ready_hooks = []
        self._grad_done_hooks = []

    def flat_grads(self):
        return self.g

    def trainable_numel(self):
        return self.n


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from repurpose_amd.distributed import GradAllReducer, MultiGPUStrategy, get_rank, get_world_size
        from repurpose_amd.metrics import gather_precisions
        # no GPU here: 'auto' resolves to single exactly as the reference (:281-282), so ask for ddp
        assert MultiGPUStrategy(strategy="auto", backend="gloo").strategy == "single"
        s = MultiGPUStrategy(strategy="ddp", backend="gloo", timeout=60)
        assert s.strategy == "ddp" and s.world_size == world and s.rank == rank
        assert s.setup() is True
        assert get_rank() == rank and get_world_size() == world
        t = s.reduce_tensor(torch.tensor([float(rank + 1)]))
        assert abs(t.item() - (1 + world) / 2) < 1e-6
        assert s.reduce_tensor(torch.tensor([1.0]), average=False).item() == world
        assert s.get_effective_batch_size(6) == 6 * world
        s.barrier()
        # DistributedSampler partitioning (utils/distributed.py:453-461): the index list (a seed 0 +
        # epoch permutation when shuffling), padded with its own head to a multiple of world, then
        # rank r takes positions r, r + world, ...
        for shuffle, epoch in ((False, 0), (True, 0), (True, 3)):
            dl = s.create_dataloader(list(range(11)), batch_size=2, shuffle=shuffle)
            dl.sampler.set_epoch(epoch)
            seen = [int(x) for b in dl for x in b]
            if shuffle:
                gen = torch.Generator()
                gen.manual_seed(0 + epoch)
                order = torch.randperm(11, generator=gen).tolist()
            else:
                order = list(range(11))
            order = order + order[:12 - 11]
            assert seen == order[rank::world], (shuffle, epoch, seen)
        # evaluate_tiou's cross-rank gather: 3 videos over 2 ranks -> rank 1's shard repeats video 0
        ids = ["a", "c"] if rank == 0 else ["b", "a"]
        prec = torch.tensor([[0.5, 0.25], [1.0, 0.0]]) if rank == 0 else torch.tensor([[0.0, 0.0], [0.5, 0.25]])
        allp = gather_precisions(prec)
        assert allp.shape == (4, 2)
        uniq = gather_precisions(prec, ids)
        assert torch.equal(uniq, torch.tensor([[0.5, 0.25], [1.0, 0.0], [0.0, 0.0]], dtype=torch.float64))
        # gradient reducer: ranges arrive in reverse order, buckets of 8 elements
        m = FakeModel(40, 36)
        r = GradAllReducer(m, bucket_mb=8 * 4 / 2 ** 20)
        m.g.copy_(torch.arange(40, dtype=torch.float32) * (rank + 1))
        for lo, hi in [(32, 40), (24, 32), (20, 24), (8, 20), (0, 8)]:
            for h in m._grad_ready_hooks:
                h(lo, hi)
        for h in m._grad_done_hooks:
            h()
        exp = torch.arange(40, dtype=torch.float32) * (1 + world) / 2
        assert torch.allclose(m.g[:36], exp[:36])
        assert torch.equal(m.g[36:], torch.arange(36, 40, dtype=torch.float32) * (rank + 1))  # untrained
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_strategy_and_reducer_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, msg in res:
        assert msg == "ok", f"rank {rank}: {msg}"


def test_detect_slurm_env_reference_priority(monkeypatch):
    """utils/distributed.py:32-74: torchrun wins over SLURM; SLURM needs NTASKS > 1; master from the
    first node of SLURM_STEP_NODELIST (compressed form too), else SLURM_LAUNCH_NODE_IPADDR / localhost."""
    from repurpose_amd.distributed import detect_slurm_env
    for k in ("RANK", "WORLD_SIZE", "SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID", "SLURM_STEP_NODELIST",
              "SLURM_LAUNCH_NODE_IPADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    assert detect_slurm_env() == {"is_slurm": False}
    monkeypatch.setenv("SLURM_PROCID", "3")
    monkeypatch.setenv("SLURM_NTASKS", "1")
    assert detect_slurm_env()["is_slurm"] is False  # a one-task allocation is not distributed
    monkeypatch.setenv("SLURM_NTASKS", "8")
    monkeypatch.setenv("SLURM_LOCALID", "1")
    info = detect_slurm_env()
    assert info == {"is_slurm": True, "rank": 3, "world_size": 8, "local_rank": 1, "master_addr": "localhost",
                    "master_port": 29500}
    monkeypatch.setenv("SLURM_LAUNCH_NODE_IPADDR", "10.0.0.7")
    assert detect_slurm_env()["master_addr"] == "10.0.0.7"
    monkeypatch.setenv("SLURM_STEP_NODELIST", "gpu[01-04]")
    monkeypatch.setenv("MASTER_PORT", "1234")
    info = detect_slurm_env()
    assert info["master_addr"] == "gpu01" and info["master_port"] == 1234
    monkeypatch.setenv("SLURM_STEP_NODELIST", "nodeA,nodeB")
    assert detect_slurm_env()["master_addr"] == "nodeA"
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert detect_slurm_env() == {"is_slurm": False}  # torchrun's variables take priority


def test_dp_strategy_one_process(monkeypatch):
    """'dp' (nn.DataParallel in the reference, utils/distributed.py:409-413): one process, world 1;
    wrap_model returns a DataParallelModel only with more than one GPU (the reference's condition,
    :409), otherwise the model itself (here: no GPU)."""
    from repurpose_amd.distributed import MultiGPUStrategy
    s = MultiGPUStrategy(strategy="dp")
    assert s.strategy == "dp" and s.world_size == 1 and not s.is_distributed
    assert s.get_effective_batch_size(4) == 4  # reference :604, the whole batch on each step
    m = torch.nn.Linear(2, 2)
    assert s.wrap_model(m) is m


def test_ddp_setup_failure_falls_back_to_dp(monkeypatch, caplog):
    """Reference utils/distributed.py:379-386: a failed DDP init falls back to DataParallel, world 1,
    and setup() still reports success."""
    import repurpose_amd.distributed as D
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(D, "setup_distributed", lambda *a, **k: False)
    s = D.MultiGPUStrategy(strategy="ddp", backend="gloo")
    with caplog.at_level("WARNING"):
        assert s.setup() is True
    assert s.strategy == "dp" and s.world_size == 1 and s.rank == 0 and not s.is_distributed
    assert any("falling back to DataParallel" in r.getMessage() for r in caplog.records)


def test_dp_batch_split_like_scatter():
    """DataParallelModel's batch cut: torch.chunk along dim 0 (nn.DataParallel's scatter) — ceil-sized
    pieces, fewer pieces than devices when the batch is short, non-tensor values shared."""
    from repurpose_amd.distributed import _split_batch
    b = {"x": torch.arange(5 * 3).view(5, 3), "m": torch.ones(5, 1, 4, dtype=torch.bool), "tag": "v"}
    pieces = _split_batch(b, 2)
    assert [p["x"].shape[0] for p in pieces] == [3, 2]
    assert torch.equal(torch.cat([p["x"] for p in pieces]), b["x"]) and all(p["tag"] == "v" for p in pieces)
    assert [p["m"].shape[0] for p in _split_batch(b, 8)] == [1] * 5
    assert [p["x"].shape[0] for p in _split_batch(b, 4)] == [c.shape[0] for c in torch.chunk(b["x"], 4)]
    with pytest.raises(ValueError):
        _split_batch({"x": torch.zeros(2, 1), "y": torch.zeros(3, 1)}, 2)


def test_single_strategy_passthrough():
    from repurpose_amd.distributed import MultiGPUStrategy
    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    s = MultiGPUStrategy(strategy="single")
    assert s.setup() and s.world_size == 1
    x = torch.tensor([3.0])
    assert s.reduce_tensor(x) is x
    m = torch.nn.Linear(2, 2)
    assert s.wrap_model(m) is m
