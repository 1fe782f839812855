"""The real data-parallel path on the GPU, two ranks: MultiGPUStrategy.setup() / wrap_model(), the
HIP backward's flat-range hooks driving GradAllReducer's bucketed all-reduce, FusedAdam on the
wrapper.  Reference semantics (utils/distributed.py:396-433 DDP around main.py:331-369): after
``loss.backward()`` every rank holds the mean over ranks of its local gradient of
``cls_loss / batch_size``, and the parameters were broadcast from rank 0 at wrap time.

Both ranks share the box's one GPU, so the rehearsal uses the gloo backend (RCCL refuses two ranks
on one device); the driver's 8-GPU bench runs the same code over RCCL (backend "nccl")."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=2, text_num_layers=3,
           cross_num_layers=3, num_heads=8)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(seed=5):
    g = torch.Generator().manual_seed(seed)
    B, T, lens = 2, 128, [128, 70]
    return {"visual_feats": torch.randn(B, T, 512, generator=g), "audio_feats": torch.relu(torch.randn(B, T, 2048, generator=g)),
            "text_feats": torch.randn(B, T, 384, generator=g),
            "masks": (torch.arange(T)[None] < torch.tensor(lens)[:, None]).unsqueeze(1),
            "labels": (torch.rand(B, T, generator=g) < 0.35).float(), "segments": torch.rand(B, T, 2, generator=g) * 10}


def _worker(rank, world, port, q, dtype="fp32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import torch.distributed as dist
        from repurpose_amd.distributed import DistributedModel, MultiGPUStrategy
        from repurpose_amd.MMCTransformer import MMCTransformer
        from repurpose_amd.optim import FusedAdam

        s = MultiGPUStrategy(strategy="auto", backend="gloo", timeout=60)
        assert s.strategy == "ddp" and s.world_size == world and s.rank == rank, (s.strategy, s.world_size)
        assert s.setup() is True
        dev = s.device
        assert dev.type == "cuda"

        def fresh(seed):
            torch.manual_seed(seed)
            # bf16: 9 layers, so the deferred grouped weight gradients flush once mid-backward (8
            # layers) and once at the end, each flush announcing its layers' ranges to the reducer
            cfg = CFG if dtype == "fp32" else dict(CFG, self_num_layers=9)
            m = MMCTransformer(**cfg, compute_dtype=dtype)
            m.DROPOUT = 0.0  # dropout off: the per-rank gradients are comparable bit for bit
            return m

        m = fresh(100 + rank)  # different init per rank: the wrap must broadcast rank 0's
        w = s.wrap_model(m)
        assert isinstance(w, DistributedModel) and w.module is m
        init0 = fresh(100).flat_params().clone()
        assert torch.equal(m.flat_params().cpu(), init0), "parameters not broadcast from rank 0"
        opt = FusedAdam(w.parameters(), lr=1e-3, weight_decay=1e-4)

        full = _batch()
        mine = {k: v[rank:rank + 1].to(dev) for k, v in full.items()}  # one sequence per rank
        w.train()
        opt.zero_grad()
        out = w(mine)
        loss = w.module.losses(*out)["cls_loss"] / 1  # main.py:331 (batch_size = 1 per rank)
        loss.backward()
        torch.cuda.synchronize()
        g_ddp = m.flat_grads().clone()

        # single-process DDP average: mean over ranks of each rank's local gradient
        ref = fresh(0)
        ref.load_state_dict(m.state_dict())
        ref.to(dev).train()
        acc = None
        for r in range(world):
            ref.zero_grad(set_to_none=True)
            o = ref({k: v[r:r + 1].to(dev) for k, v in full.items()})
            ref.losses(*o)["cls_loss"].backward()
            g = ref.flat_grads().clone()
            acc = g if acc is None else acc + g
        want = acc / world
        n = m.trainable_numel()
        rel = ((g_ddp[:n] - want[:n]).abs().max() / want[:n].abs().max()).item()
        assert rel < 1e-5, f"DDP gradient differs from the mean of per-rank gradients: rel {rel:.2e}"
        assert torch.equal(g_ddp[n:], torch.zeros_like(g_ddp[n:]))  # reg_head: no gradient anywhere

        # the averaged loss (main.py:378-380) and identical parameters on every rank after Adam
        avg = s.reduce_tensor(loss.detach())
        both = torch.zeros(world, device=dev)
        both[rank] = loss.detach()
        dist.all_reduce(both)
        assert abs(avg.item() - both.mean().item()) < 1e-5 * max(1.0, abs(avg.item()))
        opt.step()
        torch.cuda.synchronize()
        mine_p = m.flat_params().clone()
        rank0_p = mine_p.clone()
        dist.broadcast(rank0_p, src=0)
        assert torch.equal(mine_p, rank0_p), "ranks diverged after the optimizer step"
        s.barrier()
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_ddp_two_ranks_real_backward(dev, dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, dtype)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    bad = [f"rank {rank}: {msg}" for rank, msg in sorted(res) if msg != "ok"]
    assert not bad, "\n".join(bad)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_dp_strategy_replicas_sum_to_whole_batch(dev, dtype):
    """``strategy: dp`` (reference utils/distributed.py:409-413, nn.DataParallel): DataParallelModel
    cuts the batch along dim 0, runs one replica per device entry and gathers the outputs, so the
    trainer's ``model.module.losses(*out)`` / ``backward()`` give the whole batch's loss and gradient.
    Two replicas share the box's one GPU (device_ids [0, 0]); checked against the plain model on the
    whole batch over two optimizer steps (replica parameters refreshed, replica gradients re-zeroed)."""
    from repurpose_amd.distributed import DataParallelModel
    from repurpose_amd.MMCTransformer import MMCTransformer
    from repurpose_amd.optim import FusedAdam
    torch.manual_seed(7)
    ref = MMCTransformer(**CFG, compute_dtype=dtype).to(dev).train()
    ref.DROPOUT = 0.0
    m = MMCTransformer(**CFG, compute_dtype=dtype)
    m.load_state_dict(ref.state_dict())
    m.DROPOUT = 0.0
    w = DataParallelModel(m, device_ids=[0, 0])
    w.train()
    opt_ref = FusedAdam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    opt = FusedAdam(w.parameters(), lr=1e-3, weight_decay=1e-4)
    g = torch.Generator().manual_seed(11)
    B, T = 3, 128  # odd: pieces of 2 and 1 sequences
    n = m.trainable_numel()
    for step in range(2):
        full = _batch(seed=20 + step)
        full = {k: torch.cat([v, v[:1]]) for k, v in full.items()}  # B = 3
        full["visual_feats"][2] += 0.1 * torch.randn(T, 512, generator=g)
        batch = {k: v.to(dev) for k, v in full.items()}
        opt_ref.zero_grad()
        o_ref = ref(batch)
        l_ref = ref.losses(*o_ref)["cls_loss"] / B
        l_ref.backward()
        opt.zero_grad()
        out = w(batch)
        assert len(out) == 6 and out[1].shape == o_ref[1].shape and out[1].device == dev
        loss = w.module.losses(*out)["cls_loss"] / B
        loss.backward()
        torch.cuda.synchronize()
        tol = 1e-5 if dtype == "fp32" else 2e-2
        assert abs(loss.item() - l_ref.item()) <= tol * max(1.0, abs(l_ref.item())), (loss.item(), l_ref.item())
        ga, gb = m.flat_grads()[:n], ref.flat_grads()[:n]
        rel = ((ga - gb).abs().max() / gb.abs().max()).item()
        assert rel < (1e-5 if dtype == "fp32" else 3e-2), f"step {step}: dp gradient rel err {rel:.2e}"
        opt.step()
        opt_ref.step()
    torch.cuda.synchronize()
    # Adam moves a parameter by up to lr per step whatever its gradient's size, so near-zero gradients
    # whose sign differs between the two summation orders move apart by up to 2 lr per step; the
    # replica refresh itself is what the second step's gradient check above covers
    drift = (m.flat_params() - ref.flat_params()).abs().max().item()
    assert drift <= 4 * 1e-3 * 1.01, drift
