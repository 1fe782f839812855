"""Is the DP step host-bound?  One rank over RCCL (env: RANK=0 WORLD_SIZE=1 MASTER_ADDR/PORT), the
bench's eager DP step: host time to issue N steps without synchronising vs the GPU time of the same
N steps; and the host cost of an async all_reduce + wait() queued behind a long GPU kernel.
    python scripts/dp_host.py"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import MODEL_CFG, synth_batch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from repurpose_amd.distributed import GradAllReducer
    from repurpose_amd.MMCTransformer import MMCTransformer
    from repurpose_amd.optim import FusedAdam
    # 1. all_reduce + wait behind a long kernel
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    g = torch.zeros(52 * 2 ** 20, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        a @ a
    t1 = time.perf_counter()
    w = dist.all_reduce(g[: 6 * 2 ** 20], op=dist.ReduceOp.AVG, async_op=True)
    t2 = time.perf_counter()
    w.wait()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"matmuls issue {1e3 * (t1 - t0):.2f} ms, all_reduce issue {1e3 * (t2 - t1):.2f} ms, "
          f"wait {1e3 * (t3 - t2):.2f} ms, drain {1e3 * (t4 - t3):.2f} ms", flush=True)
    # 2. the DP step
    torch.manual_seed(1234)
    model = MMCTransformer(**MODEL_CFG, compute_dtype="bf16").to(dev).train()
    opt = FusedAdam(model, lr=1e-3, weight_decay=1e-4)
    red = GradAllReducer(model)
    B, T = 8, 2048
    batch = synth_batch(B, T, dev, 1000)

    def step():
        opt.zero_grad()
        out = model(batch)
        (model.losses(*out)["cls_loss"] / B).backward()
        red.wait()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for n in (1, 10):
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{n} DP steps: host issue {1e3 * (t1 - t0) / n:.2f} ms/step, GPU {1e3 * (t2 - t0) / n:.2f} ms/step",
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
