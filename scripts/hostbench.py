"""Host-side enqueue cost of one training step vs its GPU time (is the step launch-bound?).
python scripts/hostbench.py [--steps K]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from repurpose_amd.MMCTransformer import MMCTransformer  # noqa: E402
from repurpose_amd.optim import FusedAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    model = MMCTransformer(**bench.MODEL_CFG, compute_dtype="bf16").to(dev).train()
    opt = FusedAdam(model, lr=1e-3, weight_decay=1e-4)
    batch = bench.synth_batch(8, 2048, dev, 1000)

    def step():
        opt.zero_grad()
        out = model(batch)
        loss = model.losses(*out)["cls_loss"] / 8
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    host, wall = [], []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    print("host enqueue ms/step", [round(x, 2) for x in host])
    print("wall ms/step (isolated)", [round(x, 2) for x in wall])
    # enqueue while the GPU is still busy with a long kernel: pure GPU time per step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    print("pipelined wall ms/step", round((time.perf_counter() - t0) * 1e3 / a.steps, 2))


if __name__ == "__main__":
    main()
