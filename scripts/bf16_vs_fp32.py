"""bf16 (bench mode) against fp32 (parity mode) training: the same init, the same fixed batches and
dropout off, N FusedAdam steps of the L=16 tri-modal model; reports the per-step focal loss of both
and their relative deviation (weak item 12 of the round-1 verdict: does bf16 training track fp32?).

python scripts/bf16_vs_fp32.py [--steps 40] [--T 1024] [--B 2] [--out profiles/r02_bf16_vs_fp32.json]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from repurpose_amd.MMCTransformer import MMCTransformer  # noqa: E402
from repurpose_amd.optim import FusedAdam  # noqa: E402


def run(dtype, batches, steps, lr):
    torch.manual_seed(1234)
    m = MMCTransformer(**bench.MODEL_CFG, compute_dtype=dtype).to(batches[0]["labels"].device).train()
    m.DROPOUT = 0.0
    opt = FusedAdam(m, lr=lr, weight_decay=1e-4)
    out = []
    for s in range(steps):
        b = batches[s % len(batches)]
        opt.zero_grad()
        o = m(b)
        loss = m.losses(*o)["cls_loss"] / b["labels"].shape[0]
        loss.backward()
        opt.step()
        out.append(loss.item())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--out", default="gpurun_out/bf16_vs_fp32.json")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    batches = [bench.synth_batch(a.B, a.T, dev, 500 + i) for i in range(4)]
    f32 = run("fp32", batches, a.steps, a.lr)
    b16 = run("bf16", batches, a.steps, a.lr)
    rel = [abs(x - y) / abs(x) for x, y in zip(f32, b16)]
    res = {"config": f"L=16 tri-modal, T={a.T}, B={a.B}, dropout off, FusedAdam lr {a.lr} wd 1e-4, "
                     f"4 fixed synthetic batches cycled, {a.steps} steps",
           "loss_fp32": f32, "loss_bf16": b16, "rel_dev": rel, "max_rel_dev": max(rel),
           "loss_drop_fp32": f32[0] - f32[-1], "loss_drop_bf16": b16[0] - b16[-1]}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if not isinstance(v, list)}))
    for s in range(0, a.steps, max(1, a.steps // 10)):
        print(f"step {s:3d}  fp32 {f32[s]:10.5f}  bf16 {b16[s]:10.5f}  rel {rel[s]:.2e}")


if __name__ == "__main__":
    main()
