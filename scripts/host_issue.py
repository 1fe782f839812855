"""Host issue time vs GPU time of the bench training step (is the Python launch path the limit?).

python scripts/host_issue.py [--dtype bf16] : per phase host ms (no sync inside the step), then the
synchronized step time.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from repurpose_amd.MMCTransformer import MMCTransformer  # noqa: E402
from repurpose_amd.optim import FusedAdam  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(1234)
model = MMCTransformer(**bench.MODEL_CFG, compute_dtype="bf16").to(dev).train()
opt = FusedAdam(model, lr=1e-3, weight_decay=1e-4)
B, T = 8, 2048
batch = bench.synth_batch(B, T, dev, 1000)


def step(marks):
    t = time.perf_counter
    marks.append(t())
    opt.zero_grad()
    marks.append(t())
    out = model(batch)
    marks.append(t())
    loss = model.losses(*out)["cls_loss"] / B
    marks.append(t())
    loss.backward()
    marks.append(t())
    opt.step()
    marks.append(t())


for _ in range(3):
    step([])
torch.cuda.synchronize()
names = ["zero_grad", "forward", "losses", "backward", "opt.step"]
acc = [0.0] * 5
n = 5
t0 = time.perf_counter()
for _ in range(n):
    mk = []
    step(mk)
    for i in range(5):
        acc[i] += mk[i + 1] - mk[i]
host = time.perf_counter() - t0
torch.cuda.synchronize()
tot = time.perf_counter() - t0
print("host issue ms/step:", {k: round(v / n * 1e3, 3) for k, v in zip(names, acc)}, "sum", round(host / n * 1e3, 3))
print("synchronized ms/step:", round(tot / n * 1e3, 3))
