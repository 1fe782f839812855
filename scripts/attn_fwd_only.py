"""Run the attention forward (bf16, metric shape, q prescaled) N times — a short program for rocprofv3 PMC
passes of one forward variant (select it with RP_ATTN_* switches).  Tuning aid, not product.
usage: python scripts/attn_fwd_only.py [--p 0.1] [--reps 4] [--bwd]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--p", type=float, default=0.1)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--B", type=int, default=8)
ap.add_argument("--T", type=int, default=2048)
ap.add_argument("--bwd", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
B, T, H, d = a.B, a.T, 8, 512
g = torch.Generator(device="cpu").manual_seed(7)
qkv = torch.randn(B * T, 3 * d, generator=g).to(dev, torch.bfloat16)
kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
do = torch.randn(B * T, d, generator=g).to(dev, torch.bfloat16)
olo = torch.empty(B * T, d, device=dev, dtype=torch.bfloat16)
for _ in range(a.reps):
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, a.p, 11, q_prescaled=True, out_lo=olo)
    if a.bwd:
        K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, a.p, dropmask=mask, q_prescaled=True, out_lo=olo)
torch.cuda.synchronize()
print("done")
