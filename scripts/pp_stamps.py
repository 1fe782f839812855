"""Read the RP_PP_STAMPS diagnostic build's per-barrier s_memtime stamps of workgroup 0 (written over
lse) and print each wave's segment lengths (tuning aid, not product).
usage: RP_LIB_PATH=abtest/stamps/lib.so RP_ATTN_FWD_PP=1 python scripts/pp_stamps.py [--p 0.1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--p", type=float, default=0.0)
a = ap.parse_args()
dev = torch.device("cuda:0")
B, T, H, d = 8, 2048, 8, 512
g = torch.Generator(device="cpu").manual_seed(7)
qkv = torch.randn(B * T, 3 * d, generator=g).to(dev, torch.bfloat16)
kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
for rep in range(3):
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, a.p, 11, q_prescaled=True)
    torch.cuda.synchronize()
st = lse.reshape(-1).view(torch.int64)[:8 * 64].view(8, 64).cpu()
t0 = int(st[:, 0].min())
for w in range(8):
    row = [int(x) - t0 for x in st[w]]
    seg = [row[i + 1] - row[i] for i in range(min(40, len(row) - 1))]
    print(f"wave {w}: start {row[0]:6d}  segments {seg}")
