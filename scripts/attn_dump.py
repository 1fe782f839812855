"""Dump the attention forward / backward outputs at a given shape to a .pt file, so that two kernel
variants selected by environment switches (RP_ATTN_*) can be compared bit for bit across processes.
usage: python scripts/attn_dump.py out.pt [--B 8 --T 2048 --p 0.1 --ragged]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=2048)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--ragged", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, T, H, d = a.B, a.T, 8, 512
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn(M, 3 * d, generator=g).to(dev, torch.bfloat16)
    kv = torch.ones(B, T, dtype=torch.uint8)
    if a.ragged:
        for b in range(B):
            kv[b, int(torch.randint(T // 2, T + 1, (1,), generator=g)):] = 0
    kv = kv.to(dev)
    do = torch.randn(M, d, generator=g).to(dev, torch.bfloat16)
    olo = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, a.p, 11, q_prescaled=True, out_lo=olo)
    dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, a.p, dropmask=mask, q_prescaled=True, out_lo=olo)
    torch.cuda.synchronize()
    torch.save({"o": o.cpu(), "lse": lse.cpu(), "dqkv": dqkv.cpu(),
                "mask": None if mask is None else mask.cpu()}, a.out)
    print("saved", a.out, {k: float(v.float().abs().sum()) for k, v in (("o", o), ("dqkv", dqkv))})


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--cmp":
        x, y = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        for k in x:
            if x[k] is None:
                continue
            same = torch.equal(x[k], y[k])
            diff = (x[k].float() - y[k].float()).abs().max().item()
            print(f"{k:6s} bitwise={same} maxdiff={diff:.3e}")
        sys.exit(0 if all(x[k] is None or torch.equal(x[k], y[k]) for k in x) else 1)
    main()
