"""Time the attention backward at the bench shape (B = 8, T = 2048, H = 8, dropout 0.1, prescaled Q)
under the RP_ATTN_* tuning variables of the environment.  Tuning aid, not product.
usage: python scripts/attn_bwd_time.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    B, T, H, p = 8, 2048, 8, 0.1
    g = torch.Generator(device="cpu").manual_seed(1)
    qkv = torch.randn(B * T, 3 * H * 64, generator=g).to(dev).to(torch.bfloat16)
    c = 0.125 * K.LOG2E
    qkv[:, :H * 64] = (qkv[:, :H * 64].float() * c).to(torch.bfloat16)
    kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
    olo = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 5, q_prescaled=True, out_lo=olo)
    do = torch.randn(B * T, H * 64, generator=g).to(dev).to(torch.bfloat16)
    for _ in range(3):
        K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo)
    e1.record()
    torch.cuda.synchronize()
    env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("RP_ATTN"))
    print(f"attn_bwd [{env}]: {e0.elapsed_time(e1) / it * 1e3:.1f} us/call")


if __name__ == "__main__":
    main()
