"""How much of the fp32-residual forward GEMMs (out_proj / linear2 forward: y = dropout(x W^T + b) +
residual, fp32 out) is epilogue: the same launch over K = 64 .. 2048 at M = 16384, N = 512, with and
without the residual / dropout, beside a plain 64 MB device copy (the epilogue's HBM bytes).  Run it
under `rocprofv3 --kernel-trace --stats` for kernel durations.  Tuning aid, not product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M, N = 16384, 512
    g = torch.Generator().manual_seed(0)
    res = torch.randn(M, N, generator=g).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    src = torch.randn(M, 2 * N, generator=g).to(dev)
    dst = torch.empty_like(src)
    for Kd in (64, 512, 2048):
        x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
        for _ in range(20):
            K.linear_fwd(x, w, b, out_dtype=torch.float32, dropout_p=0.1, seed=3, residual=res)  # full epilogue
            K.linear_fwd(x, w, b, out_dtype=torch.float32)  # fp32 out only
            K.linear_fwd(x, w, b, out_dtype=torch.bfloat16)  # bf16 out
    for _ in range(20):
        dst.copy_(src)  # 64 MB read + 64 MB write
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
