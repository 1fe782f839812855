"""Per-K-step cost vs fixed (prologue / epilogue / launch) cost of the forward GEMM kernels: time a plain
bf16 linear_fwd at M = 16384 over K for the step's N (2048: the 256 x 256 kernel; 1536 / 512: the
128 x 128 kernel), warm caches.  Tuning aid, not product.  usage: python scripts/gemm_ksweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M = 16384
    g = torch.Generator(device="cpu").manual_seed(0)
    for N in (2048, 1536, 512):
        for Kd in (128, 256, 512, 1024, 2048):
            x = (torch.randn(M, Kd, generator=g)).to(dev, torch.bfloat16)
            w = (torch.randn(N, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
            for f32 in (False, True):
                fn = lambda: K.linear_fwd(x, w, None, out_dtype=torch.float32 if f32 else None)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                ts = []
                for _ in range(9):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    fn()
                    e.record()
                    torch.cuda.synchronize()
                    ts.append(s.elapsed_time(e) * 1e3)
                t = sorted(ts)[4]
                print(f"N {N:5d} K {Kd:5d} out {'f32 ' if f32 else 'bf16'}: {t:7.1f} us  "
                      f"{2 * M * N * Kd / t / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
