"""The encoder layer's forward / dgrad GEMM shapes at M = 16384 (bf16 in, fp32 or bf16 out, no
epilogue): rp_gemm (K.linear_fwd / K.linear_dgrad) against torch.mm (hipBLASLt), 20 back-to-back
launches between two events, warm caches.  Tuning aid, not product.  usage: python scripts/gemm_vs_blas.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def t20(fn):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / 20)
    return best


def main():
    dev = torch.device("cuda:0")
    M = 16384
    g = torch.Generator(device="cpu").manual_seed(0)
    bf, f32 = torch.bfloat16, torch.float32
    r = lambda *s: torch.randn(*s, generator=g).to(dev, bf)  # noqa: E731
    for name, kind, n, k, odt in [("qkv fwd", "fwd", 1536, 512, bf), ("out_proj fwd", "fwd", 512, 512, f32),
                                  ("linear1 fwd", "fwd", 2048, 512, bf), ("linear2 fwd", "fwd", 512, 2048, f32),
                                  ("linear2 dgrad", "dgrad", 512, 2048, bf), ("linear1 dgrad", "dgrad", 2048, 512, f32),
                                  ("out_proj dgrad", "dgrad", 512, 512, bf), ("qkv dgrad", "dgrad", 1536, 512, f32)]:
        w = r(n, k) * 0.05
        if kind == "fwd":
            x = r(M, k)
            ours = lambda: K.linear_fwd(x, w, None, out_dtype=odt)  # noqa: E731
            wt = w.t()
            blas = lambda: torch.mm(x, wt, out_dtype=odt) if odt == f32 else torch.mm(x, wt)  # noqa: E731
        else:
            dy = r(M, n)
            ours = lambda: K.linear_dgrad(dy, w, out_dtype=odt)  # noqa: E731
            blas = lambda: torch.mm(dy, w, out_dtype=odt) if odt == f32 else torch.mm(dy, w)  # noqa: E731
        try:
            tb = t20(blas)
        except Exception as ex:  # out_dtype needs a recent torch
            tb = float("nan")
            print("  blas:", ex)
        to = t20(ours)
        fl = 2 * M * n * k
        print(f"{name:16s} ours {to:7.1f} us ({fl / to / 1e6:6.1f} TF/s)   torch.mm {tb:7.1f} us ({fl / tb / 1e6:6.1f} TF/s)",
              flush=True)


if __name__ == "__main__":
    main()
