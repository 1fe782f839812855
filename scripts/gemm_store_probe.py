"""Where does the short-K GEMM's fixed cost go?  linear_fwd at M = 16384, K = 128 (two K-tiles: the
time is prologue + epilogue) with the output row stride padded (HBM channel pattern of the stores),
beside a plain torch fill of the same output bytes.  Tuning aid, not product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def timeit(fn, reps=9):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return sorted(ts)[reps // 2]


def main():
    dev = torch.device("cuda:0")
    M = 16384
    g = torch.Generator(device="cpu").manual_seed(0)
    for N, Kd in ((2048, 128), (2048, 512), (512, 128), (1536, 128)):
        x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
        for pad in (0, 64, 128, 256):
            buf = torch.empty(M, N + pad, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: K.gemm(x, w, buf, M, N, Kd, Kd, True, Kd, True, N + pad))
            print(f"N {N} K {Kd} ldc {N + pad}: {t:7.1f} us", flush=True)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: out.fill_(1.0))
        print(f"N {N}: torch fill of the output ({M * N * 2 / 1e6:.1f} MB) {t:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
