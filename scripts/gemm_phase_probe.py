"""Phase timing of the 128 x 128 LDS-DMA GEMM from the RP_GEMM_PROBE build (per-workgroup
s_memrealtime stamps: start, main loop done, epilogue issued, stores drained; 100 MHz).  Build the
probe library with -DRP_GEMM_PROBE on rp_gemm.hip and run with RP_LIB_PATH pointing at it.
Tuning aid, not product.  usage: RP_LIB_PATH=abl/probe.so python scripts/gemm_phase_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import _native as N  # noqa: E402
from repurpose_amd import kernels as K  # noqa: E402


def stamps(n):
    buf = (ctypes.c_uint64 * (4 * n))()
    rc = N.load().rp_debug_gemm_probe(buf, 4 * n)
    assert rc == 0, rc
    return np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)


def main():
    dev = torch.device("cuda:0")
    M, Nn = 16384, 512
    g = torch.Generator().manual_seed(0)
    res = torch.randn(M, Nn, generator=g).to(dev)
    b = torch.randn(Nn, generator=g).to(dev)
    for Kd in (64, 512, 2048):
        x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(Nn, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
        cases = {
            "bf16 out": lambda: K.linear_fwd(x, w, b, out_dtype=torch.bfloat16),
            "f32 out": lambda: K.linear_fwd(x, w, b, out_dtype=torch.float32),
            "f32 +res +drop": lambda: K.linear_fwd(x, w, b, out_dtype=torch.float32, dropout_p=0.1, seed=3,
                                                   residual=res),
        }
        for name, fn in cases.items():
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            nwg = (M // 128) * (Nn // 128)
            s = stamps(nwg) * 10 / 1000.0  # us
            t0 = s[:, 0] - s[:, 0].min()
            main_ = s[:, 1] - s[:, 0]
            epi = s[:, 2] - s[:, 1]
            drain = s[:, 3] - s[:, 2]
            span = s[:, 3].max() - s[:, 0].min()
            q = lambda a: f"{np.median(a):5.2f}/{a.max():5.2f}"  # noqa: E731
            print(f"K {Kd:5d} {name:15s} event {e0.elapsed_time(e1) * 1e3:6.1f} us  span {span:6.2f}  "
                  f"start spread med/max {q(t0)}  main {q(main_)}  epi-issue {q(epi)}  drain {q(drain)}",
                  flush=True)


if __name__ == "__main__":
    main()
