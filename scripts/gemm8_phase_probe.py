"""Phase timing of the 256-row phased GEMM (gemm8) from the RP_GEMM_PROBE build: per-workgroup
s_memrealtime stamps (start, main loop done, epilogue issued, stores drained; 100 MHz) for the d_ff =
2048 shapes of the step (linear1 forward with ReLU + dropout, linear2 dgrad with the gate), and the
workgroup start times by round.  Tuning aid, not product.
usage: RP_LIB_PATH=abl/probe.so python scripts/gemm8_phase_probe.py"""
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
    assert N.load().rp_debug_gemm_probe(buf, 4 * n) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)


def main():
    dev = torch.device("cuda:0")
    M, D, F = 16384, 512, 2048
    g = torch.Generator().manual_seed(0)
    h = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
    w1 = (torch.randn(F, D, generator=g) * 0.03).to(dev, torch.bfloat16)
    b1 = torch.randn(F, generator=g).to(dev) * 0.1
    dz = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
    w2 = (torch.randn(D, F, generator=g) * 0.03).to(dev, torch.bfloat16)
    f = K.linear_fwd(h, w1, b1, relu=True, dropout_p=0.1, seed=3)
    cases = {
        "linear1 fwd relu+drop": lambda: K.linear_fwd(h, w1, b1, relu=True, dropout_p=0.1, seed=3),
        "linear1 fwd plain bf16": lambda: K.linear_fwd(h, w1, b1),
        "linear2 dgrad gated": lambda: K.linear_dgrad(dz, w2, out_dtype=torch.bfloat16, gate=f, gate_scale=1.1),
        "linear2 dgrad plain": lambda: K.linear_dgrad(dz, w2, out_dtype=torch.bfloat16),
    }
    nwg = (M // 256) * (F // 256)
    for name, fn in cases.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        s = stamps(nwg) * 10 / 1000.0  # us
        t0 = s[:, 0] - s[:, 0].min()
        main_ = s[:, 1] - s[:, 0]
        epi = s[:, 2] - s[:, 1]
        drain = s[:, 3] - s[:, 2]
        span = s[:, 3].max() - s[:, 0].min()
        order = np.argsort(t0)
        r1, r2 = order[:nwg // 2], order[nwg // 2:]
        q = lambda a: f"{np.median(a):5.2f}/{a.max():5.2f}"  # noqa: E731
        print(f"{name:24s} event {e0.elapsed_time(e1) * 1e3:6.1f} us  span {span:6.2f}  main {q(main_)}  "
              f"epi {q(epi)}  drain {q(drain)}  round-2 start med {np.median(t0[r2]):5.2f} (first {t0[r2].min():5.2f})  "
              f"round-1 end med {np.median((s[r1, 3] - s[:, 0].min())):5.2f}", flush=True)


if __name__ == "__main__":
    main()
