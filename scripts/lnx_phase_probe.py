"""Phase timing of the exchange GEMM + LayerNorm kernels from the RP_GEMM_PROBE build: per-workgroup
s_memrealtime stamps (start, main loop done, payload stored, arrived, partners seen, end after the
stores drained; 100 MHz) at the bench shape.  Tuning aid, not product.
usage: RP_LIB_PATH=abl/probe.so python scripts/lnx_phase_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import _native as N  # noqa: E402
from repurpose_amd import kernels as K  # noqa: E402


def stamps(n):
    buf = (ctypes.c_uint64 * (8 * n))()
    assert N.load().rp_debug_lnx_probe(buf, 8 * n) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)


def main():
    dev = torch.device("cuda:0")
    M, D = 16384, 512
    g = torch.Generator().manual_seed(0)
    res = torch.randn(M, D, generator=g).to(dev)
    gm, bt = 1 + 0.1 * torch.randn(D, generator=g).to(dev), 0.1 * torch.randn(D, generator=g).to(dev)
    b = 0.1 * torch.randn(D, generator=g).to(dev)
    _, _, mu, rs = K.layernorm_fwd(res, gm, bt, out_f32=False, lp_dtype=torch.bfloat16)
    cases = {}
    for Kd in (512, 2048):
        x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        W = (torch.randn(D, Kd, generator=g) * 0.03).to(dev, torch.bfloat16)
        cases[f"fwd K={Kd}"] = (lambda x=x, W=W: K.linear_ln_fwd(x, W, b, res, gm, bt, dropout_p=0.1, seed=3))
    for Kd in (1536, 2048):
        dy = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        W = (torch.randn(Kd, D, generator=g) * 0.03).to(dev, torch.bfloat16)
        dg = torch.zeros(2 * D, device=dev)
        cases[f"bwd K={Kd}"] = (lambda dy=dy, W=W, dg=dg: K.linear_ln_bwd(
            dy, W, res, mu, rs, gm, dres=res, lp_dtype=torch.bfloat16, lp_dropout_p=0.1, lp_seed=5,
            dgamma=dg[:D], dbeta=dg[D:]))
    nwg = (M // 128) * 4
    names = ["main", "stage+pass1+partials", "drain+arrive", "wait", "tail (LN out, stores drained)"]
    for name, fn in cases.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        s = stamps(nwg) * 10 / 1000.0
        t0 = s[:, 0] - s[:, 0].min()
        span = s[:, 5].max() - s[:, 0].min()
        parts = "  ".join(f"{n} {np.median(s[:, i + 1] - s[:, i]):5.2f}/{(s[:, i + 1] - s[:, i]).max():5.2f}"
                          for i, n in enumerate(names))
        d = lambda a, b: f"{np.median(s[:, b] - s[:, a]):5.2f}"  # noqa: E731
        if name.startswith("fwd"):
            parts += f"\n           stage {d(1, 6)}  pass1 (x_out) {d(6, 7)}  row stats {d(7, 2)}"
        else:
            parts += f"\n           stage {d(1, 6)}  pass1 (row sums) {d(6, 2)}"
        print(f"{name:10s} event {e0.elapsed_time(e1) * 1e3:6.1f} us  span {span:6.2f}  start spread "
              f"{np.median(t0):4.2f}/{t0.max():4.2f}  {parts}", flush=True)


if __name__ == "__main__":
    main()


def spread():
    """Main-loop time per workgroup against its XCD (blockIdx % 8) and its place in the XCD's tile range."""
    dev = torch.device("cuda:0")
    M, D, Kd = 16384, 512, 2048
    g = torch.Generator().manual_seed(0)
    res = torch.randn(M, D, generator=g).to(dev)
    gm, bt = 1 + 0.1 * torch.randn(D, generator=g).to(dev), 0.1 * torch.randn(D, generator=g).to(dev)
    b = 0.1 * torch.randn(D, generator=g).to(dev)
    x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
    W = (torch.randn(D, Kd, generator=g) * 0.03).to(dev, torch.bfloat16)
    for _ in range(6):
        K.linear_ln_fwd(x, W, b, res, gm, bt, dropout_p=0.1, seed=3)
    torch.cuda.synchronize()
    nwg = (M // 128) * 4
    s = stamps(nwg) * 10 / 1000.0
    main = s[:, 1] - s[:, 0]
    start = s[:, 0] - s[:, 0].min()
    bid = np.arange(nwg)
    xcd = bid % 8
    print("fwd K=2048 main loop by XCD (median / max):",
          " ".join(f"{x}:{np.median(main[xcd == x]):.1f}/{main[xcd == x].max():.1f}" for x in range(8)))
    order = np.argsort(main)
    print("slowest 12 workgroups (bid, xcd, start, main):",
          [(int(i), int(i % 8), round(float(start[i]), 2), round(float(main[i]), 2)) for i in order[-12:]])
    print("fastest 6:", [(int(i), int(i % 8), round(float(start[i]), 2), round(float(main[i]), 2)) for i in order[:6]])
    # per CU pair? workgroups i and i + 256 dispatched to the same slot range
    print("corr(start, main):", float(np.corrcoef(start, main)[0, 1]))


if __name__ == "__main__" and os.environ.get("LNX_SPREAD"):
    spread()
