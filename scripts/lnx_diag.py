"""Where does the exchange GEMM + LayerNorm backward differ from the unfused pair?  Tuning aid."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
D = 512
for M, Kd, with_lp, has_dres in ((16384, 2048, True, True), (16384, 2048, False, True), (16384, 512, False, False),
                                 (4096, 2048, True, True), (8192, 2048, True, True)):
    g = torch.Generator().manual_seed(3 * M + Kd + 1)
    dy = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
    W = (torch.randn(Kd, D, generator=g) * 0.03).to(dev, torch.bfloat16)
    x = torch.randn(M, D, generator=g).to(dev)
    gm = 1.0 + 0.1 * torch.randn(D, generator=g).to(dev)
    _, _, mu, rs = K.layernorm_fwd(x, gm, torch.zeros(D, device=dev), out_f32=False, lp_dtype=torch.bfloat16)
    dres = torch.randn(M, D, generator=g).to(dev) if has_dres else None
    lpd = torch.bfloat16 if with_lp else None
    dh = K.linear_dgrad(dy, W, out_dtype=torch.float32)
    dx0, _ = K.layernorm_bwd(dh, x, mu, rs, gm, dres=dres, lp_dtype=lpd, lp_dropout_p=0.1, lp_seed=5)
    dx1, _ = K.linear_ln_bwd(dy, W, x, mu, rs, gm, dres=dres, lp_dtype=lpd, lp_dropout_p=0.1, lp_seed=5)
    torch.cuda.synchronize()
    ws = K._lnx_ws(dev, M)
    err = (dx1 - dx0).abs()
    bad = err > 1e-4 * dx0.abs().max()
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    print(f"M {M} K {Kd} lp {with_lp} dres {has_dres}: max err {err.max().item():.3e}, bad elems {int(bad.sum())}, "
          f"bad rows {rows.numel()} (first {rows[:8].tolist()}), bad cols {cols.numel()} (first {cols[:8].tolist()}), "
          f"err word {int(ws[:4].view(torch.int32).item())}, counters nonzero {int(ws[256:256 + (M // 128) * 4352].view(M // 128, 4352)[:, :8].count_nonzero())}")
    if rows.numel():
        rb = (rows // 128).unique()
        print("   bad row blocks", rb[:16].tolist(), "count", rb.numel(), " rows within block", (rows % 128).unique()[:16].tolist())
        r = rows[0].item()
        print("   row", r, "dx0", dx0[r, :6].tolist(), "dx1", dx1[r, :6].tolist())
