"""The eight forward / dgrad GEMM launches of one encoder layer at the bench shape (M = B*T = 16384),
with the epilogues the model gives them (MMCTransformer.py forward / backward), each timed with HIP
events around the launch alone, caches flushed before every launch (the step's working set is far
beyond the 256 MiB Infinity Cache, so in the step the operands arrive cold).  Prints per shape: us,
TFLOP/s, the HBM bytes the launch must move at least and GB/s over them, and the bound it sits on.
usage: python scripts/gemm_step.py [--reps 10] [--warm]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm", action="store_true", help="no cache flush between launches")
    ap.add_argument("--only", default="")
    ap.add_argument("--ablate", action="store_true", help="epilogue ablation of the main shapes")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, d, dff = 16384, 512, 2048
    bf, f32 = torch.bfloat16, torch.float32
    g = torch.Generator(device="cpu").manual_seed(0)
    r = lambda *s, dt=bf, sc=1.0: (torch.randn(*s, generator=g) * sc).to(dev, dt)
    h1, o, h2, f = r(M, d), r(M, d), r(M, d), torch.relu(r(M, dff))
    x, x1 = r(M, d, dt=f32), r(M, d, dt=f32)
    Wqkv, Wo, W1, W2 = r(3 * d, d, sc=0.02), r(d, d, sc=0.02), r(dff, d, sc=0.02), r(d, dff, sc=0.02)
    bqkv, bo, b1, b2 = (torch.zeros(n, device=dev) for n in (3 * d, d, dff, d))
    g2, g1, dqkv, dzf = r(M, d), r(M, d), r(M, 3 * d), r(M, dff)
    p, sd = 0.1, 1.0 / 0.9
    E = 2  # bf16 bytes
    cases = [
        ("qkv fwd", lambda: K.linear_fwd(h1, Wqkv, bqkv, col_scale_n=d, col_scale=0.18), M * 3 * d * d,
         M * d * E + 3 * d * d * E + M * 3 * d * E),
        ("out_proj fwd +res +drop f32", lambda: K.linear_fwd(o, Wo, bo, out_dtype=f32, dropout_p=p, seed=1, residual=x),
         M * d * d, M * d * E + d * d * E + 2 * M * d * 4),
        ("linear1 fwd relu+drop", lambda: K.linear_fwd(h2, W1, b1, relu=True, dropout_p=p, seed=2), M * dff * d,
         M * d * E + dff * d * E + M * dff * E),
        ("linear2 fwd +res +drop f32", lambda: K.linear_fwd(f, W2, b2, out_dtype=f32, dropout_p=p, seed=3, residual=x1),
         M * d * dff, M * dff * E + d * dff * E + 2 * M * d * 4),
        ("linear2 dgrad gated", lambda: K.linear_dgrad(g2, W2, out_dtype=bf, gate=f, gate_scale=sd), M * dff * d,
         M * d * E + d * dff * E + 2 * M * dff * E),
        ("linear1 dgrad f32", lambda: K.linear_dgrad(dzf, W1, out_dtype=f32), M * d * dff, M * dff * E + dff * d * E + M * d * 4),
        ("out_proj dgrad", lambda: K.linear_dgrad(g1, Wo, out_dtype=bf), M * d * d, 2 * M * d * E + d * d * E),
        ("qkv dgrad f32", lambda: K.linear_dgrad(dqkv, Wqkv, out_dtype=f32), M * d * 3 * d,
         M * 3 * d * E + 3 * d * d * E + M * d * 4),
    ]
    gm, bt = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    mu, rs = torch.zeros(M, device=dev), torch.ones(M, device=dev)
    flat = torch.zeros(2 * d, device=dev)
    F = 4
    cases += [
        ("out_proj fwd + LN2 (unfused)", lambda: K.layernorm_fwd(
            K.linear_fwd(o, Wo, bo, out_dtype=f32, dropout_p=p, seed=1, residual=x), gm, bt, out_f32=False,
            lp_dtype=bf), M * d * d, M * d * E + d * d * E + 2 * M * d * F + M * d * E),
        ("out_proj fwd + LN2 (fused)", lambda: K.linear_ln_fwd(o, Wo, bo, x, gm, bt, dropout_p=p, seed=1),
         M * d * d, M * d * E + d * d * E + 2 * M * d * F + M * d * E),
        ("linear2 fwd + LN1 (unfused)", lambda: K.layernorm_fwd(
            K.linear_fwd(f, W2, b2, out_dtype=f32, dropout_p=p, seed=3, residual=x1), gm, bt, out_f32=False,
            lp_dtype=bf), M * d * dff, M * dff * E + d * dff * E + 2 * M * d * F + M * d * E),
        ("linear2 fwd + LN1 (fused)", lambda: K.linear_ln_fwd(f, W2, b2, x1, gm, bt, dropout_p=p, seed=3),
         M * d * dff, M * dff * E + d * dff * E + 2 * M * d * F + M * d * E),
        ("linear1 dgrad + LN2 bwd (unfused)", lambda: K.layernorm_bwd(
            K.linear_dgrad(dzf, W1, out_dtype=f32), x1, mu, rs, gm, dres=x, lp_dtype=bf, lp_dropout_p=p, lp_seed=4,
            dgamma=flat[:d], dbeta=flat[d:]), M * d * dff, M * dff * E + dff * d * E + 3 * M * d * F + M * d * E),
        ("linear1 dgrad + LN2 bwd (fused)", lambda: K.linear_ln_bwd(
            dzf, W1, x1, mu, rs, gm, dres=x, lp_dtype=bf, lp_dropout_p=p, lp_seed=4, dgamma=flat[:d], dbeta=flat[d:]),
         M * d * dff, M * dff * E + dff * d * E + 3 * M * d * F + M * d * E),
        ("qkv dgrad + LN1 bwd (unfused)", lambda: K.layernorm_bwd(
            K.linear_dgrad(dqkv, Wqkv, out_dtype=f32), x, mu, rs, gm, dres=x1, lp_dtype=bf, lp_dropout_p=p,
            lp_seed=5, dgamma=flat[:d], dbeta=flat[d:]), M * d * 3 * d,
         M * 3 * d * E + 3 * d * d * E + 3 * M * d * F + M * d * E),
        ("qkv dgrad + LN1 bwd (fused)", lambda: K.linear_ln_bwd(
            dqkv, Wqkv, x, mu, rs, gm, dres=x1, lp_dtype=bf, lp_dropout_p=p, lp_seed=5, dgamma=flat[:d],
            dbeta=flat[d:]), M * d * 3 * d, M * 3 * d * E + 3 * d * d * E + 3 * M * d * F + M * d * E),
    ]
    if a.ablate:  # the epilogue's share: the same shapes with fewer epilogue stages
        cases = [
            ("linear1 fwd plain", lambda: K.linear_fwd(h2, W1, b1), M * dff * d, M * d * E + dff * d * E + M * dff * E),
            ("linear1 fwd relu", lambda: K.linear_fwd(h2, W1, b1, relu=True), M * dff * d,
             M * d * E + dff * d * E + M * dff * E),
            ("linear1 fwd relu+drop", lambda: K.linear_fwd(h2, W1, b1, relu=True, dropout_p=p, seed=2), M * dff * d,
             M * d * E + dff * d * E + M * dff * E),
            ("qkv fwd plain", lambda: K.linear_fwd(h1, Wqkv, bqkv), M * 3 * d * d, M * d * E + 3 * d * d * E + M * 3 * d * E),
            ("linear2 fwd f32 plain", lambda: K.linear_fwd(f, W2, b2, out_dtype=f32), M * d * dff,
             M * dff * E + d * dff * E + M * d * 4),
            ("linear2 fwd f32 +res", lambda: K.linear_fwd(f, W2, b2, out_dtype=f32, residual=x1), M * d * dff,
             M * dff * E + d * dff * E + 2 * M * d * 4),
            ("linear2 fwd f32 +res+drop", lambda: K.linear_fwd(f, W2, b2, out_dtype=f32, dropout_p=p, seed=3,
                                                               residual=x1), M * d * dff,
             M * dff * E + d * dff * E + 2 * M * d * 4),
            ("linear2 fwd bf16 plain", lambda: K.linear_fwd(f, W2, b2), M * d * dff, M * dff * E + d * dff * E + M * d * E),
        ]
    flush = torch.empty(640 << 20, dtype=torch.uint8, device=dev)
    tot = 0.0
    for name, fn, fl, by in cases:
        if a.only and a.only not in name:
            continue
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            if not a.warm:
                flush.fill_(1)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ts.sort()
        t = ts[len(ts) // 2] * 1e-3
        tot += t
        tf, gbs = 2 * fl / t / 1e12, by / t / 1e9
        bound = max(2 * fl / 2.5e15, by / 6.3e12)
        print(f"{name:30s} {t * 1e6:7.1f} us  {tf:7.1f} TF/s  {by / 1e6:6.1f} MB {gbs:7.0f} GB/s  "
              f"floor {bound * 1e6:5.1f} us ({'mfma' if 2 * fl / 2.5e15 > by / 6.3e12 else 'hbm'})", flush=True)
    print(f"total {tot * 1e6:.1f} us per layer")


if __name__ == "__main__":
    main()
