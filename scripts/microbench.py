"""Per-kernel timings at the bench shape (B=8, T=2048, d=512, H=8, dff=2048), HIP-event timed,
interleaved rounds in one process (guide rule 24).  Prints one line per kernel: avg ms and TFLOP/s
or GB/s.  Usage: python scripts/microbench.py [--only attn|gemm|ln] [--reps N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=2048)
    ap.add_argument("--gemm", default="", help="only this GEMM shape (qkv|out_proj|linear1|linear2)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, T, H, d, dff = a.B, a.T, 8, 512, 2048
    M = B * T
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(0)
    res = []
    if a.only in ("", "attn"):
        qkv = torch.randn(M, 3 * d, generator=g).to(dev, bf)
        kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
        do = torch.randn(M, d, generator=g).to(dev, bf)
        fl = 4.0 * B * H * T * T * 64
        olo = torch.empty(M, d, device=dev, dtype=bf)
        for p in (0.0, 0.1):
            # as the model calls them: Q columns prescaled by the QKV GEMM, output residual kept
            r = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 1, q_prescaled=True, out_lo=olo)
            o, lse, mask = r
            t = timeit(lambda: K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 1, q_prescaled=True, out_lo=olo), a.reps)
            res.append((f"attn_fwd p={p}", t, fl / t / 1e9, "TFLOP/s"))
            # as the step runs it (the delta pass + the two-role launch where uses_roles), untimed per phase
            t = timeit(lambda: K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True,
                                          out_lo=olo), a.reps)
            form = "delta + two-role" if K.attn_bwd_uses_roles(qkv, B, T, H, q_prescaled=True) else "dQ+delta, dK/dV"
            res.append((f"attn_bwd p={p} ({form})", t, 2 * fl / t / 1e9, "TFLOP/s alg"))
            # the per-phase kernels (the timed path's two-kernel form: fused-delta dQ, then dK/dV)
            os.environ["RP_ATTN_ROLES"] = "0"
            K.timer_start("attn_bwd_dq", "attn_bwd_dkdv")
            timeit(lambda: K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True,
                                      out_lo=olo), a.reps)
            kt = K.timer_stop()
            os.environ.pop("RP_ATTN_ROLES", None)
            res.append((f"  attn_bwd_dq p={p}", kt["attn_bwd_dq"], 2 * fl / 4 / kt["attn_bwd_dq"] / 1e9, "TFLOP/s alg"))
            res.append((f"  attn_bwd_dkdv p={p}", kt["attn_bwd_dkdv"], 6 * fl / 4 / kt["attn_bwd_dkdv"] / 1e9,
                        "TFLOP/s alg"))
    if a.only in ("", "gemm"):
        for (n, k, name) in [(3 * d, d, "qkv"), (d, d, "out_proj"), (dff, d, "linear1"), (d, dff, "linear2")]:
            if a.gemm and a.gemm != name:
                continue
            x = torch.randn(M, k, generator=g).to(dev, bf)
            w = (torch.randn(n, k, generator=g) * 0.02).to(dev, bf)
            b = torch.zeros(n, device=dev)
            fl = 2.0 * M * n * k
            t = timeit(lambda: K.linear_fwd(x, w, b, out_dtype=bf), a.reps)
            res.append((f"gemm fwd {name} {M}x{n}x{k} bf16out", t, fl / t / 1e9, "TFLOP/s"))
            dy = torch.randn(M, n, generator=g).to(dev, bf)
            t = timeit(lambda: K.linear_dgrad(dy, w, out_dtype=torch.float32), a.reps)
            res.append((f"gemm dgrad {name} f32out", t, fl / t / 1e9, "TFLOP/s"))
            dW = torch.zeros(n, k, device=dev)
            db = torch.zeros(n, device=dev)
            ws = torch.empty(64 << 20, device=dev)
            t = timeit(lambda: K.linear_wgrad(dy, x, dW, db=db, ws=ws), a.reps)
            res.append((f"gemm wgrad {name} (+bias, split-K)", t, fl / t / 1e9, "TFLOP/s"))
    if a.only in ("", "ln"):
        x = torch.randn(M, d, generator=g).to(dev)
        gm = torch.ones(d, device=dev)
        bt = torch.zeros(d, device=dev)
        t = timeit(lambda: K.layernorm_fwd(x, gm, bt, out_f32=False, lp_dtype=bf), a.reps)
        res.append(("ln fwd f32->bf16", t, M * d * 6 / t / 1e6, "GB/s"))
        _, _, mu, rs = K.layernorm_fwd(x, gm, bt, out_f32=False, lp_dtype=bf)
        dy = torch.randn(M, d, generator=g).to(dev)
        dg = torch.zeros(d, device=dev)
        t = timeit(lambda: K.layernorm_bwd(dy, x, mu, rs, gm, dres=dy, lp_dtype=bf, lp_dropout_p=0.1, dgamma=dg,
                                           dbeta=dg), a.reps)
        res.append(("ln bwd (+dres, lp out, dgamma/dbeta)", t, M * d * 18 / t / 1e6, "GB/s"))
    if a.only in ("lib",):
        # vendor-library yardsticks at the same shapes (hipBLASLt via torch.mm, torch SDPA): headroom only
        for (n, k, name) in [(3 * d, d, "qkv"), (d, d, "out_proj"), (dff, d, "linear1"), (d, dff, "linear2")]:
            x = torch.randn(M, k, generator=g).to(dev, bf)
            w = (torch.randn(n, k, generator=g) * 0.02).to(dev, bf)
            dy = torch.randn(M, n, generator=g).to(dev, bf)
            fl = 2.0 * M * n * k
            t = timeit(lambda: torch.mm(x, w.t()), a.reps)
            res.append((f"torch.mm fwd {name}", t, fl / t / 1e9, "TFLOP/s"))
            t = timeit(lambda: torch.mm(dy, w), a.reps)
            res.append((f"torch.mm dgrad {name}", t, fl / t / 1e9, "TFLOP/s"))
            t = timeit(lambda: torch.mm(dy.t(), x), a.reps)
            res.append((f"torch.mm wgrad {name}", t, fl / t / 1e9, "TFLOP/s"))
        q = torch.randn(B, H, T, 64, generator=g).to(dev, bf).requires_grad_()
        kk = torch.randn(B, H, T, 64, generator=g).to(dev, bf).requires_grad_()
        v = torch.randn(B, H, T, 64, generator=g).to(dev, bf).requires_grad_()
        fl = 4.0 * B * H * T * T * 64
        F = torch.nn.functional
        t = timeit(lambda: F.scaled_dot_product_attention(q, kk, v), a.reps)
        res.append(("torch sdpa fwd", t, fl / t / 1e9, "TFLOP/s"))
        o = F.scaled_dot_product_attention(q, kk, v)
        go = torch.randn_like(o)
        t = timeit(lambda: torch.autograd.grad(F.scaled_dot_product_attention(q, kk, v), (q, kk, v), go), a.reps)
        res.append(("torch sdpa fwd+bwd", t, 3 * fl / t / 1e9, "TFLOP/s"))
    for name, t, r, u in res:
        print(f"{name:48s} {t * 1e3:9.1f} us  {r:8.1f} {u}", flush=True)


if __name__ == "__main__":
    main()
