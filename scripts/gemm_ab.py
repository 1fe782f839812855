"""A/B the GEMM paths at the bench shapes (M = 16384 tokens) in ONE process, interleaved rounds
(guide rule 24).  Variants switch through the per-call env knob RP_GEMM8 (1: 256-row phased kernel).
Every variant is first checked against an fp32 torch product of the same bf16 operands.
Usage: python scripts/gemm_ab.py [--reps N] [--rounds R] [--variants base,g8] [--ops fwd,dgrad]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402

VARIANTS = {"base": {"RP_GEMM8": "0"}, "g8": {"RP_GEMM8": "1"}, "auto": {},
            "base_tm": {"RP_GEMM8": "0", "RP_WGRAD_SPLIT_MAJOR": "0"}, "g8_tm": {"RP_GEMM8": "1", "RP_WGRAD_SPLIT_MAJOR": "0"}}
KNOBS = ("RP_GEMM8", "RP_WGRAD_SPLIT_MAJOR")


def setenv(v):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(VARIANTS[v])


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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="base,g8")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--M", type=int, default=16384)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, d, dff = a.M, 512, 2048
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(0)
    variants = a.variants.split(",")
    ops = a.ops.split(",")
    cases = []
    ws = torch.empty(64 << 20, device=dev)
    for (n, k, name) in [(3 * d, d, "qkv"), (d, d, "out_proj"), (dff, d, "linear1"), (d, dff, "linear2"),
                         (d, 2944, "input_proj")]:
        x = torch.randn(M, k, generator=g).to(dev, bf)
        w = (torch.randn(n, k, generator=g) * 0.05).to(dev, bf)
        b = torch.randn(n, generator=g).to(dev)
        dy = torch.randn(M, n, generator=g).to(dev, bf)
        fl = 2.0 * M * n * k
        if "fwd" in ops:
            cases.append((f"fwd {name} {n}x{k} bf16", fl, lambda x=x, w=w, b=b: K.linear_fwd(x, w, b, out_dtype=bf),
                          lambda x=x, w=w, b=b: x.float() @ w.float().T + b))
            cases.append((f"fwd {name} f32", fl, lambda x=x, w=w, b=b: K.linear_fwd(x, w, b, out_dtype=torch.float32),
                          lambda x=x, w=w, b=b: x.float() @ w.float().T + b))
        if "wgrad" in ops:
            dW = torch.zeros(n, k, device=dev)
            db = torch.zeros(n, device=dev)

            def wg(dy=dy, x=x, dW=dW, db=db):
                K.linear_wgrad(dy, x, dW, db=db, ws=ws, accumulate=False)
                return dW
            cases.append((f"wgrad {name}", fl, wg, lambda dy=dy, x=x: dy.float().T @ x.float()))
        if "dgrad" in ops and name != "input_proj":
            cases.append((f"dgrad {name} f32", fl, lambda dy=dy, w=w: K.linear_dgrad(dy, w, out_dtype=torch.float32),
                          lambda dy=dy, w=w: dy.float() @ w.float()))
    bad = 0
    for v in variants:
        setenv(v)
        for (nm, fl, fn, ref) in cases:
            out = fn().float()
            r = ref()
            err = ((out - r).abs().max() / r.abs().max()).item()
            if not err < 2e-2:
                bad += 1
                print(f"check {v:6s} {nm:30s} rel err {err:.2e}  <-- MISMATCH", flush=True)
    print(f"checks done, {bad} mismatches", flush=True)
    res = {}
    for rnd in range(a.rounds):
        for (nm, fl, fn, ref) in cases:
            for v in variants:
                setenv(v)
                res.setdefault((nm, v), []).append(timeit(fn, a.reps))
    for (nm, fl, fn, ref) in cases:
        line = f"{nm:30s}"
        for v in variants:
            t = min(res[(nm, v)])
            line += f"  {v}: {t * 1e3:6.1f} us {fl / t / 1e9:5.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
