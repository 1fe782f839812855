"""Grouped weight-gradient launch (rp_gemm_wgrad_grouped) at the metric shape, alone: the 16 encoder
layers x {linear2, linear1, out_proj, in_proj} over K = 16,384 tokens, as the bf16 backward defers them
(tuning aid, not product).  Times the launch with HIP events (warm, back to back) for the item orders and
cuts given, and checks every variant bitwise against the first.
usage: python scripts/wgrad_probe.py [--reps 10] [--cut 768|256] [--env NAME=V ...]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def items(dev, L=16, T=16384, d=512, dff=2048, seed=0, pad=0, only=None):
    g = torch.Generator(device="cpu").manual_seed(seed)

    def r(n):  # [T, n] operand; pad > 0: rows `pad` elements longer than n (a non-power-of-two stride)
        x = (torch.randn(T, n, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        if pad == 0:
            return x
        buf = torch.zeros(T, n + pad, dtype=torch.bfloat16, device=dev)
        buf[:, :n] = x
        return buf[:, :n]
    out = []
    for l in reversed(range(L)):  # backward order: linear2, linear1, out_proj, in_proj per layer
        for name, (n_out, n_in) in zip(("linear2", "linear1", "out_proj", "in_proj"), ((d, dff), (dff, d), (d, d), (3 * d, d))):
            if only and name != only:
                continue
            out.append((r(n_out), r(n_in), torch.empty(n_out, n_in, device=dev), torch.empty(n_out, device=dev)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--env", nargs="*", default=[])
    ap.add_argument("--cut", type=int, default=64, help="items per launch (64 = all 16 layers in one)")
    ap.add_argument("--pad", type=int, default=0, help="operand row padding in elements")
    ap.add_argument("--only", default=None, help="one GEMM kind of the 4 (linear2 | linear1 | out_proj | in_proj)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    it = items(dev, pad=a.pad, only=a.only)
    variants = [("default", {})] + [(e, dict([e.split("=", 1)])) for e in a.env]
    ref = None
    for name, env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        times = []
        for rep in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for c in range(0, len(it), a.cut):
                K.linear_wgrad_grouped(it[c:c + a.cut], accumulate=False)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                times.append(e0.elapsed_time(e1) * 1e3)
        got = torch.cat([torch.cat([w.reshape(-1), b]) for _, _, w, b in it])
        same = "ref" if ref is None else ("bitwise" if torch.equal(ref, got) else "DIFFERENT")
        ref = got if ref is None else ref
        times.sort()
        print(f"{name:32s} median {times[len(times) // 2]:8.1f} us  min {times[0]:8.1f}  ({same})", flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
