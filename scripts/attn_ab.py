"""A/B of attention kernel variants selected by per-launch environment switches, in ONE process (tuning
aid, not product): the same inputs through variant A and variant B — keep bits compared bit for bit,
outputs / gradients compared against each other, and each kernel timed with HIP events (interleaved
repetitions).  usage: python scripts/attn_ab.py --a RP_ATTN_SPLIT=0 --b RP_ATTN_SPLIT=1 [--B 8 --T 2048
--p 0.1 --ragged --reps 10]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def setenv(spec):
    for kv in spec.split(","):
        if kv:
            k, v = kv.split("=")
            os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="")
    ap.add_argument("--b", default="")
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=2048)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--ragged", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, T, H, d = a.B, a.T, 8, 512
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn(M, 3 * d, generator=g).to(dev, torch.bfloat16)
    kv = torch.ones(B, T, dtype=torch.uint8)
    if a.ragged:
        for b in range(B):
            kv[b, int(torch.randint(T // 2, T + 1, (1,), generator=g)):] = 0
    kv = kv.to(dev)
    do = torch.randn(M, d, generator=g).to(dev, torch.bfloat16)

    def run(spec):
        setenv(spec)
        olo = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
        o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, a.p, 11, q_prescaled=True, out_lo=olo)
        dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, a.p, dropmask=mask, q_prescaled=True, out_lo=olo)
        torch.cuda.synchronize()
        return o, lse, mask, olo, dqkv

    ra, rb = run(a.a), run(a.b)
    res = {}
    if ra[2] is not None:
        res["mask_bits_equal"] = bool(torch.equal(ra[2], rb[2]))
    for i, n in ((0, "o"), (1, "lse"), (4, "dqkv")):
        x, y = ra[i].float(), rb[i].float()
        res[f"{n}_max_abs_diff"] = float((x - y).abs().max())
        res[f"{n}_max_abs"] = float(y.abs().max())
        res[f"{n}_bitwise"] = bool(torch.equal(ra[i], rb[i]))
    hi_a = ra[0].float() + ra[3].float()
    hi_b = rb[0].float() + rb[3].float()
    res["o_hi_plus_lo_max_abs_diff"] = float((hi_a - hi_b).abs().max())
    print(res, flush=True)

    times = {"A": {}, "B": {}}
    for rep in range(a.reps):
        for tag, spec in (("A", a.a), ("B", a.b)):
            setenv(spec)
            K.timer_start("attn_fwd", "attn_bwd_dq", "attn_bwd_dkdv")
            run(spec)
            for k, v in K.timer_stop().items():
                times[tag].setdefault(k, []).append(v)
    for tag in ("A", "B"):
        med = {k: sorted(v)[len(v) // 2] * 1e3 for k, v in times[tag].items()}
        print(tag, (a.a if tag == "A" else a.b), {k: f"{v:.1f} us" for k, v in med.items()}, flush=True)


if __name__ == "__main__":
    main()
