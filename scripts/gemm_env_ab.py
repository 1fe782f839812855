"""Env-switched A/B of the fp32-residual forward GEMMs (out_proj forward: K = 512, linear2 forward:
K = 2048; M = 16384, N = 512, bias, dropout 0.1, fp32 residual) in ONE process: each variant's 20
launches are captured as a HIP graph under its own env value (the launcher reads the switch per
launch), the graphs replay interleaved over several rounds, and the outputs are compared bit for bit.
Tuning aid, not product.  usage: python scripts/gemm_env_ab.py [VAR] [A] [B]  (default RP_GEMM_BM64 0 1: 128- vs
64-row tiles; the switch must be one the launcher reads per call.  Round 4 measured the removed
RP_GEMM_RESPRE switch with it)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    var, va, vb = (sys.argv[1:4] + ["RP_GEMM_BM64", "0", "1"][len(sys.argv[1:4]):])[:3]
    dev = torch.device("cuda:0")
    M, N = 16384, 512
    g = torch.Generator().manual_seed(0)
    res = torch.randn(M, N, generator=g).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    s = torch.cuda.Stream()
    calls = 20
    for Kd, name in ((512, "out_proj fwd"), (2048, "linear2 fwd")):
        x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
        graphs, outs = {}, {}
        for v in (va, vb):
            os.environ[var] = v
            with torch.cuda.stream(s):
                outs[v] = K.linear_fwd(x, w, b, out_dtype=torch.float32, dropout_p=0.1, seed=3, residual=res)
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=s):
                    for _ in range(calls):
                        K.linear_fwd(x, w, b, out_dtype=torch.float32, dropout_p=0.1, seed=3, residual=res)
            graphs[v] = gr
        torch.cuda.synchronize()
        same = torch.equal(outs[va], outs[vb])
        tot = {v: [] for v in graphs}
        for _ in range(7):
            for v, gr in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(s):
                    gr.replay()
                    e0.record(s)
                    gr.replay()
                    e1.record(s)
                torch.cuda.synchronize()
                tot[v].append(e0.elapsed_time(e1) * 1e3 / calls)
        med = {v: sorted(t)[len(t) // 2] for v, t in tot.items()}
        print(f"{name}: {var}={va} {med[va]:.2f} us, {var}={vb} {med[vb]:.2f} us; bitwise equal: {same}", flush=True)


if __name__ == "__main__":
    main()
