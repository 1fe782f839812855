"""The attention backward at the bench shape (B = 8, T = 2048, H = 8, dropout 0.1, prescaled Q) in the
sequential form (fused-delta dQ, then dK/dV) and the overlapped one (delta pass, then dQ on a side stream
beside dK/dV): time per call, eager and graph-replayed, interleaved, and the largest difference of dQKV.
Tuning aid, not product.  usage: python scripts/attn_overlap_check.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    B, T, H, p = 8, 2048, 8, 0.1
    g = torch.Generator(device="cpu").manual_seed(1)
    qkv = torch.randn(B * T, 3 * H * 64, generator=g).to(dev).to(torch.bfloat16)
    c = 0.125 * K.LOG2E
    qkv[:, :H * 64] = (qkv[:, :H * 64].float() * c).to(torch.bfloat16)
    kv = torch.ones(B, T, dtype=torch.uint8, device=dev)
    olo = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 5, q_prescaled=True, out_lo=olo)
    do = torch.randn(B * T, H * 64, generator=g).to(dev).to(torch.bfloat16)

    def run():
        return K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask, q_prescaled=True, out_lo=olo)

    res, graphs = {}, {}
    for mode in (False, True):
        K._BWD_OVERLAP = mode
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        res[mode] = run().float()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                run()
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(it):
                run()
        graphs[mode] = gr
    d = (res[True] - res[False]).abs()
    w = H * 64
    print(f"max |dQ| diff {d[:, :w].max().item():.3e} (|dQ| max {res[False][:, :w].abs().max().item():.3e}); "
          f"max |dK| diff {d[:, w:2 * w].max().item():.3e}; max |dV| diff {d[:, 2 * w:].max().item():.3e}")
    times = {False: [], True: []}
    for _ in range(4):
        for mode in (False, True):
            K._BWD_OVERLAP = mode
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(it):
                run()
            e1.record()
            torch.cuda.synchronize()
            eager = e0.elapsed_time(e1) / it * 1e3
            e0.record()
            graphs[mode].replay()
            e1.record()
            torch.cuda.synchronize()
            times[mode].append((eager, e0.elapsed_time(e1) / it * 1e3))
    for mode in (False, True):
        print(f"overlap={int(mode)}: eager " + " ".join(f"{a:.1f}" for a, _ in times[mode]) +
              " us/call; graph " + " ".join(f"{b:.1f}" for _, b in times[mode]) + " us/call")


if __name__ == "__main__":
    main()
