"""In-kernel s_memtime stamps of the forward GEMM kernels (a temporary build with RP_GEMM_STAMP support):
per workgroup the start, the end of the main loop and the end, per XCD clock.  Prints the per-shape
medians of main-loop and epilogue time and how the starts spread.  Tuning aid, not product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M = 16384
    g = torch.Generator(device="cpu").manual_seed(0)
    st = torch.zeros(65536 * 4, dtype=torch.int64, device=dev)
    for name, N, Kd, f32, res in (("out_proj fwd f32+res", 512, 512, True, True), ("linear2 fwd f32+res", 512, 2048, True, True),
                                  ("qkv fwd bf16", 1536, 512, False, False), ("linear1 fwd bf16", 2048, 512, False, False)):
        x = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
        r = torch.randn(M, N, generator=g).to(dev) if res else None
        fn = lambda: K.linear_fwd(x, w, None, out_dtype=torch.float32 if f32 else None, residual=r)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        st.zero_()
        os.environ["RP_GEMM_STAMP"] = str(st.data_ptr())
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        del os.environ["RP_GEMM_STAMP"]
        a = st.view(-1, 4).cpu()
        a = a[a[:, 2] != 0]
        t0, t1, t2, xcc = a[:, 0].double(), a[:, 1].double(), a[:, 2].double(), a[:, 3]
        main_ = (t1 - t0)
        epi = (t2 - t1)
        tot = (t2 - t0)
        spans = []
        for x_ in range(8):
            m = xcc == x_
            if m.any():
                spans.append(((t2[m].max() - t0[m].min()).item(), (t0[m].max() - t0[m].min()).item(), m.sum().item()))
        med = lambda v: v.median().item()  # noqa: E731
        print(f"{name:22s} event {s.elapsed_time(e) * 1e3:6.1f} us  wgs {len(a)}  per WG (cycles of the 100 MHz? "
              f"s_memtime clock): main {med(main_):8.0f}  epi {med(epi):8.0f}  total {med(tot):8.0f}  "
              f"XCD span/start-spread/wgs {spans[:2]}", flush=True)


if __name__ == "__main__":
    main()
