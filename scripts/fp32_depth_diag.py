"""Where does the GPU fp32 path lose accuracy against fp64?  Per layer depth: the median per-tensor
relative gradient error of the GPU fp32 model and of the CPU fp32 oracle against the fp64 oracle, and the
forward's logits error.  Diagnostic aid (test infrastructure: imports the oracle), not product.
usage: python scripts/fp32_depth_diag.py [L] [RP_* env switches as usual]"""
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.mmct_oracle import MMCTransformer as Oracle  # noqa: E402
from repurpose_amd.MMCTransformer import MMCTransformer  # noqa: E402
from tests.test_model_gpu import TRI, make_batch, to_dev  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    cfg = dict(TRI, self_num_layers=L)
    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    ref = Oracle(**cfg).eval()
    torch.manual_seed(3)
    m = MMCTransformer(**cfg, compute_dtype="fp32").to(dev).train()
    m.DROPOUT = 0.0
    b = make_batch(cfg, 2, 256, [256, 173], seed=8)
    out32 = ref(b)
    ref.losses(*out32)["cls_loss"].backward()
    g32 = {n: q.grad.detach().double().clone() for n, q in ref.named_parameters() if q.grad is not None}
    ref64 = ref.double()
    ref64.zero_grad()
    b64 = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in b.items()}
    out64 = ref64(b64)
    ref64.losses(*out64)["cls_loss"].backward()
    outm = m(to_dev(b, dev))
    m.losses(*outm)["cls_loss"].backward()
    torch.cuda.synchronize()
    for i, (o32, o64, om) in enumerate(zip(out32, out64, outm)):
        if torch.is_tensor(o64) and o64.is_floating_point():
            print(f"output {i}: cpu fp32 {rel(o32.double(), o64):.2e}  gpu fp32 {rel(om.double().cpu(), o64):.2e}")
    groups = {}
    for (n, p), (n2, q) in zip(m.named_parameters(), ref64.named_parameters()):
        if p.grad is None or q.grad is None:
            continue
        mm = re.search(r"layers\.(\d+)\.", n)
        key = f"layer {int(mm.group(1)):2d}" if mm else n.split(".")[0]
        gx = q.grad.double()
        groups.setdefault(key, []).append((n, rel(p.grad.double().cpu(), gx), rel(g32[n], gx)))
    for key in sorted(groups):
        rows = groups[key]
        eg = sorted(r[1] for r in rows)[len(rows) // 2]
        ec = sorted(r[2] for r in rows)[len(rows) // 2]
        worst = max(rows, key=lambda r: r[1] / (r[2] + 1e-12))
        print(f"{key:24s} median gpu {eg:.2e} cpu {ec:.2e}   worst ratio {worst[0]} {worst[1]:.2e} / {worst[2]:.2e}")


if __name__ == "__main__":
    main()
