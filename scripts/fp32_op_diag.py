"""Per-op accuracy of the fp32 (parity-mode) kernels against fp64, beside torch's CPU fp32 for the same
op: the attention forward / backward, the dgrad GEMM shapes and the LayerNorm backward at the depth
test's shapes (B = 2, T = 256, H = 8).  Relative norm errors.  Diagnostic aid, not product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from repurpose_amd import kernels as K  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def attn64(qkv, kv, B, T, H, scale):
    q, k, v = qkv.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    s = s.masked_fill(~kv.bool()[:, None, None, :], float("-inf"))
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * T, H * 64)


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    B, T, H, scale = 2, 256, 8, 0.125
    for amp in (1.0, 3.0):
        qkv = torch.randn(B * T, 3 * H * 64, generator=g) * amp
        kv = torch.ones(B, T, dtype=torch.uint8)
        kv[1, 173:] = 0
        do = torch.randn(B * T, H * 64, generator=g)
        x64 = qkv.double().requires_grad_(True)
        o64 = attn64(x64, kv, B, T, H, scale)
        d64, = torch.autograd.grad(o64, x64, do.double())
        x32 = qkv.clone().requires_grad_(True)
        o32 = attn64(x32, kv, B, T, H, scale)
        d32, = torch.autograd.grad(o32, x32, do)
        qd, kvd, dod = qkv.to(dev), kv.to(dev), do.to(dev)
        o, lse, _ = K.attn_fwd(qd, kvd, B, T, H, scale)
        dq = K.attn_bwd(qd, o, dod, lse, kvd, B, T, H, scale)
        # the model's path: Q prescaled by the producer
        c = scale * K.LOG2E
        qp = qd.clone()
        qp[:, :H * 64] *= c
        op, lsep, _ = K.attn_fwd(qp, kvd, B, T, H, scale, q_prescaled=True)
        dqp = K.attn_bwd(qp, op, dod, lsep, kvd, B, T, H, scale, q_prescaled=True)
        torch.cuda.synchronize()
        D = H * 64
        for nm, sl in (("dq", slice(0, D)), ("dk", slice(D, 2 * D)), ("dv", slice(2 * D, 3 * D))):
            print(f"attn amp {amp}: {nm} gpu {rel(dq[:, sl], d64[:, sl]):.2e}  gpu-prescaled "
                  f"{rel(dqp[:, sl], d64[:, sl]):.2e}  cpu fp32 {rel(d32[:, sl], d64[:, sl]):.2e}")
        print(f"attn amp {amp}: out gpu {rel(o, o64.detach()):.2e} prescaled {rel(op, o64.detach()):.2e} "
              f"cpu {rel(o32.detach(), o64.detach()):.2e}")
    M = B * T
    for (n, k) in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]:
        w = torch.randn(n, k, generator=g) * 0.05
        dy = torch.randn(M, n, generator=g)
        ref = dy.double() @ w.double()
        got = K.linear_dgrad(dy.to(dev), w.to(dev), out_dtype=torch.float32)
        torch.cuda.synchronize()
        print(f"dgrad {n}x{k}: gpu {rel(got, ref):.2e} cpu {rel(dy @ w, ref):.2e}")
    x = torch.randn(M, 512, generator=g) * 4 + 2
    gam = torch.randn(512, generator=g)
    dy = torch.randn(M, 512, generator=g)
    x64 = x.double().requires_grad_(True)
    y64 = torch.nn.functional.layer_norm(x64, (512,), gam.double(), None, 1e-5)
    dx64, = torch.autograd.grad(y64, x64, dy.double())
    x32 = x.clone().requires_grad_(True)
    y32 = torch.nn.functional.layer_norm(x32, (512,), gam, None, 1e-5)
    dx32, = torch.autograd.grad(y32, x32, dy)
    mu = x.mean(1)
    rs = 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
    dxg, _ = K.layernorm_bwd(dy.to(dev), x.to(dev), mu.to(dev), rs.to(dev), gam.to(dev))
    torch.cuda.synchronize()
    print(f"layernorm bwd: gpu {rel(dxg, dx64):.2e} cpu {rel(dx32, dx64):.2e}")


if __name__ == "__main__":
    main()
