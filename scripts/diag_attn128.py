"""Diagnose test_attention_128_blocks_ragged_dropout mismatches: where the failing gradient elements sit."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from tests.test_kernels_gpu import rnd, attn_ref
from repurpose_amd import kernels as K
dev = torch.device("cuda")
B, H, T, p = 8, 8, 1030, float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
qkv = rnd(B * T, 3 * H * 64, dev=dev, seed=T).to(torch.bfloat16)
lens = torch.tensor([T, T - 1, 1000, 777, 640, 129, 2, 1], device=dev)
kv = (torch.arange(T, device=dev)[None] < lens[:, None]).to(torch.uint8)
o, lse, mask = K.attn_fwd(qkv, kv, B, T, H, 0.125, p, 99)
ref_in = qkv.double().requires_grad_(True)
ref = attn_ref(ref_in, kv, B, T, H, p, 99)
print("fwd maxerr", (o.double() - ref).abs().max().item())
do = rnd(B * T, H * 64, dev=dev, seed=T + 1).to(torch.bfloat16)
dqkv = K.attn_bwd(qkv, o, do, lse, kv, B, T, H, 0.125, p, dropmask=mask)
g = torch.autograd.grad(ref, ref_in, do.double())[0]
err = (dqkv.double() - g).abs()
bad = err > 6e-2 + 6e-2 * g.abs()
idx = bad.nonzero()
print("bad", idx.shape[0], "block", os.environ.get("RP_ATTN_BLOCK", "auto"))
for r, c in idx[:30].tolist():
    b, t = divmod(r, T)
    part, rem = divmod(c, H * 64)
    h, d = divmod(rem, 64)
    print(f"b={b} t={t} part={'qkv'[part]} h={h} d={d} got={dqkv[r, c].item():.4f} ref={g[r, c].item():.4f}")
parts = torch.bincount((idx[:, 1] // (H * 64)), minlength=3).tolist() if idx.numel() else []
bs = torch.bincount(idx[:, 0] // T, minlength=B).tolist() if idx.numel() else []
print("by part", parts, "by batch", bs)
# per batch / part max error
for b in range(B):
    rows = slice(b * T, (b + 1) * T)
    print(b, int(lens[b]), [round(err[rows, i * H * 64:(i + 1) * H * 64].max().item(), 4) for i in range(3)],
          "ref max", [round(g[rows, i * H * 64:(i + 1) * H * 64].abs().max().item(), 3) for i in range(3)])
