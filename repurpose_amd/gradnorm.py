"""Gradient-norm logging of the reference trainer (``main.py:345-367``) without its host syncs.

Every 10 iterations rank 0 of the reference walks ``named_modules()``, takes
``module.weight.grad.norm().item()`` (and the bias's) of every ``nn.Linear`` and then the total norm
over every parameter with a gradient, one ``.item()`` per tensor (≈ 100 + 218 device->host
synchronisations at L = 16).  ``grad_norms`` returns the same dict — same keys, same order — from
one ``rp_sumsq_batched`` pass (fp64 sums of squares, one workgroup per tensor, 64 tensors per
launch) and ONE device->host copy.

    # main.py:345-367, the drop-in:
    if is_main_process() and i % 10 == 0:
        wandb.log(grad_norms(model), step=global_step)

The values are the 2-norms in fp64 arithmetic (torch's ``norm()`` accumulates in fp32); the total
is ``sqrt(sum of every parameter's sum of squares)`` where the reference sums the squares of the
fp32-rounded per-parameter norms — agreement to a few fp32 ulps.
"""
import math

import torch

from . import kernels as K


def grad_norms(model):
    """{'grad_norm/<linear name>_weight', '..._bias', ..., 'grad_norm/total'} of ``model`` (or the
    DDP / MultiGPUStrategy wrapper's ``.module``), as python floats.  Gradients must be contiguous
    fp32 on the GPU (the HIP path has no CPU fallback)."""
    m = model.module if hasattr(model, "module") else model
    grads, index = [], {}

    def slot(g):
        key = (g.data_ptr(), g.numel(), g.device)
        if key not in index:
            index[key] = len(grads)
            grads.append(g)
        return index[key]

    named = []
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Linear):
            if mod.weight.grad is not None:
                named.append((f"grad_norm/{name}_weight", slot(mod.weight.grad)))
            if mod.bias is not None and mod.bias.grad is not None:
                named.append((f"grad_norm/{name}_bias", slot(mod.bias.grad)))
    total = [slot(p.grad) for p in m.parameters() if p.grad is not None]
    ss = K.sumsq_batched(grads).cpu().tolist() if grads else []
    out = {k: math.sqrt(ss[i]) for k, i in named}
    out["grad_norm/total"] = math.sqrt(sum(ss[i] for i in total))
    return out
