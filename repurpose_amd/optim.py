"""Fused Adam over the model's flat parameter / gradient buffers (one HIP kernel per step).

Numerically the same update as ``torch.optim.Adam(params, lr, weight_decay)`` used by the
reference trainer (``main.py:190-191``, step at ``:369``): coupled L2 weight decay, bias-corrected
moments, ``denom = sqrt(v)/sqrt(bc2) + eps``.  Parameters without gradients (``reg_head``, which no
loss reaches) are skipped exactly as torch skips ``grad is None`` parameters.  In bf16 mode the
same kernel refreshes the bf16 operand copy of the weights, so the next forward needs no cast.
It is a ``torch.optim.Optimizer`` so LR schedulers (cosine, ``main.py:405-409``) drive it as usual.
"""
import torch

from . import kernels as K


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.model = model
        params = [p for n, p in model.named_parameters() if not n.startswith("reg_head.")]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._m = None
        self._v = None
        self._step = 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        model = self.model
        flat = model.flat_params()
        n = model.trainable_numel()
        g = model.flat_grads()
        if self._m is None or self._m.device != flat.device:
            self._m = torch.zeros(n, device=flat.device, dtype=torch.float32)
            self._v = torch.zeros(n, device=flat.device, dtype=torch.float32)
        self._step += 1
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        lp = None
        if model.compute_dtype == torch.bfloat16:
            lp = model.lowp_weights()[:n]
        K.adam_step(flat[:n], g[:n], self._m, self._v, grp["lr"], b1, b2, grp["eps"], grp["weight_decay"],
                    self._step, p_lp=lp)
        if lp is not None:
            model.mark_lowp_fresh()
        return loss

    def zero_grad(self, set_to_none: bool = False):
        # keep the .grad views into the flat buffer alive; zero it in one memset
        g = self.model.flat_grads()
        g.zero_()
