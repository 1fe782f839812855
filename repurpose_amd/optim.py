"""Fused Adam over the model's flat parameter / gradient buffers (one HIP kernel per step).

Numerically the same update as ``torch.optim.Adam(model.parameters(), lr, weight_decay)`` used by
the reference trainer (``main.py:190-191``, step at ``:369``): coupled L2 weight decay,
bias-corrected moments, ``denom = sqrt(v)/sqrt(bc2) + eps``.  Parameters without gradients
(``reg_head``, which no loss reaches) are skipped exactly as torch skips ``grad is None``
parameters.  In bf16 mode the same kernel refreshes the bf16 operand copy of the weights, so the
next forward needs no cast.  It is a ``torch.optim.Optimizer`` so LR schedulers (cosine,
``main.py:405-409``) drive it as usual.

Drop-in forms (all equivalent): ``FusedAdam(model.parameters(), lr=..., weight_decay=...)`` exactly
as the reference constructs ``optim.Adam`` (also through the ``wrap_model`` wrapper, whose
``parameters()`` are the module's), ``FusedAdam(model)`` or ``FusedAdam(wrapped_model)``.  The one
parameter group holds every parameter of the model in ``model.parameters()`` order, reg_head
included, so ``state_dict()`` has torch Adam's layout (per-parameter ``step`` / ``exp_avg`` /
``exp_avg_sq``, views of the flat moment buffers) and reference checkpoints (``main.py:521``,
``:729``) load with ``load_state_dict`` (``main.py:222``) and resume bit for bit.
"""
import torch

from . import kernels as K


def _owner(params):
    """The MMCTransformer whose flat buffer the given Parameters live in."""
    from .MMCTransformer import owner_of

    params = list(params)
    if not params:
        raise ValueError("FusedAdam: empty parameter list")
    if isinstance(params[0], dict):
        raise ValueError("FusedAdam: parameter groups are not supported (the model trains as one flat "
                         "buffer); pass model.parameters() or the model")
    model = owner_of(params[0])
    if model is None:
        raise ValueError("FusedAdam: the parameters do not belong to a repurpose_amd MMCTransformer")
    ids = {id(p) for p in model.parameters()}
    if any(id(p) not in ids for p in params):
        raise ValueError("FusedAdam: parameters from more than one model")
    return model


def _resolve(obj):
    from .MMCTransformer import MMCTransformer

    if isinstance(obj, MMCTransformer):
        return obj
    mod = getattr(obj, "module", None)
    if isinstance(mod, MMCTransformer):  # wrap_model's DistributedModel (or any .module wrapper)
        return mod
    if isinstance(obj, torch.nn.Module):
        raise ValueError(f"FusedAdam: {type(obj).__name__} is not an MMCTransformer")
    return _owner(obj)


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False):
        model = _resolve(params)
        self.model = model
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                        maximize=maximize)
        super().__init__(list(model.parameters()), defaults)
        self._m = None
        self._v = None
        self._step = 0
        self._step_t = None  # one shared CPU step tensor referenced by every trained param's state
        self._coef_dev = None  # graph capture (graph.py): coefficients read from this device buffer
        self._pre = []  # ranges already updated for the coming step by overlap_with's per-bucket hook
        self._pre_lp = None

    # ---------------------------------------------------------------- state <-> flat moments
    def _trained(self):
        """(param, flat offset, numel) of every parameter the kernel updates (all but reg_head)."""
        m = self.model
        out = []
        for n, p in m.named_parameters():
            if n.startswith("reg_head."):
                continue
            o, _ = m._layout[n]
            out.append((p, o, p.numel()))
        return out

    def _ensure(self):
        flat = self.model.flat_params()
        n = self.model.trainable_numel()
        if self._m is None or self._m.device != flat.device or self._m.numel() != n:
            m = torch.zeros(n, device=flat.device, dtype=torch.float32)
            v = torch.zeros(n, device=flat.device, dtype=torch.float32)
            if self._m is not None and self._m.numel() == n:
                m.copy_(self._m)
                v.copy_(self._v)
            self._m, self._v = m, v
            if self._step_t is not None:
                self._bind_state()
        return flat, n

    def _bind_state(self):
        """torch-Adam-layout state entries as views of the flat moment buffers."""
        for p, o, k in self._trained():
            self.state[p] = {"step": self._step_t, "exp_avg": self._m[o:o + k].view_as(p),
                             "exp_avg_sq": self._v[o:o + k].view_as(p)}

    def state_dict(self):
        """torch Adam's layout, detached from the live flat buffers: every parameter gets its OWN
        ``step`` tensor and its own copies of ``exp_avg`` / ``exp_avg_sq``.  (Inside the optimizer all
        trained parameters share one step tensor and view the flat moment buffers; handing those out
        would make a torch.optim.Adam that loads the dict — in process, or through torch.save /
        torch.load, which keep the sharing — add 1 to the shared step once per parameter.)"""
        sd = super().state_dict()
        sd["state"] = {i: {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                       for i, st in sd["state"].items()}
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._ensure()
        steps = set()
        with torch.no_grad():
            self._m.zero_()
            self._v.zero_()
            for p, o, k in self._trained():
                st = self.state.get(p)
                if not st:
                    continue
                self._m[o:o + k].copy_(st["exp_avg"].reshape(-1))
                self._v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"FusedAdam: parameters at different Adam steps {sorted(steps)}; the flat update "
                             "needs one step count")
        self._step = steps.pop() if steps else 0
        if self._step:
            self._step_t = torch.tensor(float(self._step))
            self._bind_state()
        else:
            self._step_t = None

    # ---------------------------------------------------------------- update
    def overlap_with(self, reducer):
        """Data parallel: update each gradient bucket as soon as its all-reduce has been waited for, on
        the step stream inside the backward (``GradAllReducer.on_bucket``), so the Adam of the first
        buckets runs while the last buckets are still being exchanged; ``step()`` then updates only what no
        bucket covered (nothing, when the buckets tile the gradient buffer) and does the bookkeeping.
        Bitwise the whole-buffer update (Adam is elementwise).  The update of a step is applied when its
        backward ends: every backward must be followed by ``step()`` with the gradients left as they are
        (the reference trainer's loop, ``main.py:331-369``; reading them for logging is fine).  A step
        captured as a HIP graph (``CapturedTrainStep``, its Adam coefficients on the device) keeps the
        whole-buffer update: with the per-bucket updates captured between the RCCL waits, the process
        group's watchdog failed on a captured event in 2 of 5 one-rank runs, never without them."""
        reducer.on_bucket = self._bucket_update

    def _coefs(self):
        grp = self.param_groups[0]
        if grp.get("amsgrad") or grp.get("maximize"):
            raise NotImplementedError("FusedAdam: amsgrad / maximize are not used by the reference trainer")
        b1, b2 = grp["betas"]
        return grp["lr"], b1, b2, grp["eps"], grp["weight_decay"]

    def _update(self, lo, hi, step, lp):
        flat, n = self._ensure()
        g = self.model.flat_grads()
        lr, b1, b2, eps, wd = self._coefs()
        K.adam_step(flat[lo:hi], g[lo:hi], self._m[lo:hi], self._v[lo:hi], lr, b1, b2, eps, wd, step,
                    p_lp=lp[lo:hi] if lp is not None else None, coef_dev=self._coef_dev)

    @torch.no_grad()
    def _bucket_update(self, lo, hi):
        n = self.model.trainable_numel()
        hi = min(hi, n)
        if lo >= hi or self._coef_dev is not None:  # being captured: step() updates the whole buffer
            return
        if any(lo < b and a < hi for a, b in self._pre):
            raise RuntimeError("FusedAdam.overlap_with: a gradient range was updated twice before step(); every "
                               "backward must be followed by optimizer.step()")
        if not self._pre:  # the step's first bucket: the bf16 copy (refreshed first when stale), once
            self._pre_lp = self._lowp()
        self._update(lo, hi, self._step + 1, self._pre_lp)
        self._pre.append((lo, hi))

    def _lowp(self):
        m = self.model
        return m.lowp_weights()[:m.trainable_numel()] if m.compute_dtype == torch.bfloat16 else None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        model = self.model
        self._coefs()
        flat, n = self._ensure()
        self._step += 1
        if self._step_t is None:
            self._step_t = torch.tensor(float(self._step))
            self._bind_state()
        else:
            self._step_t.fill_(float(self._step))
        # the whole buffer, or (overlap_with) the ranges no bucket has updated yet; the bf16 operand copy
        # is refreshed first when stale (e.g. after load_state_dict), by _lowp
        done, self._pre = sorted(self._pre), []
        lp = self._pre_lp if done else self._lowp()
        self._pre_lp = None
        lo = 0
        for a, b in done + [(n, n)]:
            if a > lo:
                self._update(lo, a, self._step, lp)
            lo = max(lo, b)
        if model.compute_dtype == torch.bfloat16:
            model.mark_lowp_fresh()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        # keep the .grad views into the flat buffer alive; zero it in one memset (the same values
        # as set_to_none: the next backward accumulates into zeros)
        self.model.flat_grads().zero_()
