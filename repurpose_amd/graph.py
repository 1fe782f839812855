"""The training step captured once as a HIP graph and replayed (MI355X launch-overhead removal).

One eager step of the reference trainer (``main.py:331-369``: ``optimizer.zero_grad()``,
``model(batch)``, ``model.losses(...)``, ``loss.backward()``, ``optimizer.step()``) is ~450 kernel
launches from Python.  ``CapturedTrainStep`` records exactly that sequence once with
``torch.cuda.graph`` (hipStreamBeginCapture under the hood: every rp_* launch goes to torch's
current stream, which is the capture stream) and replays it with one ``hipGraphLaunch`` per step.

What changes per step without re-capture lives in one small device block that the host rewrites
(pinned staging slot -> async H2D on the step's stream) before each replay:

* word 0 — the dropout base: while the step is captured the model hands this word to every dropout
  launch as its ``seed_base`` argument (per call: the library keeps no dropout state, so another
  model in the process, or an eager step between replays, keeps its own streams), and each captured
  launch draws with ``rp_hash(base, site)`` — each replay has fresh dropout streams;
* words 1..6 — the Adam coefficients ``rp_adam_coefficients(lr, betas, eps, wd, step)``
  (``rp_adam_step_dev``), computed on the host from the optimizer's current ``param_groups`` and
  step count, so LR schedulers and the bias correction behave exactly as in eager mode (the
  updates are bitwise those of ``rp_adam_step`` with the same coefficients).

The batch tensors given at construction are the graph's static inputs: ``load(batch)`` copies a new
batch of the same shape into them.  With ``input_sets=2`` the step is captured twice, over two sets
of static inputs that the replays alternate between (one shared memory pool): a loader then writes
the NEXT step's batch straight into its set while the current step runs (``input_set(ahead=1)`` gives
the dict and the event after which it is free; ``RaggedBatch.to_device(out=...)`` fills it), and no
per-step copy into the static inputs is left (``main.py:302-313``'s per-batch ``.to(device)``).
Requirements: a ``FusedAdam`` optimizer, one device, at least one eager warm-up step (it allocates the
Adam moments and binds the gradient views outside the capture: allocations or fills captured into the
graph would re-run on every replay).

Data parallel (``capture_collectives=True``): the gradient all-reduce hooks of a
``distributed.GradAllReducer`` over RCCL (``backend="nccl"``) are captured with the rest of the
step — every bucket's ``ncclAllReduce`` becomes a graph node on RCCL's stream, forked from and
joined back into the step's stream at the points the eager backward issues and waits for it — so
an N-rank step is one ``hipGraphLaunch`` per rank, the same execution mode as one GPU.  The
warm-up steps run the collectives eagerly first (communicator set-up is not capturable).  A gloo
reducer (CPU collectives) cannot be captured: it raises.
"""
import numpy as np
import torch

from . import kernels as K
from .optim import FusedAdam

_SLOTS = 4  # pinned staging slots: the host runs at most this many steps ahead of the device


class CapturedTrainStep:
    def __init__(self, model, optimizer, batch, loss_fn=None, warmup=2, seed=None, capture_collectives=False,
                 input_sets=1):
        if not isinstance(optimizer, FusedAdam):
            raise TypeError("CapturedTrainStep needs repurpose_amd.optim.FusedAdam (device-side coefficients)")
        if int(warmup) < 1:
            raise ValueError("CapturedTrainStep: warmup must be >= 1 (the first step allocates the Adam moments "
                             "and binds the gradient buffer; captured allocations would re-run every replay)")
        hooks = list(model._grad_ready_hooks) + list(model._grad_done_hooks)
        if hooks:
            if not capture_collectives:
                raise RuntimeError("CapturedTrainStep: gradient all-reduce hooks are registered; pass "
                                   "capture_collectives=True to capture the RCCL all-reduces with the step")
            for h in hooks:
                owner = getattr(h, "__self__", None)
                if getattr(owner, "backend", None) != "nccl":
                    raise RuntimeError("CapturedTrainStep: only RCCL (backend 'nccl') gradient all-reduces can be "
                                       f"captured; got hook {h!r} (backend {getattr(owner, 'backend', None)!r})")
        self.model, self.opt = model, optimizer
        if int(input_sets) < 1:
            raise ValueError("CapturedTrainStep: input_sets must be >= 1")
        self.batch = batch  # input set 0
        self.sets = [batch] + [{k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in batch.items()}
                               for _ in range(int(input_sets) - 1)]
        self._next = 0                        # the set the next step() reads
        self._used = [None] * len(self.sets)  # event after the last step that read each set
        self.loss_fn = loss_fn or (lambda m, out: m.losses(*out)["cls_loss"] / out[1].shape[0])
        self.warmup = int(warmup)
        dev = model.flat_params().device
        self.device = dev
        self._dev = torch.zeros(8, device=dev, dtype=torch.int32)  # [seed, coef0..5, pad]
        self._coef = self._dev[1:7].view(torch.float32)
        self._host = [torch.zeros(8, dtype=torch.int32).pin_memory() for _ in range(_SLOTS)]
        self._ev = [None] * _SLOTS
        self._rng = np.random.default_rng(seed)
        self._graphs = [None] * len(self.sets)
        self._losses = [None] * len(self.sets)
        self.steps = 0

    @property
    def _graph(self):  # the first set's graph (tests, callers that check the capture happened)
        return self._graphs[0]

    def input_set(self, ahead=0):
        """(static input dict, event or None) of the step ``ahead`` calls of step() from now: write a batch
        into the dict on any stream after waiting for the event (the end of the last step that read it)."""
        k = (self._next + int(ahead)) % len(self.sets)
        return self.sets[k], self._used[k]

    def load(self, batch):
        """Copy a batch of the captured shapes into the static inputs the next step() reads."""
        dsts = self.sets[self._next]
        for k, v in batch.items():
            dst = dsts.get(k)
            if isinstance(dst, torch.Tensor):
                if dst.shape != v.shape:
                    raise ValueError(f"CapturedTrainStep.load: {k} shape {tuple(v.shape)} != captured {tuple(dst.shape)}")
                dst.copy_(v, non_blocking=True)

    def _eager(self, batch, fresh=False):
        if fresh:
            # the captured step: the backward writes every gradient, so the 210 MB zero fill of the
            # flat gradient buffer and the accumulate reads of the weight-gradient epilogues drop out
            self.model._grad_fresh = True
        else:
            self.opt.zero_grad()
        out = self.model(batch)
        loss = self.loss_fn(self.model, out)
        loss.backward()
        self.opt.step()
        return loss

    def _stage(self, stream):
        """Write this step's seed and Adam coefficients and enqueue their upload on ``stream``."""
        i = self.steps % _SLOTS
        if self._ev[i] is not None:
            self._ev[i].synchronize()  # the slot's previous upload has been consumed
        grp = self.opt.param_groups[0]
        b1, b2 = grp["betas"]
        coef = K.adam_coefficients(grp["lr"], b1, b2, grp["eps"], grp["weight_decay"], self.opt._step + 1)
        h = self._host[i].numpy()
        h[0] = np.int32(np.uint32(self._rng.integers(0, 2 ** 32)).view(np.int32))
        h[1:7] = np.asarray(coef, dtype=np.float32).view(np.int32)
        with torch.cuda.stream(stream):
            self._dev.copy_(self._host[i], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._ev[i] = ev

    def _capture(self, k):
        stream = torch.cuda.current_stream(self.device)
        self._stage(stream)
        g = torch.cuda.CUDAGraph()
        first = next((x for x in self._graphs if x is not None), None)
        self.model._seed_base = self._dev[0:1]
        self.opt._coef_dev = self._coef
        step0 = self.opt._step
        try:
            # the pool is private to the graph; the eager warm-up steps ran on the caller's stream
            torch.cuda.synchronize(self.device)
            # with RCCL hooks: thread-local capture mode, so the process group's watchdog thread may
            # keep querying its own (uncaptured) events while this thread captures
            mode = "thread_local" if self.model._grad_ready_hooks else "global"
            # a second input set's graph shares the first one's memory pool (replays never overlap)
            with torch.cuda.graph(g, pool=first.pool() if first is not None else None, capture_error_mode=mode):
                self._losses[k] = self._eager(self.sets[k], fresh=True)
        finally:
            self.model._seed_base = None
            self.model._grad_fresh = False
            self.opt._coef_dev = None
        self.opt._step = step0  # capture executed nothing; replay() counts the step
        self._graphs[k] = g

    def step(self):
        """One training step (eager for the first ``warmup`` calls, then graph replays); returns the
        loss tensor of this step (device scalar, valid until the next step)."""
        k = self._next
        stream = torch.cuda.current_stream(self.device)
        if self.steps < self.warmup:
            self.steps += 1
            loss = self._eager(self.sets[k])
        else:
            if self._graphs[k] is None:
                self._capture(k)
            else:
                self._stage(stream)
            self._graphs[k].replay()
            K.lnx_status()  # an exchange seam that gave up in an earlier replay fails loudly (host-mapped word)
            self.opt._step += 1
            if self.opt._step_t is not None:
                self.opt._step_t.fill_(float(self.opt._step))
            self.steps += 1
            loss = self._losses[k]
        if len(self.sets) > 1:
            ev = torch.cuda.Event()
            ev.record(stream)
            self._used[k] = ev
            self._next = (k + 1) % len(self.sets)
        return loss
