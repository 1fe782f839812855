"""Drop-in ``utils/distributed.py`` (reference) for one process per MI355X, RCCL over xGMI.

API kept from the reference (``utils/distributed.py``): ``MultiGPUStrategy(strategy, backend,
timeout, find_unused_parameters)`` with ``setup() -> bool`` (:355-389), ``wrap_model`` (:396-433,
returns a wrapper exposing ``.module`` as the trainer needs at ``main.py:323-326``),
``create_dataloader`` (:435-473, ``DistributedSampler`` partitioning), ``reduce_tensor`` (:475-498),
``barrier``, ``cleanup``, ``print_setup_info``, ``get_effective_batch_size``, ``save_checkpoint`` /
``load_checkpoint``; free functions ``setup_distributed``, ``cleanup_distributed``, ``get_rank``,
``get_world_size``, ``is_main_process``, ``get_device``, ``detect_slurm_env``,
``auto_select_strategy`` and the ``DistributedManager`` context manager.

What changes underneath (MI355X-first, not a translation of torch DDP):

* gradients live in ONE flat fp32 buffer (``MMCTransformer.flat_grads``).  ``GradAllReducer``
  receives "this contiguous range is final" callbacks from the hand-written backward (encoder
  layers finish in reverse order), coalesces them into ~``bucket_mb`` buckets and issues one
  asynchronous RCCL all-reduce per bucket (``backend="nccl"`` is RCCL on ROCm) while the backward
  of earlier layers keeps the GPU busy; the last wait is enqueued (stream-ordered, no host sync)
  at the end of backward, so ``.grad`` is averaged when ``loss.backward()`` returns, as with DDP;
* the DDP per-forward buffer broadcast (the constant ``pe`` table) and the unused-parameter
  bitmap all-reduce are dropped: the unused set (``reg_head``) is static;
* parameters are broadcast from rank 0 once, as one flat buffer, at wrap time (C2).
"""
import datetime
import logging
import os
import socket
import threading
import time
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

log = logging.getLogger(__name__)


def find_free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def detect_slurm_env() -> Dict[str, Any]:
    """Reference ``utils/distributed.py:32-74``: torchrun's ``RANK``/``WORLD_SIZE`` win over SLURM
    (:41-45); SLURM is used only with ``SLURM_PROCID``, ``SLURM_NTASKS`` and ``SLURM_NTASKS > 1``
    (:46); the master is ``SLURM_LAUNCH_NODE_IPADDR`` (default ``localhost``), replaced by the first
    node of ``SLURM_STEP_NODELIST`` when set (compressed ``node[01-04]`` -> ``node01``, :51-63);
    port ``MASTER_PORT`` or 29500 (:66)."""
    env = os.environ
    if "RANK" in env and "WORLD_SIZE" in env:
        return {"is_slurm": False}
    if not ("SLURM_PROCID" in env and "SLURM_NTASKS" in env and int(env.get("SLURM_NTASKS", 1)) > 1):
        return {"is_slurm": False}
    master = env.get("SLURM_LAUNCH_NODE_IPADDR", "localhost")
    nodes = env.get("SLURM_STEP_NODELIST")
    if nodes is not None:
        if "[" in nodes:
            head, rest = nodes.split("[", 1)
            master = head + rest.split("-")[0].split(",")[0]
        else:
            master = nodes.split(",")[0]
    return {"is_slurm": True, "rank": int(env["SLURM_PROCID"]), "world_size": int(env["SLURM_NTASKS"]),
            "local_rank": int(env.get("SLURM_LOCALID", 0)), "master_addr": master,
            "master_port": int(env.get("MASTER_PORT", 29500))}


def setup_distributed(rank: int, world_size: int, backend: str = "nccl", master_addr: str = "127.0.0.1",
                      master_port: Optional[str] = None, timeout: int = 1800) -> bool:
    """Initialise the process group and run the reference's comm self-test (:180-193)."""
    try:
        s = detect_slurm_env()
        if s["is_slurm"]:
            rank, world_size, local_rank = s["rank"], s["world_size"], s["local_rank"]
            master_addr, master_port = s["master_addr"], str(s["master_port"])
        else:
            rank = int(os.environ.get("RANK", rank))
            world_size = int(os.environ.get("WORLD_SIZE", world_size))
            master_addr = os.environ.get("MASTER_ADDR", master_addr)
            ndev = torch.cuda.device_count() if torch.cuda.is_available() else 1
            local_rank = int(os.environ.get("LOCAL_RANK", rank % max(ndev, 1)))
            master_port = master_port or os.environ.get("MASTER_PORT") or str(find_free_port())
        os.environ.update(MASTER_ADDR=master_addr, MASTER_PORT=str(master_port), RANK=str(rank),
                          WORLD_SIZE=str(world_size), LOCAL_RANK=str(local_rank))
        kw = {}
        if backend == "nccl":
            dev = local_rank % torch.cuda.device_count()
            torch.cuda.set_device(dev)
            kw["device_id"] = torch.device("cuda", dev)
        dist.init_process_group(backend=backend, rank=rank, world_size=world_size,
                                timeout=datetime.timedelta(seconds=timeout), **kw)
        probe = torch.ones(1, device=torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else "cpu")
        dist.all_reduce(probe)
        if abs(probe.item() - world_size) > 1e-6:
            log.error("distributed self-test failed: %s != %s", probe.item(), world_size)
            return False
        return True
    except Exception as e:  # the reference reports and returns False (:197-202)
        log.error("failed to set up distributed training: %s", e)
        return False


def cleanup_distributed():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_main_process() -> bool:
    return get_rank() == 0


def get_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    return torch.device("cpu")


# ---------------------------------------------------------------------------------------------
class GradAllReducer:
    """Bucketed, backward-overlapped gradient averaging over a flat gradient buffer.

    ``ready(lo, hi)`` is called by the backward whenever flat range [lo, hi) holds final gradients
    (ranges arrive in reverse layout order); ``finish()`` closes the step: it waits for every bucket
    (stream-ordered under RCCL), so the gradients are final when ``backward()`` returns, as under DDP.
    ``on_bucket(lo, hi)``, when set (``FusedAdam.overlap_with``), runs right after bucket [lo, hi)'s wait
    on the step stream, before the next bucket's: the optimizer update of the first buckets then
    overlaps the all-reduce of the last ones.  ``timing`` (a list, bench.py): a (before, after) pair
    of HIP events around every wait, i.e. the time the step stream stalls on the exchange.  Works with
    any object exposing ``flat_grads()``, ``trainable_numel()`` and ``_grad_ready_hooks``.
    """

    def __init__(self, model, bucket_mb: float = 25.0, group=None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket_elems = max(1, int(bucket_mb * 2 ** 20 / 4))
        self.backend = dist.get_backend(group)
        self.pending = None  # [lo, hi) not yet launched
        self.works = []
        self.launched = []
        self.on_bucket = None
        self.timing = None
        model._grad_ready_hooks = [self.ready]
        model._grad_done_hooks = [self.finish]

    def _launch(self, lo, hi):
        g = self.model.flat_grads()[lo:hi]
        if self.backend == "nccl":
            # one rank: AVG == SUM, and RCCL runs a one-rank AVG as a scaling pass over the bucket
            # (oneRankReduce<PreMulSum>: 0.41 ms per step at the metric shape) where an in-place SUM
            # moves nothing
            op = dist.ReduceOp.AVG if self.world > 1 else dist.ReduceOp.SUM
            w = dist.all_reduce(g, op=op, group=self.group, async_op=True)
            self.works.append((w, None, lo, hi))
        else:  # gloo has no AVG
            w = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self.works.append((w, g, lo, hi))
        self.launched.append((lo, hi))

    def ready(self, lo, hi):
        n = self.model.trainable_numel()
        hi = min(hi, n)
        if lo >= hi:
            return
        if self.pending is None:
            self.pending = [lo, hi]
        elif hi == self.pending[0]:  # ranges arrive in reverse layout order
            self.pending[0] = lo
        elif lo == self.pending[1]:
            self.pending[1] = hi
        else:
            self._launch(*self.pending)
            self.pending = [lo, hi]
        if self.pending[1] - self.pending[0] >= self.bucket_elems:
            self._launch(*self.pending)
            self.pending = None

    def finish(self):
        if self.pending is not None:
            self._launch(*self.pending)
            self.pending = None
        works, self.works = self.works, []
        for w, g, lo, hi in works:
            e0 = None
            if self.timing is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            w.wait()  # stream-ordered for RCCL: no host synchronisation
            if g is not None:
                g.div_(self.world)
            if e0 is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                self.timing.append((e0, e1))
            if self.on_bucket is not None:
                self.on_bucket(lo, hi)

    def wait(self):
        self.finish()
        covered = sorted(self.launched)
        self.launched = []
        return covered


class DistributedModel(nn.Module):
    """What ``wrap_model`` returns under DDP: ``.module`` is the drop-in model, forward delegates,
    gradients are averaged by a ``GradAllReducer`` inside backward."""

    def __init__(self, module, bucket_mb=25.0, broadcast=True):
        super().__init__()
        self.module = module
        if broadcast:
            flat = module.flat_params()
            dist.broadcast(flat, src=0)
        self.reducer = GradAllReducer(module, bucket_mb=bucket_mb)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


def _split_batch(batch, n):
    """Per-replica pieces of a batch dict: every tensor cut along dim 0 as ``torch.chunk`` cuts it
    (nn.DataParallel's scatter: ceil-sized pieces, fewer when the batch is short); other values are
    shared.  Returns the list of piece dicts (at most n)."""
    sizes = {v.shape[0] for v in batch.values() if torch.is_tensor(v) and v.dim() > 0}
    if len(sizes) != 1:
        raise ValueError(f"DataParallelModel: batch tensors disagree on dim 0 ({sorted(sizes)})")
    B = sizes.pop()
    step = -(-B // max(1, min(n, B)))
    starts = list(range(0, B, step))
    return [{k: (v[s:s + step] if torch.is_tensor(v) and v.dim() > 0 else v) for k, v in batch.items()}
            for s in starts]


class DataParallelModel(nn.Module):
    """``strategy: dp`` (reference ``utils/distributed.py:409-413``, ``nn.DataParallel``): one
    process drives several GPUs.  The batch is cut along dim 0 (``_split_batch``), replica i runs its
    piece on ``device_ids[i]``, the six outputs are gathered onto ``output_device`` along dim 0 (with
    autograd, ``torch.nn.parallel.gather``), so ``.module.losses(*out)`` and ``loss.backward()`` read
    as the reference trainer's (``main.py:323-326``) and the gradient is that of the whole batch.

    Underneath, not ``nn.DataParallel``'s per-forward module replication: the replicas are built once
    (flat-buffer models, ``MMCTransformer._build_flat``) and refreshed by one device-to-device copy of
    the flat fp32 parameters per forward; their flat gradients are summed into ``.module``'s with one
    copy + add each, queued on the autograd engine to run once the whole backward is done (every
    replica's HIP backward has written its buffer by then).  A ``device_ids`` entry may repeat (two
    replicas on one GPU: how the one-GPU box tests this path)."""

    def __init__(self, module, device_ids=None, output_device=None):
        super().__init__()
        if device_ids is None:
            device_ids = list(range(torch.cuda.device_count()))
        if not device_ids:
            raise RuntimeError("DataParallelModel: no GPU")
        self.device_ids = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d) for d in device_ids]
        self.output_device = self.device_ids[0] if output_device is None else torch.device(
            "cuda", output_device) if isinstance(output_device, int) else torch.device(output_device)
        self.module = module.to(self.device_ids[0])
        self._replicas = []  # replicas 1.. (plain list: not sub-modules, so state_dict / parameters are .module's)
        self._queued = False
        self._done_events = []
        self._lock = threading.Lock()  # replica hooks run on the autograd engine's per-device threads

    def _replica(self, i):
        import copy
        while len(self._replicas) < i:
            j = len(self._replicas) + 1
            r = copy.deepcopy(self.module).to(self.device_ids[j])
            r._grad_ready_hooks = []
            r._grad_done_hooks = [self._on_replica_done]
            self._replicas.append(r)
        return self._replicas[i - 1]

    def _on_replica_done(self):
        # the replica's backward was enqueued on its device's current stream (this hook runs at its
        # end, on the engine's thread for that device): an event there orders the cross-device read
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        with self._lock:  # check-then-set and the event list shared by the per-device engine threads
            self._done_events.append(ev)
            queue = not self._queued
            self._queued = True
        if queue:  # once per backward: after the engine has run every replica's backward
            torch.autograd.Variable._execution_engine.queue_callback(self._reduce)

    def _reduce(self):
        with self._lock:
            self._queued = False
            events, self._done_events = self._done_events, []
        g0 = self.module.flat_grads()
        n = self.module.trainable_numel()
        s0 = torch.cuda.current_stream(g0.device)
        for ev in events:  # device 0 reads the replicas' gradients only once they are written
            s0.wait_event(ev)
        with torch.cuda.stream(s0):
            for r in self._active:
                g0[:n].add_(r.flat_grads()[:n].to(g0.device, non_blocking=True))

    def forward(self, batch):
        pieces = _split_batch(batch, len(self.device_ids))
        if len(pieces) == 1:
            return self.module({k: v.to(self.device_ids[0]) if torch.is_tensor(v) else v for k, v in batch.items()})
        src = self.module.flat_params()
        self._active = []
        outs = []
        for i, piece in enumerate(pieces):
            dev = self.device_ids[i]
            m = self.module if i == 0 else self._replica(i)
            if i:
                m.train(self.module.training)
                with torch.no_grad():
                    m.flat_params().copy_(src)
                    m.flat_grads().zero_()
                self._active.append(m)
            with torch.cuda.device(dev):
                outs.append(m({k: v.to(dev, non_blocking=True) if torch.is_tensor(v) else v for k, v in piece.items()}))
        return tuple(torch.nn.parallel.gather(outs, self.output_device, dim=0))


class MultiGPUStrategy:
    """Reference ``utils/distributed.py:242-625`` with RCCL underneath."""

    def __init__(self, strategy: str = "auto", backend: str = "nccl", timeout: int = 1800,
                 find_unused_parameters: bool = False):
        self.logger = log
        self.strategy = strategy
        self.backend = backend
        self.timeout = timeout
        self.find_unused_parameters = find_unused_parameters  # static unused set: nothing to find
        self.world_size, self.rank, self.local_rank = 1, 0, 0
        self.device = torch.device("cpu")
        self.is_distributed = False
        self.slurm_info = detect_slurm_env()
        if strategy == "auto":
            self.strategy = self._auto_detect_strategy()
        self._setup_device_info()

    def _auto_detect_strategy(self) -> str:
        """Reference :279-311, same order: no GPU -> single; SLURM with > 1 task -> ddp; torchrun's
        RANK / WORLD_SIZE with WORLD_SIZE > 1 -> ddp; one GPU -> single; several -> ddp."""
        if not torch.cuda.is_available():
            return "single"
        if self.slurm_info["is_slurm"] and self.slurm_info["world_size"] > 1:
            return "ddp"
        if "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
            return "ddp"
        return "ddp" if torch.cuda.device_count() > 1 else "single"

    def _setup_device_info(self):
        """Reference :313-353.  'dp' (nn.DataParallel in the reference, :409-413): one process on
        cuda:0 that ``wrap_model`` spreads over every visible GPU (``DataParallelModel``)."""
        if self.strategy in ("single", "dp"):
            self.device = get_device()
            self.world_size, self.rank, self.local_rank = 1, 0, 0
            return
        self.is_distributed = True
        ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
        if self.slurm_info["is_slurm"]:
            self.rank, self.world_size = self.slurm_info["rank"], self.slurm_info["world_size"]
            self.local_rank = self.slurm_info["local_rank"]
        elif "RANK" in os.environ:
            self.rank = int(os.environ["RANK"])
            self.world_size = int(os.environ["WORLD_SIZE"])
            self.local_rank = int(os.environ.get("LOCAL_RANK", self.rank % max(ndev, 1)))
        else:
            self.rank, self.local_rank = 0, 0
            self.world_size = ndev if ndev else 1
        # cuda:{local_rank} as the reference (:349-350); ranks beyond the device count (a gloo
        # rehearsal of N ranks on one GPU) share devices round robin
        self.device = torch.device("cuda", self.local_rank % ndev) if ndev else torch.device("cpu")

    def setup(self) -> bool:
        if self.strategy == "ddp" and self.world_size > 1:
            s = self.slurm_info
            addr = s["master_addr"] if s["is_slurm"] else os.environ.get("MASTER_ADDR", "127.0.0.1")
            port = str(s["master_port"]) if s["is_slurm"] else os.environ.get("MASTER_PORT")
            ok = setup_distributed(self.rank, self.world_size, self.backend, addr, port, self.timeout)
            if not ok:  # reference falls back to DataParallel and reports success (:379-386)
                self.logger.warning("DDP setup failed, falling back to DataParallel")
                self.strategy, self.is_distributed, self.world_size, self.rank = "dp", False, 1, 0
                return True
            return True
        return True

    def cleanup(self):
        if self.strategy == "ddp":
            cleanup_distributed()

    def wrap_model(self, model: nn.Module) -> nn.Module:
        model = model.to(self.device)
        if self.strategy == "dp" and torch.cuda.is_available() and torch.cuda.device_count() > 1:
            return DataParallelModel(model)
        if self.strategy == "ddp" and self.world_size > 1:
            return DistributedModel(model)
        return model

    def create_dataloader(self, dataset, batch_size: int, shuffle: bool = True, num_workers: int = 0, **kwargs):
        from torch.utils.data import DataLoader
        from torch.utils.data.distributed import DistributedSampler
        sampler = None
        if self.strategy == "ddp" and self.world_size > 1:
            sampler = DistributedSampler(dataset, num_replicas=self.world_size, rank=self.rank, shuffle=shuffle)
            shuffle = False
        return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, sampler=sampler, num_workers=num_workers,
                          pin_memory=torch.cuda.is_available(), **kwargs)

    def reduce_tensor(self, tensor: torch.Tensor, average: bool = True) -> torch.Tensor:
        if self.strategy != "ddp" or self.world_size <= 1:
            return tensor
        out = tensor.clone()
        dist.all_reduce(out, op=dist.ReduceOp.SUM)
        if average:
            out /= self.world_size
        return out

    def barrier(self):
        if self.strategy == "ddp" and self.world_size > 1:
            dist.barrier()

    def print_setup_info(self):
        if is_main_process():
            self.logger.info("strategy=%s world=%d rank=%d device=%s backend=%s", self.strategy.upper(),
                             self.world_size, self.rank, self.device, self.backend)

    def save_checkpoint(self, state_dict: Dict[str, Any], filepath: str):
        if not is_main_process():
            return
        m = state_dict.get("model")
        if hasattr(m, "module"):
            state_dict["model"] = m.module.state_dict()
        torch.save(state_dict, filepath)

    def load_checkpoint(self, model: nn.Module, filepath: str, optimizer=None) -> Dict[str, Any]:
        ckpt = torch.load(filepath, map_location=self.device, weights_only=True)
        if "model" in ckpt:
            (model.module if hasattr(model, "module") else model).load_state_dict(ckpt["model"])
        if optimizer is not None and "optimizer" in ckpt:
            optimizer.load_state_dict(ckpt["optimizer"])
        return ckpt

    def get_effective_batch_size(self, batch_size: int) -> int:
        return batch_size * self.world_size if self.strategy == "ddp" else batch_size


def auto_select_strategy() -> str:
    """Reference :628-657 recommends dp for 2-4 GPUs; on MI355X one process per GPU is always used."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        return "single"
    return "ddp"


class DistributedManager:
    def __init__(self, strategy: str = "auto", backend: str = "nccl"):
        self.strategy_manager = MultiGPUStrategy(strategy, backend)

    def __enter__(self):
        if not self.strategy_manager.setup():
            raise RuntimeError("Failed to setup distributed training")
        return self.strategy_manager

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.strategy_manager.cleanup()
