"""Benchmark: feature-timesteps/sec (fwd+bwd) of the tri-modal MMCTransformer training step.

    python bench.py [--gpus N --steps K --warmup W]

With ``--gpus N`` (N > 1) and no ``WORLD_SIZE`` in the environment, this process starts the N ranks
itself — ``python -m torch.distributed.run --nproc-per-node N ... bench.py`` as a CHILD process,
before any GPU call — relays rank 0's JSON line and exits with the launcher's status (non-zero if
any rank fails); ``--dry-run`` prints the child command instead.  Under a launcher (``WORLD_SIZE``
set) ``--gpus`` must equal the world size.

Workload (BASELINE.json metric): configs/Repurpose.yaml model — tri-modal
(512 + 2048 + 384 -> 512), 16 pre-LN encoder layers, 8 heads, d_ff 2048, heads + focal loss —
T = 2048, B = 8 sequences per GPU, bf16 MFMA compute (fp32 master weights, residual stream, LN,
softmax and accumulators), dropout 0.1 active.  One step = forward + losses + backward + gradient
all-reduce over RCCL (N > 1) + fused Adam (lr 1e-3, weight decay 1e-4).  Synthetic seeded inputs
with the feature statistics of SURVEY §8d, random-init weights (seed 1234); inputs resident in HBM.

Prints ONE JSON line (rank 0).  At N = 1 the timed steps replay the step captured as a HIP graph
(repurpose_amd/graph.py); at N > 1 they run the eager DP step (the bucketed RCCL all-reduces issued
from the backward, as DDP does) unless ``--graph on`` asks for the captured DP step (its all-reduces
captured with the step: run on one rank only so far, so it stays opt-in).  ``ms_per_step`` is the MEAN
over the K timed steps (one barrier-bracketed region: a replay loop cannot be split per step without
syncs).  Every rank reports an exact checksum of its parameters after its last step
(``param_checksums``): data parallelism must leave them identical.  `roofline` is the dominant
kernel's achieved MFMA rate measured with HIP events on its launch stream over eager steps of the same
workload right after the timed region; `cpu_baseline` is the oracle (stock torch CPU modules, fp32, the reference's own
arithmetic) timed on this host.  At N = 1 the same run also reports `parity_mode` (the fp32 step,
the reference's precision, as a graph replay) and `fresh_batch` (the trainer-shaped loop: a new
pinned ragged batch per step through the device collate and CapturedTrainStep.load()).
"""
import argparse
import datetime
import json
import math
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

# BASELINE.json "metric", verbatim (the workload it is quoted on is config["workload"])
METRIC = "feature-timesteps/sec (fwd+bwd) tri-modal T=2048; 1/2/4/8 MI355X"
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODEL_CFG = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=16, text_num_layers=3,
                 cross_num_layers=3, num_heads=8)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3   # exact-f32 MFMA (the fp32 parity mode)
PEAK_HBM_GBS = 8000.0


def flops_per_timestep(T, L=16, d=512, dff=2048, din=2944):
    """Algorithmic FLOPs per timestep, fwd+bwd: 311,167,488 + 98,304*T at L=16."""
    per_layer_linear = 2 * d * 3 * d + 2 * d * d + 2 * 2 * d * dff
    lin = 3 * L * per_layer_linear
    attn = L * (4 * T * d + 8 * T * d)
    inp = 2 * (2 * din * d)
    fm = 3 * 2 * d * d
    cls = 3 * (2 * d * 256 + 2 * 256 * 256 + 2 * 256)
    reg = 2 * d * 256 + 2 * 256 * 256 + 2 * 256 * 2
    return lin + attn + inp + fm + cls + reg


# Algorithmic FLOPs per launch of the timed attention kernels (B sequences, H heads, T, dk):
#   attn_fwd       S = QK^T and O = PV                         4*B*H*T^2*dk
#   attn_bwd_dkdv  dV = P^T dO, dP = dO V^T, dK = dS^T Q        6*B*H*T^2*dk  (its S recompute excluded)
#   attn_bwd_dq    dQ = dS K                                    2*B*H*T^2*dk  (its S, dP recompute excluded)
#   attn_bwd_roles the delta pass + the ONE two-role launch that replaces dQ + dK/dV where each grid
#                  fills the CUs once (config 4: kernels.attn_bwd_uses_roles)   8*B*H*T^2*dk
# (together the SURVEY §8d attention count: 4*T*d forward + 8*T*d backward per token and layer)
KERNEL_FLOPS = {"attn_fwd": 4.0, "attn_bwd_dkdv": 6.0, "attn_bwd_dq": 2.0, "attn_bwd_roles": 8.0}


def synth_batch(B, T, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    v = torch.randn(B, T, 512, generator=g)
    v = v / v.norm(dim=-1, keepdim=True)
    a = torch.relu(torch.randn(B, T, 2048, generator=g))
    t = torch.randn(B, T, 384, generator=g)
    t = t / t.norm(dim=-1, keepdim=True)
    t = t * (torch.rand(B, T, 1, generator=g) > 0.3)
    lab = torch.zeros(B, T)
    for b in range(B):  # run-length segments, coverage ~0.35
        pos = 0
        while pos < T:
            gap = int(torch.randint(20, 120, (1,), generator=g))
            ln = int(torch.randint(10, 70, (1,), generator=g))
            lab[b, pos + gap: pos + gap + ln] = 1
            pos += gap + ln
    batch = {"visual_feats": v, "audio_feats": a, "text_feats": t,
             "masks": torch.ones(B, 1, T, dtype=torch.bool), "labels": lab,
             "segments": torch.rand(B, T, 2, generator=g) * 30}
    return {k: x.to(dev) for k, x in batch.items()}


def host_threads():
    """Threads for the CPU baseline: every CPU this process may run on (os.cpu_count()),
    capped by a cgroup CPU quota when the host enforces one (a GPU box's CPU share: threads beyond the
    quota only contend).  Returns (threads, note)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    note = f"os.cpu_count()={os.cpu_count()}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
            if quota < n:
                note += f", cgroup cpu.max quota {quota}"
                n = quota
    except (OSError, ValueError):
        pass
    return n, note


def cpu_baseline(T, budget_s=25.0):
    """Oracle (reference arithmetic on stock torch CPU modules, fp32) fwd+bwd at the metric shape,
    B = 1, train mode; bounded sample."""
    from oracle.mmct_oracle import MMCTransformer as Oracle
    threads, note = host_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(1234)
    m = Oracle(**MODEL_CFG).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4)
    b = synth_batch(1, T, torch.device("cpu"), 999)
    times = []
    t_start = time.perf_counter()
    steps = 0
    while True:
        t0 = time.perf_counter()
        opt.zero_grad()
        out = m(b)
        loss = m.losses(*out)["cls_loss"]
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
        steps += 1
        if time.perf_counter() - t_start > budget_s or steps >= 6:
            break
    timed = times[1:] if len(times) > 1 else times
    med = sorted(timed)[len(timed) // 2]
    try:
        model = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        model = [l.split(":", 1)[1].strip() for l in model.splitlines() if l.startswith("Model name")][0]
    except Exception:
        model = "unknown"
    return {"value": T / med, "unit": "feature-timesteps/sec", "cores": threads, "kind": "port",
            "sample": f"oracle fp32 train step (fwd+focal+bwd+Adam), L=16 tri-modal, B=1, T={T}; "
                      f"{len(timed)} timed of {steps} steps, median {med:.2f}s; cpu '{model}'; {threads} threads "
                      f"({note})"}


def child_command(args_list, n, port):
    """The launcher command of the N-rank run (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(args_list)


def launch(n, argv, dry_run=False):
    """Start the N ranks as a child process tree (never an exec: the parent has not touched the GPU and
    stays a plain parent), forward rank 0's JSON line to stdout and everything else to stderr as it
    arrives, return the launcher's exit status."""
    from repurpose_amd.distributed import find_free_port
    cmd = child_command([a for a in argv if a != "--dry-run"], n, find_free_port())
    if dry_run:
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    seen = False
    for line in proc.stdout:
        st = line.strip()
        if st.startswith("{") and '"metric"' in st:
            print(st, flush=True)
            seen = True
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    if rc == 0 and not seen:
        sys.stderr.write("bench.py: the ranks exited without a result line\n")
        return 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default WORLD_SIZE or 1")
    ap.add_argument("--dry-run", action="store_true", help="print the N-rank launcher command and exit")
    ap.add_argument("--no-parity-mode", action="store_true", help="skip the fp32 parity-mode replay (N = 1)")
    ap.add_argument("--no-fresh-batch", action="store_true", help="skip the fresh-batch loop (N = 1)")
    ap.add_argument("--fresh-batch", action="store_true", help="also run the fresh-batch loop at N > 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as a captured HIP graph (auto: at N = 1 only; on: also the DP step "
                         "with its RCCL all-reduces captured)")
    ap.add_argument("--roofline-kernel", default="attn_bwd_dkdv", choices=list(KERNEL_FLOPS))
    ap.add_argument("--no-adam-overlap", action="store_true",
                    help="N > 1: one whole-buffer Adam after the exchange instead of one per all-reduce bucket "
                         "right after its wait (FusedAdam.overlap_with)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        n = args.gpus or 1
        if n > 1 or args.dry_run:
            sys.exit(launch(n, sys.argv[1:], dry_run=args.dry_run))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ranks map to GPUs one to one; RP_DIST_BACKEND=gloo and more ranks than GPUs (ranks sharing a
    # device) exist only to rehearse the multi-process path on a one-GPU box
    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev
    # RP_BENCH_DP=1 runs the DP path (process group, all-reduce hooks, barriers) even at one rank:
    # a one-GPU rehearsal of what the driver's N > 1 runs execute over RCCL
    dp = world > 1 or os.environ.get("RP_BENCH_DP") == "1"
    if dp:
        torch.cuda.set_device(gpu)
        backend = os.environ.get("RP_DIST_BACKEND", "nccl")
        # bounded: a rank that never arrives, or a collective that never completes, ends the run with an
        # error and a stack after 5 minutes instead of the default 30
        tmo = datetime.timedelta(seconds=300)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    dev = torch.device("cuda", gpu if dp else 0)

    from repurpose_amd import kernels as K
    from repurpose_amd.MMCTransformer import MMCTransformer
    from repurpose_amd.distributed import GradAllReducer
    from repurpose_amd.optim import FusedAdam

    torch.manual_seed(1234)
    model = MMCTransformer(**MODEL_CFG, compute_dtype=args.dtype).to(dev).train()
    opt = FusedAdam(model, lr=1e-3, weight_decay=1e-4)
    reducer = GradAllReducer(model) if dp else None
    if reducer is not None and not args.no_adam_overlap:
        opt.overlap_with(reducer)  # each bucket's Adam right after its wait: overlaps the exchange's tail
    B, T = args.batch, args.seq_len
    batch = synth_batch(B, T, dev, 1000 + rank)

    def eager_step():
        opt.zero_grad()
        out = model(batch)
        loss = model.losses(*out)["cls_loss"] / B
        loss.backward()
        if reducer is not None:
            reducer.wait()
        opt.step()
        return loss

    # the whole step is captured once as a HIP graph and replayed (repurpose_amd/graph.py; fresh
    # dropout streams and the Adam step / LR per replay through a device parameter block).  The DP
    # step (bucketed all-reduces issued from the backward) can be captured with its RCCL collectives
    # (--graph on); by default N > 1 runs it eagerly, the path tested with two ranks.  A gloo
    # rehearsal (CPU collectives) cannot be captured.
    capturable = not dp or reducer.backend == "nccl"
    if args.graph == "on" and not capturable:
        raise SystemExit("bench.py: --graph on needs RCCL collectives (backend nccl), not gloo")
    use_graph = args.graph == "on" or (args.graph == "auto" and not dp)
    runner = None
    if use_graph:
        from repurpose_amd.graph import CapturedTrainStep
        # two static input sets (graph.py): the fresh-batch loop writes the next batch into the free one
        runner = CapturedTrainStep(model, opt, batch, warmup=1, seed=1000 + rank, capture_collectives=dp,
                                   input_sets=1 if dp else 2)
        step = runner.step
    else:
        step = eager_step

    for _ in range(max(args.warmup, 2 if use_graph else 0)):
        step()
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    loss_val = float(loss.item())
    ranks_seen = dist.get_world_size() if dp else 1
    per_rank = [elapsed]
    if dp:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if reducer.backend == "nccl" else "cpu")
        allt = [torch.zeros_like(t) for _ in range(ranks_seen)]
        dist.all_gather(allt, t)
        per_rank = [float(x.item()) for x in allt]
        elapsed = max(per_rank)
    # per-kernel durations: the same kernels on the same data, timed with HIP events on their launch
    # stream over eager steps right after the timed region (a graph replay carries no per-launch
    # events, and ~100 event pairs per eager step would themselves add ~0.6 ms to the timed steps)
    kern_steps = min(args.steps, 5)
    K.timer_start(*KERNEL_FLOPS, "gemm_wgrad", "adam")
    if reducer is not None:
        reducer.timing = []  # (before, after) events around every bucket's wait on the step stream
    for _ in range(kern_steps):
        eager_step()
    kern = K.timer_stop(detail=True)
    waits = []
    if reducer is not None:
        waits = [a.elapsed_time(b) for a, b in reducer.timing]
        reducer.timing = None
    kern_ms = {n: v[0] for n, v in kern.items()}
    value = world * B * T * args.steps / elapsed

    fresh = None
    if (world == 1 and not args.no_fresh_batch) or args.fresh_batch:
        fresh = fresh_batch_loop(runner, eager_step, batch, B, T, dev, rank, args.steps,
                                 world, dp)
    # exact parameter checksum after this rank's last step (int64 sum of the fp32 words and an
    # order-sensitive fold): data parallelism must leave every rank's parameters identical
    csum = param_checksum(model)
    checksums = [csum]
    if dp:
        allc = [None] * ranks_seen
        dist.all_gather_object(allc, csum)
        checksums = allc
        dist.barrier()

    if rank == 0:
        fpt = flops_per_timestep(T)
        H, dk = 8, 64
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_FP32_TFLOPS
        traffic = pmc_traffic(B, T)
        # where the step runs the two-role backward (config 4) the dQ / dK/dV kernels never run alone:
        # the roofline then names the launch the step does run
        rk = args.roofline_kernel
        if kern_ms.get(rk) is None and kern_ms.get("attn_bwd_roles") is not None and rk.startswith("attn_bwd"):
            rk = "attn_bwd_roles"
        roof = roofline_of(rk, kern_ms, B, T, peak, traffic)
        roof["step_tflops"] = fpt * value / world / 1e12
        roof["step_frac"] = roof["step_tflops"] / peak
        roof["other_kernels"] = [roofline_of(n, kern_ms, B, T, peak, traffic) for n in KERNEL_FLOPS
                                 if n != rk and kern_ms.get(n) is not None]
        # the weight-gradient GEMMs (every Linear's dW = dY^T X + bias gradient, grouped or split-K):
        # algorithmic 2*N*K*T per launch summed over the timed launches
        avg, n_l, tot, fl, _ = kern["gemm_wgrad"]
        if n_l and fl:
            ach = fl / (tot * 1e-3) / 1e12
            roof["other_kernels"].append({"kernel": "gemm_wgrad (all shapes)", "bound": "mfma", "achieved": ach,
                                          "peak": peak,
                                          "unit": "TFLOP/s", "launches_per_step": n_l / kern_steps,
                                          "ms_per_step": tot / kern_steps, "avg_launch_ms": avg,
                                          "frac": ach / peak})
        roof["kernel_timing"] = "HIP events on the launch stream over %d eager steps after the timed region" % kern_steps
        res = {"metric": METRIC, "value": value,
               "unit": "feature-timesteps/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded, SURVEY §8d statistics)",
               "config": {"workload": f"tri-modal MMCTransformer L=16 d=512 H=8 dff=2048, T={T}, B={B}/GPU, "
                                      f"train step fwd+focal+bwd+allreduce+Adam",
                          "model": "MMCTransformer (configs/Repurpose.yaml)", "global_batch": B * world,
                          "seq_len": T, "parallelism": f"dp{world}"},
               "loss": loss_val, "roofline": roof, "ranks_seen": ranks_seen,
               "timing": "mean ms over the K timed steps (barrier + synchronize on both sides, max over ranks)",
               "param_checksums": checksums,
               "rank_ms_per_step": [x / args.steps * 1e3 for x in per_rank],
               "rank_spread_ms": (max(per_rank) - min(per_rank)) / args.steps * 1e3,
               "execution": ("hip-graph replay of the captured step" + (" (RCCL all-reduces captured)" if dp else ""))
               if use_graph else "eager (per-launch)"}
        if dp:
            # where the DP step's time goes: the step stream's stalls on the bucket waits (the exchange not
            # hidden behind the backward), the weight-gradient launches of one step in issue order (the
            # grouped launch cut at each full round of tiles so early buckets' exchange overlaps the rest)
            _, n_w, _, _, each_w = kern["gemm_wgrad"]
            per = n_w // kern_steps if n_w else 0
            res["comm"] = {"backend": reducer.backend, "bucket_mb": reducer.bucket_elems * 4 / 2 ** 20,
                           "allreduce_bytes_per_step": model.trainable_numel() * 4,
                           "buckets_per_step": len(waits) // kern_steps if waits else 0,
                           "exposed_ms": sum(waits) / kern_steps if waits else None,
                           "max_bucket_wait_ms": max(waits) if waits else None,
                           "wgrad_launch_ms": each_w[-per:] if per else [],
                           "adam": "per bucket after its wait" if reducer.on_bucket is not None else "whole buffer",
                           "timing": "HIP events on the step stream around each bucket's wait, eager steps "
                                     "after the timed region"}
        # SURVEY §8d reports the optimizer step separately: `value` includes it (whole train step)
        if kern.get("adam") and kern["adam"][0]:
            res["optimizer_ms_per_step"] = kern["adam"][2] / kern_steps
            res["ms_per_step_excl_optimizer"] = res["ms_per_step"] - res["optimizer_ms_per_step"]
        if fresh is not None:
            res["fresh_batch"] = fresh
    if world == 1 and not args.no_parity_mode and args.dtype != "fp32":
        del runner, model, opt, batch
        torch.cuda.empty_cache()
        pm = parity_mode(B, T, dev, rank)
        if rank == 0:
            res["parity_mode"] = pm
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(T)
            res["speedup_vs_cpu"] = value / res["cpu_baseline"]["value"]
        print(json.dumps(res), flush=True)
    if dp:
        dist.destroy_process_group()


PMC_TRAFFIC_FILES = ("r06_pmc_traffic.json", "r06_pmc_traffic_T4096_B1.json", "r06_pmc_traffic_T1024_B8.json")


def pmc_traffic(B, T, files=PMC_TRAFFIC_FILES, root=None):
    """HBM bytes per launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes of THIS round's
    kernels (scripts/pmc.sh + scripts/pmc_traffic.py; FETCH_SIZE doubled per the gfx950 correction),
    keyed by the workload shape they were measured on: {} (traffic null) when no committed file
    holds a measurement at (B, T)."""
    for name in files:
        try:
            with open(os.path.join(root or os.path.join(ROOT, "profiles"), name)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        shape = d.get("shape") or {}
        if shape.get("B") == B and shape.get("T") == T:
            return {k: v["hbm_bytes"] for k, v in d.get("kernels", {}).items()}
    return {}


def param_checksum(model):
    """Exact checksum of the trained parameters: the int64 sum of their fp32 bit patterns and of the
    bit patterns weighted by position mod 65521 (order-sensitive)."""
    n = model.trainable_numel()
    w = model.flat_params()[:n].detach().contiguous().view(torch.int32).to(torch.int64)
    pos = torch.arange(n, device=w.device, dtype=torch.int64) % 65521
    return [int(w.sum().item()), int((w * pos).sum().item())]


def roofline_of(name, kern_ms, B, T, peak, traffic, H=8, dk=64):
    ms = kern_ms.get(name)
    kflops = KERNEL_FLOPS[name] * B * H * T * T * dk
    ach = kflops / (ms * 1e-3) / 1e12 if ms else None
    return {"kernel": name, "bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
            "frac": (ach / peak) if ach else None, "traffic": traffic.get(name),
            "traffic_unit": "bytes/launch (rocprofv3 PMC)", "avg_launch_ms": ms,
            "flops_per_launch": kflops}


def parity_mode(B, T, dev, rank, warmup=2, steps=5):
    """The same train step in the reference's precision (fp32 throughout: exact-f32 MFMA, the 1e-3
    parity mode), as a graph replay; the dK/dV kernel timed with HIP events against the fp32 MFMA peak."""
    from repurpose_amd import kernels as K
    from repurpose_amd.MMCTransformer import MMCTransformer
    from repurpose_amd.optim import FusedAdam
    from repurpose_amd.graph import CapturedTrainStep

    torch.manual_seed(1234)
    model = MMCTransformer(**MODEL_CFG, compute_dtype="fp32").to(dev).train()
    opt = FusedAdam(model, lr=1e-3, weight_decay=1e-4)
    batch = synth_batch(B, T, dev, 1000 + rank)
    runner = CapturedTrainStep(model, opt, batch, warmup=1, seed=1000 + rank)
    for _ in range(warmup):
        runner.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    K.timer_start("attn_bwd_dkdv", "attn_bwd_roles")
    opt.zero_grad()
    out = model(batch)
    (model.losses(*out)["cls_loss"] / B).backward()
    kern = K.timer_stop()
    rk = "attn_bwd_dkdv" if kern.get("attn_bwd_dkdv") is not None else "attn_bwd_roles"
    ms = kern.get(rk)
    fl = KERNEL_FLOPS[rk] * B * 8 * T * T * 64
    res = {"dtype": "fp32", "steps": steps, "warmup": warmup, "ms_per_step": el / steps * 1e3,
           "value": B * T * steps / el, "unit": "feature-timesteps/sec",
           "execution": "hip-graph replay of the captured step",
           "roofline": {"kernel": rk, "bound": "mfma", "avg_launch_ms": ms,
                        "achieved": fl / (ms * 1e-3) / 1e12 if ms else None, "peak": PEAK_FP32_TFLOPS,
                        "unit": "TFLOP/s", "frac": fl / (ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS if ms else None}}
    del runner, model, opt, batch
    torch.cuda.empty_cache()
    return res


def ragged_pool(B, T, n, seed, f32=True):
    """n host batches in the layout the trainer's DataLoader hands over (repurpose_amd.data.collate_ragged:
    each modality's rows concatenated — the feature files hold fp16 CLIP, fp32 PANNs and fp64 text rows —
    labels and segments), pinned as a DataLoader's pin_memory thread leaves them.  ``f32`` (default): the
    workers also convert the rows to fp32 (collate_ragged(f32=True), as the reference's collate builds fp32
    batches), so the loop's device work is DMA only; otherwise the fp16 / fp64 rows go to rp_pad_rows."""
    from repurpose_amd.data import RaggedBatch
    pool = []
    for i in range(n):
        b = synth_batch(B, T, torch.device("cpu"), seed + i)
        vis = b["visual_feats"].reshape(B * T, -1).numpy().astype("float16")
        txt = b["text_feats"].reshape(B * T, -1).numpy().astype("float64")
        rows = {"visual": vis.astype("float32") if f32 else vis,
                "audio": b["audio_feats"].reshape(B * T, -1).numpy(),
                "text": txt.astype("float32") if f32 else txt,
                "labels": b["labels"].reshape(B * T, 1).numpy(),
                "segments": b["segments"].reshape(B * T, 2).numpy()}
        offs = {k: (torch.arange(B + 1) * T).numpy() for k in rows}
        pool.append(RaggedBatch([f"v{j}" for j in range(B)], [T] * B, rows, offs).pin())
    return pool


def fresh_batch_loop(runner, eager_step, batch, B, T, dev, rank, steps, world, dp, pool_n=3):
    """The trainer-shaped loop (main.py:302-313): every step a NEW batch goes host -> device (pinned
    ragged rows on a copy stream, overlapped with the previous step: fp32 rows by DMA straight into
    their padded places, fp16 / fp64 rows padded and converted by rp_pad_rows).  With a two-set captured
    step (CapturedTrainStep(input_sets=2)) the batch is written straight into the static inputs the
    next replay reads, so no copy is left between the replays; otherwise it is staged and copied in.
    Returns the loop's throughput beside the H2D volume."""
    pool = ragged_pool(B, T, pool_n, 5000 + 97 * rank)
    copy = torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)
    h2d = sum(v.numel() * v.element_size() for v in pool[0].rows.values())
    direct = runner is not None and len(runner.sets) > 1
    done = [0]  # steps run so far

    def stage(j):  # global step j's batch
        with torch.cuda.stream(copy):
            if direct:
                dst, used = runner.input_set(ahead=j - done[0])
                if used is not None:
                    copy.wait_event(used)  # the last step that read this set has finished
                nb = pool[j % pool_n].to_device(dev, out=dst)
            else:
                nb = pool[j % pool_n].to_device(dev)
            ev = torch.cuda.Event()
            ev.record(copy)
        return nb, ev

    def run(nxt):
        nb, ev = nxt
        main.wait_event(ev)
        if direct:
            runner.step()
        else:
            for v in nb.values():
                if torch.is_tensor(v):
                    v.record_stream(main)
            if runner is not None:
                runner.load(nb)
                runner.step()
            else:
                for k, v in nb.items():
                    if torch.is_tensor(v) and k in batch:
                        batch[k].copy_(v, non_blocking=True)
                eager_step()
        done[0] += 1

    nxt = stage(0)
    for i in range(2):  # warm-up: pinned pool, pad kernels, allocator
        cur, nxt = nxt, stage(i + 1)
        run(cur)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        cur, nxt = nxt, stage(i + 3)
        run(cur)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dp:
        t = torch.tensor([el], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return {"value": world * B * T * steps / el, "unit": "feature-timesteps/sec", "ms_per_step": el / steps * 1e3,
            "steps": steps, "h2d_bytes_per_step": h2d, "h2d_source": "pinned ragged rows (visual, audio, text, labels, "
            "segments; converted to fp32 by the loader workers as the reference's collate does) on a copy stream, "
            "overlapped with the previous replay: every modality by DMA into its padded place, masks from the host "
            "lengths",
            "into": "the captured step's free static input set (no copy between replays)" if direct
            else "staging tensors, copied into the step's inputs", "pool": pool_n}


if __name__ == "__main__":
    main()
