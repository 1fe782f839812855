"""Benchmark: feature-timesteps/sec (fwd+bwd) of the tri-modal MMCTransformer training step.

    python bench.py [--gpus N --steps K --warmup W]          (N > 1: under torch.distributed.run)

Workload (BASELINE.json metric): configs/Repurpose.yaml model — tri-modal
(512 + 2048 + 384 -> 512), 16 pre-LN encoder layers, 8 heads, d_ff 2048, heads + focal loss —
T = 2048, B = 8 sequences per GPU, bf16 MFMA compute (fp32 master weights, residual stream, LN,
softmax and accumulators), dropout 0.1 active.  One step = forward + losses + backward + gradient
all-reduce over RCCL (N > 1) + fused Adam (lr 1e-3, weight decay 1e-4).  Synthetic seeded inputs
with the feature statistics of SURVEY §8d, random-init weights (seed 1234); inputs resident in HBM.

Prints ONE JSON line (rank 0).  On one GPU the timed steps replay the step captured as a HIP graph
(repurpose_amd/graph.py; the DP path, N > 1, runs eager).  `roofline` is the dominant kernel's
achieved MFMA rate measured with HIP events on its launch stream over eager steps of the same
workload right after the timed region; `cpu_baseline` is the oracle
(stock torch CPU modules, fp32, the reference's own arithmetic) timed on this host.
"""
import argparse
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
# (together the SURVEY §8d attention count: 4*T*d forward + 8*T*d backward per token and layer)
KERNEL_FLOPS = {"attn_fwd": 4.0, "attn_bwd_dkdv": 6.0, "attn_bwd_dq": 2.0}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as a captured HIP graph (auto: on for one GPU)")
    ap.add_argument("--roofline-kernel", default="attn_bwd_dkdv", choices=list(KERNEL_FLOPS))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
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
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu if dp else 0)

    from repurpose_amd import kernels as K
    from repurpose_amd.MMCTransformer import MMCTransformer
    from repurpose_amd.distributed import GradAllReducer
    from repurpose_amd.optim import FusedAdam

    torch.manual_seed(1234)
    model = MMCTransformer(**MODEL_CFG, compute_dtype=args.dtype).to(dev).train()
    opt = FusedAdam(model, lr=1e-3, weight_decay=1e-4)
    reducer = GradAllReducer(model) if dp else None
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

    # one GPU: the whole step is captured once as a HIP graph and replayed (repurpose_amd/graph.py;
    # fresh dropout streams and the Adam step / LR per replay through a device parameter block); the
    # DP path (N > 1) keeps the eager step, whose all-reduce hooks overlap the backward
    use_graph = args.graph == "on" or (args.graph == "auto" and not dp)
    if use_graph:
        from repurpose_amd.graph import CapturedTrainStep
        runner = CapturedTrainStep(model, opt, batch, warmup=1, seed=1000 + rank)
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
    # per-kernel durations: the same kernels on the same data, timed with HIP events on their launch
    # stream over eager steps right after the timed region (a graph replay carries no per-launch
    # events, and ~100 event pairs per eager step would themselves add ~0.6 ms to the timed steps)
    kern_steps = min(args.steps, 5)
    K.timer_start(*KERNEL_FLOPS, "gemm_wgrad", "adam")
    for _ in range(kern_steps):
        eager_step()
    kern = K.timer_stop(detail=True)
    kern_ms = {n: v[0] for n, v in kern.items()}
    if dp:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    value = world * B * T * args.steps / elapsed
    if rank == 0:
        fpt = flops_per_timestep(T)
        H, dk = 8, 64
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_FP32_TFLOPS

        def roofline(name):
            ms = kern_ms.get(name)
            kflops = KERNEL_FLOPS[name] * B * H * T * T * dk
            ach = kflops / (ms * 1e-3) / 1e12 if ms else None
            return {"kernel": name, "bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                    "frac": (ach / peak) if ach else None, "traffic": traffic.get(name),
                    "traffic_unit": "bytes/launch (rocprofv3 PMC)", "avg_launch_ms": ms,
                    "flops_per_launch": kflops}

        # HBM bytes per launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
        # (scripts/pmc.sh + scripts/pmc_traffic.py; FETCH_SIZE doubled per the gfx950 correction)
        try:
            with open(os.path.join(ROOT, "profiles", "r02_pmc_traffic.json")) as f:
                traffic = {k: v["hbm_bytes"] for k, v in json.load(f).items()}
        except (OSError, ValueError, KeyError):
            traffic = {}
        roof = roofline(args.roofline_kernel)
        roof["step_tflops"] = fpt * value / world / 1e12
        roof["step_frac"] = roof["step_tflops"] / peak
        roof["other_kernels"] = [roofline(n) for n in KERNEL_FLOPS if n != args.roofline_kernel]
        # the weight-gradient GEMMs (split-K dW = dY^T X + bias gradient, every Linear of the step): the
        # largest GEMM time slice; algorithmic 2*N*K*T per launch summed over the timed launches
        avg, n_l, tot, fl = kern["gemm_wgrad"]
        if n_l and fl:
            ach = fl / (tot * 1e-3) / 1e12
            roof["other_kernels"].append({"kernel": "gemm_wgrad (all shapes)", "bound": "mfma", "achieved": ach,
                                          "peak": peak,
                                          "unit": "TFLOP/s", "launches_per_step": n_l / kern_steps,
                                          "ms_per_step": tot / kern_steps, "avg_launch_ms": avg,
                                          "frac": ach / peak})
        res = {"metric": METRIC, "value": value,
               "unit": "feature-timesteps/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded, SURVEY §8d statistics)",
               "config": {"workload": f"tri-modal MMCTransformer L=16 d=512 H=8 dff=2048, T={T}, B={B}/GPU, "
                                      f"train step fwd+focal+bwd+allreduce+Adam",
                          "model": "MMCTransformer (configs/Repurpose.yaml)", "global_batch": B * world,
                          "seq_len": T, "parallelism": f"dp{world}"},
               "loss": loss_val, "roofline": roof,
               "execution": "hip-graph replay of the captured step" if use_graph else "eager (per-launch)"}
        roof["kernel_timing"] = "HIP events on the launch stream over %d eager steps after the timed region" % kern_steps
        # SURVEY §8d reports the optimizer step separately: `value` includes it (whole train step)
        if kern.get("adam") and kern["adam"][0]:
            res["optimizer_ms_per_step"] = kern["adam"][2] / kern_steps
            res["ms_per_step_excl_optimizer"] = res["ms_per_step"] - res["optimizer_ms_per_step"]
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(T)
            res["speedup_vs_cpu"] = value / res["cpu_baseline"]["value"]
        print(json.dumps(res), flush=True)
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
