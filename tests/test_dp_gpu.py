"""The data-parallel step as the driver's multi-GPU bench runs it (config 3: DDP over RCCL,
``/root/reference/utils/distributed.py:415-428`` around ``main.py:331-386``), on the one-GPU box:

* ``bench.py --gpus 2`` end to end: the launcher starts two ranks (gloo: RCCL refuses two ranks on one
  device), each runs the eager DP step with the bucketed all-reduce; one JSON line, ``n_gpus`` and
  ``ranks_seen`` 2, a finite loss and bitwise identical parameters on both ranks after the last step;
* the all-reduce buckets of every weight-gradient schedule the DP backward can take (the default
  256 + 512 tile cut of the grouped launch, ``RP_WGRAD_GROUP_LAYERS`` cuts, per-layer split-K, fp32)
  tile ``[0, trainable_numel)`` exactly once, in reverse layout order;
* the captured DP step (``CapturedTrainStep(capture_collectives=True)``: RCCL all-reduces captured into
  the HIP graph, tile cut active, backward writing the gradients) on a one-rank RCCL group gives bitwise
  the parameters and Adam moments of eager DP steps.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _heartbeat(request, msg):
    """A progress line on the terminal, past pytest's capture: a long multi-process test is not then
    taken for a hang by a runner that watches the output."""
    capman = request.config.pluginmanager.getplugin("capturemanager")
    if capman is None:  # capture disabled (-p no:capture): plain print reaches the terminal
        print(f"\n[{msg}]", flush=True)
        return
    with capman.global_and_fixture_disabled():
        print(f"\n[{msg}]", flush=True)


def _wait(q, p, request, name, limit, trace=None):
    """The worker's (status, result), polling every 20 s with a progress line; ("timeout", log tail)
    when it has not answered within ``limit`` seconds or died without answering."""
    import queue
    import time
    t0 = time.time()
    try:
        while True:
            try:
                return q.get(timeout=20)
            except queue.Empty:
                log = ""
                if trace and os.path.exists(trace):
                    with open(trace) as f:
                        log = f.read()
                if time.time() - t0 > limit or not p.is_alive():
                    return "timeout", log[-6000:] or f"{name}: no answer after {time.time() - t0:.0f}s"
                last = log.strip().splitlines()[-1] if log.strip() else "running"
                _heartbeat(request, f"{name} {time.time() - t0:.0f}s: {last}")
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(420)
def test_bench_two_ranks_gloo(dev, request, tmp_path):
    import time
    env = dict(os.environ, RP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    out, err = tmp_path / "bench.out", tmp_path / "bench.err"
    with open(out, "w") as fo, open(err, "w") as fe:
        proc = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                                 "--warmup", "1"], stdout=fo, stderr=fe, text=True, env=env, cwd=ROOT)
        t0 = time.time()
        while True:
            try:
                proc.wait(timeout=20)
                break
            except subprocess.TimeoutExpired:
                if time.time() - t0 > 400:
                    proc.kill()
                    proc.wait()
                    break
                _heartbeat(request, f"bench.py --gpus 2 (gloo) {time.time() - t0:.0f}s")
    stdout, stderr = out.read_text(), err.read_text()
    assert proc.returncode == 0, stderr[-4000:]
    lines = [l for l in stdout.strip().splitlines() if l.strip()]
    assert len(lines) == 1, stdout
    res = json.loads(lines[0])
    print({k: res[k] for k in ("value", "ms_per_step", "n_gpus", "ranks_seen", "param_checksums", "execution")})
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2
    assert res["config"]["parallelism"] == "dp2" and res["comm"]["backend"] == "gloo"
    assert res["execution"].startswith("eager")
    assert torch.isfinite(torch.tensor(res["loss"])).item()
    assert res["value"] > 0 and len(res["rank_ms_per_step"]) == 2
    cs = res["param_checksums"]
    assert len(cs) == 2 and cs[0] == cs[1], cs


def _tiling_worker(port, q, cases):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    try:
        import torch.distributed as dist
        from repurpose_amd.distributed import GradAllReducer
        from repurpose_amd.MMCTransformer import MMCTransformer
        from tests.test_model_gpu import TRI, make_batch, to_dev
        dist.init_process_group("gloo", rank=0, world_size=1)
        dev = torch.device("cuda", 0)
        b = to_dev(make_batch(TRI, 2, 128, [128, 90], seed=3), dev)
        out = []
        for name, dtype, env in cases:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                torch.manual_seed(1)
                m = MMCTransformer(**dict(TRI, self_num_layers=16), compute_dtype=dtype).to(dev).train()
                m.DROPOUT = 0.0
                red = GradAllReducer(m, bucket_mb=4.0)
                (m.losses(*m(b))["cls_loss"] / 2).backward()
                launched = list(red.launched)
                red.wait()
                torch.cuda.synchronize()
                out.append((name, m.trainable_numel(), launched))
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        q.put(("ok", out))
    except Exception:
        import traceback
        q.put(("err", traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_buckets_tile_the_gradient_buffer(dev, request):
    cases = [("tile cut (default)", "bf16", {}),
             ("8-layer groups", "bf16", {"RP_WGRAD_GROUP_LAYERS": "8"}),
             ("4-layer groups", "bf16", {"RP_WGRAD_GROUP_LAYERS": "4"}),
             ("one 16-layer group", "bf16", {"RP_WGRAD_GROUP_LAYERS": "16"}),
             ("per-layer split-K", "bf16", {"RP_WGRAD_GROUPED": "0"}),
             ("fp32", "fp32", {})]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_tiling_worker, args=(_port(), q, cases))
    p.start()
    status, res = _wait(q, p, request, "bucket tiling worker", 240)
    assert status == "ok", res
    for name, n, launched in res:
        assert launched, name
        # reverse layout order: each bucket ends where the previous one began
        assert launched[0][1] == n, (name, launched[0], n)
        for a, c in zip(launched, launched[1:]):
            assert c[1] == a[0], (name, a, c)
        assert launched[-1][0] == 0, (name, launched[-1])
        assert sum(hi - lo for lo, hi in launched) == n, name  # exactly once
        print(f"{name}: {len(launched)} buckets")


def _captured_worker(q, trace):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import faulthandler
    import time
    tf = open(trace, "w", buffering=1)
    t0 = time.time()

    def mark(stage):  # stage log (stacks on stderr every 30 s) for a run that does not finish
        tf.write(f"{time.time() - t0:7.1f}s {stage}\n")
        sys.stderr.write(f"[captured worker] {time.time() - t0:7.1f}s {stage}\n")
        sys.stderr.flush()

    faulthandler.dump_traceback_later(30, repeat=True, file=sys.stderr)
    try:
        import torch.distributed as dist
        from repurpose_amd.distributed import GradAllReducer
        from repurpose_amd.graph import CapturedTrainStep
        from repurpose_amd.MMCTransformer import MMCTransformer
        from repurpose_amd.optim import FusedAdam
        from tests.test_model_gpu import TRI, make_batch, to_dev
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        mark("init_process_group")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        mark("process group up")
        cfg = dict(TRI, self_num_layers=16)
        batches = [{k: v for k, v in to_dev(make_batch(cfg, 2, 128, [128, 100], seed=40 + i), dev).items()
                    if torch.is_tensor(v)} for i in range(4)]

        def fresh():
            torch.manual_seed(5)
            m = MMCTransformer(**cfg, compute_dtype="bf16").to(dev).train()
            m.DROPOUT = 0.0
            return m, FusedAdam(m, lr=1e-3, weight_decay=1e-4), GradAllReducer(m)

        me, oe, re_ = fresh()
        for i, b in enumerate(batches):
            oe.zero_grad()
            (me.losses(*me(b))["cls_loss"] / 2).backward()
            re_.wait()
            oe.step()
            torch.cuda.synchronize()
            mark(f"eager DP step {i}")
        mg, og, rg = fresh()
        run = CapturedTrainStep(mg, og, {k: v.clone() for k, v in batches[0].items()}, warmup=1,
                                capture_collectives=True)
        torch.cuda.synchronize()
        mark("captured")
        for i, b in enumerate(batches):
            run.load(b)
            run.step()
            torch.cuda.synchronize()
            mark(f"replay {i}")
        n = me.trainable_numel()
        ok = (run._graph is not None, len(rg.launched) > 0,
              torch.equal(mg.flat_params()[:n], me.flat_params()[:n]),
              torch.equal(og._m, oe._m), torch.equal(og._v, oe._v))
        q.put(("ok", ok))
    except Exception:
        import traceback
        q.put(("err", traceback.format_exc()))
    finally:
        faulthandler.cancel_dump_traceback_later()
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
        mark("done")


@pytest.mark.timeout(300)
def test_captured_rccl_dp_step_equals_eager_dp(dev, tmp_path, request):
    trace = str(tmp_path / "captured_worker.log")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_captured_worker, args=(q, trace))
    p.start()
    status, res = _wait(q, p, request, "captured DP worker", 240, trace)
    assert status == "ok", res
    captured, hooked, params, m1, m2 = res
    assert captured, "the DP step was not captured"
    assert hooked, "the captured backward issued no all-reduce"
    assert params and m1 and m2, res
