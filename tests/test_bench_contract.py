"""CPU checks of bench.py's reporting contract: the metric string is BASELINE.json's, and the
algorithmic FLOP count per timestep matches SURVEY.md §8(d) (311,167,488 + 98,304*T at L=16)."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_metric_is_baseline_metric():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert _bench().METRIC == json.load(f)["metric"]


def test_flops_per_timestep_matches_survey():
    b = _bench()
    for T in (128, 1024, 2048, 4096):
        assert b.flops_per_timestep(T) == 311_167_488 + 98_304 * T


def _run(args, env=None):
    import subprocess
    import sys
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=120)


def test_gpus_n_launches_n_ranks_as_a_child():
    """`bench.py --gpus N` without WORLD_SIZE starts N ranks through torch.distributed.run (a child
    process: the parent never touches the GPU, never execs) and forwards every other argument."""
    r = _run(["--gpus", "8", "--steps", "7", "--warmup", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(c.startswith("--master-port=") for c in cmd)
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "7", "--warmup", "2"]  # --dry-run is not forwarded


def test_gpus_must_match_world_size_under_a_launcher():
    r = _run(["--gpus", "4", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus 4 but WORLD_SIZE=2" in r.stderr


def test_launcher_relays_only_the_result_line_and_the_exit_status(monkeypatch, tmp_path, capsys):
    """launch(): rank 0's JSON line goes to stdout, other child output to stderr; a failing rank
    (non-zero launcher status) fails the bench."""
    b = _bench()
    script = tmp_path / "fake.py"
    script.write_text("import json,sys\nprint('rank chatter')\nprint(json.dumps({'metric': 'm', 'value': 1}))\n"
                      "sys.exit(int(sys.argv[-1]))\n")

    def fake_cmd(args_list, n, port):
        import sys
        return [sys.executable, str(script)] + list(args_list)

    monkeypatch.setattr(b, "child_command", fake_cmd)
    assert b.launch(2, ["0"]) == 0
    out = capsys.readouterr()
    assert out.out.strip() == json.dumps({"metric": "m", "value": 1})
    assert "rank chatter" in out.err
    assert b.launch(2, ["3"]) == 3


def test_traffic_is_keyed_by_the_measured_shape(tmp_path):
    """roofline.traffic comes from a committed PMC file of the SAME (B, T) workload, else null."""
    b = _bench()
    (tmp_path / "a.json").write_text(json.dumps({"shape": {"B": 8, "T": 2048},
                                                 "kernels": {"attn_bwd_dkdv": {"hbm_bytes": 123.0}}}))
    (tmp_path / "b.json").write_text(json.dumps({"shape": {"B": 1, "T": 4096},
                                                 "kernels": {"attn_bwd_dkdv": {"hbm_bytes": 45.0}}}))
    assert b.pmc_traffic(8, 2048, files=("a.json", "b.json"), root=str(tmp_path)) == {"attn_bwd_dkdv": 123.0}
    assert b.pmc_traffic(1, 4096, files=("a.json", "b.json"), root=str(tmp_path)) == {"attn_bwd_dkdv": 45.0}
    assert b.pmc_traffic(8, 1024, files=("a.json", "b.json"), root=str(tmp_path)) == {}
    assert b.roofline_of("attn_bwd_dkdv", {"attn_bwd_dkdv": 0.1}, 8, 1024, 2500.0, {})["traffic"] is None
    # an old-format (shape-less) file never matches
    (tmp_path / "c.json").write_text(json.dumps({"attn_bwd_dkdv": {"hbm_bytes": 1.0}}))
    assert b.pmc_traffic(8, 2048, files=("c.json",), root=str(tmp_path)) == {}


def test_committed_traffic_files_are_this_rounds():
    """bench.py reads only r06 PMC files (the kernels changed in every round)."""
    assert all(n.startswith("r06_") for n in _bench().PMC_TRAFFIC_FILES)
