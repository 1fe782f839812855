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
