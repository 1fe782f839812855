"""configs/Repurpose.yaml, unchanged, drives the drop-in exactly where the reference trainer uses it
(main.py:139 MMCTransformer(**cfg['model']), :69 MultiGPUStrategy(**cfg['distributed']),
:190-191 Adam(lr, weight_decay from cfg['train']), :674 inference_(batch, cfg['test_cfg'])).

CPU test: reads the reference's config file in place when the reference tree is present (this
container; the GPU box has no /root/reference and skips), with yaml.safe_load (the file is plain
YAML; the reference's FullLoader would execute nothing more on it).  The inference settings every GPU
test uses (tests/test_infer_gpu.py, scripts/val_atiou.py) are checked equal to the file's test_cfg,
so the GPU parity runs exercise the shipped settings."""
import inspect
import os
import sys

import pytest
import torch
import yaml

from repurpose_amd.distributed import MultiGPUStrategy
from repurpose_amd.MMCTransformer import MMCTransformer
from repurpose_amd.optim import FusedAdam

CFG_PATH = "/root/reference/configs/Repurpose.yaml"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cfg():
    if not os.path.exists(CFG_PATH):
        pytest.skip("reference tree not present (GPU box)")
    with open(CFG_PATH) as f:
        return yaml.safe_load(f)


def test_model_from_cfg(cfg):
    m = MMCTransformer(**cfg["model"])
    assert sum(p.numel() for p in m.parameters()) == 52_608_771
    assert m.num_layers == 16 and m.num_heads == 8 and m.d_model == 512
    opt = FusedAdam(m.parameters(), lr=cfg["train"]["lr"], weight_decay=cfg["train"]["weight_decay"])
    assert opt.param_groups[0]["lr"] == 1e-3 and opt.param_groups[0]["weight_decay"] == 1e-4


def test_distributed_section(cfg):
    s = MultiGPUStrategy(**cfg["distributed"])
    assert s.backend == "nccl" and s.timeout == 1800 and s.find_unused_parameters is True
    assert s.strategy in ("single", "ddp")


def test_test_cfg_is_what_the_gpu_tests_run(cfg):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import val_atiou
    from tests import test_infer_gpu
    assert test_infer_gpu.CFG == cfg["test_cfg"]
    assert val_atiou.CFG == cfg["test_cfg"]
    # every key inference_ / inference_single_video read is in the file
    src = "".join(inspect.getsource(f) for f in (MMCTransformer.inference_, MMCTransformer._infer_batch,
                                                  MMCTransformer.inference_single_video))
    for k in cfg["test_cfg"]:
        assert f'"{k}"' in src, k
