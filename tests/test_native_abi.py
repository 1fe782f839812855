"""CPU checks of the C ABI: the library loads, exports every entry point include/rp_api.h declares,
and rejects bad arguments with a readable error (no GPU work is launched here)."""
import ctypes
import os
import re

import pytest

from repurpose_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "rp_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rp_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(N.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = N.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.rp_version() == 1


def test_argument_errors_are_reported():
    with pytest.raises(RuntimeError, match="K=7 must be a multiple of 8"):
        N.call("rp_gemm", 0, 8, 8, 7, ctypes.c_void_p(16), 8, 1, ctypes.c_void_p(16), 8, 1, ctypes.c_void_p(16), 8, 0,
               1.0, None, None)
    with pytest.raises(RuntimeError, match="head dim"):
        N.call("rp_attn_fwd", 0, None, None, 1, 1, 1, 32, 1.0, 0.0, 0, None, None, None, None, None, None)
    fake = ctypes.c_void_p(16)
    assert N.load().rp_softnms_workspace(2, 1000) == 0 and N.load().rp_softnms_workspace(2, 7000) == 2 * 5 * 7000 * 4
    with pytest.raises(RuntimeError, match="needs rp_softnms_workspace"):
        N.call("rp_softnms", fake, fake, fake, 1, 7000, 0.5, 0.01, fake, fake, fake, None, None, 0, None)
    with pytest.raises(RuntimeError, match="D=300 unsupported"):
        a = N.LnFwdArgs()
        a.x, a.gamma, a.beta, a.x_dtype = 16, 16, 16, 0
        N.call("rp_layernorm_fwd", 4, 300, ctypes.byref(a), None)


def test_zero_sized_calls_are_noops():
    N.call("rp_gemm", 1, 0, 16, 16, None, 16, 1, None, 16, 1, None, 16, 1, 1.0, None, None)
    N.call("rp_cast_f32_to_bf16", None, None, 0, None)
    N.call("rp_focal_elementwise", None, None, 0, 0.7, 2.0, None, None)


def test_workspace_queries():
    lib = N.load()
    assert lib.rp_colsum_workspace(16384, 2048) == 256 * 2048
    assert lib.rp_gemm_wgrad_workspace(2048, 512, 16384) >= 2048 * 512 * 4
    assert lib.rp_layernorm_bwd_blocks(16384) == 16384 // 32  # 32 rows per block (8 waves x 4 rows)
    assert lib.rp_layernorm_bwd_blocks(1) == 1
