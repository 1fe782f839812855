"""Host sanitizer build of the C ABI (SURVEY.md §5 "sanitizers on the CPU build"): `make asan`
compiles the launchers with AddressSanitizer + UndefinedBehaviorSanitizer on the host side and
links tests/native/abi_errors.cpp, which drives every rp_* entry point's argument validation
(null / misaligned pointers, bad shapes, dtypes, dropout ranges, item counts), the workspace queries,
rp_last_error's truncation and rp_adam_coefficients' host arithmetic.  No device work is enqueued,
so it runs without a GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs make and hipcc")
def test_abi_error_paths_under_asan_ubsan():
    b = subprocess.run(["make", "-j8", "asan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "build", "asan", "abi_errors")], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out, out[-3000:]
    assert r.returncode == 0, out[-3000:]
    assert ", 0 failed" in r.stdout
