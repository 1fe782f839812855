#!/bin/bash
# Exchange seams: phase probe (RP_GEMM_PROBE build), parity tests, whole-step A/B against HEAD, and the
# metric-shape PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RP_LIB_PATH=abl/probe.so timeout -k 10 120 python -u scripts/lnx_phase_probe.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_ln_gpu.py \
  > gpurun_out/r05z_tests.log 2>&1 || { echo "tests FAILED"; grep -E "FAIL|Error|assert" gpurun_out/r05z_tests.log | tail -20; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05z_tests.log)"
timeout -k 10 900 bash scripts/ab_libs_bench.sh 3 abl/head.so tree
