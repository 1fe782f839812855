#!/bin/bash
# 256-row GEMM keep bits drawn in the DMA prologue: tests, phase probe, whole-step A/B vs HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "gemm or wgrad" > gpurun_out/r05w_tests.log 2>&1 || { echo "tests FAILED"; tail -20 gpurun_out/r05w_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05w_tests.log)"
RP_LIB_PATH=abl/probe.so timeout -k 10 120 python -u scripts/gemm8_phase_probe.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 bash scripts/ab_libs_bench.sh 3 abl/head.so tree
