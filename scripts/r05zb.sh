#!/bin/bash
# GEMM epilogue bias chunk loaded once per thread: GEMM tests, whole-step A/B against HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "gemm or wgrad or linear or dout_delta" > gpurun_out/r05zb_tests.log 2>&1 || { echo "tests FAILED"; tail -20 gpurun_out/r05zb_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05zb_tests.log)"
timeout -k 10 900 bash scripts/ab_libs_bench.sh 3 abl/head.so tree
