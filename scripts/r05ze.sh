#!/bin/bash
# 8-lane delta sums on DPP: the fused delta epilogue bitwise the delta pass, attention tests, A/B vs HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "delta or attn or attention" > gpurun_out/r05ze_tests.log 2>&1 || { echo "tests FAILED"; tail -20 gpurun_out/r05ze_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05ze_tests.log)"
timeout -k 10 900 bash scripts/ab_libs_bench.sh 3 abl/head.so tree
