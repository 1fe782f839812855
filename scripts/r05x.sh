#!/bin/bash
# Exchange seams with the epilogue operand prefetched in the main loop: parity tests, then A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_ln_gpu.py \
  > gpurun_out/r05x_tests.log 2>&1 || { echo "tests FAILED"; grep -E "FAIL|Error|assert" gpurun_out/r05x_tests.log | tail -20; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05x_tests.log)"
timeout -k 10 900 bash scripts/ab_envs.sh 3 RP_LNX_PF=0 RP_LNX_PF=1
