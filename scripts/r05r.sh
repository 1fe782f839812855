#!/bin/bash
# GEMM + LayerNorm exchange kernels: parity tests, then whole-step A/B of the fused seams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_gemm_ln_gpu.py \
  -k "exchange_mixed or model_fused_seams_exchange" > gpurun_out/r05r_tests.log 2>&1 || { echo "tests FAILED"; grep -E "PASS|FAIL|Error|assert|step grad" gpurun_out/r05r_tests.log | tail -30; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05r_tests.log)"; grep "step gradients" gpurun_out/r05r_tests.log
timeout -k 10 900 bash scripts/ab_envs.sh 3 RP_GEMM_LN=0 RP_GEMM_LN=fwd RP_GEMM_LN=bwd RP_GEMM_LN=1
