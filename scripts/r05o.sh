#!/bin/bash
# Attention store-policy A/B: keep bits / O / dQ dK dV stores nt; tests under all three, then steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RP_STORE_POLICY_KB=2 RP_STORE_POLICY_AO=2 RP_STORE_POLICY_AG=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention" > gpurun_out/r05o_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -20 gpurun_out/r05o_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05o_tests.log)"
timeout -k 10 900 bash scripts/ab_envs.sh 3 - RP_STORE_POLICY_KB=2 RP_STORE_POLICY_AO=2 RP_STORE_POLICY_AG=2
