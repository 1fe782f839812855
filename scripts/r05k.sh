#!/bin/bash
# LayerNorm output store policy A/B (GEMMs at their nt default): LN tests under nt, then interleaved steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RP_STORE_POLICY_LN=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "layernorm or ln_" > gpurun_out/r05k_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -20 gpurun_out/r05k_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r05k_tests.log)"
timeout -k 10 900 bash scripts/ab_env_bench.sh RP_STORE_POLICY_LN 3 "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch" 0 2
