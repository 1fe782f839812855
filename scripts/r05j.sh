#!/bin/bash
# Output store cache policy A/B (RP_STORE_POLICY 0 plain / 1 sc1 write-through / 2 nt): GEMM tests
# under each non-default policy, the step's GEMM shapes, then interleaved whole steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in 1 2; do
  RP_STORE_POLICY=$p timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "gemm or wgrad or dout_delta" > gpurun_out/r05j_tests_$p.log 2>&1 \
    || { echo "tests FAILED policy $p"; tail -20 gpurun_out/r05j_tests_$p.log; exit 1; }
  echo "tests ok policy $p: $(tail -1 gpurun_out/r05j_tests_$p.log)"
done
for p in 0 1 2; do
  echo "=== policy $p"; RP_STORE_POLICY=$p timeout -k 10 120 python -u scripts/gemm_step.py --reps 10 2>&1 | grep -E "fwd|dgrad|total"
done
A="--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch"
for i in 1 2 3; do
  for p in 0 1 2; do
    lg=gpurun_out/r05j_step_$p.log
    RP_STORE_POLICY=$p timeout -k 10 300 python -u bench.py $A > $lg 2>&1 || { echo "FAILED $p"; tail -5 $lg; exit 1; }
    echo "policy=$p $(grep -o '"ms_per_step": [0-9.]*' $lg | head -1)"
  done
done
