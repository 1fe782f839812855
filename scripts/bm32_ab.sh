#!/bin/bash
# 32 x 128 GEMM tiles (RP_GEMM_BM32): bitwise test, then interleaved config-4 step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py \
  -k "64_row or metric_shapes" > gpurun_out/bm32_t.log 2>&1 || { tail -40 gpurun_out/bm32_t.log; exit 1; }
tail -2 gpurun_out/bm32_t.log
bash scripts/ab_env_bench.sh RP_GEMM_BM32 ${1:-3} \
  "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch --batch 1 --seq-len 4096" || exit 1
