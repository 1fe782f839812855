#!/bin/bash
# 32 x 128 GEMM tiles: config 4 with the automatic choice vs off, config 2 forced on vs off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py \
  -k "64_row" > gpurun_out/bm32_t.log 2>&1 || { tail -40 gpurun_out/bm32_t.log; exit 1; }
tail -1 gpurun_out/bm32_t.log
C="--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch"
bash scripts/ab_env_bench.sh RP_GEMM_BM32 2 "$C --batch 1 --seq-len 4096" auto 0 || exit 1
bash scripts/ab_env_bench.sh RP_GEMM_BM32 2 "$C --batch 8 --seq-len 1024" 1 0 || exit 1
