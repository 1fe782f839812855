#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 0 6000 12000 0 20000 30000; do
  echo "=== stagger $c"; RP_GEMM_STAGGER=$c timeout -k 10 120 python -u scripts/gemm_step.py --reps 10 2>&1 | grep -E "out_proj fwd \+res|linear2 fwd \+res|linear1 dgrad f32|qkv dgrad f32|out_proj dgrad   |total"
done
timeout -k 10 700 bash scripts/ab_env_bench.sh RP_GEMM_STAGGER 2 "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch" 0 12000
timeout -k 10 700 bash scripts/ab_env_bench.sh RP_GEMM_STAGGER 2 "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch" 0 24000
