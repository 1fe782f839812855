#!/bin/bash
# Configs 2 (B = 8, T = 1024) and 4 (B = 1, T = 4096): fused exchange seams forced on vs the auto rule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in "8 1024" "1 4096"; do
  set -- $c
  echo "== B=$1 T=$2"
  AB_ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch --batch $1 --seq-len $2" \
    timeout -k 10 600 bash scripts/ab_envs.sh 3 RP_GEMM_LN=auto RP_GEMM_LN=1 || exit 1
done
