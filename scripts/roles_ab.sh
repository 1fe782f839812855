#!/bin/bash
# The two-role attention backward (RP_ATTN_ROLES): its GPU tests, then interleaved whole-step A/B at
# config 4 (B = 1, T = 4096) and one pair at the metric shape (where it is not selected).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py \
  -k "roles or overlap or fused_delta or split" > gpurun_out/roles_t.log 2>&1 || { tail -40 gpurun_out/roles_t.log; exit 1; }
tail -2 gpurun_out/roles_t.log
bash scripts/ab_env_bench.sh RP_ATTN_ROLES ${1:-3} \
  "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch --batch 1 --seq-len 4096" 1 0 || exit 1
bash scripts/ab_env_bench.sh RP_ATTN_ROLES 1 || exit 1
