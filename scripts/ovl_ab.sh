#!/bin/bash
# The overlapped attention backward (RP_ATTN_BWD_OVERLAP): kernel-level check, its GPU tests, then
# interleaved whole-step A/B at the metric shape and at config 4 (B = 1, T = 4096).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 240 python -u scripts/attn_overlap_check.py 20 > gpurun_out/ovl.log 2>&1 || { tail -20 gpurun_out/ovl.log; exit 1; }
cat gpurun_out/ovl.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "overlap or fused_delta" > gpurun_out/ovl_t.log 2>&1 || { tail -30 gpurun_out/ovl_t.log; exit 1; }
tail -2 gpurun_out/ovl_t.log
bash scripts/ab_env_bench.sh RP_ATTN_BWD_OVERLAP ${1:-2} || exit 1
bash scripts/ab_env_bench.sh RP_ATTN_BWD_OVERLAP ${2:-2} \
  "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch --batch 1 --seq-len 4096" || exit 1
