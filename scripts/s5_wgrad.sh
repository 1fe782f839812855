#!/bin/bash
# wgrad split-K target sweep (GEMM microbench, wgrad rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
for t in 256 384 512 768; do
  RP_WGRAD_BLOCKS=$t timeout -k 10 200 python -u scripts/microbench.py --only gemm > gpurun_out/s5wg.log 2>&1 || exit 1
  echo "== r$r target $t"; grep wgrad gpurun_out/s5wg.log | sed 's/  */ /g'
done
done
