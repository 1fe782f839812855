#!/bin/bash
# wgrad: DMA LDS configuration x split target (GEMM microbench, wgrad rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 0 1 2; do
for t in 512 1024; do
  RP_GEMM_CFG=$c RP_WGRAD_BLOCKS=$t timeout -k 10 200 python -u scripts/microbench.py --only gemm > gpurun_out/s5wg2.log 2>&1 || exit 1
  echo "== cfg $c target $t"; grep wgrad gpurun_out/s5wg2.log | sed 's/  */ /g'
done
done
