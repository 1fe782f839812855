#!/bin/bash
# attention block-size A/B: RP_ATTN_BLOCK unset (size rule) vs forced 64 / 128, metric and config-4 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
for shape in "--B 8 --T 2048" "--B 1 --T 4096"; do
for blk in auto 64 128; do
  if [ $blk = auto ]; then unset RP_ATTN_BLOCK; else export RP_ATTN_BLOCK=$blk; fi
  timeout -k 10 200 python -u scripts/microbench.py --only attn $shape > gpurun_out/s5blk.log 2>&1 || exit 1
  echo "== r$r $shape block $blk"; grep -v amdgpu.ids gpurun_out/s5blk.log | sed 's/  */ /g'
done
done
done
