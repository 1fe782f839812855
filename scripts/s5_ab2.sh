#!/bin/bash
# GEMM / LayerNorm microbench + step A/B of abtest/{gemmnoslp,allnoslp}.so against the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in cur gemmnoslp allnoslp; do
  if [ $lib = cur ]; then unset RP_LIB_PATH; else export RP_LIB_PATH=abtest/$lib.so; fi
  timeout -k 10 300 python -u scripts/microbench.py --only "${MB:-gemm}" > gpurun_out/s5ab2_mb_$lib.log 2>&1 || exit 1
  echo "== micro $lib"; grep -v amdgpu.ids gpurun_out/s5ab2_mb_$lib.log
done
unset RP_LIB_PATH
for lib in gemmnoslp allnoslp; do
  echo "== step A=$lib B=cur"; bash scripts/ab_bench.sh abtest/$lib.so 3 || exit 1
done
