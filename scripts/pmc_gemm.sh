#!/bin/bash
# SQ stall counters over the per-shape GEMM and attention microbenches -> gpurun_out/<tag>_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmcg}
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for shape in ${SHAPES:-qkv linear2 attn}; do
  if [ $shape = attn ]; then CMD="python3 scripts/microbench.py --only attn --reps 3"; else CMD="python3 scripts/microbench.py --only gemm --gemm $shape --reps 3"; fi
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/${TAG}_$shape -o run --output-format csv -- $CMD > gpurun_out/${TAG}_$shape.log 2>&1
  rc=$?
  echo "$shape rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$shape.log; exit $rc; fi
done
