#!/bin/bash
# LDS / issue counters over the per-shape GEMM microbench -> gpurun_out/<tag>_<shape>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmcl}
C="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY"
for shape in linear1 linear2; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/${TAG}_$shape -o run --output-format csv -- python3 scripts/microbench.py --only gemm --gemm $shape --reps 3 > gpurun_out/${TAG}_$shape.log 2>&1
  rc=$?
  echo "$shape rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$shape.log; exit $rc; fi
done
