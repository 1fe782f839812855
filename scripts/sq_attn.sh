#!/bin/bash
# SQ counters of the attention microbench (one rocprofv3 --pmc run per pass, counters filtered
# against rocprofv3 -L so a name the box lacks is dropped instead of failing the pass).
# usage: scripts/sq_attn.sh <tag>   -> gpurun_out/<tag>_pN/ (+ counters list gpurun_out/<tag>_list.txt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-sq}
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_list.txt 2>&1
CMD=${PMC_CMD:-"python3 scripts/microbench.py --only attn --reps 2"}
PASSES=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
 "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"
 "SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_WAVES SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE"
)
i=0
for pass in "${PASSES[@]}"; do
  i=$((i+1))
  keep=""
  for c in $pass; do grep -qw "$c" gpurun_out/${TAG}_list.txt && keep="$keep $c"; done
  echo "pass $i: $keep"
  [ -z "$keep" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $keep -d gpurun_out/${TAG}_p$i -o run --output-format csv -- $CMD > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; fi
done
