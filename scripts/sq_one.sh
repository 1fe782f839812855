#!/bin/bash
# SQ counter passes (separate rocprofv3 --pmc runs) over one command: scripts/sq_one.sh <tag> <cmd...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
PASSES=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
 "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"
 "SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
)
i=0
for pass in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/${TAG}_p$i -o run --output-format csv -- "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; fi
done
