#!/bin/bash
# HBM traffic per launch of every kernel of the training step: two rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE: separate runs, the TCC slots do not hold both) over a short eager bench at (B, T), then
# scripts/pmc_traffic.py -> gpurun_out/<out> (only gpurun_out/ comes back from the box; copy the file
# into profiles/ to commit it).  usage: scripts/pmc_step.sh <out.json> [B T]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; B=${2:-8}; T=${3:-2048}
CMD="python3 bench.py --steps 2 --warmup 1 --graph off --no-parity-mode --no-fresh-batch --no-cpu-baseline --batch $B --seq-len $T"
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc_${c}_${T} -o run --output-format csv -- $CMD > gpurun_out/pmc_${c}_${T}.log 2>&1
  rc=$?
  echo "pass $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${c}_${T}.log; exit $rc; fi
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE_${T} gpurun_out/pmc_WRITE_SIZE_${T} gpurun_out/$OUT $B $T
