#!/bin/bash
# Round-5 record run: GPU suite, smoke, the default bench line, its rocprofv3 kernel-trace stats, the
# PMC traffic passes of configs 2 and 4, and the one-rank RCCL DP rehearsal.  Stops at a crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05f}
STEPS="gputests smoke benchfull" bash scripts/gpu_run.sh $TAG || exit $?
bash scripts/prof.sh ${TAG}_prof --no-parity-mode --no-fresh-batch || exit $?
bash scripts/pmc_step.sh r05_pmc_traffic_T1024_B8.json 8 1024 || exit $?
bash scripts/pmc_step.sh r05_pmc_traffic_T4096_B1.json 1 4096 || exit $?
STEPS="dp1 dp1eager" bash scripts/gpu_run.sh $TAG || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch \
  --batch 8 --seq-len 1024 > gpurun_out/${TAG}_cfg2.json 2>gpurun_out/${TAG}_cfg2.err || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch \
  --batch 1 --seq-len 4096 > gpurun_out/${TAG}_cfg4.json 2>gpurun_out/${TAG}_cfg4.err || exit $?
echo ALLDONE
