#!/bin/bash
# PMC HBM traffic refresh (attention microbench + eager bench step) and the bf16-vs-fp32 trajectory
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bf16_vs_fp32.py --steps 40 --out gpurun_out/bf16_vs_fp32.json > gpurun_out/bf16_vs_fp32.log 2>&1; rc=$?
tail -13 gpurun_out/bf16_vs_fp32.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc.sh pmcA FETCH_SIZE WRITE_SIZE || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmcA_p1 gpurun_out/pmcA_p2 gpurun_out/pmc_attn.json || exit $?
PMC_CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --graph off" bash scripts/pmc.sh pmcB FETCH_SIZE WRITE_SIZE || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmcB_p1 gpurun_out/pmcB_p2 gpurun_out/pmc_step.json
