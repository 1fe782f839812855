#!/bin/bash
# Interleaved whole-step A/B of one environment switch: bench.py with VAR=0 and VAR=1, N pairs.
# usage: scripts/ab_env_bench.sh VAR [pairs] [bench args] [value A (0)] [value B (1)]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$1; N=${2:-3}; ARGS=${3:-"--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch"}; VA=${4:-0}; VB=${5:-1}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in $VA $VB; do
    lg=gpurun_out/abenv_$(echo "$v" | tr -c 'A-Za-z0-9_\n' _).log
    env $V=$v timeout -k 10 300 python -u bench.py $ARGS > $lg 2>&1 || { echo "FAILED $V=$v"; tail -5 $lg; exit 1; }
    echo "$V=$v $(grep -o '"ms_per_step": [0-9.]*' $lg | head -1)"
  done
done
