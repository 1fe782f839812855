#!/bin/bash
# Interleaved whole-step A/B over environment settings, N rounds.
# usage: scripts/ab_envs.sh ROUNDS "VAR=a VAR2=b" "VAR=c" ...   ("-" = no extra variables)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=$1; shift
ARGS=${AB_ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch"}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  k=0
  for E in "$@"; do
    k=$((k + 1)); lg=gpurun_out/abenvs_$k.log
    EV=$E; [ "$E" = - ] && EV=""
    env $EV timeout -k 10 300 python -u bench.py $ARGS > $lg 2>&1 || { echo "FAILED $E"; tail -5 $lg; exit 1; }
    echo "[$E] $(grep -o '"ms_per_step": [0-9.]*' $lg | head -1)"
  done
done
