#!/bin/bash
# Interleaved microbench A/B of two builds of the library: A = $1 (.so path), B = the in-tree build.
# usage: scripts/ab_lib.sh <libA.so> [rounds] [microbench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; R=${2:-2}; ARGS=${3:-"--only attn --reps 30"}
for r in $(seq $R); do
  for v in A B; do
    echo "--- $v round $r"
    if [ $v = A ]; then L=$A; else L=repurpose_amd/_native/librepurpose_amd.so; fi
    RP_LIB_PATH=$L timeout -k 10 180 python -u scripts/microbench.py $ARGS || exit $?
  done
done
