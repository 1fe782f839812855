#!/bin/bash
# Interleaved whole-step A/B of several builds of the library (RP_LIB_PATH), N rounds.
# usage: scripts/ab_libs_bench.sh ROUNDS LIB [LIB ...]   ("tree" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=$1; shift
ARGS=${AB_ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch"}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for L in "$@"; do
    P=$L; [ "$L" = tree ] && P=repurpose_amd/_native/librepurpose_amd.so
    lg=gpurun_out/ablib_$(echo "$L" | tr -c 'A-Za-z0-9_\n' _).log
    RP_LIB_PATH=$P timeout -k 10 300 python -u bench.py $ARGS > $lg 2>&1 || { echo "FAILED $L"; tail -5 $lg; exit 1; }
    echo "$L $(grep -o '"ms_per_step": [0-9.]*' $lg | head -1)"
  done
done
