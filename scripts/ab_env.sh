#!/bin/bash
# usage: scripts/ab_env.sh ROUNDS STEPS "ENV1" "ENV2" ... : interleaved bench runs per env setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; ST=$2; shift 2
for i in $(seq 1 $R); do
  k=0
  for E in "$@"; do
    k=$((k+1))
    env $E timeout -k 10 200 python -u bench.py --steps $ST --warmup 3 --no-cpu-baseline > gpurun_out/abm_$k.log 2>&1 || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/abm_$k.log') if l.startswith('{')][0]; print('$E', round(d['ms_per_step'],3))"
  done
done
