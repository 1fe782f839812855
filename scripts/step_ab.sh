#!/bin/bash
# Whole-step A/B/...: alternate bench.py runs under several environments (interleaved, one box).
# usage: R=3 scripts/step_ab.sh "<envA>" "<envB>" ...   e.g. scripts/step_ab.sh "RP_GEMM8=0" "RP_GEMM8="
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${R:-3}
for i in $(seq 1 $R); do
  k=0
  for E in "$@"; do
    k=$((k+1))
    env $E timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/stepab_$k.$i.log 2>&1 || { echo "bench $k.$i failed"; tail -5 gpurun_out/stepab_$k.$i.log; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/stepab_$k.$i.log') if l.startswith('{')][0]; print('$k', '$E', round(d['ms_per_step'],3))"
  done
done
