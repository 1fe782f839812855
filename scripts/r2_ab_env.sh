#!/bin/bash
# usage: scripts/r2_ab_env.sh VAR "v1 v2" ROUNDS STEPS : interleaved bench runs under VAR=v
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; VALS=$2; R=${3:-4}; ST=${4:-20}
for i in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --steps $ST --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]; r=d['roofline']; print('$VAR=$v', round(d['ms_per_step'],3), 'dkdv', round(r['avg_launch_ms']*1e3,1), [(k['kernel'], round(k['avg_launch_ms']*1e3,1)) for k in r['other_kernels'][:2]])"
  done
done
