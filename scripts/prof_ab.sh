#!/bin/bash
# kernel traces of a short bench run under two settings of one env var: scripts/prof_ab.sh TAG VAR VAL_A VAL_B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; VAR=$2
for v in "$3" "$4"; do
  if [ "$v" = unset ]; then unset "$VAR"; else export "$VAR=$v"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$v.log 2>&1 || exit 1
  python3 scripts/steptrace.py gpurun_out/${TAG}_$v/run_kernel_trace.csv -1 > gpurun_out/${TAG}_$v.txt
  echo "== $VAR=$v"; head -30 gpurun_out/${TAG}_$v.txt
done
