#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run -> gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-prof}
shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/$TAG.log 2>&1
rc=$?
echo "prof rc=$rc"
grep '"metric"' gpurun_out/$TAG.log | head -1
exit $rc
