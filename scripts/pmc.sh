#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass) over the attention microbench -> gpurun_out/<tag>_pN/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
CMD=${PMC_CMD:-"python3 scripts/microbench.py --only attn --reps 3"}
i=0
for pass in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/${TAG}_p$i -o run --output-format csv -- $CMD > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i ($pass) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; fi
done
