#!/bin/bash
# Run GPU steps given as "name|limit|command" lines on stdin; stop at the first step that ends other
# than 0 / 1 (fault, abort, timeout), as gpurun requires.  Logs in gpurun_out/<tag>_<name>.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-g}
while IFS='|' read -r name lim cmd; do
  [ -z "$name" ] && continue
  echo "=== $name (limit ${lim}s) ==="
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/${TAG}_${name}.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 8 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
echo ALLDONE
