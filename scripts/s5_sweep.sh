#!/bin/bash
# full GPU tests on the in-tree build, then the attention microbench for each abtest/<lib>.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/s5sw_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s5sw_tests.log
[ $rc -eq 0 ] || exit $rc
fi
for lib in cur $LIBS; do
  if [ $lib = cur ]; then unset RP_LIB_PATH; else export RP_LIB_PATH=abtest/$lib.so; fi
  timeout -k 10 200 python -u scripts/microbench.py --only "${MB:-attn}" > gpurun_out/s5sw_mb_$lib.log 2>&1 || exit 1
  echo "== micro $lib"; grep -v amdgpu.ids gpurun_out/s5sw_mb_$lib.log
done
