#!/bin/bash
# change under test: the given GPU tests, then a same-box step A/B against the abtest/base build
# usage: scripts/ab_check.sh ROUNDS "pytest targets"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PYT $2 > gpurun_out/abc_tests.log 2>&1; rc=$?
tail -2 gpurun_out/abc_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_tree.sh abtest/base ${1:-3} "--steps 20 --warmup 3 --no-cpu-baseline" | grep -v avg_launch
