#!/bin/bash
# GPU tests, then config-4 / metric bench (small-problem attention blocks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/s5qt_tests.log 2>&1; rc=$?
tail -5 gpurun_out/s5qt_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --seq-len 4096 --batch 1 --no-cpu-baseline > gpurun_out/s5qt_cfg4.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/s5qt_metric.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"workload": "[^"]*"' gpurun_out/s5qt_cfg4.log gpurun_out/s5qt_metric.log
