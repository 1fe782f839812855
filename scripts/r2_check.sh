#!/bin/bash
# round-2 check: host issue probe, graph + model + kernel GPU tests, bench graph vs eager
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 240 $PYT tests/test_graph_gpu.py tests/test_model_gpu.py > gpurun_out/r2_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r2_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/host_issue.py > gpurun_out/host_issue.log 2>&1 || exit $?
cat gpurun_out/host_issue.log
for g in on off; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph $g > gpurun_out/r2_bench_$g.log 2>&1 || exit $?
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r2_bench_$g.log') if l.startswith('{')][0]; print('$g', round(d['ms_per_step'],3), d['execution'], round(d['roofline']['avg_launch_ms'],4))"
done
