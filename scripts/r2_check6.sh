#!/bin/bash
# full GPU suite, smoke, bench (graph), rocprof kernel stats of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2c6}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PYT -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/${TAG}_bench.log') if l.startswith('{')][0]; print('ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1; echo prof rc=$?
