#!/bin/bash
# Record run: full GPU suite, smoke, full bench (with the CPU baseline), rocprof kernel stats and the
# per-kernel breakdown of one graph-replayed step.  usage: scripts/gpu_check.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2f}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PYT -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', round(d['ms_per_step'],3), 'value', round(d['value']), 'frac', round(d['roofline']['frac'],3), 'cpu', round(d['cpu_baseline']['value'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1; echo prof rc=$?
python3 scripts/stepsum.py gpurun_out/prof_${TAG}/run_kernel_trace.csv 4 > gpurun_out/${TAG}_step_kernels.txt; head -12 gpurun_out/${TAG}_step_kernels.txt
