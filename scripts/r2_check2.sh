#!/bin/bash
# grouped wgrad: kernel + model tests, bench (graph), rocprof kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py > gpurun_out/r2c2_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r2c2_tests.log; [ $rc -le 1 ] || exit $rc
for v in 1 0 1 0; do
  RP_WGRAD_GROUPED=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2c2_bench_$v.log 2>&1 || exit $?
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r2c2_bench_$v.log') if l.startswith('{')][0]; print('grouped=$v', round(d['ms_per_step'],3), [ (k['kernel'], round(k.get('ms_per_step',0) or 0,3)) for k in d['roofline']['other_kernels'] if 'wgrad' in k['kernel']])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2c2 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r2c2.log 2>&1; echo prof rc=$?
