#!/bin/bash
# LDS-DMA dQ kernel: attention + model tests, attention microbench A/B, whole-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_transformer.py tests/test_configs_gpu.py > gpurun_out/r2c11_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2c11_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  RP_ATTN_PIPE=$v timeout -k 10 120 python -u scripts/microbench.py --only attn --reps 20 > gpurun_out/r2c11_mb_$v.log 2>&1 || exit $?
  echo "pipe=$v"; grep -i "bwd\|fwd" gpurun_out/r2c11_mb_$v.log | head -6
done
for v in 1 0 1 0; do
  RP_ATTN_PIPE=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2c11_bench_$v.log 2>&1 || exit $?
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r2c11_bench_$v.log') if l.startswith('{')][0]; print('pipe=$v', round(d['ms_per_step'],3), [(k['kernel'], round(k['avg_launch_ms']*1e3,1)) for k in d['roofline']['other_kernels'][:2]])"
done
