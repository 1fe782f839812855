#!/bin/bash
# DP path with grouped weight gradients: two-rank GPU tests (gloo) and a 2-rank bench rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_distributed_gpu.py tests/test_model_gpu.py > gpurun_out/r2c4_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r2c4_tests.log; [ $rc -eq 0 ] || exit $rc
RP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r2c4_bench2.log 2>&1; rc=$?
grep '"metric"' gpurun_out/r2c4_bench2.log | cut -c1-400; echo bench2 rc=$rc
