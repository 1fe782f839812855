#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT tests/test_kernels_gpu.py tests/test_depth_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py > gpurun_out/r05g_tests.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/r05g_tests.log
timeout -k 10 700 bash scripts/ab_env_bench.sh RP_DOUT_DELTA 3 "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch" 0 1
