#!/bin/bash
# Runs GPU steps in order; stops at the first step that did not end in success / plain test failure.
# usage: scripts/gpu_run.sh <tag> ; steps chosen by $STEPS (default: tests smoke bench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-run}
STEPS=${STEPS:-"kernels model infer smoke bench"}
step() {
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s) ==="
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider"
for s in $STEPS; do
  case $s in
    kernels) step kernels 400 $PYT tests/test_kernels_gpu.py ;;
    model)   step model 400 $PYT tests/test_model_gpu.py ;;
    infer)   step infer 300 $PYT tests/test_infer_gpu.py ;;
    gputests) step gputests 1000 $PYT -m gpu tests ;;
    smoke)   step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   step bench 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benchfull) step benchfull 500 python -u bench.py ;;
    gloo2)   RP_DIST_BACKEND=gloo step gloo2 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 ;;
    dp1)     RP_BENCH_DP=1 step dp1 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
               --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph on ;;
    dp1eager) RP_BENCH_DP=1 step dp1eager 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
               --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph off ;;
    dptests) step dptests 900 $PYT --timeout 450 tests/test_dp_gpu.py ;;
    cfg2)    step cfg2 700 $PYT --timeout 650 tests/test_configs_gpu.py -k config2 ;;
    tq0)     step tq0 300 $PYT tests/test_transformer.py -k "without_queries or parity" ;;
    prof)    step prof 450 bash scripts/prof.sh ${TAG}_prof ;;
    b1)      step b1 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch ;;
  esac
done
echo ALLDONE
