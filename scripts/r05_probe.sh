#!/bin/bash
# Round-5 probe call: DP tests, grouped weight-gradient order / cut A/B with PMC passes, attention SQ
# counters.  Each GPU step under its own time limit; stops at a crash / timeout (rc not 0 or 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05b}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 8 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
for s in ${STEPS:-dp wgrad wpmc roles sq}; do
  case $s in
    dp) run dp 600 $PYT tests/test_dp_gpu.py tests/test_distributed_gpu.py ;;
    wgrad) run wgrad 240 python -u scripts/wgrad_probe.py --reps 10 --env RP_WGRAD_ORDER=1 RP_WGRAD_ORDER=2 RP_WGRAD_ORDER=0
           run wgradcut 240 python -u scripts/wgrad_probe.py --reps 10 --cut 21 --env RP_WGRAD_ORDER=1 ;;
    wpmc) timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
          for o in 0 1 2; do
            for c in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
              d=gpurun_out/${TAG}_wpmc_o${o}_$(echo $c | cut -d' ' -f1)
              RP_WGRAD_ORDER=$o timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o run --output-format csv -- \
                python3 scripts/wgrad_probe.py --reps 2 > $d.log 2>&1
              rc=$?; echo "wpmc o=$o $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
            done
          done ;;
    sq) run sq 400 bash scripts/sq_attn.sh ${TAG}_sq ;;
    wpad) for pd in 0 64 128 0; do run wpad$pd 200 python -u scripts/wgrad_probe.py --reps 10 --pad $pd; done
          for pd in 0 64; do
            for c in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
              d=gpurun_out/${TAG}_wpad${pd}_$(echo $c | cut -d' ' -f1)
              timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o run --output-format csv -- \
                python3 scripts/wgrad_probe.py --reps 2 --pad $pd > $d.log 2>&1
              rc=$?; echo "wpad pmc pad=$pd $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
            done
          done ;;
    roles) run roles 900 bash scripts/ab_env_bench.sh RP_ATTN_ROLES 3 "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch" 1 2 ;;
  esac
done
echo ALLDONE
