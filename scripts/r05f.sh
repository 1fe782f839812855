#!/bin/bash
# round-5 probes: GEMM tile variants per layer shape (cold caches), grouped-wgrad single-kind L2 reuse
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "X=0" "RP_GEMM_CFG=0 RP_GEMM_BM64=1" "RP_GEMM8=1" "RP_GEMM_CFG=1" "X=0"; do
  echo "=== $v"; env $v timeout -k 10 120 python -u scripts/gemm_step.py --reps 10 2>&1 | grep -v amdgpu.ids
done
for o in linear2 in_proj; do
  for c in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    d=gpurun_out/r05f_w_${o}_$(echo $c | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python3 scripts/wgrad_probe.py --reps 2 --only $o > $d.log 2>&1
    echo "wpmc $o $c rc=$?"
  done
done
echo ALLDONE
