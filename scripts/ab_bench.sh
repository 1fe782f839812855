#!/bin/bash
# Same-box A/B of the training step: library A (RP_LIB_PATH=$1) vs the in-tree build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; N=${2:-3}
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then export RP_LIB_PATH=$A; else unset RP_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
