#!/bin/bash
# Same-box A/B of the training step between two source trees (A = $1, e.g. a git worktree of an
# older commit built in place; B = this tree), interleaved N times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; N=${2:-3}; ARGS=${3:-"--steps 10 --warmup 3 --no-cpu-baseline"}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then D=$A; else D=.; fi
    (cd $D && timeout -k 10 200 python -u bench.py $ARGS) > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ab_$v.log | tr '\n' ' ')"
  done
done
