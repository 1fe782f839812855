#!/bin/bash
# A/B of one attention switch: bitwise compare of the two variants' outputs (ragged, dropout), then
# interleaved microbench runs.  usage: scripts/ab_attn.sh <ENVVAR> [rounds] [value A (0)] [value B (1)]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$1; R=${2:-2}; VA=${3:-0}; VB=${4:-1}
run() { timeout -k 10 "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
env $V=$VA timeout -k 10 180 python -u scripts/attn_dump.py /tmp/ab_${V}_0.pt --ragged || exit $?
env $V=$VB timeout -k 10 180 python -u scripts/attn_dump.py /tmp/ab_${V}_1.pt --ragged || exit $?
python scripts/attn_dump.py --cmp /tmp/ab_${V}_0.pt /tmp/ab_${V}_1.pt
echo "cmp rc=$?"
for r in $(seq $R); do
  for v in $VA $VB; do
    echo "--- $V=$v round $r"
    env $V=$v timeout -k 10 180 python -u scripts/microbench.py --only attn --reps 30 || exit $?
  done
done
