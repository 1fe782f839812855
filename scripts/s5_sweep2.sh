#!/bin/bash
# interleaved attention microbench over abtest/<lib>.so (R rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${R:-2}); do
for lib in cur $LIBS; do
  if [ $lib = cur ]; then unset RP_LIB_PATH; else export RP_LIB_PATH=abtest/$lib.so; fi
  timeout -k 10 200 python -u scripts/microbench.py --only "${MB:-attn}" > gpurun_out/s5sw2_mb.log 2>&1 || exit 1
  echo "== r$r $lib"; grep -v amdgpu.ids gpurun_out/s5sw2_mb.log | sed 's/  */ /g'
done
done
