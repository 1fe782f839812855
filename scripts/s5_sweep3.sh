#!/bin/bash
# schedule-bias sweep (attention microbench, interleaved) + GEMM microbench of gemmb10
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=2 LIBS="bias0 bias5 bias10 bias20 bias40" bash scripts/s5_sweep2.sh || exit 1
for lib in bias10 gemmb10 bias10 gemmb10; do
  RP_LIB_PATH=abtest/$lib.so timeout -k 10 200 python -u scripts/microbench.py --only gemm > gpurun_out/s5sw3.log 2>&1 || exit 1
  echo "== gemm $lib"; grep -v amdgpu.ids gpurun_out/s5sw3.log | sed 's/  */ /g'
done
