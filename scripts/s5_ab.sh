#!/bin/bash
# attention tests on the in-tree build, then attention microbench + step A/B against abtest/*.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "attn or mha" > gpurun_out/s5ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s5ab_tests.log
[ $rc -eq 0 ] || exit $rc
for lib in ${LIBS:-base noslp}; do
  RP_LIB_PATH=abtest/$lib.so timeout -k 10 200 python -u scripts/microbench.py --only attn > gpurun_out/s5ab_mb_$lib.log 2>&1 || exit 1
  echo "== micro $lib"; cat gpurun_out/s5ab_mb_$lib.log | grep -v amdgpu.ids
done
timeout -k 10 200 python -u scripts/microbench.py --only attn > gpurun_out/s5ab_mb_cur.log 2>&1 || exit 1
echo "== micro cur"; grep -v amdgpu.ids gpurun_out/s5ab_mb_cur.log
for lib in ${LIBS:-base noslp}; do
  echo "== step A=$lib B=cur"; bash scripts/ab_bench.sh abtest/$lib.so 3 || exit 1
done
