#!/bin/bash
# GEMM phase probe (in-kernel stamps) beside rocprofv3 kernel durations, plain vs nt epilogue stores.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 2; do
  RP_LIB_PATH=abl/probe.so RP_STORE_POLICY=$p RP_LOAD_POLICY_RES=$p timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r05q_p$p \
    -o run --output-format csv -- python scripts/gemm_phase_probe.py > gpurun_out/r05q_p$p.log 2>&1 || { echo "FAILED $p"; tail gpurun_out/r05q_p$p.log; exit 1; }
  echo "== policy $p"; grep "^K" gpurun_out/r05q_p$p.log
done
