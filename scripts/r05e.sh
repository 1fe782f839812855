cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_dp_gpu.py -k oracle > gpurun_out/r05e_dp.log 2>&1; echo dp rc=$?; grep -E "passed|failed|worst|Error" gpurun_out/r05e_dp.log | tail -4
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k roles > gpurun_out/r05e_roles.log 2>&1; echo roles rc=$?; tail -2 gpurun_out/r05e_roles.log
for r in 1 2; do for v in 0 1; do RP_ATTN_ROLES_IL=$v timeout -k 10 120 python -u scripts/microbench.py --only attn --reps 30 2>&1 | grep "attn_bwd p" | sed "s/^/IL=$v /"; done; done
timeout -k 10 600 bash scripts/ab_env_bench.sh RP_ATTN_ROLES_IL 3 "--steps 20 --warmup 3 --no-cpu-baseline --no-parity-mode --no-fresh-batch" 0 1
