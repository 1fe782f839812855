cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT tests/test_dp_gpu.py -k oracle tests/test_kernels_gpu.py -k "attention or oracle or delta" > gpurun_out/r05d_tests.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/r05d_tests.log
timeout -k 10 400 bash scripts/ab_lib.sh ablibs/pre_delta.so 2 "--only attn --reps 30" > gpurun_out/r05d_abmicro.log 2>&1; echo abmicro rc=$?
timeout -k 10 600 bash scripts/ab_libs_bench.sh 3 ablibs/pre_delta.so tree > gpurun_out/r05d_abstep.log 2>&1; echo abstep rc=$?; cat gpurun_out/r05d_abstep.log
