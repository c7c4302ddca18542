set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpu_check.sh smoke tests || exit 3
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/tests.log | head; exit 3; }
LIBS="a_base i_tq" CFGS="cfg3 cfg2" VARS=" " bash scripts/libbench.sh || exit 3
EXTRA=--no-cpu-baseline VARS=" " REPS=3 bash scripts/driverwin.sh
