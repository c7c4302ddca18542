set -u
cd $GRAFT_REPO_ROOT
SNAKE_ROWS1=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/tests_rows1.log 2>&1; echo "rows1 tests rc=$?"; tail -3 gpurun_out/tests_rows1.log
LIBS="h_rows1" CFGS="cfg3 cfg2" VARS="SNAKE_ROWS1=0;SNAKE_ROWS1=1;SNAKE_ROWS1=0;SNAKE_ROWS1=1" bash scripts/libbench.sh || exit 3
