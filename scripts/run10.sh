set -u
cd $GRAFT_REPO_ROOT
SNAKE_BG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/tests_bg.log 2>&1; echo "bg tests rc=$?"; tail -2 gpurun_out/tests_bg.log
LIBS="g_bgf" CFGS="cfg2 cfg3" VARS="SNAKE_BG=0;SNAKE_BG=1;SNAKE_BG=1 SNAKE_SPAWN_THR=3;SNAKE_BG=1 SNAKE_SPAWN_SLOTS=512" bash scripts/libbench.sh || exit 3
