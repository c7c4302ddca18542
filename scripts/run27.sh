set -u
cd $GRAFT_REPO_ROOT
# k_post_lean correctness first (cfg5-shaped cases of the parity suite), each under its own limit
SNAKE_POST_LEAN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_pl.log 2>&1; rc=$?; echo "post_lean tests rc=$rc"; tail -3 gpurun_out/tests_pl.log
[ $rc -eq 0 ] || exit 3
LIBS="m_pl" CFGS="cfg5" VARS="SNAKE_POST_LEAN=0;SNAKE_POST_LEAN=1;SNAKE_POST_LEAN=0;SNAKE_POST_LEAN=1" bash scripts/libbench.sh
