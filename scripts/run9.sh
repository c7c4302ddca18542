set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpu_check.sh smoke tests || exit 3
SNAKE_LOGIC_MS=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "oracle or full_size or golden or crafted" --timeout 200 --timeout-method thread > gpurun_out/tests_ms16.log 2>&1; echo "ms16 tests rc=$?"; tail -2 gpurun_out/tests_ms16.log
LIBS="f_ms" CFGS="cfg2 cfg3" VARS="SNAKE_LOGIC_MS=4;SNAKE_LOGIC_MS=8;SNAKE_LOGIC_MS=16" bash scripts/libbench.sh || exit 3
for c in cfg3 cfg2 cfg5; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 && tail -1 gpurun_out/bench_$c.log | cut -c1-1200; done
