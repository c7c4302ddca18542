#!/bin/bash
# fp32 DQN: the 4x2 wave-tile conv variant (SNAKE_DQN32_WT=1) against the 8x1
# default -- parity (tests/test_dqn.py fp32 cases) and per-layer kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/dqnwt}
mkdir -p $OUT
export TMPDIR=/tmp
SNAKE_DQN32_WT=1 timeout -k 10 300 python -u -m pytest tests/test_dqn.py -x -q -m gpu -k fp32 --timeout 200 --timeout-method thread > $OUT/tests_wt.log 2>&1; echo "wt tests rc=$?"; tail -3 $OUT/tests_wt.log
for wt in 0 1 0 1; do
  SNAKE_DQN32_WT=$wt timeout -k 10 200 python scripts/dqn_bench.py --precision fp32 --envs 4096 --vr 0 --no-torch > $OUT/bench_wt$wt.log 2>&1 || { echo "bench fail"; tail -3 $OUT/bench_wt$wt.log; exit 3; }
  echo "wt=$wt $(tail -1 $OUT/bench_wt$wt.log | cut -c1-400)"
done
for wt in 0 1; do
  SNAKE_DQN32_WT=$wt timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$wt -o run --output-format csv -- python3 scripts/dqn_bench.py --precision fp32 --envs 4096 --vr 0 --no-torch --steps 5 --warmup 2 > $OUT/prof$wt.log 2>&1 || exit 3
  grep -h "conv32\|fc32\|gemm32" $OUT/prof$wt/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/wt=$wt /"
done
