#!/bin/bash
# fp32 DQN consumer: parity tests, A/B bench (matrix-core convs vs the vector
# GEMM), per-kernel rocprof stats. Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/dqn32}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -20 $OUT/$name.log; exit 3; }; tail -n 2 $OUT/$name.log | cut -c1-600; }
run tests 300 python -u -m pytest tests/test_dqn.py -x -q -m gpu --timeout 120 --timeout-method thread
run bench_full 300 python scripts/dqn_bench.py --precision fp32 --envs 4096 --vr 0
SNAKE_DQN32_MFMA=0 run bench_full_vec 300 python scripts/dqn_bench.py --precision fp32 --envs 4096 --vr 0 --no-torch
run bench_vr5 300 python scripts/dqn_bench.py --precision fp32 --envs 16384
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 scripts/dqn_bench.py --precision fp32 --envs 4096 --vr 0 --no-torch --steps 5 --warmup 2

# PMC pass over the matrix-core kernels (one counter set per run)
run pmc 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY --kernel-include-regex "mfma" --output-format csv -d $OUT/pmc -o pmc -- python3 scripts/dqn_bench.py --precision fp32 --envs 4096 --vr 0 --no-torch --steps 2 --warmup 1
echo all-ok
