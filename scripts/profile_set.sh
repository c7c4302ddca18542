#!/bin/bash
# One round's measurement set on the GPU box: GPU suite (optional), bench lines
# per config and the driver's 20/5 window, rocprofv3 kernel stats per config,
# PMC passes (HBM traffic and SQ instruction counts, one pass each), and the
# device-side spawn-ahead counters. Each GPU step runs under its own time limit;
# the script stops at the first failure. Collect with scripts/collect_set.py.
#   OUT=gpurun_out/r05 TESTS=1 PMC=1 COUNT=1 bash scripts/profile_set.sh
# Knobs: CONFIGS, PMC_CONFIGS (default: CONFIGS), BENCH/PROF (default 1),
# BENCH_STEPS/BENCH_WARMUP (default 2000/200).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/set}
CONFIGS=${CONFIGS:-"cfg3 cfg4 cfg2 cfg5"}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -15 $OUT/$name.log; exit 3; }; tail -n 1 $OUT/$name.log | cut -c1-400; }
if [ "${TESTS:-0}" = 1 ]; then
  run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
if [ "${BENCH:-1}" = 1 ]; then
  run driverwin 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 10
  for c in $CONFIGS; do
    run bench_$c 300 python bench.py --config $c --steps ${BENCH_STEPS:-2000} --warmup ${BENCH_WARMUP:-200} --no-cpu-baseline
  done
fi
if [ "${PROF:-1}" = 1 ]; then
  for c in $CONFIGS; do
    run prof_$c 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 300 --warmup 100 --no-cpu-baseline --timing-stride 0
  done
fi
if [ "${PMC:-0}" = 1 ]; then
  K='k_logic|k_post|k_autoreset|k_encode|k_spawn'
  for c in ${PMC_CONFIGS:-$CONFIGS}; do
    B="python3 bench.py --config $c --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
    run pmcF_$c 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcF_$c -o pmc -- $B
    run pmcW_$c 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcW_$c -o pmc -- $B
    run pmcSQ_$c 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$K" --output-format csv -d $OUT/pmcSQ_$c -o pmc -- $B
  done
fi
if [ "${COUNT:-0}" = 1 ]; then
  run counters 300 python -u scripts/spawn_counters.py --cfg $CONFIGS
fi
echo all-ok
