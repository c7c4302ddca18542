#!/bin/bash
# Round-4 measurement set: GPU suite (optional), bench lines for cfg3/cfg4/cfg2/cfg5
# and the driver's 20/5 window, rocprofv3 kernel stats per config and (optional)
# PMC traffic passes. Each GPU step under its own time limit; stops at the first
# failure.  Usage: OUT=gpurun_out/r04a TESTS=1 PMC=1 bash scripts/r04_profiles.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04}
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
    run bench_$c 300 python bench.py --config $c --no-cpu-baseline
  done
fi
if [ "${PROF:-1}" = 1 ]; then
  for c in $CONFIGS; do
    run prof_$c 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 300 --warmup 100 --no-cpu-baseline --timing-stride 0
  done
fi
if [ "${PMC:-0}" = 1 ]; then
  K='k_logic|k_post|k_autoreset|k_encode|k_spawn'
  for c in ${PMC_CONFIGS:-cfg3 cfg5}; do
    B="python3 bench.py --config $c --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
    run pmcF_$c 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcF_$c -o pmc -- $B
    run pmcW_$c 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcW_$c -o pmc -- $B
    run pmcSQ_$c 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$K" --output-format csv -d $OUT/pmcSQ_$c -o pmc -- $B
  done
fi
echo all-ok
