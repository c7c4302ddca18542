#!/bin/bash
# cfg5 on the final tree (k_post_lean): rocprofv3 kernel stats + PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r03e}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $OUT/$name.log; exit 3; }; }
run prof_cfg5 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cfg5 -o run --output-format csv -- python3 bench.py --config cfg5 --steps 300 --warmup 100 --no-cpu-baseline --timing-stride 0
K='k_logic|k_post|k_spawn'
B="python3 bench.py --config cfg5 --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
run pmcF_cfg5 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcF_cfg5 -o pmc -- $B
run pmcW_cfg5 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcW_cfg5 -o pmc -- $B
echo all-ok
