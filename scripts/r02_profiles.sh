#!/bin/bash
# Round-2 measurement set: bench lines + rocprofv3 kernel stats for cfg2/cfg3/cfg5,
# and the HBM-traffic PMC passes for the cfg3 step kernels. Each GPU step under
# its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r02}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $OUT/$name.log; exit 3; }; tail -n 1 $OUT/$name.log | cut -c1-300; }
run bench_cfg3 300 python bench.py --cpu-seconds 10
run bench_cfg3_2 300 python bench.py --no-cpu-baseline
run bench_cfg3_short 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_cfg3_short2 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run compat 200 python scripts/compat_bench.py
run bench_cfg2 200 python bench.py --config cfg2 --no-cpu-baseline
run bench_cfg5 200 python bench.py --config cfg5 --no-cpu-baseline
run early 200 python scripts/early_steps.py
for c in cfg3 cfg2 cfg5; do
  run prof_$c 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 300 --warmup 100 --no-cpu-baseline --timing-stride 0
done
K='k_logic|k_autoreset|k_encode'
B='python3 bench.py --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0'
run pmcF 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcF -o pmc -- $B
run pmcW 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcW -o pmc -- $B
echo all-ok
