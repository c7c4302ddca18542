#!/bin/bash
# Round-3 measurement set (final tree: k_post, NT obs stores, whole-deque tail queue): bench lines (cfg3 with the CPU baseline, cfg2, cfg5),
# rocprofv3 kernel stats per config, and the PMC passes (HBM traffic; SQ
# instruction counts) for the cfg3 and cfg5 step kernels. Each GPU step under
# its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r03d}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $OUT/$name.log; exit 3; }; tail -n 1 $OUT/$name.log | cut -c1-300; }
run bench_cfg3 300 python bench.py --cpu-seconds 10
run bench_cfg3_2 300 python bench.py --no-cpu-baseline
run bench_cfg2 200 python bench.py --config cfg2 --no-cpu-baseline
run bench_cfg5 200 python bench.py --config cfg5 --no-cpu-baseline
run driverwin 200 python bench.py --gpus 1 --steps 20 --warmup 5
run hostov 200 python scripts/host_overhead.py
run graph 200 python scripts/graph_probe.py
for c in cfg3 cfg2 cfg5; do
  run prof_$c 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 300 --warmup 100 --no-cpu-baseline --timing-stride 0
done
K='k_logic|k_post|k_autoreset|k_encode|k_spawn'
for c in cfg3 cfg5; do
  B="python3 bench.py --config $c --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
  run pmcF_$c 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcF_$c -o pmc -- $B
  run pmcW_$c 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $OUT/pmcW_$c -o pmc -- $B
  run pmcSQ_$c 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$K" --output-format csv -d $OUT/pmcSQ_$c -o pmc -- $B
done
echo all-ok
