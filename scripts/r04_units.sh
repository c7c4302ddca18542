#!/bin/bash
# Round 4: k_post's instructions per unit of work at cfg3 from
# PMC SQ passes on the product build and a diagnostic build whose encode blocks
# return at once (SNAKE_DIAG_NO_ENCODE; results not valid): the difference is the
# encodes' share. (An attempt-free build is not possible without changing the
# workload: resets without draws spawn every snake at the same poses.)
# Libraries from scripts/build_variants.sh base noenc:-DSNAKE_DIAG_NO_ENCODE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04u}
mkdir -p $OUT
export TMPDIR=/tmp
for l in base noenc; do
  export SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex 'k_post' --output-format csv -d $OUT/sq_$l -o pmc -- python3 bench.py --config cfg3 --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 1 > $OUT/sq_$l.log 2>&1 || { echo "fail $l"; tail -5 $OUT/sq_$l.log; exit 3; }
  tail -1 $OUT/sq_$l.log | cut -c1-120
done
echo all-ok
