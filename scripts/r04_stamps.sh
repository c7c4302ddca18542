#!/bin/bash
# k_logic timelines from the stamps build (scripts/logic_stamps.py) per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04s}
mkdir -p $OUT
LIB=${LIB:-marl-snake_amd/build/var/libsnake_stamps.so}
for c in ${CONFIGS:-cfg2 cfg4 cfg3 cfg5}; do
  echo "== stamps $c"
  timeout -k 10 240 python scripts/logic_stamps.py $LIB --cfg $c > $OUT/stamps_$c.json 2> $OUT/stamps_$c.err || { echo "stamps $c failed"; tail -5 $OUT/stamps_$c.err; exit 3; }
  cat $OUT/stamps_$c.json
done
echo all-ok
