#!/bin/bash
# Round-4 A/B: persistent k_logic (k_logic_pf, pf<waves per CU>) and the table
# encode in k_post (tbl<envs per wave>) against the current forms: parity of the
# variant builds, bench per build, k_logic timelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04c}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -15 $OUT/$name.log; exit 3; }; tail -n 2 $OUT/$name.log | cut -c1-300; }
echo "== dpp_check"; timeout -k 10 60 scripts/microbench/dpp_check > $OUT/dpp.log 2>&1 || { echo "dpp_check failed"; cat $OUT/dpp.log; exit 3; }; cat $OUT/dpp.log
if [ "${TESTS:-1}" = 1 ]; then
  run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
K="oracle or full_size or golden or crafted or shards or invisible or snapshot"
for v in ${TLIBS:-pf8 tbl4}; do
  SNAKE_LIB=marl-snake_amd/build/var/libsnake_$v.so run tests_$v 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "$K"
done
OUT=$OUT/lb LIBS="${LIBS:-base pf4 pf8 tbl2 tbl4 pf8tbl4}" CFGS="${CFGS:-cfg3 cfg2}" VARS=" " timeout -k 10 900 bash scripts/libbench.sh || exit 3
OUT=$OUT LIB=marl-snake_amd/build/var/libsnake_stamps.so CONFIGS="cfg3 cfg2" bash scripts/r04_stamps.sh || exit 3
mkdir -p $OUT/pf8 && OUT=$OUT/pf8 LIB=marl-snake_amd/build/var/libsnake_stampspf8.so CONFIGS="cfg3 cfg2" bash scripts/r04_stamps.sh || exit 3
echo all-ok
