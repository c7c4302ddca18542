#!/bin/bash
# Round-4: the GPU suite on the default build (table encode on), bench of the
# table-encode variants (envs per wave) against the staged encode, and the
# k_logic / k_post timelines with and without the table encode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04e}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > $OUT/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -15 $OUT/$name.log; exit 3; }; tail -n 2 $OUT/$name.log | cut -c1-300; }
if [ "${TESTS:-1}" = 1 ]; then
  run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
OUT=$OUT/lb LIBS="${LIBS:-base prev notbl tbl8}" CFGS="${CFGS:-cfg3 cfg4 cfg2}" VARS=" " timeout -k 10 900 bash scripts/libbench.sh || exit 3
for v in stamps stampsnotbl; do
  mkdir -p $OUT/$v && OUT=$OUT/$v LIB=marl-snake_amd/build/var/libsnake_$v.so CONFIGS="cfg3 cfg2" bash scripts/r04_stamps.sh || exit 3
done
echo all-ok
