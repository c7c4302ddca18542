#!/bin/bash
# Diagnosis of the compat-env failure: the DPP micro-check, then the compat
# golden replays with the default build and with the __shfl fallback build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04d}
mkdir -p $OUT
export TMPDIR=/tmp
echo "== dpp_check"; timeout -k 10 60 scripts/microbench/dpp_check > $OUT/dpp.log 2>&1; echo "rc=$?"; cat $OUT/dpp.log
for v in default nodpp; do
  lib=""; [ $v != default ] && lib=marl-snake_amd/build/var/libsnake_$v.so
  echo "== compat $v"
  SNAKE_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "compat or batch_matches" > $OUT/compat_$v.log 2>&1; echo "rc=$?"; tail -4 $OUT/compat_$v.log
done
