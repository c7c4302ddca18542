#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out/obsprof
for c in ${OPCFGS:-cfg5}; do for l in ${OPLIBS:-st1 st3}; do
  echo "== $c $l"
  timeout -k 10 200 python scripts/obs_profile.py marl-snake_amd/build/var/libsnake_$l.so --cfg $c > gpurun_out/obsprof/${c}_$l.log 2>&1 || { tail -5 gpurun_out/obsprof/${c}_$l.log; exit 3; }
  tail -3 gpurun_out/obsprof/${c}_$l.log
done; done
