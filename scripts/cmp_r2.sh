#!/bin/bash
# The round-2 tree's bench (worktree in _ab_old/r2, built there) beside this
# tree's, alternating, for the configs in CMPCFGS (bench.py's default window).
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out/cmp
B="--steps ${STEPS:-1000} --warmup 200 --no-cpu-baseline"
for c in ${CMPCFGS:-cfg3}; do for i in 1 2; do
  (cd _ab_old/r2 && timeout -k 10 200 python bench.py --config $c $B > ../../gpurun_out/cmp/r2_${c}_$i.log 2>&1) || exit 3
  timeout -k 10 200 python bench.py --config $c $B > gpurun_out/cmp/cur_${c}_$i.log 2>&1 || exit 3
  for t in r2 cur; do echo "$t $c $i: $(tail -1 gpurun_out/cmp/${t}_${c}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'])")"; done
done; done
