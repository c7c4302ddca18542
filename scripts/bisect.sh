#!/bin/bash
# Bench the trees in _ab_old/<name> (git worktrees, built there) and this tree,
# alternating, for one config; extra SNAKE_LIB builds of this tree via LIBS.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out/bisect
B="--config ${CFG:-cfg3} --steps ${STEPS:-1000} --warmup 200 --no-cpu-baseline"
for i in 1 2; do
  for t in ${TREES:-r2 c1}; do
    (cd _ab_old/$t && timeout -k 10 200 python bench.py $B > ../../gpurun_out/bisect/${t}_$i.log 2>&1) || exit 3
    echo "$t $i: $(tail -1 gpurun_out/bisect/${t}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'])")"
  done
  timeout -k 10 200 python bench.py $B > gpurun_out/bisect/cur_$i.log 2>&1 || exit 3
  echo "cur $i: $(tail -1 gpurun_out/bisect/cur_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'])")"
  for l in ${LIBS:-}; do
    SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so timeout -k 10 200 python bench.py $B > gpurun_out/bisect/${l}_$i.log 2>&1 || exit 3
    echo "$l $i: $(tail -1 gpurun_out/bisect/${l}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'])")"
  done
done
