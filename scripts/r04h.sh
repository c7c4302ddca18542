#!/bin/bash
# Round-4: spawn-ahead threshold (live snakes at which an env is queued) per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04h}
mkdir -p $OUT
i=0
for c in ${CONFIGS:-cfg5 cfg3 cfg4 cfg2}; do
  for thr in ${THRS:-2 3 4}; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 1000 --warmup 200 --spawn-ahead $thr > $OUT/$i.log 2>&1 || { echo "fail $c $thr"; tail -5 $OUT/$i.log; exit 3; }
    echo "$c thr=$thr $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'))")"
  done
done
echo all-ok
