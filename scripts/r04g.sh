#!/bin/bash
# Round-4: where the missed spawn-ahead records come from, and whether two
# attempts per in-step job (tries2) or a threshold of 3 live snakes cut them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04g}
mkdir -p $OUT
i=0
for c in cfg3 cfg4 cfg2; do
  for l in base tries2; do
    for thr in 0 3; do
      i=$((i+1))
      SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 1000 --warmup 200 --spawn-ahead $thr > $OUT/$i.log 2>&1 || { echo "fail $c $l $thr"; tail -5 $OUT/$i.log; exit 3; }
      echo "$c $l thr=$thr $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels']['k_logic'], d['kernels']['k_post'], d['resets_per_timed_step'], d.get('spawn_ahead'))")"
    done
  done
done
echo all-ok
