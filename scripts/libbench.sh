#!/bin/bash
# bench.py per (library, config): LIBS="a b" -> marl-snake_amd/build/var/libsnake_<x>.so,
# CFGS="cfg3 cfg2"; prints ms per step, per-kernel averages and spawn-ahead stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/lb}
mkdir -p $OUT
# VARS="A=1 B=2;A=3": each ';'-separated environment setting per (library, config)
IFS=';' read -ra sets <<< "${VARS:- }"
i=0
for c in ${CFGS:-cfg3}; do
  for l in ${LIBS:-a_base}; do
    for kv in "${sets[@]}"; do
      i=$((i+1))
      env $kv SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps ${STEPS:-1000} --warmup 200 > $OUT/$i.log 2>&1 || { echo "fail $l $c $kv"; tail -5 $OUT/$i.log; exit 3; }
      echo "$c $l [$kv] $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead',{}).get('hit_rate'))")"
    done
  done
done
