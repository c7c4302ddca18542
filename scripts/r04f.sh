#!/bin/bash
# Round-4: k_logic's own encode (lenc build) and background spawn-ahead at 20x20:
# parity of the lenc build, then bench per (build, spawn_background, config).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04f}
mkdir -p $OUT
export TMPDIR=/tmp
K="oracle or full_size or golden or crafted or shards or invisible or snapshot or info or invalid or every_step"
SNAKE_LIB=marl-snake_amd/build/var/libsnake_lenc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $OUT/tests_lenc.log 2>&1 || { echo "lenc tests failed"; tail -30 $OUT/tests_lenc.log; exit 3; }
tail -1 $OUT/tests_lenc.log
i=0
for c in cfg3 cfg4; do
  for rep in 1 2; do
    for l in base lenc; do
      for bg in -1 1; do
        i=$((i+1))
        SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 1000 --warmup 200 --spawn-background $bg > $OUT/$i.log 2>&1 || { echo "fail $c $l $bg"; tail -5 $OUT/$i.log; exit 3; }
        echo "$c $l bg=$bg $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'))")"
      done
    done
  done
done
echo all-ok
