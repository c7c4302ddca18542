#!/bin/bash
# The driver's bench window (python bench.py --gpus 1 --steps 20 --warmup 5) per
# environment setting (VARS="A=1;B=2"), REPS runs each: ms per step, kernels,
# spawn-ahead stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/dw}
mkdir -p $OUT
IFS=';' read -ra sets <<< "${VARS:- }"
i=0
for kv in "${sets[@]}"; do
  for r in $(seq ${REPS:-2}); do
    i=$((i+1))
    env $kv timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 ${EXTRA:-} > $OUT/$i.log 2>&1 || { echo "fail [$kv]"; tail -5 $OUT/$i.log; exit 3; }
    echo "[$kv] $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('resets_per_step'), d.get('spawn_ahead'))")"
  done
done
