#!/bin/bash
# Bench sweep: one short bench.py run per ';'-separated "ENV=.. ENV=.. | args" set,
# printing ms/step, kernel times and spawn-ahead stats. Each run under its own limit.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out/sweep
IFS=';' read -ra sets <<< "$SETS"
i=0
for s in "${sets[@]}"; do
    i=$((i+1))
    envs=${s%%|*}; args=${s#*|}
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-400} --warmup ${WARM:-200} $args > gpurun_out/sweep/$i.log 2>&1
    rc=$?
    echo "[$i] $s rc=$rc :: $(tail -1 gpurun_out/sweep/$i.log | python3 -c "import json,sys
try:
    d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'), d['resets_per_step'])
except Exception as e: print('parse error', e)")"
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "fault-like exit $rc"; exit $rc; }
done
exit 0
