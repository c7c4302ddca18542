#!/bin/bash
# A/B timings of the DQN consumer: one dqn_bench run per "ENV=..;ENV=.." set.
# Usage: VARS="SNAKE_DQN_WAVES=1;SNAKE_DQN_WAVES=2" bash scripts/dqn_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra sets <<< "$VARS"
i=0
for kv in "${sets[@]}"; do
    i=$((i+1))
    env $kv timeout -k 10 200 python scripts/dqn_bench.py --no-torch > gpurun_out/dqnab$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "set $i ($kv) rc=$rc"; tail -3 gpurun_out/dqnab$i.log; exit $rc; fi
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/dqnab$i.log') if l.startswith('{')][0]; print('$kv', round(d['ms_per_forward'],3), round(d['roofline']['frac'],4))"
done
