#!/bin/bash
# usage: abrun.sh "ENV=.. ENV2=..;ENV=.." [bench args]  -> one bench per set
IFS=';' read -ra sets <<< "$1"; shift
i=0
for kv in "${sets[@]}"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$i.log 2>&1
  rc=$?
  echo "[$kv] rc=$rc $(tail -1 gpurun_out/ab_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'])" 2>&1)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
