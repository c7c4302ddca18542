#!/bin/bash
# In-process A/B of every build in marl-snake_amd/build/var (scripts/ab_probe.py)
# for the configs in ABCFGS, with the environment in ABENV.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out/ab2
for c in ${ABCFGS:-cfg3}; do
  n=65536; [ $c = cfg2 ] && n=4096; [ $c = cfg5 ] && n=8192
  env ${ABENV:-X=1} timeout -k 10 300 python scripts/ab_probe.py --cfg $c --N $n marl-snake_amd/build/var/*.so > gpurun_out/ab2/$c.log 2>&1 || exit 3
  tail -1 gpurun_out/ab2/$c.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); print('$c', {k[9:-3]:(v['auto']['median_ms'],v['fresh']['median_ms']) for k,v in d.items() if isinstance(v,dict)})"
done
