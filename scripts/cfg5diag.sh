set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/d5
for l in a_base b_kargs c_lane; do
  SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --steps 400 --warmup 100 > gpurun_out/d5/$l.log 2>&1 || { echo fail $l; tail -5 gpurun_out/d5/$l.log; exit 3; }
  echo $l; tail -1 gpurun_out/d5/$l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'))"
done
timeout -k 10 300 python scripts/ab_probe.py --cfg cfg3 marl-snake_amd/build/var/libsnake_a_base.so marl-snake_amd/build/var/libsnake_c_lane.so > gpurun_out/d5/ab3.log 2>&1 && tail -1 gpurun_out/d5/ab3.log
