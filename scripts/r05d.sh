set -u
O=gpurun_out/r05d; mkdir -p $O
L=marl-snake_amd/build/var/libsnake_stamps.so
run() { n=$1; shift; timeout -k 10 200 python scripts/post_items.py $L "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 3; }; echo "$n $(cat $O/$n.json)"; }
run c3_old --cfg cfg3 --spawn-ahead 3
run c3_new --cfg cfg3
run win_old --cfg cfg3 --spawn-ahead 3 --skip 5 --steps 20
run win_new --cfg cfg3 --skip 5 --steps 20
run c2_old --cfg cfg2 --spawn-ahead 3
run c2_new --cfg cfg2
run c4_old --cfg cfg4 --spawn-ahead 3
