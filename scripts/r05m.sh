set -u
O=gpurun_out/r05m; mkdir -p $O
V=marl-snake_amd/build/var
run() { n=$1; shift; timeout -k 10 200 python scripts/$@ > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 3; }; echo "$n $(cut -c1-1500 $O/$n.json)"; }
run items_c3 post_items.py $V/libsnake_stamps.so --cfg cfg3
run items_win post_items.py $V/libsnake_stamps.so --cfg cfg3 --skip 5 --steps 20
run logic_c3 logic_stamps.py $V/libsnake_stamps.so --cfg cfg3
