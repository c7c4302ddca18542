set -u
O=gpurun_out/r05g; mkdir -p $O
V=marl-snake_amd/build/var
run() { n=$1; L=$2; shift 2; timeout -k 10 200 python scripts/post_items.py $V/$L "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 3; }; echo "$n $(python3 -c "import json; d=json.load(open('$O/$n.json')); print(d['span_ns'], d['enc_end_ns'], d['last_to_end'], d['encode_blocks'])")"; }
run c3 libsnake_stamps.so --cfg cfg3 --spawn-ahead 3
run c3_enconly libsnake_stenc2.so --cfg cfg3 --spawn-ahead 3
run c4 libsnake_stamps.so --cfg cfg4 --spawn-ahead 3
run c4_enconly libsnake_stenc2.so --cfg cfg4 --spawn-ahead 3
run win libsnake_stamps.so --cfg cfg3 --spawn-ahead 3 --skip 5 --steps 20
