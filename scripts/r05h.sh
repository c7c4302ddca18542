set -u
O=gpurun_out/r05h; mkdir -p $O
V=marl-snake_amd/build/var
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "full_size or batch_matches or spawn_ahead_is or snapshot or shards" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 900 python -u scripts/ab.py --out $O --rounds 2 \
  "win_base=SNAKE_LIB=$V/libsnake_base.so;--steps 20 --warmup 5" "win_new=--steps 20 --warmup 5" \
  "c3_base=SNAKE_LIB=$V/libsnake_base.so;--config cfg3" "c3_new=--config cfg3" \
  "c4_base=SNAKE_LIB=$V/libsnake_base.so;--config cfg4" "c4_new=--config cfg4" \
  "c2_base=SNAKE_LIB=$V/libsnake_base.so;--config cfg2" "c2_new=--config cfg2" \
  "c3_enc2=SNAKE_LIB=$V/libsnake_enc2.so;--config cfg3" "c4_enc2=SNAKE_LIB=$V/libsnake_enc2.so;--config cfg4"
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l)
    if 'enc2' in d['ab_name']: print(d['ab_name'], d['ab_round'], {k:round(v*1e3,1) for k,v in d['kernels'].items()})
"
