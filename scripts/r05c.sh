set -u
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
L=SNAKE_LIB=marl-snake_amd/build/var/libsnake_t1.so
timeout -k 10 900 python -u scripts/ab.py --out $O --rounds 2 \
  "win_old=--steps 20 --warmup 5 --spawn-ahead 3" "win_new=--steps 20 --warmup 5" "win_t1=$L;--steps 20 --warmup 5" \
  "c3_old=--config cfg3 --spawn-ahead 3" "c3_new=--config cfg3" "c3_t1=$L;--config cfg3" \
  "c4_old=--config cfg4 --spawn-ahead 3" "c4_new=--config cfg4" "c4_t1=$L;--config cfg4" \
  "c2_old=--config cfg2 --spawn-ahead 3" "c2_new=--config cfg2" "c2_t1=$L;--config cfg2"
