set -u
O=gpurun_out/r05o; mkdir -p $O
V=marl-snake_amd/build/var
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 600 python -u scripts/ab.py --out $O --rounds 3 \
  "c2_p2=SNAKE_LIB=$V/libsnake_prio2.so;--config cfg2" "c2_p3=--config cfg2" \
  "c4_p2=SNAKE_LIB=$V/libsnake_prio2.so;--config cfg4" "c4_p3=--config cfg4" | grep median
