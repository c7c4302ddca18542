set -u
O=gpurun_out/r05j; mkdir -p $O
V=marl-snake_amd/build/var
timeout -k 10 120 scripts/microbench/storebw > $O/storebw.txt 2>&1 || { echo storebw failed; exit 3; }
cat $O/storebw.txt
timeout -k 10 200 python scripts/attemptbench.py $V/libsnake_dbench.so > $O/attempt.txt 2>&1 || { echo attemptbench failed; tail -20 $O/attempt.txt; exit 3; }
tail -1 $O/attempt.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "cfg5 or 40 or big_44 or snapshot" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 600 python -u scripts/ab.py --out $O --rounds 2 "c5_nocoop=SNAKE_LIB=$V/libsnake_nocoop.so;--config cfg5" "c5_coop=--config cfg5" | grep median
