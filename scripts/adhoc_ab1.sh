set -e
V=marl-snake_amd/build/var
timeout -k 10 400 python scripts/ab.py --out gpurun_out/r06_ab_fork --rounds 3 "old=SNAKE_LIB=$V/libsnake_old.so;--config cfg3s8" "new=--config cfg3s8" "bgt2=SNAKE_LIB=$V/libsnake_bgt2.so;--config cfg3s8" "bgt4=SNAKE_LIB=$V/libsnake_bgt4.so;--config cfg3s8" > gpurun_out/r06_ab_fork_cfg3s8.txt 2>&1
timeout -k 10 300 python scripts/ab.py --out gpurun_out/r06_ab_fork --rounds 3 "old=SNAKE_LIB=$V/libsnake_old.so;--config cfg2" "new=--config cfg2" "bgt2=SNAKE_LIB=$V/libsnake_bgt2.so;--config cfg2" > gpurun_out/r06_ab_fork_cfg2.txt 2>&1
timeout -k 10 300 python scripts/ab.py --out gpurun_out/r06_ab_fork --rounds 3 "old=SNAKE_LIB=$V/libsnake_old.so;--config cfg5" "new=--config cfg5" > gpurun_out/r06_ab_fork_cfg5.txt 2>&1
