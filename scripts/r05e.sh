set -u
O=gpurun_out/r05e; mkdir -p $O
V=marl-snake_amd/build/var
timeout -k 10 900 python -u scripts/ab.py --out $O --rounds 2 \
  "win_old=--steps 20 --warmup 5 --spawn-ahead 3" "win_hyb=SNAKE_LIB=$V/libsnake_hyb.so;--steps 20 --warmup 5" "win_hyb1=SNAKE_LIB=$V/libsnake_hyb1.so;--steps 20 --warmup 5" \
  "c3_old=--config cfg3 --spawn-ahead 3" "c3_hyb=SNAKE_LIB=$V/libsnake_hyb.so;--config cfg3" "c3_hyb1=SNAKE_LIB=$V/libsnake_hyb1.so;--config cfg3" \
  "c2_old=--config cfg2 --spawn-ahead 3" "c2_hyb=SNAKE_LIB=$V/libsnake_hyb.so;--config cfg2" "c2_hyb1=SNAKE_LIB=$V/libsnake_hyb1.so;--config cfg2" \
  "win_enc2=SNAKE_LIB=$V/libsnake_enc2.so;--steps 20 --warmup 5" "c3_enc2=SNAKE_LIB=$V/libsnake_enc2.so;--config cfg3" \
  "c4_enc2=SNAKE_LIB=$V/libsnake_enc2.so;--config cfg4" "c2_enc2=SNAKE_LIB=$V/libsnake_enc2.so;--config cfg2"
