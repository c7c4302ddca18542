set -u
O=gpurun_out/r05k; mkdir -p $O
V=marl-snake_amd/build/var
B="SNAKE_LIB=$V/libsnake_base.so;"; N="SNAKE_LIB=$V/libsnake_nocoop.so;"; W="SNAKE_LIB=$V/libsnake_wbnocoop.so;"
timeout -k 10 1000 python -u scripts/ab.py --out $O --rounds 2 \
  "win_base=$B--steps 20 --warmup 5" "win_nt=$N--steps 20 --warmup 5" "win_wb=$W--steps 20 --warmup 5" \
  "c3_base=$B--config cfg3" "c3_nt=$N--config cfg3" "c3_wb=$W--config cfg3" \
  "c4_base=$B--config cfg4" "c4_nt=$N--config cfg4" "c4_wb=$W--config cfg4" \
  "c2_base=$B--config cfg2" "c2_wb=$W--config cfg2" \
  "c5_base=$B--config cfg5" "c5_wb=$W--config cfg5" | grep median
