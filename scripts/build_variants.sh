#!/bin/bash
# Build alternative libsnake_amd.so variants into marl-snake_amd/build/var/ for
# in-process A/B timing (scripts/ab_probe.py). Usage: build_variants.sh tag:flags ...
#   tag:flags   -> current sources compiled with extra flags (e.g. lb4:-DSNAKE_STEP_MIN_WAVES=4)
#   tag@commit  -> the sources of a git commit
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/marl-snake_amd/build/var
mkdir -p "$OUT"
FLAGS="-O3 -fPIC -std=c++17 -ffp-contract=off --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None"
for spec in "$@"; do
    if [[ $spec == *@* ]]; then
        tag=${spec%@*}; rev=${spec#*@}
        src=$OUT/src_$tag; mkdir -p "$src/csrc" "$src/include"
        for f in snake_kernels.hip snake_capi.cpp snake_internal.h dqn_kernels.hip dqn32_kernels.hip; do
            git -C "$ROOT" show "$rev:marl-snake_amd/csrc/$f" > "$src/csrc/$f"
        done
        git -C "$ROOT" show "$rev:include/snake_env.h" | sed "s/define SNAKE_ABI_VERSION .*/define SNAKE_ABI_VERSION ${ABI:-8}/" > "$src/include/snake_env.h"
        sed -i 's#"../../include/snake_env.h"#"../include/snake_env.h"#' "$src/csrc/snake_internal.h"
        extra=""; dir=$src/csrc
    else
        tag=${spec%%:*}; extra=${spec#*:}; dir=$ROOT/marl-snake_amd/csrc
        [[ $extra == "$spec" ]] && extra=""
    fi
    dqn=""; [[ -f $dir/dqn_kernels.hip ]] && dqn=$dir/dqn_kernels.hip; [[ -f $dir/dqn32_kernels.hip ]] && dqn="$dqn $dir/dqn32_kernels.hip"
    /opt/rocm/bin/hipcc $FLAGS $extra -shared -o "$OUT/libsnake_$tag.so" "$dir/snake_kernels.hip" "$dir/snake_capi.cpp" $dqn &
done
wait
ls -la "$OUT"/*.so
