#!/bin/bash
# Kernel-trace timelines of several library builds (scripts/trace_gaps.py per
# build): scripts/prof_libs.sh tag ... -> marl-snake_amd/build/var/libsnake_<tag>.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for tag in "$@"; do
    SNAKE_LIB=marl-snake_amd/build/var/libsnake_$tag.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pl_$tag -o run --output-format csv -- python3 bench.py --steps ${STEPS:-300} --warmup 100 --no-cpu-baseline --timing-stride 0 > gpurun_out/pl_$tag.log 2>&1 || exit $?
    f=$(find gpurun_out/pl_$tag -name '*kernel_trace.csv' | head -1)
    echo "== $tag"
    python3 scripts/trace_gaps.py "$f"
done
