#!/bin/bash
# One GPU-box session: smoke -> parity tests -> short bench (+ optional rocprof).
# Each GPU step has its own time limit; a fault-like exit (abort, segfault,
# timeout) ends the script, an ordinary test failure (rc 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fault-like exit $rc: stopping"; exit $rc; fi
}
for s in "$@"; do
    case $s in
        build) step build 300 python -c "import __graft_entry__ as g; g.build()" ;;
        smoke) step smoke 300 python __graft_entry__.py smoke ;;
        tests) step tests 900 python -m pytest tests -x -q -m gpu ;;
        testsv) step tests 900 python -m pytest tests -q -m gpu -rf ;;
        bench) step bench 600 python bench.py ;;
        benchq) step bench 300 python bench.py --steps 200 --warmup 50 --cpu-seconds 5 ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
