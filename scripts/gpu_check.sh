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
        tests) step tests 1100 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread ;;
        testsv) step tests 1100 python -u -m pytest tests -v -m gpu -rf --timeout 400 --timeout-method thread ;;
        testsk) step tests 1100 python -u -m pytest tests -x -v -m gpu -k "$TESTK" --timeout 400 --timeout-method thread ;;
        bench) step bench 600 python bench.py ;;
        benchq) step bench 300 python bench.py --steps 200 --warmup 50 --cpu-seconds 5 ;;
        benchthr) for t in ${THRS:--1 1 2 3}; do
                      export SNAKE_SPAWN_THR=$t
                      step benchthr$t 300 python bench.py --no-cpu-baseline --steps 1000
                  done
                  unset SNAKE_SPAWN_THR ;;
        benchab) # VARS="A=1 B=2;A=3" : one short bench per ';'-separated env setting
                 IFS=';' read -ra sets <<< "$VARS"
                 i=0
                 for kv in "${sets[@]}"; do
                     i=$((i+1))
                     echo "-- set $i: $kv"
                     env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1000 > gpurun_out/benchab$i.log 2>&1
                     rc=$?
                     echo "benchab$i rc=$rc"; tail -1 gpurun_out/benchab$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'))"
                     if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fault-like exit $rc: stopping"; exit $rc; fi
                 done ;;
        benchnt) step benchnt 300 python bench.py --timing-stride 0 --no-cpu-baseline ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 300 --warmup 100 --no-cpu-baseline ;;
        probe) step probe 600 python scripts/perf_probe.py ;;
        rlat) step rlat 300 python scripts/perf_probe.py --reset-latency ;;
        stamps) step stamps 300 python scripts/reset_stamps.py marl-snake_amd/build/libsnake_stamps.so ;;
        lat) step lat 120 scripts/microbench/lat ;;
        gap) step gap 300 scripts/microbench/gap ;;
        forkjoin) step forkjoin 300 scripts/microbench/forkjoin ;;
        profserial) export SNAKE_LIB=marl-snake_amd/build/var/libsnake_${PROFLIB:-serial}.so
                    step profserial 600 rocprofv3 --kernel-trace -d gpurun_out/prof_${PROFLIB:-serial} -o run --output-format csv -- python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline --timing-stride 0
                    unset SNAKE_LIB ;;
        dbpmc) step dbpmc 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM --kernel-include-regex drawbench --output-format csv -d gpurun_out/dbpmc -o pmc -- python3 scripts/drawbench.py marl-snake_amd/build/db/libsnake_base.so ;;
        drawbench) for f in marl-snake_amd/build/db/*.so; do step drawbench 120 python scripts/drawbench.py $f; done ;;
        obsprof) step obsprof 300 python scripts/obs_profile.py marl-snake_amd/build/libsnake_stamps.so ;;
        ab) step ab 600 python scripts/ab_probe.py marl-snake_amd/build/var/*.so ;;
        ab2) step ab2 600 python scripts/ab_probe.py --cfg cfg2 --N 4096 marl-snake_amd/build/var/*.so ;;
        ab5) step ab5 600 python scripts/ab_probe.py --cfg cfg5 --N 8192 marl-snake_amd/build/var/*.so ;;
        pmc) K='k_logic|k_autoreset|k_encode'
             B='python3 bench.py --steps 40 --warmup 60 --no-cpu-baseline'
             step pmcF 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcF -o pmc -- $B
             step pmcW 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcW -o pmc -- $B
             step pmcSQ 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcSQ -o pmc -- $B ;;
        hostov) step hostov 300 python scripts/host_overhead.py ;;
        counters) step counters 60 rocprofv3 -L ;;
        prof3) for c in ${CFGS:-cfg3}; do
                   step prof_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 300 --warmup 100 --no-cpu-baseline --timing-stride 0
               done ;;
        pmcA) K='k_logic|k_autoreset|k_encode'
              B="python3 bench.py --config ${CFG:-cfg3} --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
              step pmcA 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcA -o pmc -- $B ;;
        pmcB) K='k_logic|k_autoreset|k_encode'
              B="python3 bench.py --config ${CFG:-cfg3} --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
              step pmcB 300 rocprofv3 --pmc $PMCB --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcB -o pmc -- $B ;;
        pmcTr) K='k_logic|k_autoreset|k_encode'
               B="python3 bench.py --config ${CFG:-cfg3} --steps 40 --warmup 60 --no-cpu-baseline --timing-stride 0"
               step pmcF 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcF -o pmc -- $B
               step pmcW 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcW -o pmc -- $B ;;
        dqn) step dqn 300 python scripts/dqn_bench.py ;;
        dqnprof) step dqnprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dqnprof -o run --output-format csv -- python3 scripts/dqn_bench.py --no-torch ;;
        dqnpmc) step dqnpmc 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-include-regex k_dqn --output-format csv -d gpurun_out/dqnpmc -o pmc -- python3 scripts/dqn_bench.py --no-torch --steps 3 --warmup 1 ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
