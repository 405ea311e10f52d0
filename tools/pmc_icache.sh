#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
A="--replicas 1024 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --companion-replicas 0 --plain-companion 0 --config1-seconds 0"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_WAVES SQ_IFETCH" \
           "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES"; do
    i=$((i+1))
    echo "== pass $i: $grp"
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/ic$i -o run -- python3 bench.py $A > gpurun_out/ic$i.log 2>&1
    st=$?; echo "status $st"; case $st in 0) ;; *) tail -3 gpurun_out/ic$i.log; exit $st;; esac
done
