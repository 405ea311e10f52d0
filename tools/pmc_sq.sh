#!/bin/bash
# SQ counters per kernel (one rocprofv3 --pmc pass per counter group), 1024 replicas.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${PROF_ARGS:-"--replicas 1024 --steps 1 --warmup 1 --no-cpu-baseline"}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    echo "== pmc pass $i: $grp"
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sq$i -o run \
        -- python3 bench.py $ARGS > gpurun_out/sq$i.log 2>&1
    st=$?; echo "status $st"; tail -2 gpurun_out/sq$i.log
    case $st in 0) ;; *) exit $st;; esac
done
