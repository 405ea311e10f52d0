#!/bin/bash
# k_doctree phase times (probe build) of automerge-paper and seph-blog1 documents with one lane
# and with two lanes (the other lane's level 0 beside it); $ARGS: extra bench arguments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for L in 1 2; do for p in 0 3; do
    CRDT_HIP_LIB=libcrdt_hip_probe.so CRDT_HIP_PROBE=$p timeout -k 10 120 python bench.py --replicas 1024 --steps 1 --warmup 1 --lanes $L \
        --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 $ARGS > gpurun_out/probe_$p.log 2>&1
    st=$?; echo "lanes $L $ARGS: $(grep 'doctree\]' gpurun_out/probe_$p.log | tail -1)"
    case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/probe_$p.log; exit $st;; esac
done; done
