#!/bin/bash
# experiment library ($LIB) with the probe on one document of each trace ($DOCS), one lane
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for p in ${DOCS:-0 1 2 3}; do
    CRDT_HIP_LIB=${LIB:-libcrdt_hip_exp.so} CRDT_HIP_PROBE=$p timeout -k 10 120 python bench.py --replicas ${REPL:-4096} --steps 1 --warmup 1 \
        --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 --lanes 1 > gpurun_out/exp_$p.log 2>&1
    st=$?; grep "doctree\]\|twice\]" gpurun_out/exp_$p.log | tail -${TAILN:-3}
    case $st in 0|1) ;; *) echo "status $st"; tail -5 gpurun_out/exp_$p.log; exit $st;; esac
done
