#!/bin/bash
# k_doctree phase timings (probe build) with ONE lane (no level-0 kernels of another lane beside
# it), one document of each trace; then the GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for p in 0 1 2 3; do
    CRDT_HIP_LIB=libcrdt_hip_probe.so CRDT_HIP_PROBE=$p timeout -k 10 120 python bench.py --replicas ${REPL:-4096} --steps 1 --warmup 1 \
        --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 --lanes 1 > gpurun_out/probe1_$p.log 2>&1
    st=$?; grep "doctree\]" gpurun_out/probe1_$p.log | tail -1
    case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/probe1_$p.log; exit $st;; esac
done
