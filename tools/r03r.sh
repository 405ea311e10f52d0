#!/bin/bash
# k_doctree phase probe per document for builds with 12 / 8 / 4 runs per thread (CRDT_DOC_J);
# batches without the documents a build cannot hold in LDS (CRDT_BENCH_TRACES)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() {  # lib traces probe-doc
    CRDT_BENCH_TRACES=$2 CRDT_HIP_LIB=libcrdt_hip_$1.so CRDT_HIP_PROBE=$3 timeout -k 10 120 python bench.py --replicas 256 \
        --steps 1 --warmup 1 --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 > gpurun_out/pr_$1_$3.log 2>&1
    st=$?; echo "$1 $(grep "doctree\]" gpurun_out/pr_$1_$3.log | tail -1 | cut -c1-40) ... $(grep "doctree\]" gpurun_out/pr_$1_$3.log | tail -1 | grep -o 'total [0-9.]*')"
    case $st in 0|1) ;; *) echo "status $st"; tail -5 gpurun_out/pr_$1_$3.log; exit $st;; esac
}
for rep in 1 2; do
    for lib in pj12 pj8; do
        run $lib automerge-paper,rustcode,sveltecomponent 0
        run $lib automerge-paper,rustcode,sveltecomponent 1
        run $lib automerge-paper,rustcode,sveltecomponent 2
    done
    for lib in pj12 pj8 pj4; do run $lib sveltecomponent 0; done
done
