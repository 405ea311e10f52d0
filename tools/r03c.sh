#!/bin/bash
# k_doctree staging / text-out change: GPU tests, probe, A/B against the previous engine, and the
# incremental-merge bench with a kernel trace.
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
st=$?; tail -4 gpurun_out/gpu_tests.log; grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20; case $st in 0|1) ;; *) exit $st;; esac
REPL=1024 bash tools/probe.sh || exit 1
LIBS="libcrdt_hip_head.so libcrdt_hip.so" bash tools/ab_libs.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/upinc_kt -o run -- python3 bench.py --workload upstream_inc --steps 1 --warmup 1 > gpurun_out/upinc.json 2> gpurun_out/upinc.err
st=$?; tail -2 gpurun_out/upinc.err; head -c 2500 gpurun_out/upinc.json; echo; exit $st
