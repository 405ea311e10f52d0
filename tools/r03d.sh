#!/bin/bash
# incremental-merge tests and a per-phase profile of the incremental loop
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_incr.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/incr_tests.log 2>&1
st=$?; tail -12 gpurun_out/incr_tests.log; case $st in 0|1) ;; *) exit $st;; esac
CRDT_INC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 1 --warmup 0 > gpurun_out/upinc_prof.json 2> gpurun_out/upinc_prof.err
st=$?; grep "^\[inc\]" gpurun_out/upinc_prof.err | tail -5; head -c 600 gpurun_out/upinc_prof.json; echo; exit $st
