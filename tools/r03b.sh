#!/bin/bash
# Round 3 session 2: incremental-merge tests + bench, k_doctree probe, Fugue line.
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_incr.py tests/test_fugue.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/incr_tests.log 2>&1
st=$?; tail -15 gpurun_out/incr_tests.log; case $st in 0|1) ;; *) exit $st;; esac
timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 3 --warmup 1 > gpurun_out/upinc.json 2> gpurun_out/upinc.err
st=$?; tail -3 gpurun_out/upinc.err; head -c 2500 gpurun_out/upinc.json; echo; case $st in 0|1) ;; *) exit $st;; esac
REPL=1024 bash tools/probe.sh || exit 1
timeout -k 10 300 python -u bench.py --order fugue --steps 5 --warmup 2 --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 > gpurun_out/fugue.json 2> gpurun_out/fugue.err
st=$?; tail -2 gpurun_out/fugue.err; exit $st
