#!/bin/bash
# key list A/B (k_runs) + incremental tests/bench + batch parity tests
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_incr.py tests/test_gpu_merge.py tests/test_fugue.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
st=$?; tail -3 gpurun_out/t.log; grep -E "FAILED|ERROR" gpurun_out/t.log | head; case $st in 0|1) ;; *) exit $st;; esac
LIBS="libcrdt_hip_nokey.so libcrdt_hip.so" ARGS="--lanes 1" bash tools/ab_libs.sh || exit 1
timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 3 --warmup 1 > gpurun_out/upinc.json 2> gpurun_out/upinc.err
st=$?; python3 -c "import json;d=json.load(open('gpurun_out/upinc.json'));print({k:d[k] for k in ('len_speedup_mean','len_speedup_median','lens_ok')}, round(d['incremental']['len_ms_mean']*1e3,1), round(d['full']['len_ms_mean']*1e3,1))"; exit $st
