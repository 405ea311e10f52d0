#!/bin/bash
# 2-byte character column + incremental run contraction: all GPU tests, cp2 A/B, incremental bench
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
st=$?; tail -3 gpurun_out/gpu_tests.log; grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20; case $st in 0|1) ;; *) exit $st;; esac
A="--cp2 0" B="--cp2 1" LANES=1 bash tools/ab_args.sh || exit 1
CRDT_INC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 1 --warmup 0 > gpurun_out/upinc_prof.json 2> gpurun_out/upinc_prof.err
st=$?; grep "^\[inc\]" gpurun_out/upinc_prof.err | sed -n '100,104p'; case $st in 0|1) ;; *) exit $st;; esac
timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 3 --warmup 1 > gpurun_out/upinc.json 2> gpurun_out/upinc.err
st=$?; python3 -c "import json;d=json.load(open('gpurun_out/upinc.json'));print({k:d[k] for k in ('len_speedup_mean','len_speedup_median','lens_ok')}, d['incremental'], d['full'])"; exit $st
