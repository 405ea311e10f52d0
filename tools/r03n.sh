#!/bin/bash
# j-list A/B (k_runs seq-head keys) + merge parity tests
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_scale.py tests/test_fugue.py tests/test_store.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
st=$?; tail -3 gpurun_out/t.log; grep -E "FAILED|ERROR" gpurun_out/t.log | head; case $st in 0|1) ;; *) exit $st;; esac
LIBS="libcrdt_hip_noj.so libcrdt_hip.so" ARGS="--lanes 1" bash tools/ab_libs.sh || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --companion-replicas 0 --config1-seconds 0 > gpurun_out/b2.json 2> gpurun_out/b2.err
st=$?; python3 -c "import json;d=json.load(open('gpurun_out/b2.json'));print('2 lanes', round(d['ms_per_step'],3), '1 lane', round(d['ms_per_step_1_lane'],3), d['digests_ok'])"; exit $st
