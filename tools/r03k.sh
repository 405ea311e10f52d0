#!/bin/bash
# incremental merge variants (LDS-staged words; 512 threads; no run contraction) + tests
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_incr.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/incr_tests.log 2>&1
st=$?; tail -2 gpurun_out/incr_tests.log; case $st in 0|1) ;; *) exit $st;; esac
for rep in 1 2; do
for lib in libcrdt_hip.so libcrdt_hip_t512.so libcrdt_hip_noruns.so; do
  CRDT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 3 --warmup 1 > gpurun_out/upinc_$lib.json 2> gpurun_out/upinc_$lib.err
  st=$?; python3 -c "import json,sys;d=json.load(open('gpurun_out/upinc_$lib.json'));print('$lib', {k:round(d[k],3) for k in ('len_speedup_mean','len_speedup_median')}, d['lens_ok'], round(d['incremental']['len_ms_mean']*1e3,1), round(d['full']['len_ms_mean']*1e3,1))"; case $st in 0|1) ;; *) exit $st;; esac
done
done
