#!/bin/bash
# GPU tests, then an A/B bench of the libraries named in $LIBS (default: the in-tree build).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for L in ${LIBS:-libcrdt_hip.so libcrdt_hip.so}; do
  CRDT_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab_$L.json 2> gpurun_out/bench.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$L.json'));print('$L',round(d['ms_per_step'],3),d['digests_ok'],{k:round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
done
