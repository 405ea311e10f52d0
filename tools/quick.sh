#!/bin/bash
# GPU tests (all), then the headline bench and the side workloads, each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));print(round(d['ms_per_step'],3),d['digests_ok'],round(d['roofline']['frac'],3),{k:round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
for W in ${SIDE:-}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload $W --steps 5 --warmup 2 > gpurun_out/side_$W.json 2> gpurun_out/side_$W.err || { tail gpurun_out/side_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/side_$W.json'));print('$W',round(d['ms_per_step'],3),d['digests_ok'],{k:round(v,3) for k,v in d.get('kernels_ms',{}).items()})"
done
