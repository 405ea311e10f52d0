#!/bin/bash
# Gather mode (text_scatter 2): its text-path tests, then the headline A/B against phase C and
# the byte-scatter kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_merge.py \
    -k "text_paths" > gpurun_out/ga_tests.log 2>&1
st=$?; tail -12 gpurun_out/ga_tests.log; [ $st -eq 0 ] || exit $st
for rep in 1 2; do
  for lanes in 1 2; do
    for ts in 0 1 2; do
      timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --companion-replicas 0 --config1-seconds 0 \
          --raw-companion 0 --plain-companion 0 --lanes $lanes --text-scatter $ts > gpurun_out/ga.json 2> gpurun_out/ga.err
      st=$?; case $st in 0|1) ;; *) echo "status $st"; tail -5 gpurun_out/ga.err; exit $st;; esac
      python3 -c "import json; d=json.loads(open('gpurun_out/ga.json').read().strip().splitlines()[-1]); print('lanes $lanes ts $ts', round(d['ms_per_step'],3), d['digests_ok'], {k: round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
    done
  done
done
