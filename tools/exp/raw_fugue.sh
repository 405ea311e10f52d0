#!/bin/bash
# Raw encode (4 slots per lane): its tests and the raw companion line; then the Fugue line with
# waves grouped by trace (default) against ungrouped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_merge.py -k "raw_soa" > gpurun_out/rf_tests.log 2>&1
st=$?; tail -2 gpurun_out/rf_tests.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u bench.py --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 --plain-companion 0 \
    > gpurun_out/rf_raw.json 2> gpurun_out/rf_raw.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/rf_raw.json').read().strip().splitlines()[-1]); r=d['companion_raw_soa']; print('raw', r['ms_per_step'], r['encode_ms'], r['digests_ok'], 'main', d['ms_per_step'], d['digests_ok'])"
for rep in 1 2; do
  for g in -1 0; do
    timeout -k 10 300 python -u bench.py --order fugue --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 \
        --plain-companion 0 --raw-companion 0 --steps 6 --group-docs $g > gpurun_out/rf_f$g.json 2> gpurun_out/rf_f$g.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/rf_f$g.json').read().strip().splitlines()[-1]); print('fugue group $g', round(d['ms_per_step'],3), d['digests_ok'], d['config']['waves'], {k: round(v['ms'],2) for k,v in d['kernels'].items() if v['launches']})"
  done
done
