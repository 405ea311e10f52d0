#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
A="--cp2 0" B="--cp2 1" LANES=1 bash tools/ab_args.sh || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --companion-replicas 0 --config1-seconds 0 --cp2 0 > gpurun_out/b2.json 2> gpurun_out/b2.err
st=$?; python3 -c "import json;d=json.load(open('gpurun_out/b2.json'));print('2 lanes', round(d['ms_per_step'],3), '1 lane', round(d['ms_per_step_1_lane'],3), d['digests_ok'])"; exit $st
