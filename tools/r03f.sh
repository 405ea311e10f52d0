#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CRDT_INC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 1 --warmup 0 > gpurun_out/upinc_prof.json 2> gpurun_out/upinc_prof.err
st=$?; grep "^\[inc-forest\]" gpurun_out/upinc_prof.err | sed -n '100,110p'; exit $st
