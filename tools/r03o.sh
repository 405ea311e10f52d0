#!/bin/bash
# SQ counter passes of the end-of-round-3 build at the headline config (tools/pmc_sq.sh), and a
# kernel trace of the incremental len() workload (k_inc launch durations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PROF_ARGS="--replicas 4096 --steps 1 --warmup 1 --no-cpu-baseline --companion-replicas 0" \
    bash tools/pmc_sq.sh || exit $?
python3 tools/sq_summary.py gpurun_out > gpurun_out/r03o_sq_summary_4096.txt || exit 1
echo "== kernel trace of upstream_inc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03o_inc_kt -o run \
    -- python3 bench.py --workload upstream_inc --steps 2 --warmup 1 \
    > gpurun_out/r03o_inc.json 2> gpurun_out/r03o_inc.err
st=$?; echo "status $st"; head -c 300 gpurun_out/r03o_inc.json; echo
exit $st
