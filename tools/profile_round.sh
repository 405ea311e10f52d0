#!/bin/bash
# Round profile: kernel trace + PMC passes at 1024 replicas (tools/profile.sh), then the
# kernel trace alone at the headline config (4096 replicas; its PMC pass hangs in rocprofv3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R=${ROUND:-r01d}
TAG=${R}_1024 PROF_ARGS="--replicas 1024 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/profile.sh || exit $?
echo "== kernel trace at 4096"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_4096_kt -o run \
    -- python3 bench.py --replicas 4096 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/${R}_4096_bench.json 2> gpurun_out/${R}_4096_kt.log
st=$?; echo "status $st"; tail -2 gpurun_out/${R}_4096_kt.log; exit $st
