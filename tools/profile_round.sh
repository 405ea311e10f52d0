#!/bin/bash
# Round profile at the headline config (4 traces x 4096 replicas): rocprofv3 kernel trace + stats
# of the default bench command, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (one lane:
# the profiler serialises dispatches anyway), summarised per kernel in bytes per item.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R=${ROUND:-r02a}
mkdir -p gpurun_out
echo "== kernel trace at 4096 (default bench command)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_kt -o run \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --companion-replicas 0 \
    --raw-companion 0 > gpurun_out/${R}_bench_4096.json 2> gpurun_out/${R}_kt.log
st=$?; echo "status $st"; tail -2 gpurun_out/${R}_kt.log
case $st in 0) ;; *) exit $st;; esac
for ctr in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $ctr at 4096"
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${R}_${ctr} -o run \
        -- python3 bench.py --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --companion-replicas 0 \
        --plain-companion 0 --raw-companion 0 \
        > gpurun_out/${R}_${ctr}.log 2>&1
    st=$?; echo "status $st"; tail -2 gpurun_out/${R}_${ctr}.log
    case $st in 0) ;; *) exit $st;; esac
done
