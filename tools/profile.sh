#!/bin/bash
# Per-kernel profile of bench.py: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate PMC passes (gfx950: FETCH_SIZE reports half of wide streaming reads).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-prof}
ARGS=${PROF_ARGS:-"--replicas 512 --steps 3 --warmup 1 --no-cpu-baseline"}
mkdir -p gpurun_out
echo "== kernel trace: $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run \
    -- python3 bench.py $ARGS > gpurun_out/${TAG}_kt.log 2>&1
st=$?; echo "status $st"; tail -3 gpurun_out/${TAG}_kt.log
case $st in 0) ;; *) exit $st;; esac
for ctr in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $ctr"
    timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${TAG}_${ctr} -o run \
        -- python3 bench.py $ARGS > gpurun_out/${TAG}_${ctr}.log 2>&1
    st=$?; echo "status $st"; tail -2 gpurun_out/${TAG}_${ctr}.log
    case $st in 0) ;; *) exit $st;; esac
done
find gpurun_out/${TAG}_* -name "*.csv" | head -20
