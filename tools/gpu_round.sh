#!/bin/bash
# GPU check of the current build: every -m gpu test (one process), smoke, the default bench line,
# then optional extra bench lines ($EXTRA: ';'-separated argument lists).  Every GPU step has its
# own time limit; a crash / abort / timeout stops the script (no further GPU work in that call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
stop_if_fatal() {  # $1 = exit status of a GPU step
    case "$1" in 0) ;; 124|134|137|139) echo "fatal status $1: stopping"; exit "$1";; *) echo "status $1";; esac
}
if [ -z "$SKIP_TESTS" ]; then
    echo "== pytest -m gpu ${TESTS:-tests}"
    timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests.log 2>&1
    st=$?; tail -4 gpurun_out/gpu_tests.log; grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20
    stop_if_fatal $st
    echo "== smoke"
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    st=$?; tail -2 gpurun_out/smoke.log; stop_if_fatal $st
fi
i=0
IFS=';' read -ra LINES <<< "${BENCH:-}"
for args in "${LINES[@]}"; do
    i=$((i+1))
    echo "== bench $i: $args"
    timeout -k 10 600 python -u bench.py $args > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err
    st=$?; tail -3 gpurun_out/bench_$i.err; head -c 1500 gpurun_out/bench_$i.json; echo
    stop_if_fatal $st
done
