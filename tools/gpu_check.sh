#!/bin/bash
# GPU round check: parity tests, smoke, a short bench.  Every GPU step has its own time limit;
# a crash / abort / timeout stops the script (no further GPU work in that call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
stop_if_fatal() {  # $1 = exit status of a GPU step
    case "$1" in 124|134|137|139) echo "fatal status $1: stopping"; exit "$1";; esac
}
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
st=$?; echo "pytest status $st"; tail -5 gpurun_out/gpu_tests.log; stop_if_fatal $st
echo "== smoke"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
st=$?; echo "smoke status $st"; cat gpurun_out/smoke.log | tail -3; stop_if_fatal $st
echo "== bench ${BENCH_ARGS}"
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
st=$?; echo "bench status $st"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $st
