#!/bin/bash
# GPU tests only (optionally a -k filter in $K), then smoke; every GPU step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/gpu_tests.log 2>&1
st=$?; echo "pytest status $st"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
case $st in 0) ;; *) grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $st;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
st=$?; echo "smoke status $st"; tail -2 gpurun_out/smoke.log; exit $st
