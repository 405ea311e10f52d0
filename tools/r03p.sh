#!/bin/bash
# incremental tests on the new forest, A/B against the base build, then SQ passes + k_inc trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_incr.py > gpurun_out/r03p_incr_tests.log 2>&1
st=$?; tail -3 gpurun_out/r03p_incr_tests.log; [ $st = 0 ] || exit $st
LIBS="libcrdt_hip_base.so libcrdt_hip.so" REPS=3 bash tools/ab_inc.sh || exit $?
bash tools/r03o.sh
