#!/bin/bash
# GPU tests on the current build, then A/B against libcrdt_hip_base.so (headline bench, 1 and 2 lanes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03s_gpu_tests.log 2>&1
st=$?; tail -3 gpurun_out/r03s_gpu_tests.log; [ $st = 0 ] || exit $st
LIBS="libcrdt_hip_base.so libcrdt_hip.so" STEPS=8 bash tools/ab_libs.sh || exit $?
LIBS="libcrdt_hip_base.so libcrdt_hip.so" STEPS=8 ARGS="--lanes 1" bash tools/ab_libs.sh
