#!/bin/bash
# k_classify change: the GPU suite, then the headline A/B against the committed build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/cls_tests.log 2>&1
st=$?; tail -3 gpurun_out/cls_tests.log; [ $st -eq 0 ] || exit $st
LIBS="libcrdt_hip_head.so libcrdt_hip.so" ARGS="--lanes 1 --raw-companion 0 --plain-companion 0" bash tools/ab_libs.sh || exit 1
LIBS="libcrdt_hip_head.so libcrdt_hip.so" ARGS="--raw-companion 0 --plain-companion 0 --order fugue" bash tools/ab_libs.sh
