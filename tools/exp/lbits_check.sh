#!/bin/bash
# Fugue left-child bits in LDS: Fugue and merge tests, then the Fugue and RGA A/B against HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/lb_tests.log 2>&1
st=$?; tail -3 gpurun_out/lb_tests.log; [ $st -eq 0 ] || exit $st
LIBS="libcrdt_hip_head.so libcrdt_hip.so" ARGS="--raw-companion 0 --plain-companion 0 --order fugue" bash tools/ab_libs.sh || exit 1
LIBS="libcrdt_hip_head.so libcrdt_hip.so" ARGS="--raw-companion 0 --plain-companion 0 --lanes 1" bash tools/ab_libs.sh
