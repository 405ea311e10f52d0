#!/bin/bash
# keyseq change: the affected GPU tests, then the headline A/B against the committed build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_merge.py -k "seq_head_keys or raw_soa or runs_slots or trace_merge_byte_exact or malformed or text_paths or contraction or replica_batch or mixed_ascii or learnt_plan" \
    > gpurun_out/ks_tests.log 2>&1
st=$?; tail -3 gpurun_out/ks_tests.log; [ $st -eq 0 ] || exit $st
LIBS="libcrdt_hip_head.so libcrdt_hip.so" ARGS="--lanes 1 --raw-companion 0 --plain-companion 0" bash tools/ab_libs.sh || exit 1
LIBS="libcrdt_hip_head.so libcrdt_hip.so" ARGS="--raw-companion 0 --plain-companion 0" bash tools/ab_libs.sh
timeout -k 10 300 python -u bench.py --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 --plain-companion 0 \
    > gpurun_out/ks_raw.json 2> gpurun_out/ks_raw.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/ks_raw.json').read().strip().splitlines()[-1]); r=d['companion_raw_soa']; print('raw', r['ms_per_step'], r['encode_ms'], r['digests_ok'], 'main', d['ms_per_step'], d['digests_ok'])"
