#!/bin/bash
# One development iteration on the GPU: merge parity tests ($TESTS), the k_doctree probe of the
# in-tree probe build (one lane), then an A/B of $LIBS (alternating, one lane unless $LANES).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_merge.py tests/test_fugue.py} -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/iter_tests.log 2>&1
st=$?; tail -1 gpurun_out/iter_tests.log
case $st in 0|5) ;; *) grep -E "FAILED|Error|assert" gpurun_out/iter_tests.log | head -20; exit $st;; esac
for pl in ${PLIBS:-libcrdt_hip_probe.so}; do
for p in ${DOCS:-1 2}; do
    CRDT_HIP_LIB=$pl CRDT_HIP_PROBE=$p timeout -k 10 120 python bench.py --replicas 4096 --steps 1 --warmup 1 \
        --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 --lanes 1 > gpurun_out/iter_probe_$p.log 2>&1
    st=$?; grep "doctree\]\|walk\]" gpurun_out/iter_probe_$p.log | tail -2
    case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/iter_probe_$p.log; exit $st;; esac
done
done
for rep in 1 2; do
    for lib in ${LIBS:-libcrdt_hip_base.so libcrdt_hip.so}; do
        CRDT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-8} --warmup 2 \
            --companion-replicas 0 --config1-seconds 0 --lanes ${LANES:-1} $ARGS > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err
        st=$?
        case $st in 0|1) ;; *) echo "status $st for $lib"; tail -5 gpurun_out/ab_$lib.err; exit $st;; esac
        python3 - "$lib" gpurun_out/ab_$lib.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {n: round(v["ms"], 2) for n, v in d["kernels"].items() if v["launches"]}
print(f"{sys.argv[1]:28s} {d['ms_per_step']:7.3f} ms ok={d['digests_ok']} {k}")
PY
    done
done
