#!/bin/bash
# A/B of library builds ($LIBS: space-separated .so names in crdt-benches_amd/), each run twice in
# alternation with the same short headline bench; prints ms/step per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
    for lib in $LIBS; do
        CRDT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-8} --warmup 2 \
            --companion-replicas 0 --config1-seconds 0 $ARGS > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err
        st=$?
        # (status 1: the line was printed but a check failed, e.g. a timing experiment whose
        # results are wrong on purpose; anything else ends the run)
        case $st in 0|1) ;; *) echo "status $st for $lib"; tail -5 gpurun_out/ab_$lib.err; exit $st;; esac
        python3 - "$lib" gpurun_out/ab_$lib.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {n: round(v["ms"], 2) for n, v in d["kernels"].items() if v["launches"]}
print(f"{sys.argv[1]:28s} {d['ms_per_step']:7.3f} ms ok={d['digests_ok']} {k}")
PY
    done
done
