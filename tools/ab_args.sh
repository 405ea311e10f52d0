#!/bin/bash
# A/B of bench argument sets ($A and $B) on the in-tree library, alternating, one lane.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
    for v in A B; do
        args=${!v}
        timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-8} --warmup 2 \
            --companion-replicas 0 --config1-seconds 0 --lanes ${LANES:-1} $args > gpurun_out/abx_$v.json 2> gpurun_out/abx_$v.err
        st=$?
        case $st in 0|1) ;; *) echo "status $st for $v"; tail -5 gpurun_out/abx_$v.err; exit $st;; esac
        python3 - "$v: $args" gpurun_out/abx_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {n: round(v["ms"], 2) for n, v in d["kernels"].items() if v["launches"]}
print(f"{sys.argv[1]:28s} {d['ms_per_step']:7.3f} ms ok={d['digests_ok']} {k}")
PY
    done
done
