#!/bin/bash
# (Experiment, removed after measuring: 8.39-8.57 ms default vs 8.9-12.8 with any CU share.)
# A/B: level-1 stream held to a CU share (--l1-split 1 --l1-cus N) against the default two lanes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
run() {
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --companion-replicas 0 \
        --config1-seconds 0 --raw-companion 0 --plain-companion 0 $1 > gpurun_out/cum.json 2> gpurun_out/cum.err
    st=$?
    case $st in 0|1) ;; *) echo "status $st for $1"; tail -5 gpurun_out/cum.err; exit $st;; esac
    python3 - "$1" gpurun_out/cum.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:44s} {d['ms_per_step']:7.3f} ms ok={d['digests_ok']}")
PY
}
for rep in 1 2; do
    run "--lanes 2"
    run "--lanes 1 --l1-split 1"
    run "--lanes 1 --l1-split 1 --l1-cus 128"
    run "--lanes 1 --l1-split 1 --l1-cus 192"
    run "--lanes 2 --l1-split 1 --l1-cus 160"
    run "--lanes 2 --l1-split 1 --l1-cus 208"
done
