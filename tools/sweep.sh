#!/bin/bash
# Parameter sweep of bench.py (each run its own time limit; stops at the first failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${SWEEP_BASE:-"--replicas 512 --steps 5 --warmup 2 --no-cpu-baseline"}
for arg in ${SWEEP_ARGS:-"--splitter-stride=64"}; do
    a=${arg//=/ }
    timeout -k 10 300 python3 -u bench.py $BASE $a > gpurun_out/sweep.json 2> gpurun_out/sweep.err
    st=$?
    if [ $st != 0 ]; then echo "$arg: status $st"; tail -3 gpurun_out/sweep.err; exit $st; fi
    python3 - "$arg" <<'PY'
import json, sys
d = json.load(open("gpurun_out/sweep.json"))
k = {n: round(v["ms"], 2) for n, v in d["kernels"].items()}
print(sys.argv[1], "ms/step %.2f" % d["ms_per_step"], "Gpatch/s %.2f" % (d["value"] / 1e9),
      "ok" if d["digests_ok"] else "BAD", k, flush=True)
PY
done
