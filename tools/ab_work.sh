#!/bin/bash
# A/B of library builds ($LIBS, names in crdt-benches_amd/) over a set of workloads ($WORK:
# ';'-separated "name:args"), saved as gpurun_out/${ROUND}_<name>_<lib>.json, one line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
R=${ROUND:-ab}
IFS=';' read -ra SETS <<< "$WORK"
for set in "${SETS[@]}"; do
    name=${set%%:*}; args=${set#*:}
    for lib in $LIBS; do
        b=${lib%.so}
        echo "== ${name}_$b: $args"
        CRDT_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline $args \
            > gpurun_out/${R}_${name}_$b.json 2> gpurun_out/${R}_${name}_$b.err
        st=$?
        case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/${R}_${name}_$b.err; exit $st;; esac
        python3 - gpurun_out/${R}_${name}_$b.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = ({n: round(v["ms"], 2) for n, v in d["kernels"].items() if v["launches"]} if "kernels" in d
     else {n: round(v, 2) for n, v in d.get("kernels_ms", {}).items()})
print(f"{d['ms_per_step']:.3f} ok={d.get('digests_ok')} {k}")
PY
    done
done
