#!/bin/bash
# A/B of library builds ($LIBS) on side workloads ($SETS: ';'-separated bench argument lists),
# alternating, $REPS rounds: ms per step of each line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
IFS=';' read -ra SETS_A <<< "${SETS:---workload downstream --steps 30 --warmup 3;--workload seph --steps 30 --warmup 3}"
for rep in $(seq ${REPS:-2}); do
    for lib in $LIBS; do
        for a in "${SETS_A[@]}"; do
            CRDT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline $a \
                > gpurun_out/abs.json 2> gpurun_out/abs.err
            st=$?
            case $st in 0) ;; *) echo "status $st for $lib $a"; tail -5 gpurun_out/abs.err; exit $st;; esac
            python3 - "$lib" "$a" gpurun_out/abs.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:24s} {sys.argv[2][:40]:40s} {d['ms_per_step']:8.4f} ms")
PY
        done
    done
done
