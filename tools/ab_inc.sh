#!/bin/bash
# A/B of library builds ($LIBS, in crdt-benches_amd/) on the incremental len() workload
# (bench.py --workload upstream_inc), alternating, $REPS rounds: mean / median ms per len().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
    for lib in $LIBS; do
        CRDT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 3 \
            --warmup 1 $ARGS > gpurun_out/abi_$lib.json 2> gpurun_out/abi_$lib.err
        st=$?
        case $st in 0) ;; *) echo "status $st for $lib"; tail -5 gpurun_out/abi_$lib.err; exit $st;; esac
        python3 - "$lib" gpurun_out/abi_$lib.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
i, f = d["incremental"], d["full"]
print(f"{sys.argv[1]:28s} inc {i['len_ms_mean']*1e3:6.1f} / {i['len_ms_median']*1e3:6.1f} us  "
      f"full {f['len_ms_mean']*1e3:6.1f} / {f['len_ms_median']*1e3:6.1f} us  "
      f"x{d['len_speedup_mean']:.2f} / x{d['len_speedup_median']:.2f} ok={d['lens_ok']}")
PY
    done
done
