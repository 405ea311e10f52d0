#!/bin/bash
# incremental tests on the current build, then k_inc launch durations (rocprofv3 kernel trace of
# the upstream_inc workload) for each library in $LIBS, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_incr.py > gpurun_out/r03q_incr_tests.log 2>&1
st=$?; tail -3 gpurun_out/r03q_incr_tests.log; [ $st = 0 ] || exit $st
for rep in 1 2; do
    for lib in $LIBS; do
        CRDT_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d gpurun_out/q_$lib -o run -- python3 bench.py --workload upstream_inc --steps 2 \
            --warmup 1 > gpurun_out/q_$lib.json 2> gpurun_out/q_$lib.err
        st=$?; [ $st = 0 ] || { echo "status $st for $lib"; tail -5 gpurun_out/q_$lib.err; exit $st; }
        python3 - "$lib" gpurun_out/q_$lib.json gpurun_out/q_$lib/run_kernel_stats.csv <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = [r for r in csv.DictReader(open(sys.argv[3])) if "k_inc(" in r["Name"]][0]
print(f"{sys.argv[1]:26s} k_inc {float(k['AverageNs'])/1e3:6.2f} us x{k['Calls']}  len() "
      f"{d['incremental']['len_ms_mean']*1e3:6.1f} / {d['incremental']['len_ms_median']*1e3:6.1f} us, "
      f"full {d['full']['len_ms_mean']*1e3:6.1f} us")
PY
    done
done
