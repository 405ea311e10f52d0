#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of one bench command ($ARGS, e.g. "--workload
# downstream --steps 20"), summarised: total kernel time and the top kernels by time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R=${ROUND:-ktw}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R} -o run \
    -- python3 bench.py --no-cpu-baseline $ARGS > gpurun_out/${R}.json 2> gpurun_out/${R}.log
st=$?; echo "status $st"
case $st in 0) ;; *) tail -5 gpurun_out/${R}.log; exit $st;; esac
python3 - gpurun_out/${R} <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print(f"total kernel time {sum(float(r['TotalDurationNs']) for r in rows) / 1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{r["Name"][:48]:48s} {float(r["TotalDurationNs"]) / 1e6:8.2f} ms {r["Calls"]:>7s} x '
          f'{float(r["AverageNs"]) / 1e3:8.1f} us')
PY
