#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of a short headline bench with $LANES lanes
# (default 1), summarised per kernel: ms per step and mean us per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R=${ROUND:-kt}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R} -o run \
    -- python3 bench.py --steps 5 --warmup 2 --lanes ${LANES:-1} --no-cpu-baseline --companion-replicas 0 \
    --config1-seconds 0 --raw-companion 0 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}.log
st=$?; echo "status $st"
case $st in 0) ;; *) tail -5 gpurun_out/${R}.log; exit $st;; esac
python3 - gpurun_out/${R} <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
steps = 7  # 2 warmup + 5 timed
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:40]:40s} {float(r["TotalDurationNs"]) / 1e6 / steps:7.3f} ms/step '
          f'{float(r["AverageNs"]) / 1e3:8.1f} us x {r["Calls"]}')
PY
