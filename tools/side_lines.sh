#!/bin/bash
# Side workloads of the current build, one bench line each (SURVEY configs 2, 4, 5 and the
# downstream group), saved as gpurun_out/${ROUND}_side_<name>.json for profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
R=${ROUND:-r02}
run() {  # name, args...
    local name=$1; shift
    echo "== $name: $*"
    timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" \
        > gpurun_out/${R}_side_$name.json 2> gpurun_out/${R}_side_$name.err
    local st=$?
    tail -1 gpurun_out/${R}_side_$name.json | cut -c1-400; echo
    case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/${R}_side_$name.err; exit $st;; esac
}
run seph --workload seph --steps 20 --warmup 3
run agents64 --workload agents64 --steps 10 --warmup 2
run big1b --workload big1b --steps 5 --warmup 1
run big1b_p0 --workload big1b --p-chain 0 --steps 3 --warmup 1
run downstream --workload downstream --steps 20 --warmup 3
run downstream_pcie --workload downstream --pcie --steps 10 --warmup 2
run upstream_inc --workload upstream_inc --steps 3 --warmup 1
run downstream_fugue --workload downstream --order fugue --steps 20 --warmup 3
run shuffle --relabel shuffle --replicas 1024 --steps 3 --warmup 1 --companion-replicas 0 --plain-companion 0
