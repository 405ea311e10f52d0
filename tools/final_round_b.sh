#!/bin/bash
# End-of-round record, second half: side lines, the Fugue line, SQ counters (headline at 4096
# replicas with one lane, and config 5 with uniform parents).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r06}
[ -n "$SKIP_SIDE" ] || ROUND=$R bash tools/side_lines.sh || exit 1
timeout -k 10 400 python -u bench.py --order fugue --steps 10 --no-cpu-baseline --companion-replicas 0 \
    > gpurun_out/${R}_side_fugue.json 2> gpurun_out/${R}_side_fugue.err || exit 1
tail -c 300 gpurun_out/${R}_side_fugue.json
PROF_ARGS="--steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --companion-replicas 0 --config1-seconds 0 --plain-companion 0 --raw-companion 0" \
    bash tools/pmc_sq.sh || exit 1
mkdir -p gpurun_out/${R}_sq4096 && mv gpurun_out/sq1 gpurun_out/sq2 gpurun_out/${R}_sq4096/
PROF_ARGS="--workload big1b --p-chain 0 --steps 1 --warmup 1 --no-cpu-baseline" bash tools/pmc_sq.sh || exit 1
mkdir -p gpurun_out/${R}_sqbig && mv gpurun_out/sq1 gpurun_out/sq2 gpurun_out/${R}_sqbig/
