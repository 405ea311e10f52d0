#!/bin/bash
# End-of-round record of the current build: GPU tests + smoke, the default bench line, the round
# profile (2-lane kernel trace + FETCH/WRITE PMC passes), a 1-lane kernel trace, the side lines
# and the Fugue line; every GPU step under its own limit, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r02g}
BENCH=" " bash tools/gpu_round.sh || exit 1
cp gpurun_out/bench_1.json gpurun_out/${R}_bench_default.json
ROUND=$R bash tools/profile_round.sh || exit 1
python3 tools/kt_timed.py gpurun_out/${R}_kt/run_kernel_trace.csv gpurun_out/${R}_bench_4096.json \
    > gpurun_out/${R}_kernel_timed_4096.txt
ROUND=${R}_1lane LANES=1 bash tools/kt1.sh || exit 1
ROUND=$R bash tools/side_lines.sh || exit 1
timeout -k 10 400 python -u bench.py --order fugue --steps 10 > gpurun_out/${R}_side_fugue.json 2> gpurun_out/${R}_side_fugue.err || exit 1
tail -c 300 gpurun_out/${R}_side_fugue.json
