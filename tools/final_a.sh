#!/bin/bash
# First half of tools/final_round.sh (one gpurun call each): GPU tests + smoke, the default bench
# line, the round profile and the 1-lane kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r02g}
BENCH=" " bash tools/gpu_round.sh || exit 1
cp gpurun_out/bench_1.json gpurun_out/${R}_bench_default.json
ROUND=$R bash tools/profile_round.sh || exit 1
python3 tools/kt_timed.py gpurun_out/${R}_kt/run_kernel_trace.csv gpurun_out/${R}_bench_4096.json \
    > gpurun_out/${R}_kernel_timed_4096.txt
ROUND=${R}_1lane LANES=1 bash tools/kt1.sh || exit 1
