#!/bin/bash
# End-of-round record, first half (tools/final_round.sh split in two gpurun calls): GPU tests +
# smoke, the default bench line, the round profile (2-lane kernel trace + FETCH/WRITE PMC passes)
# and a 1-lane kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r06}
BENCH=" " bash tools/gpu_round.sh || exit 1
cp gpurun_out/bench_1.json gpurun_out/${R}_bench_default.json
cp gpurun_out/gpu_tests.log gpurun_out/${R}_gpu_tests.log
ROUND=$R bash tools/profile_round.sh || exit 1
python3 tools/kt_timed.py gpurun_out/${R}_kt/run_kernel_trace.csv gpurun_out/${R}_bench_4096.json \
    > gpurun_out/${R}_kernel_timed_4096.txt
ROUND=${R}_1lane LANES=1 bash tools/kt1.sh > gpurun_out/${R}_1lane_summary.txt || exit 1
