#!/bin/bash
# Second half of tools/final_round.sh: the side lines and the Fugue line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r02g}
ROUND=$R bash tools/side_lines.sh || exit 1
timeout -k 10 400 python -u bench.py --order fugue --steps 10 > gpurun_out/${R}_side_fugue.json 2> gpurun_out/${R}_side_fugue.err || exit 1
tail -c 300 gpurun_out/${R}_side_fugue.json
