#!/bin/bash
# Scheduling knobs of the headline merge on the current build: each argument set ($SETS,
# ';'-separated; default: the engine's defaults and a few alternatives), run twice in alternation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${SETS:- ;--tail-wave-div 0;--l1-split 0;--lanes 3;--wave-slots-log2 29}"
for rep in 1 2; do
for args in "${SETS[@]}"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --companion-replicas 0 \
      --config1-seconds 0 $args > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo fail; tail -3 gpurun_out/sw.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]);print('$args'.ljust(36), round(d['ms_per_step'],3), d['digests_ok'], d['config']['waves'])"
done; done
