#!/bin/bash
# Fugue line: scheduling knobs (wave size, lanes) on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
for rep in 1 2; do
  for a in "" "--wave-slots-log2 29" "--lanes 3" "--lanes 1" "--wave-slots-log2 29 --lanes 3"; do
    timeout -k 10 300 python -u bench.py --order fugue --no-cpu-baseline --steps 6 --warmup 2 --companion-replicas 0 \
        --config1-seconds 0 --plain-companion 0 $a > gpurun_out/fs.json 2> gpurun_out/fs.err
    st=$?; case $st in 0) ;; *) echo "status $st"; tail -3 gpurun_out/fs.err; exit $st;; esac
    python3 -c "import json; d=json.loads(open('gpurun_out/fs.json').read().strip().splitlines()[-1]); print('[$a]', round(d['ms_per_step'],3), d['digests_ok'], d['config']['waves'])"
  done
done
