#!/bin/bash
# level-1 stream on a CU subset (l1_split + CRDT_L1_CU_KEEP) against the default, same box
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "0 0" "1 0" "1 6" "1 7" "1 5"; do
    set -- $cfg
    CRDT_L1_CU_KEEP=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --companion-replicas 0 --config1-seconds 0 --l1-split $1 > gpurun_out/cu.json 2> gpurun_out/cu.err
    st=$?; case $st in 0|1) ;; *) echo "status $st"; tail -5 gpurun_out/cu.err; exit $st;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/cu.json'));print('split $1 keep $2', round(d['ms_per_step'],3), d['digests_ok'])"
  done
done
