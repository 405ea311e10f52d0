#!/bin/bash
# upstream_inc / downstream / config 2 on the round-5 tree (tmp_r05, a git worktree of 21a6b96)
# against this tree, alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
ROOTD=$(pwd)
for rep in 1 2; do
  for tree in tmp_r05 .; do
    for w in "--workload upstream_inc --steps 3 --warmup 1" "--workload downstream --steps 20 --warmup 3" "--workload seph --steps 20 --warmup 3"; do
      (cd $ROOTD/$tree && timeout -k 10 300 python -u bench.py --no-cpu-baseline $w > $ROOTD/gpurun_out/ia.json 2> $ROOTD/gpurun_out/ia.err)
      st=$?; case $st in 0) ;; *) echo "status $st"; tail -3 gpurun_out/ia.err; exit $st;; esac
      python3 -c "import json; d=json.loads(open('gpurun_out/ia.json').read().strip().splitlines()[-1]); print('$tree', '$w'.split()[1], round(d['ms_per_step'],3), {k: round(d[k]['len_ms_mean'],4) for k in ('incremental','full') if k in d})"
    done
  done
done
