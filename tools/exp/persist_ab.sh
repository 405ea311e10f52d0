#!/bin/bash
# k_runs persistent against one workgroup per tile: digests, then the headline A/B (1 and 2 lanes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
for rep in 1 2; do
  for lanes in 1 2; do
    for p in 0 1; do
      timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --companion-replicas 0 --config1-seconds 0 \
          --raw-companion 0 --plain-companion 0 --lanes $lanes --runs-persist $p > gpurun_out/pa.json 2> gpurun_out/pa.err
      st=$?; case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/pa.err; exit $st;; esac
      python3 -c "import json; d=json.loads(open('gpurun_out/pa.json').read().strip().splitlines()[-1]); print('lanes $lanes persist $p', round(d['ms_per_step'],3), d['digests_ok'], {k: round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
    done
  done
done
