#!/bin/bash
# One GPU iteration: the GPU tests (all, or a -k filter in $K; none with K=none), then each bench
# line named in $LINES ("name:args;name:args"), every step under its own time limit, stopping at
# the first failure.  Outputs under gpurun_out/ (tag $R).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=${R:-iter}
if [ "${K:-}" != none ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
      ${K:+-k "$K"} > gpurun_out/${R}_gpu_tests.log 2>&1
  st=$?; echo "pytest status $st"; grep -E "passed|failed|error" gpurun_out/${R}_gpu_tests.log | tail -3
  case $st in 0) ;; *) grep -E "FAILED|Error|assert" gpurun_out/${R}_gpu_tests.log | head -30; exit $st;; esac
fi
IFS=';' read -ra L <<< "${LINES:-}"
# ABLIBS="libA.so libB.so": every line once per library build (CRDT_HIP_LIB), in alternation
for item0 in "${L[@]}"; do
 for lib in ${ABLIBS:-libcrdt_hip.so}; do
  item=$item0
  [ -z "$item" ] && continue
  name=${item%%:*}; args=${item#*:}
  [ -n "${ABLIBS:-}" ] && name=${name}_${lib%.so}
  echo "== $name: $args"
  CRDT_HIP_LIB=$lib timeout -k 10 ${BT:-300} python -u bench.py --no-cpu-baseline $args > gpurun_out/${R}_$name.json 2> gpurun_out/${R}_$name.err
  st=$?
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${R}_$name.json').read().strip().splitlines()[-1])
ks=d.get('kernels_ms') or {k:v['ms'] for k,v in d.get('kernels',{}).items() if v.get('launches')}
print(round(d['ms_per_step'],3),'ok' if d.get('digests_ok') else 'DIGEST?',{k:round(v,3) for k,v in ks.items()})" 2>/dev/null
  case $st in 0) ;; *) echo "status $st"; tail -5 gpurun_out/${R}_$name.err; exit $st;; esac
 done
done
# optional kernel trace of one bench line: PROF="name:args"
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  name=${PROF%%:*}; args=${PROF#*:}
  echo "== rocprof $name: $args"
  timeout -k 10 ${BT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof_$name -o run \
      -- python3 bench.py --no-cpu-baseline $args > gpurun_out/${R}_prof_$name.log 2>&1
  st=$?; echo "status $st"
  case $st in 0) ;; *) tail -5 gpurun_out/${R}_prof_$name.log; exit $st;; esac
  f=$(find gpurun_out/${R}_prof_$name -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:25]:
    n=r["Name"].replace("crdt::(anonymous namespace)::","")[:70]
    print(f'{n:70s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
fi
