#!/bin/bash
# A/B of bench.py argument sets ($AB: ';'-separated), one short headline run each, summarised.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
i=0
IFS=';' read -ra SETS <<< "$AB"
for args in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 $args \
        > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
    st=$?
    case $st in 0) ;; *) echo "status $st for: $args"; tail -5 gpurun_out/ab_$i.err; exit $st;; esac
    python3 - "$args" gpurun_out/ab_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {n: round(v["ms"], 2) for n, v in d["kernels"].items() if v["launches"]}
iso = (d.get("stream_kernel") or {}).get("isolated_1_lane") or {}
print(f"{sys.argv[1]:40s} {d['ms_per_step']:7.3f} ms ok={d['digests_ok']} {k} "
      f"1lane={iso.get('ms_per_step_1_lane', 0):.2f}/{iso.get('kernel_ms_sum_1_lane', 0):.2f}")
PY
done
