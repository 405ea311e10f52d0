#!/bin/bash
# cp2 variants: 3-byte column vs 2-byte (xpre early / late), same box, alternating
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "libcrdt_hip.so --cp2 0" "libcrdt_hip.so --cp2 1" "libcrdt_hip_late.so --cp2 1"; do
    set -- $cfg; lib=$1; shift
    CRDT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --companion-replicas 0 --config1-seconds 0 --lanes 1 "$@" > gpurun_out/v.json 2> gpurun_out/v.err
    st=$?; case $st in 0|1) ;; *) echo "status $st"; tail -5 gpurun_out/v.err; exit $st;; esac
    python3 - "$cfg" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/v.json").read().strip().splitlines()[-1])
k = {n: round(v["ms"], 2) for n, v in d["kernels"].items() if v["launches"]}
print(f"{sys.argv[1]:34s} {d['ms_per_step']:7.3f} ms ok={d['digests_ok']} {k}")
PY
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py -m gpu -k "mixed_ascii or tiles_above" -v --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
timeout -k 10 300 python -u bench.py --workload upstream_inc --steps 3 --warmup 1 > gpurun_out/upinc.json 2> gpurun_out/upinc.err
st=$?; python3 -c "import json;d=json.load(open('gpurun_out/upinc.json'));print({k:d[k] for k in ('len_speedup_mean','len_speedup_median','lens_ok')}, d['incremental'], d['full'])"; exit $st
