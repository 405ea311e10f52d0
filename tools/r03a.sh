#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
REPL=4096 bash tools/probe.sh || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --companion-replicas 0 --config1-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));print(round(d['ms_per_step'],3),d['digests_ok'],round(d['roofline']['frac'],3),{k:round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --companion-replicas 0 --config1-seconds 0 --lanes 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail gpurun_out/bench1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench1.json'));print(round(d['ms_per_step'],3),d['digests_ok'],round(d['roofline']['frac'],3),{k:round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
