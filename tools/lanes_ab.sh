#!/bin/bash
# A/B of the engine's wave lanes at the headline config: one bench line per "lanes gate" pair.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for cfg in ${CFGS:-4,1,30 2,1,30 3,1,30 4,0,30 1,1,30}; do  # lanes,gate,log2(wave slots)
    set -- ${cfg//,/ }
    timeout -k 10 200 python bench.py --no-cpu-baseline --lanes $1 --lane-gate $2 --wave-slots-log2 $3 \
        > gpurun_out/lanes_$1_$2_$3.json 2> gpurun_out/lanes_$1_$2_$3.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/lanes_$1_$2_$3.json'));print('lanes $1 gate $2 waves 2^$3',round(d['ms_per_step'],3),d['digests_ok'],round(d['roofline']['frac'],3),{k:round(v['ms'],3) for k,v in d['kernels'].items() if v['launches']})"
done
