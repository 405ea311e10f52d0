#!/bin/bash
# One rocprofv3 PMC pass per argument group over a short bench run ($PROF_ARGS), summed per kernel.
#   PMC="SQ_WAVES SQ_BUSY_CYCLES;SQC_ICACHE_HITS SQC_ICACHE_MISSES" bash tools/pmc_pass.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${PROF_ARGS:-"--replicas 1024 --steps 1 --warmup 1 --no-cpu-baseline --lanes 1"}
TAG=${TAG:-pmc}
i=0
IFS=';' read -ra GROUPS_ <<< "$PMC"
for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    echo "== pmc pass $i: $grp"
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}$i -o run \
        -- python3 bench.py $ARGS > gpurun_out/${TAG}$i.log 2>&1
    st=$?; echo "status $st"
    case $st in 0) ;; *) tail -5 gpurun_out/${TAG}$i.log; exit $st;; esac
    python3 - gpurun_out/${TAG}$i/run_counter_collection.csv <<'PY'
import csv, collections, re, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    nm = r["Kernel_Name"].replace("crdt::(anonymous namespace)::", "").replace("void ", "")
    # (template instances apart: k_rs_pass<uint4, 0, ...> vs <uint2, 1, ...>)
    k = re.split(r"\(", nm, 1)[0].replace("HIP_vector_type<unsigned int, ", "u").replace("u>", "")[:48]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[k] += 1  # (rows: dispatches x counters of the pass)
for k in sorted(agg, key=lambda k: -sum(agg[k].values())):
    if k.startswith("k_"):
        print(f"  {k:48s} n={n[k]} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(agg[k].items())))
PY
done
