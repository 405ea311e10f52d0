#!/usr/bin/env python3
"""Summarise rocprofv3 csv outputs of one round profile (tools/profile_round.sh):
per-kernel mean duration (kernel trace) and HBM bytes per item from the separate FETCH_SIZE and
WRITE_SIZE passes, summed over every dispatch of the kernel and divided by the items all merges
of the profiled run processed (items per merge x merges).  FETCH_SIZE is doubled: gfx950 counts
half of wide streaming reads (MI355X_MICROARCH.md, HBM).

usage: pmc_summary.py <prefix> <items per merge> <merges> [json out]"""
import collections
import csv
import json
import re
import sys


def short(name: str) -> str:
    name = name.replace("crdt::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[<(]", name, 1)[0]


def load_pmc(path):
    agg = collections.defaultdict(float)
    with open(path) as f:
        for r in csv.DictReader(f):
            agg[short(r["Kernel_Name"])] += float(r["Counter_Value"])
    return agg


def main(prefix, items, merges, json_out=None):
    total = float(items) * float(merges)
    dur = collections.defaultdict(list)
    with open(f"{prefix}_kt/run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fe = load_pmc(f"{prefix}_FETCH_SIZE/run_counter_collection.csv")
    wr = load_pmc(f"{prefix}_WRITE_SIZE/run_counter_collection.csv")
    print(f"{'kernel':18s} {'calls':>5s} {'mean_us':>10s} {'FETCH B/it':>10s} {'x2':>7s} {'WRITE B/it':>10s}")
    table = {}
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if not k.startswith("k_"):
            continue
        f = fe.get(k, 0.0) * 1024 / total
        w = wr.get(k, 0.0) * 1024 / total
        print(f"{k:18s} {len(dur[k]):5d} {sum(dur[k]) / len(dur[k]) / 1e3:10.1f} {f:10.3f} {2 * f:7.3f} {w:10.3f}")
        table[k] = {"mean_us": sum(dur[k]) / len(dur[k]) / 1e3, "fetch_x2_per_item": 2 * f,
                    "write_per_item": w}
    if json_out:
        with open(json_out, "w") as fh:
            json.dump({"items_per_merge": float(items), "merges": int(merges), "source": prefix,
                       "kernels": table}, fh, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
