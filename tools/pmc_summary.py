#!/usr/bin/env python3
"""Summarise rocprofv3 csv outputs: per-kernel mean duration (kernel trace) and per-dispatch
FETCH_SIZE / WRITE_SIZE (KB) of the last dispatch of each kernel, in bytes per item."""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("crdt::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[<(]", name, 1)[0] + ("<order>" if "<true>" in name else "")


def load_pmc(path):
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return agg


def main(prefix, items, json_out=None):
    items = float(items)
    dur = collections.defaultdict(list)
    with open(f"{prefix}_kt/run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fe = load_pmc(f"{prefix}_FETCH_SIZE/run_counter_collection.csv")
    wr = load_pmc(f"{prefix}_WRITE_SIZE/run_counter_collection.csv")
    print(f"{'kernel':18s} {'calls':>5s} {'mean_us':>10s} {'FETCH B/it':>10s} {'x2':>7s} {'WRITE B/it':>10s}")
    table = {}
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        f = fe.get(k, [0])[-1] * 1024 / items
        w = wr.get(k, [0])[-1] * 1024 / items
        print(f"{k:18s} {len(dur[k]):5d} {sum(dur[k]) / len(dur[k]) / 1e3:10.1f} {f:10.2f} {2 * f:7.2f} {w:10.2f}")
        table[k] = {"mean_us": sum(dur[k]) / len(dur[k]) / 1e3, "fetch_x2_per_item": 2 * f,
                    "write_per_item": w}
    if json_out:
        import json
        with open(json_out, "w") as fh:
            json.dump({"items_per_launch": items, "source": prefix, "kernels": table}, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
