#!/usr/bin/env python3
"""Summarise the SQ counter passes of tools/pmc_sq.sh per kernel: every counter summed over the
kernel's dispatches, plus the ratios the LDS/latency analysis in DESIGN.md uses (per-wave
instruction mix, LDS bank conflicts per active LDS cycle, the share of wave cycles spent waiting).

usage: sq_summary.py <dir with sq1/, sq2/ ...> [kernel ...]"""
import collections
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    name = name.replace("crdt::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[<(]", name, 1)[0]


def main(root, *kernels):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for path in sorted(glob.glob(os.path.join(root, "sq*", "run_counter_collection.csv"))):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size"])
    names = kernels or sorted(k for k in agg if k.startswith("k_"))
    for k in names:
        c = agg.get(k)
        if not c:
            continue
        v, s, lds, wg = meta[k]
        print(f"== {k}: VGPR {v} SGPR {s} LDS {lds} B, workgroup {wg}")
        for n in sorted(c):
            print(f"   {n:24s} {c[n]:18.0f}")
        waves = c.get("SQ_WAVES", 0.0)
        if waves:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
                if n in c:
                    print(f"   {n + ' / wave':24s} {c[n] / waves:18.1f}")
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for n in ("SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    print(f"   {n + ' / wave cyc':24s} {c[n] / wc:18.3f}")
        if c.get("SQ_ACTIVE_INST_LDS"):
            print(f"   {'bank conflict / LDS act':24s} {c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_ACTIVE_INST_LDS']:18.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
