#!/usr/bin/env python3
"""Per-kernel mean duration over the TIMED merges of a bench run profiled with
rocprofv3 --kernel-trace (tools/profile_round.sh), to set beside the bench line's HIP-event
launch times: rocprofv3's --stats average covers every launch of the process, including the
warmup merges (the first one synchronous, without lane overlap) and the two one-lane merges
bench.py runs after the timed region for `stream_kernel.isolated_1_lane`.

usage: kt_timed.py <run_kernel_trace.csv> <bench line json> [warmup=2]"""
import csv
import json
import sys


def main(trace, bench, warmup=2):
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    waves, steps = int(b["config"]["waves"]), int(b["steps"])
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    lo, hi = int(warmup) * waves, (int(warmup) + steps) * waves
    print(f"timed merges {int(warmup) + 1}..{int(warmup) + steps} of the run ({waves} waves each): "
          f"launches {lo}..{hi - 1} of each per-wave kernel")
    print(f"{'kernel':14s} {'launches':>8s} {'all (us)':>9s} {'timed (us)':>10s} {'bench HIP events (us)':>22s}")
    ev = {"k_doctree": b["roofline"]["launch_us"] if b["roofline"]["kernel"] == "k_doctree" else None,
          "k_classify": b["stream_kernel"]["launch_us"]}
    for k in ("k_doctree", "k_classify", "k_runs<", "k_heads", "k_leafhash"):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
             if k in r["Kernel_Name"]]
        if not d:
            continue
        t = d[lo:hi]
        e = ev.get(k)
        print(f"{k.rstrip('<'):14s} {len(d):8d} {sum(d) / len(d):9.0f} {sum(t) / max(1, len(t)):10.0f} "
              f"{'' if e is None else f'{e:22.0f}'}")


if __name__ == "__main__":
    main(*sys.argv[1:])
