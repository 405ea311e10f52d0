#!/usr/bin/env python3
"""k_doctree time per document by trace, each trace alone in a batch (LDS sized for it) and with
the launch forced to take the whole LDS (one workgroup per CU): what occupancy is worth."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "crdt-benches_amd"))
import crdt_hip  # noqa: E402

TRACES = ["automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
ctx = crdt_hip.Context(0)
ctx.set_param("lanes", 1)
for name in TRACES:
    lg = crdt_hip.Trace(os.path.join(ROOT, "traces", f"{name}.json.gz")).resolve().arrays()
    b = ctx.batch([lg], replicas=reps, relabel="rotate", seed=1)
    row = []
    for force in (0, 1):
        ctx.set_param("doctree_lds_max", force)
        ctx.set_param("plan_cache", 0)
        st = [b.merge()[2] for _ in range(3)][-1]
        ns = st["stage_ns"]["doctree"]
        row.append(f"lds{'max' if force else 'fit'} {ns / 1e6:.3f} ms = {ns / 1e3 / reps:.2f} us/doc "
                   f"(x256 CUs: {ns / 1e3 / reps * 256:.1f} us per doc per CU)")
    b.close()
    print(f"{name:16s} runs/doc {st['runs'] // reps:6d}  " + " | ".join(row), flush=True)
