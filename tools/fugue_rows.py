"""Level-1 rows (runs) per document of each trace, RGA and Fugue anchors: one document per merge
(crdt_hip stats "runs"); the capacity of k_doctree is 12 runs per thread (12,288), of
k_doctree_wide 12 and of k_doctree_wide17 17 (17,408).  GPU."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "crdt-benches_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import crdt_hip  # noqa: E402
from conftest import TRACES, trace_path  # noqa: E402

ctx = crdt_hip.Context(0)
for name in TRACES:
    t = crdt_hip.Trace(trace_path(name))
    row = []
    for fugue in (False, True):
        lg = t.resolve(fugue=fugue).arrays()
        dig, lens, st = ctx.merge_batch([lg], stats=True)
        row.append(st["runs"] - 1)
    print(f"{name:18s} rga {row[0]:6d}  fugue {row[1]:6d}")
