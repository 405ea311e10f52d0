"""Diagnostic: merge each random Fugue log of tests/test_fugue.py alone (both level-1 paths)
and report errors / mismatches against the oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "crdt-benches_amd")]
import numpy as np
import crdt_hip
from oracle_bind import Oracle
from test_fugue import random_fugue, to_anchor
o = Oracle()
cases = []
for s in range(10):
    cases.append((f"rand{s}", random_fugue(20000, s, agents=1 + s % 5, p_chain=0.3 + 0.1 * (s % 6),
                                          p_left=0.1 + 0.15 * (s % 5), cps=(0x61, 0xE9, 0x4E2D, 0x1F600))))
cases.append(("leftheavy", random_fugue(30000, 77, p_chain=0.0, p_left=0.9, p_del=0.0)))
for n in (300, 3000):
    cases.append((f"small{n}", random_fugue(n, 5, p_chain=0.5, p_left=0.5, p_del=0.0)))
    cases.append((f"smallnl{n}", random_fugue(n, 5, p_chain=0.5, p_left=0.0, p_del=0.0)))
for level1 in (0, 1):
    c = crdt_hip.Context(0)
    c.set_param("level1", level1)
    for name, lg in cases:
        ref = o.merge_fugue(to_anchor(lg))
        try:
            text, _ = c.merge(lg)
            st = "ok" if text == ref else f"MISMATCH len {len(text)} vs {len(ref)}"
            if text != ref:
                order = c.merge_order(lg)
                os.makedirs("gpurun_out", exist_ok=True)
                np.save(f"gpurun_out/order_{name}_{level1}.npy", order)
        except crdt_hip.CrdtHipError as e:
            st = f"ERR {e}"
        print(level1, name, lg.n, int(lg.side.sum()), st, flush=True)
    c.close()
