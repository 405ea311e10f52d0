"""Debug: replica-from-log merge vs context merge under different engine states."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "crdt-benches_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import crdt_hip
from conftest import trace_path

log = crdt_hip.Trace(trace_path("sveltecomponent")).resolve()
for case in ["fresh", "after_empty", "no_plan_cache"]:
    ctx = crdt_hip.Context(0)
    if case == "no_plan_cache":
        ctx.set_param("plan_cache", 0)
    if case == "after_empty":
        print("empty:", crdt_hip.Replica(ctx).merge()[0])
    ref = ctx.merge(log)
    r = crdt_hip.Replica(ctx, log)
    got = r.merge()
    got2 = r.merge()
    print(case, "ok" if got == ref else "BAD", "second", "ok" if got2 == ref else "BAD", len(ref[0]), got[0][:40])
    del r, ctx
