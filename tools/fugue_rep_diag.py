"""Diagnostic: Fugue replica states midway through random batches (which path fails)."""
import random
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "crdt-benches_amd")
import crdt_hip
from test_fugue import fugue_updates

t, up, updates = fugue_updates("rustcode")
ctx = crdt_hip.Context(0)
at0 = len(updates) // 5
host = crdt_hip.OpLog(fugue=True)
for u in updates[:at0]:
    host.apply_update(u)
r = crdt_hip.Replica(ctx, host)
rng = random.Random(11)
i = at0
checks = 0


def tryit(tag, fn):
    try:
        out = fn()
        return "ok" if out else "MISMATCH"
    except crdt_hip.CrdtHipError as e:
        return "ERR " + str(e)


while i < len(updates):
    batch = updates[i: i + rng.choice([1, 3, 50, 700, 4000])]
    r.apply_updates(batch)
    for u in batch:
        host.apply_update(u)
    i += len(batch)
    ref = ctx.merge(host)[0]
    res = [tryit("r", lambda: r.merge()[0] == ref),
           tryit("clone", lambda: r.clone().merge()[0] == ref),
           tryit("fresh", lambda: crdt_hip.Replica(ctx, host).merge()[0] == ref)]
    if any(x != "ok" for x in res):
        print(i, host.view().n, res, flush=True)
        checks += 1
        if checks > 10:
            break
print("done", i, flush=True)
