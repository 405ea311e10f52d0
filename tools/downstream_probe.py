#!/usr/bin/env python3
"""Host wall time of each call of the downstream step (clone, device decode, merge) per trace."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "crdt-benches_amd"))
import crdt_hip  # noqa: E402

ctx = crdt_hip.Context(0)
for name in ["automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"]:
    t = crdt_hip.Trace(os.path.join(ROOT, "traces", f"{name}.json.gz"))
    patches = [t.patch(i) for i in range(len(t))]
    up, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
    init = crdt_hip.Replica(ctx, up.log if up.log.view().n else None)
    ub = crdt_hip.UpdateBatch(ctx, *crdt_hip.pack_updates(updates))
    acc = [0.0, 0.0, 0.0, 0.0]
    N = 30
    if "--replay" in sys.argv:
        for i in range(N + 3):
            t0 = time.perf_counter()
            init.replay(ub)
            if i >= 3:
                acc[0] += time.perf_counter() - t0
        print(f"{name:16s} replay {acc[0] / N * 1e6:7.1f} us", flush=True)
        continue
    for i in range(N + 3):
        t0 = time.perf_counter()
        r = init.clone()
        t1 = time.perf_counter()
        r.apply_resident(ub)
        t2 = time.perf_counter()
        cps, n, d = r.merge_len()
        t3 = time.perf_counter()
        r.close()
        t4 = time.perf_counter()
        if i >= 3:
            for k, v in enumerate((t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                acc[k] += v
    print(f"{name:16s} clone {acc[0] / N * 1e6:7.1f} us  decode {acc[1] / N * 1e6:7.1f} us  "
          f"merge {acc[2] / N * 1e6:7.1f} us  free {acc[3] / N * 1e6:7.1f} us", flush=True)
