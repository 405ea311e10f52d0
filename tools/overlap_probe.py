#!/usr/bin/env python3
"""Probe: do merges on separate engine streams overlap on one GPU?  The headline replica set is
split over K contexts (each its own engine, scratch and non-blocking HIP stream); one step merges
every batch, first one after the other, then from K host threads at once (ctypes releases the
GIL).  Prints ms/step of both and whether every digest checks."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from bench import crdt_hip  # noqa: E402


def main(k: int, replicas: int, steps: int) -> int:
    bases, patches, items, survivors, golden = bench.load_bases()
    ctxs = [crdt_hip.Context(0) for _ in range(k)]
    batches = [c.batch(bases, replicas=replicas // k, relabel=1, seed=0x5EED0003 + i)
               for i, c in enumerate(ctxs)]
    expect = bench.expected_digests(golden, batches[0].docs)
    ok = True
    for b in batches:
        dig, _, _ = b.merge()
        ok &= bool(np.array_equal(dig, expect))

    def seq():
        for b in batches:
            b.merge()

    res = [None] * k

    def one(i):
        res[i] = batches[i].merge()

    def par():
        ts = [threading.Thread(target=one, args=(i,)) for i in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    for name, fn in (("sequential", seq), ("concurrent", par), ("sequential", seq), ("concurrent", par)):
        fn()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        el = (time.perf_counter() - t0) / steps * 1e3
        print(f"{name} x{k}: {el:.2f} ms/step", flush=True)
    for r in res:
        ok &= bool(np.array_equal(r[0], expect))
    print("digests_ok", ok, flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 2,
                  int(sys.argv[2]) if len(sys.argv) > 2 else 4096,
                  int(sys.argv[3]) if len(sys.argv) > 3 else 5))
