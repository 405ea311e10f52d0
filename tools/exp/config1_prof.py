"""Config 1's len() path timed piece by piece (resolve, merge_len on a resolved log), for a
rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --stats run."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "crdt-benches_amd"))
import crdt_hip  # noqa: E402

t = crdt_hip.Trace(os.path.join(ROOT, "traces", "automerge-paper.json.gz"))
ctx = crdt_hip.Context(0)
lg = t.resolve()
for _ in range(20):
    ctx.merge_len(lg)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
a = time.perf_counter()
for _ in range(N):
    ctx.merge_len(lg)
b = time.perf_counter()
for _ in range(N):
    x = t.resolve()
    del x
c = time.perf_counter()
for _ in range(N):
    x = t.resolve()
    ctx.merge_len(x)
    del x
d = time.perf_counter()
print(f"merge_len {1e3 * (b - a) / N:.3f} ms, resolve {1e3 * (c - b) / N:.3f} ms, "
      f"loop {1e3 * (d - c) / N:.3f} ms per iteration")
ctx.close()
