"""The C++ bench harness (crdt-benches_amd/crdt_bench), the restatement of the reference's
/root/reference/src/main.rs:17-81 with the device engine registered as the CRDT under test.

Each group runs once end to end in its own process: the upstream closure (main.rs:28-36), the
downstream closure with host and device decode (main.rs:63-69), and the batched group over two
replicas of every trace.  The harness aborts on any length or digest mismatch (main.rs:35,68),
so rc 0 is the check; it also guards the exit path: the shared device is deliberately never
destroyed at exit (csrc/hipmerge.hpp), because a static destructor running after the HIP
runtime's own teardown segfaulted (status -11) once every group had passed.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "crdt-benches_amd", "crdt_bench")

pytestmark = pytest.mark.gpu


def run(*args, timeout=240):
    assert os.path.exists(BIN), "crdt_bench is not built (make -C crdt-benches_amd)"
    # traces are found relative to the working directory, as main.rs:19 does
    return subprocess.run([BIN, *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("order", ["rga", "fugue"])
def test_crdt_bench_all_groups_exit_cleanly(order):
    p = run("all", "--iters", "1", "--replicas", "2", "--order", order)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    out = p.stdout
    for t in ("automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"):
        assert f"upstream/{t}/" in out and f"downstream/{t}/" in out, out
    assert "batched/all-4-traces/" in out and "all digests match endContent" in out, out
