"""The C-ABI library loads and exports every symbol include/crdt_hip.h declares (CPU only)."""
import ctypes as C
import sys
import os
import re

import crdt_hip
from conftest import ROOT


def header_functions():
    with open(os.path.join(ROOT, "include", "crdt_hip.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(crdt_hip_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    L = crdt_hip.lib()
    declared = header_functions()
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(crdt_hip.EXPORTS) == declared


def test_abi_version():
    assert crdt_hip.lib().crdt_hip_abi_version() == 2


def test_library_is_native_gfx950():
    so = crdt_hip.LIB_PATH
    with open(so, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob, "libcrdt_hip.so carries no gfx950 code object"


def test_device_count_does_not_crash():
    n = crdt_hip.device_count()
    assert n >= 0


def test_errors_are_codes_not_crashes():
    L = crdt_hip.lib()
    h = C.c_void_p()
    rc = L.crdt_hip_trace_load(b"/nonexistent.json.gz", C.byref(h))
    assert rc == -7
    assert b"cannot open" in L.crdt_hip_last_error(None)
    log = crdt_hip.OpLog()
    try:
        log.insert(5, "x")
        raise AssertionError("expected ERANGE")
    except crdt_hip.CrdtHipError as e:
        assert e.code == -2
    assert L.crdt_hip_set_param(None, b"splitter_stride", 64) == -1


def test_host_digest_helpers_match_oracle(oracle):
    data = bytes(range(256)) * 50
    assert crdt_hip.xxh64(data, 7) == oracle.xxh64(data, 7)
    assert crdt_hip.tree_digest(data) == oracle.tree_digest(data)
    assert crdt_hip.tree_digest(b"") == oracle.tree_digest(b"")


def test_tree_digest_groups_above_16mib(oracle):
    """Documents of more than 4096 leaves hash their leaf digests in groups of 4096: the host
    library, the oracle and the pure-Python restatement (make_golden.py) agree."""
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import tree_digest as py_tree_digest
    rng = np.random.default_rng(3)
    for n in (4096 * 4096, 4096 * 4096 + 1, 20_000_003):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        d = crdt_hip.tree_digest(data)
        assert d == oracle.tree_digest(data) == py_tree_digest(data), n
