"""ctypes binding of the CPU oracle (oracle/liboracle.so) plus a pure-Python trace loader.

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The trace loader restates crdt-testdata's `load_testing_data` (called at
/root/reference/src/main.rs:19,52): gunzip + JSON {startContent, endContent, txns[{patches}]},
patches flattened in txn order (the replay order of src/main.rs:30-31).
"""
from __future__ import annotations

import ctypes as C
import gzip
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
TRACES = ["automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"]  # src/main.rs:10-15


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


class Patches(C.Structure):
    _fields_ = [
        ("npatch", C.c_size_t),
        ("pos", C.POINTER(C.c_uint64)),
        ("dele", C.POINTER(C.c_uint64)),
        ("ins_off", C.POINTER(C.c_uint64)),
        ("ins_len", C.POINTER(C.c_uint64)),
        ("ins_cp", C.POINTER(C.c_uint32)),
        ("start_cp", C.POINTER(C.c_uint32)),
        ("start_n", C.c_size_t),
    ]


class OrcLog(C.Structure):
    _fields_ = [
        ("n", C.c_uint32),
        ("parent", C.POINTER(C.c_uint32)),
        ("lamport", C.POINTER(C.c_uint32)),
        ("agent", C.POINTER(C.c_uint16)),
        ("deleted", C.POINTER(C.c_uint8)),
        ("cp", C.POINTER(C.c_uint32)),
    ]


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class TraceData:
    """Flattened trace: numpy arrays of patches + start/end content."""

    def __init__(self, name: str, start: str, end: str, patches: list):
        self.name = name
        self.start_content = start
        self.end_content = end
        n = len(patches)
        self.pos = np.fromiter((p[0] for p in patches), dtype=np.uint64, count=n)
        self.dele = np.fromiter((p[1] for p in patches), dtype=np.uint64, count=n)
        lens = [len(p[2]) for p in patches]
        self.ins_len = np.asarray(lens, dtype=np.uint64)
        self.ins_off = np.zeros(n, dtype=np.uint64)
        if n:
            self.ins_off[1:] = np.cumsum(self.ins_len)[:-1]
        joined = "".join(p[2] for p in patches)
        self.ins_cp = np.frombuffer(joined.encode("utf-32-le"), dtype=np.uint32).copy()
        if self.ins_cp.size == 0:
            self.ins_cp = np.zeros(1, dtype=np.uint32)
        self.start_cp = np.frombuffer(start.encode("utf-32-le"), dtype=np.uint32).copy()
        if self.start_cp.size == 0:
            self.start_cp = np.zeros(1, dtype=np.uint32)
        self.start_n = len(start)

    def __len__(self) -> int:  # TestData::len == number of patches (src/main.rs:25)
        return int(self.pos.size)

    @property
    def n_items(self) -> int:
        return self.start_n + int(self.ins_len.sum())

    def cstruct(self) -> Patches:
        return Patches(len(self), _p(self.pos, C.c_uint64), _p(self.dele, C.c_uint64),
                       _p(self.ins_off, C.c_uint64), _p(self.ins_len, C.c_uint64),
                       _p(self.ins_cp, C.c_uint32), _p(self.start_cp, C.c_uint32), self.start_n)


def load_trace(name: str, traces_dir: str | None = None) -> TraceData:
    path = os.path.join(traces_dir or os.path.join(ROOT, "traces"), f"{name}.json.gz")
    with gzip.open(path, "rb") as f:
        d = json.loads(f.read())
    patches = [p for txn in d["txns"] for p in txn["patches"]]
    return TraceData(name, d["startContent"], d["endContent"], patches)


def from_patch_list(start: str, patches: list, end: str = "") -> TraceData:
    return TraceData("adhoc", start, end, patches)


class AnchorLog:
    """Anchor op log SoA (ids 1..n; id 0 = document start)."""

    def __init__(self, n: int):
        self.n = n
        self.parent = np.zeros(max(n, 1), np.uint32)
        self.oright = np.zeros(max(n, 1), np.uint32)
        self.lamport = np.zeros(max(n, 1), np.uint32)
        self.agent = np.zeros(max(n, 1), np.uint16)
        self.deleted = np.zeros(max(n, 1), np.uint8)
        self.cp = np.zeros(max(n, 1), np.uint32)
        self.side = np.zeros(max(n, 1), np.uint8)  # Fugue: 1 = left child of parent

    def trimmed(self, n: int) -> "AnchorLog":
        out = AnchorLog(n)
        for f in ("parent", "oright", "lamport", "agent", "deleted", "cp", "side"):
            getattr(out, f)[:n] = getattr(self, f)[:n]
        return out

    def orclog(self) -> OrcLog:
        return OrcLog(self.n, _p(self.parent, C.c_uint32), _p(self.lamport, C.c_uint32),
                      _p(self.agent, C.c_uint16), _p(self.deleted, C.c_uint8),
                      _p(self.cp, C.c_uint32))


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        L = C.CDLL(path)
        L.orc_xxh64.restype = C.c_uint64
        L.orc_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_tree_digest.restype = C.c_uint64
        L.orc_tree_digest.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_replay.restype = C.c_int64
        L.orc_replay.argtypes = [C.POINTER(Patches), C.c_void_p, C.c_size_t]
        L.orc_replay_len.restype = C.c_int64
        L.orc_replay_len.argtypes = [C.POINTER(Patches)]
        L.orc_resolve.restype = C.c_int64
        L.orc_resolve.argtypes = [C.POINTER(Patches)] + [C.c_void_p] * 6
        for fn in ("orc_merge_rga",):
            getattr(L, fn).restype = C.c_int64
            getattr(L, fn).argtypes = [C.c_uint32] + [C.c_void_p] * 6 + [C.c_size_t, C.c_void_p]
        L.orc_merge_rga_naive.restype = C.c_int64
        L.orc_merge_rga_naive.argtypes = [C.c_uint32] + [C.c_void_p] * 6 + [C.c_size_t]
        L.orc_resolve_fugue.restype = C.c_int64
        L.orc_resolve_fugue.argtypes = [C.POINTER(Patches)] + [C.c_void_p] * 6
        L.orc_merge_fugue.restype = C.c_int64
        L.orc_merge_fugue.argtypes = [C.c_uint32] + [C.c_void_p] * 7 + [C.c_size_t, C.c_void_p]
        L.orc_merge_many.restype = C.c_int
        L.orc_merge_many.argtypes = [C.POINTER(OrcLog), C.c_uint32, C.c_int, C.c_void_p,
                                     C.c_void_p]
        self.L = L

    def xxh64(self, data: bytes, seed: int = 0) -> int:
        return int(self.L.orc_xxh64(data, len(data), seed))

    def tree_digest(self, data: bytes) -> int:
        return int(self.L.orc_tree_digest(data, len(data)))

    def replay(self, t: TraceData) -> bytes:
        cap = 4 * (t.n_items + 1)
        buf = C.create_string_buffer(cap)
        st = t.cstruct()
        k = self.L.orc_replay(C.byref(st), buf, cap)
        if k < 0:
            raise ValueError(f"orc_replay failed ({k})")
        return buf.raw[:k]

    def replay_len(self, t: TraceData) -> int:
        st = t.cstruct()
        return int(self.L.orc_replay_len(C.byref(st)))

    def resolve(self, t: TraceData) -> AnchorLog:
        a = AnchorLog(t.n_items)
        st = t.cstruct()
        n = self.L.orc_resolve(C.byref(st), a.parent.ctypes.data, a.oright.ctypes.data,
                               a.lamport.ctypes.data, a.agent.ctypes.data,
                               a.deleted.ctypes.data, a.cp.ctypes.data)
        if n < 0:
            raise ValueError("orc_resolve failed")
        assert n == t.n_items
        return a

    def merge(self, log: AnchorLog, want_order: bool = False):
        cap = 4 * log.n + 4
        buf = C.create_string_buffer(cap)
        order = np.zeros(max(log.n, 1), np.uint32) if want_order else None
        k = self.L.orc_merge_rga(log.n, log.parent.ctypes.data, log.lamport.ctypes.data,
                                 log.agent.ctypes.data, log.deleted.ctypes.data,
                                 log.cp.ctypes.data, buf, cap,
                                 order.ctypes.data if want_order else None)
        if k < 0:
            raise ValueError(f"orc_merge_rga failed ({k})")
        return (buf.raw[:k], order[: log.n]) if want_order else buf.raw[:k]

    def resolve_fugue(self, t: TraceData) -> AnchorLog:
        a = AnchorLog(t.n_items)
        st = t.cstruct()
        n = self.L.orc_resolve_fugue(C.byref(st), a.parent.ctypes.data, a.side.ctypes.data,
                                     a.lamport.ctypes.data, a.agent.ctypes.data,
                                     a.deleted.ctypes.data, a.cp.ctypes.data)
        if n < 0:
            raise ValueError("orc_resolve_fugue failed")
        assert n == t.n_items
        return a

    def merge_fugue(self, log: AnchorLog, want_order: bool = False):
        cap = 4 * log.n + 4
        buf = C.create_string_buffer(cap)
        order = np.zeros(max(log.n, 1), np.uint32) if want_order else None
        k = self.L.orc_merge_fugue(log.n, log.parent.ctypes.data, log.side.ctypes.data,
                                   log.lamport.ctypes.data, log.agent.ctypes.data,
                                   log.deleted.ctypes.data, log.cp.ctypes.data, buf, cap,
                                   order.ctypes.data if want_order else None)
        if k < 0:
            raise ValueError(f"orc_merge_fugue failed ({k})")
        return (buf.raw[:k], order[: log.n]) if want_order else buf.raw[:k]

    def merge_naive(self, log: AnchorLog) -> bytes:
        cap = 4 * log.n + 4
        buf = C.create_string_buffer(cap)
        k = self.L.orc_merge_rga_naive(log.n, log.parent.ctypes.data, log.lamport.ctypes.data,
                                       log.agent.ctypes.data, log.deleted.ctypes.data,
                                       log.cp.ctypes.data, buf, cap)
        if k < 0:
            raise ValueError(f"orc_merge_rga_naive failed ({k})")
        return buf.raw[:k]

    def merge_many(self, logs: list, threads: int):
        arr = (OrcLog * len(logs))(*[l.orclog() for l in logs])
        dig = np.zeros(len(logs), np.uint64)
        lens = np.zeros(len(logs), np.uint64)
        rc = self.L.orc_merge_many(arr, len(logs), threads, dig.ctypes.data, lens.ctypes.data)
        if rc != 0:
            raise ValueError(f"orc_merge_many failed ({rc})")
        return dig, lens
