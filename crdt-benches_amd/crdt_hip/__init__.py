"""Python ctypes binding of libcrdt_hip.so (include/crdt_hip.h).

Host plumbing for the tests and bench.py.  The merge itself always runs in the HIP kernels of
libcrdt_hip.so; there is no Python or CPU fallback: if the library is missing, or no device is
present, calls raise.

Mirrors the reference's per-CRDT interface (/root/reference/src/rope.rs:6-33 `Upstream`,
:185-191 `Downstream`) through `HipMerge`, so tests read like the reference's bench loop
(/root/reference/src/main.rs:28-36, :63-69).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# CRDT_HIP_LIB selects another in-tree build (e.g. libcrdt_hip_probe.so: `make probe`)
LIB_PATH = os.path.join(PKG_DIR, os.environ.get("CRDT_HIP_LIB", "libcrdt_hip.so"))

OK = 0
ERRORS = {
    -1: "EINVAL", -2: "ERANGE", -3: "ENOMEM", -4: "EDEVICE", -5: "EBADLOG", -6: "ESPACE",
    -7: "EIO", -8: "ECOMM",
}
STAGES = ["classify", "runs", "sortb", "count", "scan", "place", "link", "walk1", "rank",
          "walk2", "expand", "digest", "doctree", "text", "encode"]

# Every symbol include/crdt_hip.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "crdt_hip_abi_version", "crdt_hip_device_count", "crdt_hip_init", "crdt_hip_destroy",
    "crdt_hip_last_error", "crdt_hip_set_param", "crdt_hip_oplog_new", "crdt_hip_oplog_set_fugue",
    "crdt_hip_oplog_set_agent", "crdt_hip_oplog_clone", "crdt_hip_trace_resolve_fugue",
    "crdt_hip_replica_merge_inc",
    "crdt_hip_oplog_free", "crdt_hip_oplog_insert", "crdt_hip_oplog_remove",
    "crdt_hip_oplog_replace", "crdt_hip_oplog_visible_len", "crdt_hip_oplog_get_view",
    "crdt_hip_oplog_version", "crdt_hip_oplog_encode_from", "crdt_hip_oplog_apply_update",
    "crdt_hip_trace_load", "crdt_hip_trace_free", "crdt_hip_trace_len", "crdt_hip_trace_txns",
    "crdt_hip_trace_patch", "crdt_hip_trace_start_content", "crdt_hip_trace_end_content",
    "crdt_hip_trace_chars_to_bytes", "crdt_hip_trace_resolve", "crdt_hip_trace_resolve_many",
    "crdt_hip_trace_save",
    "crdt_hip_oplog_save", "crdt_hip_oplog_load", "crdt_hip_logfile_open",
    "crdt_hip_logfile_close", "crdt_hip_synth_agents",
    "crdt_hip_synth_tree", "crdt_hip_synth_tree_visible", "crdt_hip_merge", "crdt_hip_merge_batch", "crdt_hip_merge_order",
    "crdt_hip_batch_create", "crdt_hip_batch_synth_tree", "crdt_hip_batch_free", "crdt_hip_batch_info",
    "crdt_hip_batch_merge", "crdt_hip_batch_raw", "crdt_hip_replica_new", "crdt_hip_replica_clone",
    "crdt_hip_replica_free", "crdt_hip_replica_apply_updates", "crdt_hip_replica_info",
    "crdt_hip_updates_upload", "crdt_hip_updates_free", "crdt_hip_replica_apply_resident",
    "crdt_hip_replica_merge", "crdt_hip_comm_unique_id", "crdt_hip_comm_init",
    "crdt_hip_allgather_u64", "crdt_hip_comm_destroy", "crdt_hip_xxh64",
    "crdt_hip_tree_digest", "crdt_hip_merge_len", "crdt_hip_replica_merge_len",
    "crdt_hip_replica_replay",
]


class CrdtHipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class View(C.Structure):
    _fields_ = [
        ("n", C.c_uint32),
        ("parent", C.POINTER(C.c_uint32)),
        ("origin_right", C.POINTER(C.c_uint32)),
        ("lamport", C.POINTER(C.c_uint32)),
        ("agent", C.POINTER(C.c_uint16)),
        ("deleted", C.POINTER(C.c_uint8)),
        ("cp", C.POINTER(C.c_uint32)),
        ("side", C.POINTER(C.c_uint8)),  # Fugue (NULL: RGA)
    ]


class Stats(C.Structure):
    _fields_ = [
        ("items", C.c_uint64),
        ("docs", C.c_uint64),
        ("text_bytes", C.c_uint64),
        ("runs", C.c_uint64),
        ("waves", C.c_uint32),
        ("nstages", C.c_uint32),
        ("stage_ns", C.c_uint64 * 16),
        ("stage_launches", C.c_uint32 * 16),
        ("total_ns", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {
            "items": self.items, "docs": self.docs, "text_bytes": self.text_bytes,
            "runs": self.runs, "waves": self.waves, "total_ns": self.total_ns,
            "stage_ns": {STAGES[i]: int(self.stage_ns[i]) for i in range(self.nstages)},
            "stage_launches": {STAGES[i]: int(self.stage_launches[i]) for i in range(self.nstages)},
        }


_LIB = None


def lib() -> C.CDLL:
    """Load libcrdt_hip.so from the package directory (fails loudly if it is not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is not built: run `make -C {PKG_DIR}` "
                           "(or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, sz, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
    P = C.POINTER
    sig = {
        "crdt_hip_abi_version": (i32, []),
        "crdt_hip_device_count": (i32, [P(i32)]),
        "crdt_hip_init": (i32, [i32, P(vp)]),
        "crdt_hip_destroy": (i32, [vp]),
        "crdt_hip_last_error": (C.c_char_p, [vp]),
        "crdt_hip_set_param": (i32, [vp, C.c_char_p, u64]),
        "crdt_hip_oplog_new": (i32, [P(vp)]),
        "crdt_hip_oplog_set_fugue": (i32, [vp, i32]),
        "crdt_hip_oplog_set_agent": (i32, [vp, C.c_uint16]),
        "crdt_hip_oplog_clone": (i32, [vp, P(vp)]),
        "crdt_hip_oplog_free": (None, [vp]),
        "crdt_hip_oplog_insert": (i32, [vp, sz, C.c_char_p, sz]),
        "crdt_hip_oplog_remove": (i32, [vp, sz, sz]),
        "crdt_hip_oplog_replace": (i32, [vp, sz, sz, C.c_char_p, sz]),
        "crdt_hip_oplog_visible_len": (sz, [vp]),
        "crdt_hip_oplog_get_view": (i32, [vp, P(View)]),
        "crdt_hip_oplog_version": (u64, [vp]),
        "crdt_hip_oplog_encode_from": (i32, [vp, u64, vp, sz, P(sz)]),
        "crdt_hip_oplog_apply_update": (i32, [vp, vp, sz]),
        "crdt_hip_trace_load": (i32, [C.c_char_p, P(vp)]),
        "crdt_hip_trace_free": (None, [vp]),
        "crdt_hip_trace_len": (sz, [vp]),
        "crdt_hip_trace_txns": (sz, [vp]),
        "crdt_hip_trace_patch": (i32, [vp, sz, P(sz), P(sz), P(C.c_char_p), P(sz)]),
        "crdt_hip_trace_start_content": (i32, [vp, P(vp), P(sz)]),
        "crdt_hip_trace_end_content": (i32, [vp, P(vp), P(sz)]),
        "crdt_hip_trace_chars_to_bytes": (i32, [vp]),
        "crdt_hip_trace_resolve": (i32, [vp, P(vp)]),
        "crdt_hip_trace_resolve_fugue": (i32, [vp, P(vp)]),
        "crdt_hip_trace_resolve_many": (i32, [P(vp), u32, u32, P(vp)]),
        "crdt_hip_trace_save": (i32, [vp, C.c_char_p]),
        "crdt_hip_oplog_save": (i32, [vp, C.c_char_p]),
        "crdt_hip_oplog_load": (i32, [C.c_char_p, P(vp)]),
        "crdt_hip_logfile_open": (i32, [C.c_char_p, P(vp), P(View)]),
        "crdt_hip_logfile_close": (i32, [vp]),
        "crdt_hip_synth_agents": (i32, [u32, u32, u64, P(vp)]),
        "crdt_hip_synth_tree": (i32, [u32, u32, u32, u64, P(vp)]),
        "crdt_hip_synth_tree_visible": (i32, [u32, u32, u64, P(u64)]),
        "crdt_hip_merge": (i32, [vp, P(View), vp, sz, P(sz), P(u64)]),
        "crdt_hip_merge_batch": (i32, [vp, P(View), u32, vp, vp, P(Stats)]),
        "crdt_hip_merge_order": (i32, [vp, P(View), vp]),
        "crdt_hip_batch_create": (i32, [vp, P(View), u32, u32, u32, u64, P(vp)]),
        "crdt_hip_batch_synth_tree": (i32, [vp, u32, u32, u32, u64, P(vp)]),
        "crdt_hip_batch_free": (i32, [vp]),
        "crdt_hip_batch_info": (i32, [vp, P(u64), P(u64), P(u64)]),
        "crdt_hip_batch_merge": (i32, [vp, vp, vp, vp, P(Stats)]),
        "crdt_hip_batch_raw": (i32, [vp, vp, i32]),
        "crdt_hip_replica_new": (i32, [vp, P(View), P(vp)]),
        "crdt_hip_replica_clone": (i32, [vp, vp, P(vp)]),
        "crdt_hip_replica_free": (i32, [vp]),
        "crdt_hip_replica_apply_updates": (i32, [vp, vp, vp, sz, vp, u32]),
        "crdt_hip_updates_upload": (i32, [vp, vp, sz, vp, u32, P(vp)]),
        "crdt_hip_updates_free": (i32, [vp]),
        "crdt_hip_replica_apply_resident": (i32, [vp, vp, vp]),
        "crdt_hip_replica_info": (i32, [vp, P(u64), P(u64), P(u64)]),
        "crdt_hip_replica_merge": (i32, [vp, vp, vp, sz, P(sz), P(u64)]),
        "crdt_hip_replica_merge_len": (i32, [vp, vp, P(u64), P(u64), P(u64)]),
        "crdt_hip_replica_merge_inc": (i32, [vp, vp, vp, sz, P(sz), P(u64), P(u32)]),
        "crdt_hip_replica_replay": (i32, [vp, vp, vp, P(u64), P(u64), P(u64)]),
        "crdt_hip_merge_len": (i32, [vp, P(View), P(u64), P(u64), P(u64)]),
        "crdt_hip_comm_unique_id": (i32, [vp]),
        "crdt_hip_comm_init": (i32, [vp, i32, i32, vp]),
        "crdt_hip_allgather_u64": (i32, [vp, vp, sz, vp]),
        "crdt_hip_comm_destroy": (i32, [vp]),
        "crdt_hip_xxh64": (u64, [vp, sz, u64]),
        "crdt_hip_tree_digest": (u64, [vp, sz]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def _check(rc: int, ctx=None) -> None:
    if rc != OK:
        msg = lib().crdt_hip_last_error(ctx)
        raise CrdtHipError(rc, msg.decode("utf-8", "replace") if msg else "")


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().crdt_hip_device_count(C.byref(n))
    return int(n.value) if rc == OK else 0


def xxh64(data: bytes, seed: int = 0) -> int:
    return int(lib().crdt_hip_xxh64(data, len(data), seed))


def tree_digest(data: bytes) -> int:
    return int(lib().crdt_hip_tree_digest(data, len(data)))


# ------------------------------------------------------------------------------------------------
_NO_SIDE = (C.c_uint8 * 1)(0)  # the side column of an empty Fugue log (never read)


class LogArrays:
    """Anchor op log as numpy SoA (ids 1..n).  Keeps the arrays alive for a View.  `side`
    (optional): 1 = the item is a LEFT child of its parent (Fugue order); None = RGA."""

    FIELDS = ("parent", "origin_right", "lamport", "agent", "deleted", "cp")

    def __init__(self, parent, lamport, agent, deleted, cp, origin_right=None, side=None):
        self.parent = np.ascontiguousarray(parent, dtype=np.uint32)
        n = self.parent.size
        self.lamport = np.ascontiguousarray(lamport, dtype=np.uint32)
        self.agent = np.ascontiguousarray(agent, dtype=np.uint16)
        self.deleted = np.ascontiguousarray(deleted, dtype=np.uint8)
        self.cp = np.ascontiguousarray(cp, dtype=np.uint32)
        self.origin_right = (np.full(n, 0xFFFFFFFF, np.uint32) if origin_right is None
                             else np.ascontiguousarray(origin_right, dtype=np.uint32))
        self.side = None if side is None else np.ascontiguousarray(side, dtype=np.uint8)
        for f in self.FIELDS:
            assert getattr(self, f).size == n, f
        assert self.side is None or self.side.size == n

    @property
    def n(self) -> int:
        return int(self.parent.size)

    def view(self) -> View:
        def p(a, t):
            return a.ctypes.data_as(C.POINTER(t)) if a.size else None
        # a Fugue log stays a Fugue log when empty: a null side means RGA, so an empty side
        # column points at a dummy byte (as the C API's kNoSide does, capi.cpp)
        if self.side is None:
            side = None
        elif self.side.size:
            side = p(self.side, C.c_uint8)
        else:
            side = C.cast(_NO_SIDE, C.POINTER(C.c_uint8))
        return View(self.n, p(self.parent, C.c_uint32), p(self.origin_right, C.c_uint32),
                    p(self.lamport, C.c_uint32), p(self.agent, C.c_uint16),
                    p(self.deleted, C.c_uint8), p(self.cp, C.c_uint32), side)

    def copy(self) -> "LogArrays":
        return LogArrays(self.parent.copy(), self.lamport.copy(), self.agent.copy(),
                         self.deleted.copy(), self.cp.copy(), self.origin_right.copy(),
                         None if self.side is None else self.side.copy())


class OpLog:
    """Host-side resolver (positional patches -> anchor op log), crdt_hip_oplog_*."""

    def __init__(self, handle=None, fugue: bool = False, agent: int = 0):
        if handle is None:
            h = C.c_void_p()
            _check(lib().crdt_hip_oplog_new(C.byref(h)))
            handle = h
            if fugue:
                _check(lib().crdt_hip_oplog_set_fugue(h, 1))
        self._h = handle
        if agent:
            _check(lib().crdt_hip_oplog_set_agent(self._h, agent))

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_oplog_free(self._h)
            self._h = None

    def clone(self) -> "OpLog":
        h = C.c_void_p()
        _check(lib().crdt_hip_oplog_clone(self._h, C.byref(h)))
        return OpLog(h)

    def insert(self, pos: int, text: str) -> None:
        b = text.encode("utf-8")
        _check(lib().crdt_hip_oplog_insert(self._h, pos, b, len(b)))

    def remove(self, start: int, end: int) -> None:
        _check(lib().crdt_hip_oplog_remove(self._h, start, end))

    def replace(self, start: int, end: int, text: str) -> None:
        b = text.encode("utf-8")
        _check(lib().crdt_hip_oplog_replace(self._h, start, end, b, len(b)))

    def visible_len(self) -> int:
        return int(lib().crdt_hip_oplog_visible_len(self._h))

    def view(self) -> View:
        v = View()
        _check(lib().crdt_hip_oplog_get_view(self._h, C.byref(v)))
        return v

    def arrays(self) -> LogArrays:
        v = self.view()
        n = v.n

        def arr(ptr, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True)
        side = None
        if v.side:
            side = arr(v.side, np.uint8)
        return LogArrays(arr(v.parent, np.uint32), arr(v.lamport, np.uint32),
                         arr(v.agent, np.uint16), arr(v.deleted, np.uint8),
                         arr(v.cp, np.uint32), arr(v.origin_right, np.uint32), side)

    def version(self) -> int:
        return int(lib().crdt_hip_oplog_version(self._h))

    def encode_from(self, version: int) -> bytes:
        need = C.c_size_t(0)
        rc = lib().crdt_hip_oplog_encode_from(self._h, version, None, 0, C.byref(need))
        if rc not in (OK, -6):
            _check(rc)
        buf = C.create_string_buffer(max(need.value, 1))
        _check(lib().crdt_hip_oplog_encode_from(self._h, version, buf, need.value,
                                                C.byref(need)))
        return buf.raw[: need.value]

    def apply_update(self, update: bytes) -> None:
        _check(lib().crdt_hip_oplog_apply_update(self._h, update, len(update)))

    def save(self, path: str) -> None:
        """Op-log file (crdt_hip_oplog_save): 64-byte-aligned SoA arrays."""
        _check(lib().crdt_hip_oplog_save(self._h, path.encode()))

    @staticmethod
    def load(path: str) -> "OpLog":
        h = C.c_void_p()
        _check(lib().crdt_hip_oplog_load(path.encode(), C.byref(h)))
        return OpLog(h)

    @staticmethod
    def synth_agents(n_items: int, agents: int, seed: int) -> "OpLog":
        h = C.c_void_p()
        _check(lib().crdt_hip_synth_agents(n_items, agents, seed, C.byref(h)))
        return OpLog(h)

    @staticmethod
    def synth_tree(n_items: int, p_chain_pct: int, del_pct: int, seed: int) -> "OpLog":
        h = C.c_void_p()
        _check(lib().crdt_hip_synth_tree(n_items, p_chain_pct, del_pct, seed, C.byref(h)))
        return OpLog(h)


class Trace:
    """josephg trace loaded by the native loader (crdt_hip_trace_*)."""

    def __init__(self, path: str):
        h = C.c_void_p()
        _check(lib().crdt_hip_trace_load(path.encode(), C.byref(h)))
        self._h = h
        self.path = path

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_trace_free(self._h)
            self._h = None

    def __len__(self) -> int:
        return int(lib().crdt_hip_trace_len(self._h))

    @property
    def txns(self) -> int:
        return int(lib().crdt_hip_trace_txns(self._h))

    def patch(self, i: int):
        pos, dele, n = C.c_size_t(), C.c_size_t(), C.c_size_t()
        ins = C.c_char_p()
        _check(lib().crdt_hip_trace_patch(self._h, i, C.byref(pos), C.byref(dele),
                                          C.byref(ins), C.byref(n)))
        return int(pos.value), int(dele.value), C.string_at(ins, n.value).decode("utf-8")

    def _content(self, fn) -> str:
        p, n = C.c_void_p(), C.c_size_t()
        _check(fn(self._h, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value).decode("utf-8") if n.value else ""

    @property
    def start_content(self) -> str:
        return self._content(lib().crdt_hip_trace_start_content)

    @property
    def end_content(self) -> str:
        return self._content(lib().crdt_hip_trace_end_content)

    def chars_to_bytes(self) -> None:
        _check(lib().crdt_hip_trace_chars_to_bytes(self._h))

    def resolve(self, fugue: bool = False) -> OpLog:
        """Positional patches -> anchor op log (RGA anchors; `fugue`: Fugue anchors)."""
        h = C.c_void_p()
        fn = lib().crdt_hip_trace_resolve_fugue if fugue else lib().crdt_hip_trace_resolve
        _check(fn(self._h, C.byref(h)))
        return OpLog(h)

    @staticmethod
    def resolve_many(traces, threads: int = 0):
        """resolve() of every trace, on up to `threads` host threads (0: one per trace)."""
        n = len(traces)
        ins = (C.c_void_p * n)(*[t._h for t in traces])
        outs = (C.c_void_p * n)()
        _check(lib().crdt_hip_trace_resolve_many(ins, n, threads, outs))
        return [OpLog(C.c_void_p(outs[i])) for i in range(n)]

    def save(self, path: str) -> None:
        """Trace cache (crdt_hip_trace_save); Trace(path) reads it back without gunzip + JSON."""
        _check(lib().crdt_hip_trace_save(self._h, path.encode()))


class LogFile:
    """An op-log file mapped read-only (crdt_hip_logfile_open): view() points into the mapping,
    so it can be merged, batched or uploaded without a host copy."""

    def __init__(self, path: str):
        h = C.c_void_p()
        self._v = View()
        _check(lib().crdt_hip_logfile_open(path.encode(), C.byref(h), C.byref(self._v)))
        self._h = h
        self.path = path

    def close(self) -> None:
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_logfile_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def view(self) -> View:
        if not self._h:
            raise ValueError("log file is closed")
        return self._v

    def arrays(self) -> LogArrays:
        v, n = self.view(), self._v.n

        def arr(ptr, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True)
        return LogArrays(arr(v.parent, np.uint32), arr(v.lamport, np.uint32),
                         arr(v.agent, np.uint16), arr(v.deleted, np.uint8),
                         arr(v.cp, np.uint32), arr(v.origin_right, np.uint32),
                         arr(v.side, np.uint8) if v.side else None)


def _as_view(log) -> tuple:
    """(View, keepalive) for an OpLog or LogArrays."""
    if isinstance(log, OpLog):
        return log.view(), log
    if isinstance(log, (LogArrays, LogFile)):
        return log.view(), log
    raise TypeError(type(log))


class Context:
    """One HIP device + its merge engine (crdt_hip_init)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(lib().crdt_hip_init(device, C.byref(h)))
        self._h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_destroy(self._h)
            self._h = None

    __del__ = close

    def set_param(self, key: str, value: int) -> None:
        _check(lib().crdt_hip_set_param(self._h, key.encode(), value), self._h)

    def merge(self, log) -> tuple:
        """Merged document: (utf8 bytes, tree digest)."""
        v, keep = _as_view(log)
        cap = 4 * v.n + 16
        buf = np.empty(cap, np.uint8)  # (not zeroed: the engine writes the n bytes returned)
        n, dig = C.c_size_t(), C.c_uint64()
        _check(lib().crdt_hip_merge(self._h, C.byref(v), buf.ctypes.data, cap, C.byref(n),
                                    C.byref(dig)), self._h)
        del keep
        return buf[: n.value].tobytes(), int(dig.value)

    def merge_digest(self, log) -> tuple:
        v, keep = _as_view(log)
        n, dig = C.c_size_t(), C.c_uint64()
        _check(lib().crdt_hip_merge(self._h, C.byref(v), None, 0, C.byref(n), C.byref(dig)),
               self._h)
        return int(n.value), int(dig.value)

    def merge_len(self, log) -> tuple:
        """Upstream::len on the device: (codepoints, UTF-8 bytes, tree digest) of the merged
        document, without copying the text back (crdt_hip_merge_len)."""
        v, keep = _as_view(log)
        c, n, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().crdt_hip_merge_len(self._h, C.byref(v), C.byref(c), C.byref(n), C.byref(d)),
               self._h)
        return int(c.value), int(n.value), int(d.value)

    def merge_batch(self, logs: list, stats: bool = False):
        views = []
        keep = []
        for lg in logs:
            v, k = _as_view(lg)
            views.append(v)
            keep.append(k)
        arr = (View * len(views))(*views)
        dig = np.zeros(len(views), np.uint64)
        lens = np.zeros(len(views), np.uint64)
        st = Stats()
        _check(lib().crdt_hip_merge_batch(self._h, arr, len(views), dig.ctypes.data,
                                          lens.ctypes.data, C.byref(st)), self._h)
        return (dig, lens, st.as_dict()) if stats else (dig, lens)

    def merge_order(self, log) -> np.ndarray:
        v, keep = _as_view(log)
        out = np.zeros(max(v.n, 1), np.uint32)
        _check(lib().crdt_hip_merge_order(self._h, C.byref(v), out.ctypes.data), self._h)
        return out[: v.n]

    def batch(self, bases: list, replicas: int, relabel: int = 0, seed: int = 0) -> "Batch":
        return Batch(self, bases, replicas, relabel, seed)

    # RCCL
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        _check(lib().crdt_hip_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        _check(lib().crdt_hip_comm_init(self._h, nranks, rank, uid), self._h)

    def allgather_u64(self, values: np.ndarray, nranks: int) -> np.ndarray:
        v = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.zeros(v.size * nranks, np.uint64)
        _check(lib().crdt_hip_allgather_u64(self._h, v.ctypes.data, v.size, out.ctypes.data),
               self._h)
        return out


def synth_tree_visible(n_items: int, del_pct: int, seed: int) -> int:
    """Visible items (= merged bytes) of OpLog.synth_tree(n_items, *, del_pct, seed)."""
    out = C.c_uint64()
    _check(lib().crdt_hip_synth_tree_visible(n_items, del_pct, seed, C.byref(out)))
    return int(out.value)


class Batch:
    """Device-resident replica batch (crdt_hip_batch_*)."""

    RELABEL = {"none": 0, "rotate": 1, "shuffle": 2}

    def __init__(self, ctx: Context, bases: list, replicas: int, relabel=0, seed: int = 0,
                 _handle=None):
        if _handle is not None:
            h = _handle
        else:
            if isinstance(relabel, str):
                relabel = self.RELABEL[relabel]
            views = []
            keep = []
            for b in bases:
                v, k = _as_view(b)
                views.append(v)
                keep.append(k)
            arr = (View * len(views))(*views)
            h = C.c_void_p()
            _check(lib().crdt_hip_batch_create(ctx._h, arr, len(views), replicas, relabel, seed,
                                               C.byref(h)), ctx._h)
        self._h = h
        self.ctx = ctx
        docs, items, dev = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().crdt_hip_batch_info(h, C.byref(docs), C.byref(items), C.byref(dev)))
        self.docs, self.items, self.device_bytes = int(docs.value), int(items.value), int(dev.value)

    @classmethod
    def synth_tree(cls, ctx: Context, n_items: int, p_chain_pct: int, del_pct: int,
                   seed: int) -> "Batch":
        """One config-5 document generated on the device (= OpLog.synth_tree, no host copy)."""
        h = C.c_void_p()
        _check(lib().crdt_hip_batch_synth_tree(ctx._h, n_items, p_chain_pct, del_pct, seed,
                                               C.byref(h)), ctx._h)
        return cls(ctx, [], 0, _handle=h)

    def close(self) -> None:
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_batch_free(self._h)
            self._h = None

    __del__ = close

    def merge(self):
        dig = np.zeros(self.docs, np.uint64)
        lens = np.zeros(self.docs, np.uint64)
        st = Stats()
        _check(lib().crdt_hip_batch_merge(self.ctx._h, self._h, dig.ctypes.data,
                                          lens.ctypes.data, C.byref(st)), self.ctx._h)
        return dig, lens, st.as_dict()

    def set_raw(self, on: bool = True) -> None:
        """Raw SoA mode (crdt_hip_batch_raw): every merge derives its input encoding on the device
        from reference-shaped columns (lamport, agent, deleted, codepoint beside the parents)."""
        _check(lib().crdt_hip_batch_raw(self.ctx._h, self._h, int(bool(on))), self.ctx._h)


def pack_updates(updates) -> tuple:
    """Concatenate encoded updates: (bytes as np.uint8, n + 1 byte offsets as np.uint64)."""
    lens = np.fromiter((len(u) for u in updates), np.uint64, count=len(updates))
    offsets = np.zeros(len(updates) + 1, np.uint64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.frombuffer(b"".join(updates), np.uint8) if updates else np.zeros(0, np.uint8)
    return buf, offsets


class UpdateBatch:
    """Encoded updates uploaded to HBM once (crdt_hip_updates_*), applied to any replica of the
    context by Replica.apply_resident: Downstream's update vector (main.rs:58) kept on the device."""

    def __init__(self, ctx: "Context", buf: np.ndarray, offsets: np.ndarray):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        h = C.c_void_p()
        _check(lib().crdt_hip_updates_upload(ctx._h, buf.ctypes.data if buf.size else None,
                                             buf.size, offsets.ctypes.data,
                                             max(0, offsets.size - 1), C.byref(h)), ctx._h)
        self._h = h
        self.ctx = ctx
        self.n = max(0, offsets.size - 1)

    def close(self) -> None:
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_updates_free(self._h)
            self._h = None

    __del__ = close


class Replica:
    """Device-resident replica (crdt_hip_replica_*): Downstream on the device.

    Updates (OpLog.encode_from's wire format) are decoded by the HIP kernels straight into the
    replica's HBM slot arrays, a whole batch per call, and the replica is merged where it lies.
    """

    def __init__(self, ctx: Context, init=None, _handle=None):
        if _handle is None:
            h = C.c_void_p()
            if init is None:
                rc = lib().crdt_hip_replica_new(ctx._h, None, C.byref(h))
            else:
                v, keep = _as_view(init)
                rc = lib().crdt_hip_replica_new(ctx._h, C.byref(v), C.byref(h))
            _check(rc, ctx._h)
            _handle = h
        self._h = _handle
        self.ctx = ctx

    def close(self) -> None:
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.crdt_hip_replica_free(self._h)
            self._h = None

    __del__ = close

    def clone(self) -> "Replica":
        h = C.c_void_p()
        _check(lib().crdt_hip_replica_clone(self.ctx._h, self._h, C.byref(h)), self.ctx._h)
        return Replica(self.ctx, _handle=h)

    def apply_packed(self, buf: np.ndarray, offsets: np.ndarray) -> None:
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        if n <= 0:
            return
        _check(lib().crdt_hip_replica_apply_updates(
            self.ctx._h, self._h, buf.ctypes.data if buf.size else None, buf.size,
            offsets.ctypes.data, n), self.ctx._h)

    def apply_updates(self, updates) -> None:
        self.apply_packed(*pack_updates(list(updates)))

    def apply_resident(self, batch: "UpdateBatch") -> None:
        """Apply a batch already in HBM (crdt_hip_replica_apply_resident): no PCIe transfer."""
        _check(lib().crdt_hip_replica_apply_resident(self.ctx._h, self._h, batch._h), self.ctx._h)

    def info(self) -> tuple:
        """(items, visible codepoints, visible UTF-8 bytes)."""
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().crdt_hip_replica_info(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return int(a.value), int(b.value), int(c.value)

    def merge(self) -> tuple:
        """Merged document: (utf8 bytes, tree digest)."""
        cap = self.info()[2] + 16
        buf = C.create_string_buffer(cap)
        n, dig = C.c_size_t(), C.c_uint64()
        _check(lib().crdt_hip_replica_merge(self.ctx._h, self._h, buf, cap, C.byref(n),
                                            C.byref(dig)), self.ctx._h)
        return buf.raw[: n.value], int(dig.value)

    def merge_digest(self) -> tuple:
        n, dig = C.c_size_t(), C.c_uint64()
        _check(lib().crdt_hip_replica_merge(self.ctx._h, self._h, None, 0, C.byref(n),
                                            C.byref(dig)), self.ctx._h)
        return int(n.value), int(dig.value)

    def merge_inc(self, text: bool = False) -> tuple:
        """Incremental len() (crdt_hip_replica_merge_inc): (codepoints, UTF-8 bytes, path, text or
        None); path 1 = only the items appended since the previous call were ranked, 0 = a full
        merge (first call, concurrent update, > 4096 new items, Fugue)."""
        cap = self.info()[2] + 16 if text else 0
        buf = C.create_string_buffer(cap) if text else None
        n, c, p = C.c_size_t(), C.c_uint64(), C.c_uint32()
        _check(lib().crdt_hip_replica_merge_inc(self.ctx._h, self._h, buf, cap, C.byref(n),
                                                C.byref(c), C.byref(p)), self.ctx._h)
        return int(c.value), int(n.value), int(p.value), (buf.raw[: n.value] if text else None)

    def replay(self, batch: "UpdateBatch") -> tuple:
        """The downstream closure (main.rs:63-69) in one device call: a copy of this replica
        receives the whole resident batch and is merged; returns (codepoints, UTF-8 bytes, tree
        digest) and leaves this replica unchanged (crdt_hip_replica_replay)."""
        c, n, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().crdt_hip_replica_replay(self.ctx._h, self._h, batch._h, C.byref(c),
                                             C.byref(n), C.byref(d)), self.ctx._h)
        return int(c.value), int(n.value), int(d.value)

    def merge_len(self) -> tuple:
        """(codepoints, UTF-8 bytes, tree digest) of the merged document; the codepoints are
        counted on the device from the merged bytes (crdt_hip_replica_merge_len)."""
        c, n, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().crdt_hip_replica_merge_len(self.ctx._h, self._h, C.byref(c), C.byref(n),
                                                C.byref(d)), self.ctx._h)
        return int(c.value), int(n.value), int(d.value)


class HipMerge:
    """Mirror of the reference's per-CRDT adapter for the GPU engine.

    `Upstream` (/root/reference/src/rope.rs:6-33): NAME, EDITS_USE_BYTE_OFFSETS, from_str,
    insert, remove, replace, len.  `Downstream` (:185-191): upstream_updates, apply_update.
    len() is where the merge happens (as Dt::len -> checkout_tip, rope.rs:133-136): it calls
    crdt_hip_merge on the shared device context.
    """

    NAME = "mi355x"
    EDITS_USE_BYTE_OFFSETS = False
    _ctx: Context | None = None

    def __init__(self, log: OpLog):
        self.log = log

    @classmethod
    def context(cls) -> Context:
        if cls._ctx is None:
            cls._ctx = Context(0)
        return cls._ctx

    @classmethod
    def from_str(cls, s: str) -> "HipMerge":
        log = OpLog()
        if s:
            log.insert(0, s)
        return cls(log)

    def insert(self, at: int, text: str) -> None:
        self.log.insert(at, text)

    def remove(self, start: int, end: int) -> None:
        self.log.remove(start, end)

    def replace(self, start: int, end: int, text: str) -> None:
        self.log.replace(start, end, text)

    def clone(self) -> "HipMerge":
        return HipMerge(self.log.clone())

    def text(self) -> str:
        data, _ = self.context().merge(self.log)
        return data.decode("utf-8")

    def len(self) -> int:
        # the merge (Dt::len -> checkout_tip, rope.rs:133-136): codepoints of the merged text,
        # counted on the device (EDITS_USE_BYTE_OFFSETS = false)
        return self.context().merge_len(self.log)[0]

    # Downstream
    @classmethod
    def upstream_updates(cls, start_content: str, patches) -> tuple:
        up = cls.from_str(start_content)
        updates = []
        for pos, dele, ins in patches:
            v = up.log.version()
            up.replace(pos, pos + dele, ins)
            updates.append(up.log.encode_from(v))
        return cls.from_str(start_content), updates

    def apply_update(self, update: bytes) -> None:
        self.log.apply_update(update)


class HipDownstream:
    """`Downstream` (/root/reference/src/rope.rs:185-191) with the replica on the device.

    apply_update() queues the encoded update on the host; len() decodes every queued update on
    the device in one batch (crdt_hip_replica_apply_updates), merges the replica there and
    returns its visible codepoints.  clone() copies the replica device to device.  This is the
    shape of the Rust adapter in INTEGRATION.md.
    """

    NAME = "mi355x-device"
    EDITS_USE_BYTE_OFFSETS = False

    def __init__(self, replica: Replica):
        self.replica = replica
        self.pending: list = []

    @classmethod
    def upstream_updates(cls, start_content: str, patches) -> tuple:
        up, updates = HipMerge.upstream_updates(start_content, patches)
        ctx = HipMerge.context()
        return cls(Replica(ctx, up.log if up.log.view().n else None)), updates

    def clone(self) -> "HipDownstream":
        c = HipDownstream(self.replica.clone())
        c.pending = list(self.pending)
        return c

    def apply_update(self, update: bytes) -> None:
        self.pending.append(update)

    def flush(self) -> None:
        if self.pending:
            self.replica.apply_updates(self.pending)
            self.pending = []

    def text(self) -> str:
        self.flush()
        return self.replica.merge()[0].decode("utf-8")

    def len(self) -> int:
        """Codepoints of the merged document (main.rs:68 asserts them): the merge's own count,
        cross-checked against the decoder's visible-codepoint counter."""
        self.flush()
        cps, _, _ = self.replica.merge_len()
        counter = self.replica.info()[1]
        if cps != counter:
            raise CrdtHipError(-5, f"merged text has {cps} codepoints, the decoder counted {counter}")
        return cps
