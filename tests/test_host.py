"""Host-side product code vs the oracle (CPU only): native trace loader (crdt-testdata
restatement), resolver (positional patches -> anchor op log), update wire format, synthetic
generators."""
import numpy as np
import pytest

import crdt_hip
from conftest import TRACES, trace_path
from oracle_bind import AnchorLog, from_patch_list


def to_anchor(arrs: crdt_hip.LogArrays) -> AnchorLog:
    a = AnchorLog(arrs.n)
    for f in ("parent", "lamport", "agent", "deleted", "cp"):
        getattr(a, f)[: arrs.n] = getattr(arrs, f)
    a.oright[: arrs.n] = arrs.origin_right
    return a


@pytest.mark.parametrize("name", TRACES)
def test_native_loader_matches_python_loader(name, py_trace):
    t = crdt_hip.Trace(trace_path(name))
    p = py_trace(name)
    assert len(t) == len(p)  # TestData::len (main.rs:25)
    assert t.end_content == p.end_content and t.start_content == p.start_content
    rng = np.random.default_rng(0)
    idx = set(rng.integers(0, len(p), 2000).tolist()) | {0, len(p) - 1}
    for i in sorted(idx):
        pos, dele, ins = t.patch(i)
        assert pos == int(p.pos[i]) and dele == int(p.dele[i])
        off, n = int(p.ins_off[i]), int(p.ins_len[i])
        exp = p.ins_cp[off: off + n].tobytes().decode("utf-32-le") if n else ""
        assert ins == exp


@pytest.mark.parametrize("name", ["rustcode", "seph-blog1", "sveltecomponent"])
def test_chars_to_bytes_replay(name, py_trace):
    """After chars_to_bytes, a byte-offset replay reproduces endContent."""
    t = crdt_hip.Trace(trace_path(name))
    t.chars_to_bytes()
    doc = bytearray(t.start_content.encode())
    for i in range(len(t)):
        pos, dele, ins = t.patch(i)
        doc[pos: pos + dele] = ins.encode()
    assert bytes(doc) == t.end_content.encode()


def test_chars_to_bytes_changes_expected_patch_counts():
    """exactly 7 rustcode and 2 seph-blog1 patches change coordinates."""
    for name, exp in (("rustcode", 7), ("seph-blog1", 2), ("sveltecomponent", 0)):
        a = crdt_hip.Trace(trace_path(name))
        b = crdt_hip.Trace(trace_path(name))
        b.chars_to_bytes()
        changed = sum(a.patch(i)[:2] != b.patch(i)[:2] for i in range(len(a)))
        assert changed == exp, name


@pytest.mark.parametrize("name", TRACES)
def test_native_resolver_matches_oracle_bit_exact(name, oracle, py_trace):
    t = crdt_hip.Trace(trace_path(name))
    log = t.resolve().arrays()
    ref = oracle.resolve(py_trace(name))
    assert log.n == ref.n
    for f, g in (("parent", "parent"), ("lamport", "lamport"), ("agent", "agent"),
                 ("deleted", "deleted"), ("cp", "cp"), ("origin_right", "oright")):
        assert np.array_equal(getattr(log, f), getattr(ref, g)[: ref.n]), f
    # and the oracle merges the product's resolved log to endContent
    assert oracle.merge(to_anchor(log)) == py_trace(name).end_content.encode()


@pytest.mark.parametrize("threads", [0, 1, 3])
def test_parallel_resolve_matches_sequential(threads):
    """crdt_hip_trace_resolve_many (documents resolved in parallel) gives
    every trace's log exactly as resolve() does, whatever the thread count."""
    traces = [crdt_hip.Trace(trace_path(n)) for n in TRACES] * 2
    logs = crdt_hip.Trace.resolve_many(traces, threads)
    for t, lg in zip(traces, logs):
        a, b = lg.arrays(), t.resolve().arrays()
        assert a.n == b.n
        for f in ("parent", "lamport", "agent", "deleted", "cp", "origin_right"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert crdt_hip.Trace.resolve_many([], 2) == []


def test_resolver_upstream_api_semantics(oracle):
    log = crdt_hip.OpLog()
    log.insert(0, "hello")
    log.insert(5, " world")
    log.replace(0, 1, "J")           # Upstream::replace: remove then insert
    log.remove(5, 11)
    log.insert(5, "!€\U0001F600")
    assert log.visible_len() == 8
    assert oracle.merge(to_anchor(log.arrays())) == "Jello!€\U0001F600".encode()
    with pytest.raises(crdt_hip.CrdtHipError):
        log.remove(3, 100)
    assert crdt_hip.lib().crdt_hip_oplog_insert(log._h, 0, b"\xff", 1) == -2  # invalid UTF-8


def test_update_wire_roundtrip(oracle, py_trace):
    """Downstream: upstream_updates (one update per patch) + apply_update == the upstream log."""
    t = py_trace("sveltecomponent")
    patches = [(int(t.pos[i]), int(t.dele[i]),
                t.ins_cp[int(t.ins_off[i]): int(t.ins_off[i] + t.ins_len[i])].tobytes().decode("utf-32-le"))
               for i in range(2000)]
    down, updates = crdt_hip.HipMerge.upstream_updates("", patches)
    assert len(updates) == len(patches)
    for u in updates:
        down.apply_update(u)
    up = crdt_hip.OpLog()
    for pos, dele, ins in patches:
        up.replace(pos, pos + dele, ins)
    a, b = down.log.arrays(), up.arrays()
    for f in crdt_hip.LogArrays.FIELDS:
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    # re-applying is idempotent, a gap is rejected
    down.log.apply_update(updates[-1])
    fresh = crdt_hip.OpLog()
    with pytest.raises(crdt_hip.CrdtHipError):
        fresh.apply_update(updates[5])
    # positional edits after remote updates rebuild the resolver index from the log
    down.log.insert(0, "Z")
    up.insert(0, "Z")
    assert oracle.merge(to_anchor(down.log.arrays())) == oracle.merge(to_anchor(up.arrays()))


def test_synth_agents_is_valid_and_oracles_agree(oracle):
    log = crdt_hip.OpLog.synth_agents(20000, 64, 0x5EED0001).arrays()
    assert log.n == 20000
    ids = np.arange(1, log.n + 1)
    assert np.all(log.parent < ids)  # causal
    par = log.parent.astype(np.int64)
    has_p = par > 0
    assert np.all(log.lamport[has_p] > log.lamport[par[has_p] - 1])
    keys = log.lamport.astype(np.uint64) << np.uint64(16) | log.agent.astype(np.uint64)
    assert np.unique(keys).size == log.n  # (lamport, agent) unique
    assert len(set(log.agent.tolist())) == 64
    a = to_anchor(log)
    assert oracle.merge(a) == oracle.merge_naive(a)
    # heavy sibling conflicts exist
    counts = np.bincount(log.parent, minlength=log.n + 1)
    assert counts.max() >= 3


def test_synth_tree_shape():
    log = crdt_hip.OpLog.synth_tree(100000, 90, 50, 0x5EED0002).arrays()
    ids = np.arange(1, log.n + 1)
    chain = np.mean(log.parent == ids - 1)
    assert 0.88 < chain < 0.93
    assert 0.48 < log.deleted.mean() < 0.52
    assert np.all(log.lamport == ids) and np.all(log.agent == ids % 64)
    log2 = crdt_hip.OpLog.synth_tree(1000, 90, 50, 0x5EED0002).arrays()
    assert np.array_equal(log2.parent, log.parent[:1000])  # counter-based: prefix-stable


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_span_resolver_random_edits_match_oracle(oracle, seed):
    """Random positional edits (typing runs, pastes, long deletes spanning many spans and chunks,
    edits at both ends) through the span index == the oracle's linked-list resolver, bit-exact."""
    rng = np.random.default_rng(seed)
    text, patches, cursor = [], [], 0
    for _ in range(6000):
        n = len(text)
        r = rng.random()
        if r < 0.05:
            cursor = int(rng.integers(0, n + 1))
        cursor = min(cursor, n)
        if r < 0.55 or n == 0:  # type on at the cursor
            s = "".join(chr(int(c)) for c in rng.choice([97, 98, 233, 0x20AC, 0x1F600], size=int(rng.integers(1, 4))))
            pos = 0 if rng.random() < 0.03 else (n if rng.random() < 0.03 else cursor)
            patches.append((pos, 0, s))
            text[pos:pos] = list(s)
            cursor = pos + len(s)
        elif r < 0.85:  # backspace / forward delete
            k = int(min(n, rng.integers(1, 4) if rng.random() < 0.9 else rng.integers(1, 400)))
            pos = int(rng.integers(0, n - k + 1))
            patches.append((pos, k, ""))
            del text[pos:pos + k]
            cursor = pos
        else:  # replace a range with a paste
            k = int(rng.integers(0, min(n, 50) + 1))
            pos = int(rng.integers(0, n - k + 1))
            s = "xyz" * int(rng.integers(1, 30))
            patches.append((pos, k, s))
            text[pos:pos + k] = list(s)
            cursor = pos + len(s)
    log = crdt_hip.OpLog()
    for pos, k, s in patches:
        log.replace(pos, pos + k, s)
    assert log.visible_len() == len(text)
    got = log.arrays()
    ref = oracle.resolve(from_patch_list("", patches))
    assert got.n == ref.n
    for f, g in (("parent", "parent"), ("lamport", "lamport"), ("deleted", "deleted"),
                 ("cp", "cp"), ("origin_right", "oright")):
        assert np.array_equal(getattr(got, f), getattr(ref, g)[: ref.n]), f
    assert oracle.merge(to_anchor(got)) == "".join(text).encode()
    # a remote item forces an index rebuild from the log (spans rebuilt from the RGA order)
    down, updates = crdt_hip.HipMerge.upstream_updates("", patches[:300])
    for u in updates:
        down.apply_update(u)
    up = crdt_hip.OpLog()
    for pos, k, s in patches[:300]:
        up.replace(pos, pos + k, s)
    for pos, k, s in patches[300:900]:
        down.log.replace(pos, pos + k, s)
        up.replace(pos, pos + k, s)
    a, b = down.log.arrays(), up.arrays()
    for f in ("parent", "origin_right", "deleted", "cp"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_rejected_update_leaves_the_log_unchanged():
    """The host decoder validates a whole update before applying any of it (as the device
    decoder does with a batch): a bad parent, an unknown delete target or a delete index past
    the log's deletes changes neither size() nor version()."""
    import struct
    up = crdt_hip.OpLog()
    up.insert(0, "hello")
    v0 = up.version()
    up.insert(5, " world")
    up.remove(0, 2)
    good = up.encode_from(v0)
    log = crdt_hip.OpLog()
    log.insert(0, "hello")
    before = (log.arrays().n, log.version())
    words = list(struct.unpack(f"<{len(good) // 4}I", good))
    n, m = words[3], words[5]
    bad_parent = words.copy()
    bad_parent[6 + n - 1] = 10_000  # the last new item's parent: unknown
    bad_delete = words.copy()
    bad_delete[-1] = 10_000  # the last delete: unknown item
    bad_del_index = words.copy()
    bad_del_index[4] = 7  # first_del beyond the log's deletes
    for w in (bad_parent, bad_delete, bad_del_index):
        with pytest.raises(crdt_hip.CrdtHipError):
            log.apply_update(struct.pack(f"<{len(w)}I", *w))
        assert (log.arrays().n, log.version()) == before
    log.apply_update(good)
    assert log.arrays().n == up.arrays().n and log.version() == up.version()
    assert m == 2


def test_parsers_survive_corrupted_inputs(tmp_path):
    """Byte-flipped and truncated trace caches, op-log files and update buffers either parse or
    fail with an error code; run under tools/asan_tests.sh (ASan + UBSan) nothing may overrun."""
    rng = np.random.default_rng(2024)
    t = crdt_hip.Trace(trace_path("sveltecomponent"))
    cache = tmp_path / "t.bin"
    t.save(str(cache))
    log = t.resolve()
    lpath = tmp_path / "l.bin"
    log.save(str(lpath))
    v0 = log.version()
    up = log.clone()
    up.insert(3, "xyzé’")
    up.remove(10, 20)
    upd = up.encode_from(v0)
    for src, kind in ((cache.read_bytes(), "trace"), (lpath.read_bytes(), "log")):
        for i in range(60):
            b = bytearray(src)
            if i % 3 == 0:
                b = b[: int(rng.integers(0, len(b)))]
            else:
                for _ in range(int(rng.integers(1, 16))):
                    k = int(rng.integers(0, min(len(b), 4096)))  # headers and index tables
                    b[k] = int(rng.integers(0, 256))
            p = tmp_path / f"bad_{kind}_{i}"
            p.write_bytes(bytes(b))
            try:
                if kind == "trace":
                    x = crdt_hip.Trace(str(p))
                    len(x)
                else:
                    crdt_hip.OpLog.load(str(p))
                    crdt_hip.LogFile(str(p)).close()
            except crdt_hip.CrdtHipError:
                pass
    for i in range(300):
        b = bytearray(upd)
        if i % 4 == 0:
            b = b[: int(rng.integers(0, len(b)))]
        else:
            for _ in range(int(rng.integers(1, 6))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        fresh = log.clone()
        try:
            fresh.apply_update(bytes(b))
        except crdt_hip.CrdtHipError:
            pass
