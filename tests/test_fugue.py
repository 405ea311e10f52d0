"""Fugue mode ("side u8 (Fugue)", "in-order (Fugue)").

Every item is a left or a right child of its parent; the document is the in-order walk (left
children, the item, right children; each side by (lamport, agent) descending).  Parity pins:
  * the four traces resolved with Fugue anchors merge to their endContent (the reference-held
    fixture), through the oracle and through the device;
  * the oracle's in-order merge equals a third, recursive Python restatement on random trees
    (concurrent sibling order is parity unpinned, as for RGA: no reference fixture exercises it);
  * a log without left children merges exactly as RGA.
The product resolver's Fugue anchors are checked bit-exact against the oracle's resolver.
"""
import random
import struct
import sys

import numpy as np
import pytest

import crdt_hip
from conftest import TRACES, trace_path
from oracle_bind import AnchorLog, load_trace

sys.setrecursionlimit(100000)


def random_fugue(n, seed, agents=4, p_chain=0.6, p_left=0.4, p_del=0.3, cps=(0x61,)):
    """A random Fugue tree: item i hangs off i-1 (right) with p_chain, else off a random earlier
    item on a random side (never left of the document start)."""
    rng = np.random.default_rng(seed)
    ids = np.arange(1, n + 1, dtype=np.int64)
    rnd = rng.integers(0, np.maximum(ids, 1))
    chain = rng.random(n) < p_chain
    parent = np.where(chain, ids - 1, rnd).astype(np.uint32)
    side = ((~chain) & (rng.random(n) < p_left) & (parent > 0)).astype(np.uint8)
    # ids (lamport, agent) are unique, as every CRDT's are; lamports repeat across agents
    agent = (ids % agents).astype(np.uint16)
    lamport = (ids // agents + 1).astype(np.uint32)
    deleted = (rng.random(n) < p_del).astype(np.uint8)
    cp = rng.choice(np.asarray(cps, np.uint32), n)
    return crdt_hip.LogArrays(parent, lamport, agent, deleted, cp, side=side)


def to_anchor(arrs) -> AnchorLog:
    a = AnchorLog(arrs.n)
    for f in ("parent", "lamport", "agent", "deleted", "cp"):
        getattr(a, f)[: arrs.n] = getattr(arrs, f)
    if arrs.side is not None:
        a.side[: arrs.n] = arrs.side
    return a


def py_fugue_order(arrs):
    """Recursive restatement: in-order over (left kids desc, item, right kids desc)."""
    n = arrs.n
    kids = {}
    for i in range(1, n + 1):
        kids.setdefault((int(arrs.parent[i - 1]), int(arrs.side[i - 1])), []).append(i)

    def key(i):
        return (int(arrs.lamport[i - 1]), int(arrs.agent[i - 1]), i)
    out = []

    def walk(v):
        for c in sorted(kids.get((v, 1), []), key=key, reverse=True):
            walk(c)
        if v:
            out.append(v)
        for c in sorted(kids.get((v, 0), []), key=key, reverse=True):
            walk(c)
    walk(0)
    return out


def text_of(arrs, order):
    return "".join(chr(int(arrs.cp[v - 1])) for v in order if not arrs.deleted[v - 1]).encode()


# ---- CPU: oracle and host resolver ------------------------------------------------------------
@pytest.mark.parametrize("name", TRACES)
def test_oracle_fugue_resolve_merge_is_end_content(oracle, name):
    t = load_trace(name)
    a = oracle.resolve_fugue(t)
    assert oracle.merge_fugue(a) == t.end_content.encode()
    assert a.side[: a.n].any()  # the traces do produce left children


@pytest.mark.parametrize("seed", range(6))
def test_oracle_fugue_matches_recursive_restatement(oracle, seed):
    lg = random_fugue(3000, seed, agents=1 + seed)
    text, order = oracle.merge_fugue(to_anchor(lg), want_order=True)
    ref = py_fugue_order(lg)
    assert order.tolist() == ref
    assert text == text_of(lg, ref)


def test_oracle_fugue_without_left_children_is_rga(oracle):
    lg = random_fugue(5000, 9, p_left=0.0)
    a = to_anchor(lg)
    assert oracle.merge_fugue(a) == oracle.merge(a)


def test_oracle_fugue_rejects_left_child_of_start(oracle):
    a = AnchorLog(2)
    a.parent[:2] = [0, 0]
    a.side[:2] = [0, 1]
    a.lamport[:2] = [1, 2]
    with pytest.raises(ValueError):
        oracle.merge_fugue(a)


@pytest.mark.parametrize("name", TRACES)
def test_host_fugue_resolver_matches_oracle(oracle, name):
    lg = crdt_hip.Trace(trace_path(name)).resolve(fugue=True).arrays()
    ref = oracle.resolve_fugue(load_trace(name))
    n = lg.n
    assert n == ref.n
    for f in ("parent", "lamport", "deleted", "cp", "side"):
        assert np.array_equal(getattr(lg, f), getattr(ref, f)[:n]), f


def test_host_fugue_oplog_api(oracle):
    log = crdt_hip.OpLog(fugue=True)
    for pos, text in [(0, "hello"), (0, ">> "), (3, "[x]"), (8, "!"), (2, "~")]:
        log.insert(pos, text)
    log.remove(1, 4)
    lg = log.arrays()
    assert lg.side is not None and lg.side.any()
    # the resolver's own sequence is the in-order: replay the same edits positionally
    s = ""
    for pos, text in [(0, "hello"), (0, ">> "), (3, "[x]"), (8, "!"), (2, "~")]:
        s = s[:pos] + text + s[pos:]
    s = s[:1] + s[4:]
    assert oracle.merge_fugue(to_anchor(lg)) == s.encode()
    upd = log.encode_from(0)
    assert struct.unpack_from("<2I", upd) == (0x55445243, 2)  # "CRDU", version 2 (Fugue)
    with pytest.raises(crdt_hip.CrdtHipError):
        crdt_hip.OpLog().apply_update(upd)  # an RGA log takes no Fugue update
    rga = crdt_hip.OpLog()
    rga.insert(0, "a")
    assert crdt_hip.lib().crdt_hip_oplog_set_fugue(rga._h, 1) != 0  # only on an empty log


# ---- CPU: the update wire format (version 2: cp bit 31 = left child) --------------------------
def fugue_updates(name, limit=None):
    """(sender log, per-patch updates) of a trace replayed on a Fugue log."""
    t = crdt_hip.Trace(trace_path(name))
    up = crdt_hip.OpLog(fugue=True)
    up.insert(0, t.start_content)
    updates = [up.encode_from(0)]
    for i in range(len(t) if limit is None else min(limit, len(t))):
        pos, dele, ins = t.patch(i)
        v = up.version()
        up.replace(pos, pos + dele, ins)
        updates.append(up.encode_from(v))
    return t, up, updates


def same_log(a, b):
    x, y = a.arrays(), b.arrays()
    assert x.n == y.n
    for f in ("parent", "lamport", "agent", "deleted", "cp", "side"):
        assert np.array_equal(getattr(x, f), getattr(y, f)), f


def test_host_fugue_updates_round_trip(oracle):
    t, up, updates = fugue_updates("sveltecomponent")
    down = crdt_hip.OpLog(fugue=True)
    for u in updates:
        down.apply_update(u)
    same_log(up, down)
    assert oracle.merge_fugue(to_anchor(down.arrays())) == t.end_content.encode()
    # one update from version 0, and every update twice (idempotent)
    one = crdt_hip.OpLog(fugue=True)
    one.apply_update(up.encode_from(0))
    one.apply_update(updates[len(updates) // 2])
    same_log(up, one)


def edit_and_check(oracle, log, rng, k):
    """k random local edits on a log whose index was rebuilt from remote items: each must land
    at its position in the oracle's in-order merge of the log."""
    for _ in range(k):
        text = oracle.merge_fugue(to_anchor(log.arrays())).decode()
        if text and rng.random() < 0.3:
            a = rng.randrange(len(text))
            b = min(len(text), a + rng.randint(1, 4))
            log.remove(a, b)
            want = text[:a] + text[b:]
        else:
            p = rng.randint(0, len(text))
            ins = rng.choice(["x", "yz", "\u00e9", "\U0001f600w", "pq r"])
            log.insert(p, ins)
            want = text[:p] + ins + text[p:]
        assert oracle.merge_fugue(to_anchor(log.arrays())).decode() == want


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode"])
def test_host_fugue_rebuilt_index_takes_local_edits(oracle, name):
    """A log that received a whole trace as remote updates rebuilds its positional index as the
    Fugue in-order (OpLog::rebuild_index_fugue): local edits made on it land where asked."""
    t, up, updates = fugue_updates(name, limit=20000)
    down = crdt_hip.OpLog(fugue=True, agent=7)
    for u in updates:
        down.apply_update(u)
    same_log(up, down)
    assert down.arrays().side.any()
    edit_and_check(oracle, down, random.Random(5), 60)
    lg = down.arrays()
    assert (lg.agent[up.arrays().n:] == 7).all()  # the local agent (crdt_hip_oplog_set_agent)


# ---- GPU: device merge vs oracle --------------------------------------------------------------
_FUG = {}


def fugue_resolved(name):
    if name not in _FUG:
        _FUG[name] = crdt_hip.Trace(trace_path(name)).resolve(fugue=True).arrays()
    return _FUG[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", TRACES)
def test_gpu_fugue_trace_merge_is_end_content(ctx, oracle, golden, name):
    lg = fugue_resolved(name)
    text, dig = ctx.merge(lg)
    assert text == oracle.merge_fugue(to_anchor(lg))
    assert "%016x" % dig == golden[name]["tree_digest"]
    order = ctx.merge_order(lg)
    _, ref = oracle.merge_fugue(to_anchor(lg), want_order=True)
    assert np.array_equal(order, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("relabel", ["rotate", "shuffle"])
def test_gpu_fugue_replica_batch(ctx, golden, relabel):
    bases = [fugue_resolved(n) for n in TRACES] + [crdt_hip.Trace(trace_path(TRACES[0])).resolve().arrays()]
    b = ctx.batch(bases, replicas=3, relabel=relabel, seed=99)
    dig, lens, _ = b.merge()
    for r in range(b.docs):
        name = TRACES[r % 5] if r % 5 < 4 else TRACES[0]
        assert "%016x" % dig[r] == golden[name]["tree_digest"], (relabel, r)
        assert lens[r] == golden[name]["end_bytes"]
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("level1", [0, 1])
def test_gpu_fugue_random_trees_match_oracle(oracle, level1):
    c = crdt_hip.Context(0)
    c.set_param("level1", level1)
    logs = [random_fugue(20000, s, agents=1 + s % 5, p_chain=0.3 + 0.1 * (s % 6),
                         p_left=0.1 + 0.15 * (s % 5), cps=(0x61, 0xE9, 0x4E2D, 0x1F600))
            for s in range(10)]
    logs.append(random_fugue(30000, 77, p_chain=0.0, p_left=0.9, p_del=0.0))  # left-heavy
    # pasted runs typed backwards: every char a left child of the one typed before it
    n = 5000
    logs.append(crdt_hip.LogArrays(np.r_[0, np.arange(1, n)].astype(np.uint32),
                                   np.arange(1, n + 1), np.zeros(n), np.zeros(n), np.full(n, 0x62),
                                   side=np.r_[0, np.ones(n - 1)]))
    logs.append(crdt_hip.Trace(trace_path("sveltecomponent")).resolve().arrays())  # RGA beside
    dig, lens = c.merge_batch(logs)
    for i, lg in enumerate(logs):
        ref = oracle.merge_fugue(to_anchor(lg)) if lg.side is not None else oracle.merge(to_anchor(lg))
        assert lens[i] == len(ref), i
        assert dig[i] == oracle.tree_digest(ref), i
    for i in (0, 3, 10, 11):
        text, _ = c.merge(logs[i])
        assert text == oracle.merge_fugue(to_anchor(logs[i])), i
        order = c.merge_order(logs[i])
        _, ref = oracle.merge_fugue(to_anchor(logs[i]), want_order=True)
        assert np.array_equal(order, ref), i
    c.close()


@pytest.mark.gpu
def test_gpu_fugue_left_child_of_start_is_rejected(ctx):
    bad = crdt_hip.LogArrays([0, 0], [1, 2], [0, 0], [0, 0], [97, 98], side=[0, 1])
    with pytest.raises(crdt_hip.CrdtHipError) as e:
        ctx.merge(bad)
    assert e.value.code == -5
    assert ctx.merge(crdt_hip.LogArrays([0, 1], [1, 2], [0, 0], [0, 0], [97, 98], side=[0, 1]))[0] == b"ba"


@pytest.mark.gpu
def test_gpu_fugue_large_log_and_relabelled_replicas(ctx, oracle):
    """A 3 M-item Fugue log (typing chains, 30 % of the other inserts left children, several
    agents) against the oracle, then as a resident batch relabelled three ways: every replica
    must give the same digest (rows, ranks and sides do not depend on the slot order)."""
    lg = random_fugue(3_000_000, 2024, agents=8, p_chain=0.85, p_left=0.3, p_del=0.5,
                      cps=(0x61, 0x62, 0xE9, 0x4E2D))
    ref = oracle.merge_fugue(to_anchor(lg))
    text, dig = ctx.merge(lg)
    assert text == ref and dig == oracle.tree_digest(ref)
    for relabel in ("none", "rotate", "shuffle"):
        b = ctx.batch([lg], replicas=2, relabel=relabel, seed=5)
        d2, l2, _ = b.merge()
        assert all(int(x) == dig for x in d2) and all(int(x) == len(ref) for x in l2), relabel
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 3])
def test_gpu_fugue_multi_wave_lanes(golden, lanes):
    """Fugue and RGA documents in small waves merged on several lanes (learnt plans on the
    second merge, documents in longest-processing-time order): every replica gives its trace's
    endContent digest."""
    c = crdt_hip.Context(0)
    c.set_param("lanes", lanes)
    c.set_param("max_wave_slots", 1 << 20)
    bases = [fugue_resolved(n) for n in TRACES] + [crdt_hip.Trace(trace_path(n)).resolve().arrays()
                                                   for n in TRACES]
    b = c.batch(bases, replicas=2, relabel="rotate", seed=11)
    for _ in range(2):
        dig, lens, st = b.merge()
    assert st["waves"] >= 3
    for r in range(b.docs):
        name = TRACES[(r % 8) % 4]
        assert "%016x" % dig[r] == golden[name]["tree_digest"], r
        assert lens[r] == golden[name]["end_bytes"], r
    b.close()
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("lanes,slots", [(1, 32), (2, 32), (2, 64)])
def test_gpu_fugue_grouped_batch_takes_the_lds_level1(golden, lanes, slots):
    """group_docs: the replicas are placed base by base, each base in waves of its own.  The
    Fugue rows of every trace fit the per-document LDS level 1: sveltecomponent (4.5 k rows) in
    k_doctree, automerge-paper (11.8 k), rustcode (10.7 k) and seph-blog1 (16.6 k) in
    k_doctree_wide (32-bit sibling keys, the up-arc successors in the key slots, up to 17 rows
    per thread; tools/fugue_rows.py).  Results come back in the caller's (replica-major) order,
    equal to every trace's endContent digest."""
    c = crdt_hip.Context(0)
    c.set_param("lanes", lanes)
    c.set_param("group_docs", 1)
    c.set_param("runs_slots", slots)  # (k_runs<true>: 32 or 64 slots per thread)
    bases = [fugue_resolved(n) for n in TRACES]
    b = c.batch(bases, replicas=3, relabel="rotate", seed=21)
    for _ in range(2):  # (the second merge runs on the learnt plans)
        dig, lens, st = b.merge()
    for r in range(b.docs):
        name = TRACES[r % 4]
        assert "%016x" % dig[r] == golden[name]["tree_digest"], r
        assert lens[r] == golden[name]["end_bytes"], r
    assert st["waves"] == 4
    # (two launches per LDS wave: k_doctotals and k_doctree / k_doctree_wide)
    assert st["stage_launches"]["doctree"] == 2 * 4 and st["stage_launches"]["walk1"] == 0, st
    b.close()
    c.close()


# ---- GPU: Fugue replicas (device decode of version-2 updates) --------------------------------
_FUPD = {}


def fugue_updates_cached(name):
    if name not in _FUPD:
        _FUPD[name] = fugue_updates(name)
    return _FUPD[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", TRACES)
def test_gpu_fugue_replica_decodes_trace(ctx, oracle, golden, name):
    """Every per-patch update of a trace replayed on a Fugue log, decoded into an (empty) Fugue
    replica in one batch: the trace's endContent, the sender's log bit for bit."""
    t, up, updates = fugue_updates_cached(name)
    r = crdt_hip.Replica(ctx, crdt_hip.OpLog(fugue=True))
    r.apply_updates(updates)
    text, dig = r.merge()
    assert text == t.end_content.encode()
    assert "%016x" % dig == golden[name]["tree_digest"]
    items, vis_cp, vis_b = r.info()
    assert (items, vis_cp, vis_b) == (up.view().n, len(t.end_content), len(text))
    assert (text, dig) == ctx.merge(up)


@pytest.mark.gpu
def test_gpu_fugue_replica_random_batches_and_clone(ctx, oracle):
    """Random-sized batches into a replica made from a partial Fugue log, a device clone taken
    midway, against the host decoder fed the same updates one at a time."""
    t, up, updates = fugue_updates_cached("rustcode")
    at0 = len(updates) // 5
    host = crdt_hip.OpLog(fugue=True)
    for u in updates[:at0]:
        host.apply_update(u)
    r = crdt_hip.Replica(ctx, host)          # a non-empty Fugue view
    rng = random.Random(11)
    i, snap = at0, None
    while i < len(updates):
        batch = updates[i: i + rng.choice([1, 3, 50, 700, 4000])]
        r.apply_updates(batch)
        for u in batch:
            host.apply_update(u)
        i += len(batch)
        if snap is None and i >= len(updates) // 2:
            snap = (r.clone(), host.clone(), i)
    text, _ = r.merge()
    assert text == t.end_content.encode() == oracle.merge_fugue(to_anchor(host.arrays()))
    rc, hc, at = snap
    assert rc.merge()[0] == oracle.merge_fugue(to_anchor(hc.arrays()))
    rc.apply_updates(updates[at:])
    assert rc.merge()[0] == text


@pytest.mark.gpu
def test_gpu_fugue_replay_closure(ctx, golden):
    """crdt_hip_replica_replay (clone + decode + merge as one graph) on a Fugue replica."""
    name = "sveltecomponent"
    t, up, updates = fugue_updates_cached(name)
    init = crdt_hip.Replica(ctx, crdt_hip.OpLog(fugue=True))
    init.apply_updates(updates[:1])          # the start content
    ub = crdt_hip.UpdateBatch(ctx, *crdt_hip.pack_updates(updates[1:]))
    want = (len(t.end_content), len(t.end_content.encode()), int(golden[name]["tree_digest"], 16))
    before = init.info()
    for _ in range(3):
        assert init.replay(ub) == want
    assert init.info() == before
    ub.close()
    init.close()


@pytest.mark.gpu
def test_gpu_fugue_replica_update_checks(ctx):
    """An RGA replica rejects a version-2 update; a Fugue replica takes RGA (version-1) updates
    and rejects a left child of the document start, leaving itself unchanged."""
    t, up, updates = fugue_updates_cached("sveltecomponent")
    rga = crdt_hip.Replica(ctx)
    with pytest.raises(crdt_hip.CrdtHipError):
        rga.apply_updates(updates[:3])
    assert rga.info()[0] == 0
    _, rga_updates = crdt_hip.HipMerge.upstream_updates("", [(0, 0, "abc"), (1, 1, "XY")])
    f = crdt_hip.Replica(ctx, crdt_hip.OpLog(fugue=True))
    f.apply_updates(rga_updates)
    assert f.merge()[0] == b"aXYc"
    bad = crdt_hip.OpLog(fugue=True)
    bad.insert(0, "ab")
    u = bytearray(bad.encode_from(0))
    # item 1 (parent 0) marked as a left child: cp words follow 6 header words + 3 columns of 2
    struct.pack_into("<I", u, 24 + 3 * 8, ord("a") | 0x80000000)
    with pytest.raises(crdt_hip.CrdtHipError):
        crdt_hip.OpLog(fugue=True).apply_update(bytes(u))
    info = f.info()
    struct.pack_into("<I", u, 8, info[0] + 1)  # new ids for the replica (first id, word 2)
    with pytest.raises(crdt_hip.CrdtHipError):
        f.apply_updates([bytes(u)])
    assert f.info() == info and f.merge()[0] == b"aXYc"


@pytest.mark.gpu
def test_gpu_fugue_replica_from_empty_fugue_arrays(ctx, golden):
    """A replica built from the numpy arrays of an EMPTY Fugue log is a Fugue replica: its side
    column is a zero-length array, which the view passes as a non-null pointer (null = RGA), so
    version-2 updates apply."""
    name = "sveltecomponent"
    t, up, updates = fugue_updates_cached(name)
    arrs = crdt_hip.OpLog(fugue=True).arrays()
    assert arrs.side is not None and arrs.side.size == 0
    r = crdt_hip.Replica(ctx, arrs)
    r.apply_updates(updates)
    text, dig = r.merge()
    assert text == t.end_content.encode()
    assert "%016x" % dig == golden[name]["tree_digest"]


def test_empty_fugue_arrays_view_keeps_side():
    """CPU half of the above: the view of an empty Fugue log's arrays carries a non-null side."""
    v = crdt_hip.OpLog(fugue=True).arrays().view()
    assert v.n == 0 and bool(v.side)
    assert not bool(crdt_hip.OpLog().arrays().view().side)
