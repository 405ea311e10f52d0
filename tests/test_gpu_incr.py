"""GPU parity tests of the incremental len() (crdt_hip_replica_merge_inc, csrc/incr.hip).

SURVEY §8(f) row 3: the reference's len() (Dt::len -> checkout_tip, /root/reference/src/rope.rs:135)
re-materialises the whole document each call; the upstream loop (/root/reference/src/main.rs:28-36)
with a len() every K patches pays a full merge per call.  The replica keeps its order and text
and ranks only the items appended since the previous call.  Every checkpoint is compared with
the CPU oracle's merge of the same log (oracle/oracle.c orc_merge_rga) and with the replica's own
counters; the path taken (1 = incremental, 0 = full) is asserted where it is determined.
"""
import struct

import pytest

import crdt_hip
from conftest import trace_path
from test_gpu_merge import to_anchor
from test_gpu_replica import trace_updates
from test_fugue import fugue_updates, to_anchor as fugue_anchor

pytestmark = pytest.mark.gpu


def _checkpoints(ctx, oracle, name, K, every_oracle=1):
    t, patches, updates = trace_updates(name)
    r = crdt_hip.Replica(ctx)
    host = crdt_hip.OpLog()
    paths = []
    for c, i in enumerate(range(0, len(updates), K)):
        batch = updates[i:i + K]
        n_before = r.info()[0]
        r.apply_updates(batch)
        for u in batch:
            host.apply_update(u)
        cps, nb, path, text = r.merge_inc(text=True)
        # (local edits: the fast path applies unless the batch appended more than 4096 items)
        paths.append(path if r.info()[0] - n_before <= 4096 else "big")
        items, vis_cp, vis_b = r.info()
        assert (cps, nb) == (vis_cp, vis_b) == (len(text.decode()), len(text))
        if c % every_oracle == 0 or i + K >= len(updates):
            assert text == oracle.merge(to_anchor(host.arrays())), f"checkpoint {c} ({i + K} patches)"
    assert text.decode() == t.end_content
    return paths


def test_incremental_len_every_1000_patches_sveltecomponent(ctx, oracle):
    paths = _checkpoints(ctx, oracle, "sveltecomponent", 1000)
    # the first call builds the state; every later one is a local edit batch (keys increase)
    assert paths[0] in (0, "big") and all(p in (1, "big") for p in paths[1:]), paths
    assert paths.count(1) >= len(paths) // 2, paths


def test_incremental_len_every_1000_patches_automerge_paper(ctx, oracle):
    """The verdict's case: automerge-paper, len() every 1000 patches, oracle at every checkpoint."""
    paths = _checkpoints(ctx, oracle, "automerge-paper", 1000)
    assert paths[0] in (0, "big") and all(p in (1, "big") for p in paths[1:]), paths
    assert paths.count(1) >= len(paths) - 10, paths


@pytest.mark.parametrize("K", [1, 7, 4096])
def test_incremental_len_small_and_large_steps(ctx, oracle, K):
    """One patch per call, an odd step, and steps large enough that some batches carry more than
    4096 items (then the full path runs and rebuilds the state)."""
    t, patches, updates = trace_updates("sveltecomponent")
    n = 3000 if K < 100 else len(updates)
    r = crdt_hip.Replica(ctx)
    host = crdt_hip.OpLog()
    for i in range(0, n, K):
        batch = updates[i:i + K]
        r.apply_updates(batch)
        for u in batch:
            host.apply_update(u)
        if K == 1 and i % 97 and i + 1 < n:
            continue  # (len() at every 97th patch: the others accumulate)
        cps, nb, path, text = r.merge_inc(text=True)
        assert text == oracle.merge(to_anchor(host.arrays()))


def _with_item_id(u: bytes, k: int, lamport: int, agent: int) -> bytes:
    """Update u (OpLog.encode_from's wire layout: 24-byte header, then parent, origin-right,
    lamport and codepoint words, then u16 agents) with item k's (lamport, agent) replaced."""
    n = struct.unpack_from("<I", u, 12)[0]
    b = bytearray(u)
    struct.pack_into("<I", b, 24 + 8 * n + 4 * k, lamport)
    struct.pack_into("<H", b, 24 + 16 * n + 2 * k, agent)
    return bytes(b)


def test_concurrent_update_takes_the_incremental_path(ctx, oracle):
    """An update whose item sorts below an older sibling (a concurrent insert that lost the
    race: its key is below the replica's largest key) is placed by a search of its parent's old
    subtree: after the older sibling's subtree, as the oracle does, without a full merge."""
    a = crdt_hip.OpLog(agent=1)
    h = crdt_hip.OpLog(agent=1)  # the host log fed the same (patched) updates
    r = crdt_hip.Replica(ctx)

    def ship(u):
        r.apply_updates([u])
        h.apply_update(u)

    a.insert(0, "hello")
    ship(a.encode_from(0))
    assert r.merge_inc(text=True)[3] == b"hello"
    v = a.version()
    a.insert(5, " world")
    ship(a.encode_from(v))
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == b"hello world"
    v = a.version()
    a.insert(0, "XY")                            # X: a new child of the document start
    u = _with_item_id(a.encode_from(v), 0, 1, 0)  # X's key (1, agent 0) < 'h' (1, agent 1)
    ship(u)
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1
    assert text == oracle.merge(to_anchor(h.arrays())) == b"hello worldXY"
    # a later local edit goes the fast way too
    v = a.version()
    a.insert(2, "--")
    ship(a.encode_from(v))
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == oracle.merge(to_anchor(h.arrays()))


def test_deletes_only_and_many_roots(ctx, oracle):
    """A batch of deletes only (no new items: the order is kept, the text re-weighed), and a batch
    whose items hang off many different old parents (roots ordered by anchor)."""
    log = crdt_hip.OpLog()
    log.insert(0, "abcdefghijklmnopqrstuvwxyz" * 40)
    r = crdt_hip.Replica(ctx)
    r.apply_updates([log.encode_from(0)])
    r.merge_inc()
    v = log.version()
    for k in range(0, 900, 37):
        log.remove(k, k + 3)
    r.apply_updates([log.encode_from(v)])
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == oracle.merge(to_anchor(log.arrays()))
    v = log.version()
    for k in range(0, 800, 13):
        log.insert(k, "é中😀"[k % 3])
    r.apply_updates([log.encode_from(v)])
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == oracle.merge(to_anchor(log.arrays()))
    assert cps == len(text.decode())


def test_incremental_state_survives_clone_and_fugue_state_starts_with_a_full_merge(ctx, oracle):
    t, patches, updates = trace_updates("sveltecomponent")
    r = crdt_hip.Replica(ctx)
    r.apply_updates(updates[:5000])
    r.merge_inc()
    c = r.clone()                 # a clone starts without state: its first call is a full merge
    c.apply_updates(updates[5000:5200])
    assert c.merge_inc()[2] == 0
    r.apply_updates(updates[5000:5200])
    assert r.merge_inc()[2] == 1
    assert r.merge_inc(text=True)[3] == c.merge_inc(text=True)[3]
    # a Fugue replica's first call builds its state (full merge)
    up = crdt_hip.OpLog(fugue=True)
    up.insert(0, "fugue text")
    f = crdt_hip.Replica(ctx, crdt_hip.OpLog(fugue=True))
    f.apply_updates([up.encode_from(0)])
    cps, nb, path, text = f.merge_inc(text=True)
    assert path == 0 and text == b"fugue text"


def test_incremental_len_on_a_document_with_more_tiles_than_cus(ctx, oracle):
    """A 2.2 M-item document: 538 tiles of 4096 old ranks, more than the GPU has CUs (k_inc holds
    ~136 KB of LDS, one workgroup per CU), so later workgroups start after earlier ones have
    spliced.  Every batch is a set of small local edits whose roots hang under parents spread
    over the whole document; each checkpoint's text is compared with the oracle's merge.  (Reads
    of the old ranks and writes of the new ones are separate arrays, incr.hip rank / rank2.)"""
    import random
    rng = random.Random(0x1C4)
    log = crdt_hip.OpLog()
    base = "".join(chr(ord("a") + i % 26) for i in range(2_200_000))
    log.insert(0, base)
    r = crdt_hip.Replica(ctx)
    r.apply_updates([log.encode_from(0)])
    assert r.merge_inc()[2] == 0
    length = len(base)
    for c in range(4):
        v = log.version()
        for _ in range(150):
            pos = rng.randrange(0, length)
            if rng.random() < 0.3 and pos + 2 < length:
                log.remove(pos, pos + 2)
                length -= 2
            else:
                s = "".join(rng.choice("XYZ") for _ in range(rng.randint(1, 4)))
                log.insert(pos, s)
                length += len(s)
        r.apply_updates([log.encode_from(v)])
        cps, nb, path, text = r.merge_inc(text=True)
        assert path == 1, c
        assert nb == length
        assert text == oracle.merge(to_anchor(log.arrays())), f"checkpoint {c}"


def test_concurrent_roots_placed_by_search_match_oracle(ctx, oracle):
    """Local edit batches in which every 5th update's items carry a key below the replica's
    largest (a random lamport, an agent of their own): their roots are placed by searching the
    parent's old subtree.  The oracle's merge of the same log at every checkpoint."""
    import random
    rng = random.Random(0xC0C0)
    t, patches, updates = trace_updates("sveltecomponent")
    r = crdt_hip.Replica(ctx)
    host = crdt_hip.OpLog(agent=0)
    paths = []
    maxlam = 0
    for c, i in enumerate(range(0, 2000, 10)):
        batch = []
        for j, u in enumerate(updates[i:i + 10]):
            n = struct.unpack_from("<I", u, 12)[0]
            if n and (i + j) % 5 == 0 and maxlam > 2:
                lam = rng.randint(1, maxlam - 1)
                for k in range(n):
                    u = _with_item_id(u, k, lam + k, 1000 + i + j)
            for k in range(n):
                maxlam = max(maxlam, struct.unpack_from("<I", u, 24 + 8 * n + 4 * k)[0])
            batch.append(u)
        r.apply_updates(batch)
        for u in batch:
            host.apply_update(u)
        cps, nb, path, text = r.merge_inc(text=True)
        paths.append(path)
        assert text == oracle.merge(to_anchor(host.arrays())), f"checkpoint {c}"
    assert paths[0] == 0 and paths[1:].count(1) >= len(paths) - 5, paths


def test_concurrent_root_whose_search_runs_out_of_range_falls_back(ctx, oracle):
    """A concurrent root under the document start of a 70,000-item document: its place would be
    after the whole document (one typing chain under the first item), beyond the search's 65,536
    ranks (incr.hip kIncScan), so the call merges in full; the next local edit is incremental."""
    a = crdt_hip.OpLog(agent=1)
    h = crdt_hip.OpLog(agent=1)
    r = crdt_hip.Replica(ctx)

    def ship(u):
        r.apply_updates([u])
        h.apply_update(u)

    a.insert(0, "".join(chr(ord("a") + i % 26) for i in range(70_000)))
    ship(a.encode_from(0))
    assert r.merge_inc()[2] == 0
    v = a.version()
    a.insert(0, "XY")
    ship(_with_item_id(a.encode_from(v), 0, 1, 0))  # X sorts below the first item (1, agent 1)
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 0
    assert text == oracle.merge(to_anchor(h.arrays()))
    assert text.endswith(b"XY")
    v = h.version()
    h.insert(5, "--")
    r.apply_updates([h.encode_from(v)])
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == oracle.merge(to_anchor(h.arrays()))


@pytest.mark.parametrize("nroots,path", [(200, 1), (300, 0)])
def test_many_concurrent_roots_in_one_batch(ctx, oracle, nroots, path):
    """One batch of `nroots` concurrent inserts, each a new child of a different old item with a
    key below every old one: up to 256 of them (incr.hip kIncHard) are placed by the searches, one
    workgroup each (k_inc_search); more than that merges in full."""
    log = crdt_hip.OpLog(agent=1)
    log.insert(0, "abcdefghijklmnopqrstuvwxyz" * 80)
    base = log.encode_from(0)
    r = crdt_hip.Replica(ctx)
    r.apply_updates([base])
    assert r.merge_inc()[2] == 0
    v = log.version()
    for k in range(nroots):  # descending positions: every new item's parent is an old item
        log.insert(6 * (nroots - k), "XYZ"[k % 3])
    u = log.encode_from(v)
    n = struct.unpack_from("<I", u, 12)[0]
    assert n == nroots
    for k in range(n):
        u = _with_item_id(u, k, 1 + k, 0)
    h = crdt_hip.OpLog(agent=1)
    h.apply_update(base)
    h.apply_update(u)
    r.apply_updates([u])
    cps, nb, p, text = r.merge_inc(text=True)
    assert p == path
    assert text == oracle.merge(to_anchor(h.arrays()))


@pytest.mark.parametrize("name,K", [("sveltecomponent", 300), ("automerge-paper", 1000)])
def test_fugue_incremental_len_matches_oracle(ctx, oracle, name, K):
    """Fugue replicas on the incremental path: the trace replayed on a Fugue upstream, its
    version-2 updates applied to a Fugue replica K patches at a time, len() after each batch.
    Local edits give a new item either a right child's place (right after its old parent) or a
    left child's place under the leftmost node of a right subtree (right before that node, which
    has no left child): every batch after the first takes the fast path (path 1) unless it holds
    more than 4096 items, and every checkpoint is the oracle's in-order merge of the same log."""
    t, up, updates = fugue_updates(name)
    r = crdt_hip.Replica(ctx, crdt_hip.OpLog(fugue=True))
    host = crdt_hip.OpLog(fugue=True)
    paths = []
    for c, i in enumerate(range(0, len(updates), K)):
        batch = updates[i:i + K]
        n_before = r.info()[0]
        r.apply_updates(batch)
        for u in batch:
            host.apply_update(u)
        cps, nb, path, text = r.merge_inc(text=True)
        paths.append(path if r.info()[0] - n_before <= 4096 else "big")
        assert (cps, nb) == (len(text.decode()), len(text))
        assert text == oracle.merge_fugue(fugue_anchor(host.arrays())), f"checkpoint {c}"
    assert text.decode() == t.end_content
    assert paths[0] in (0, "big") and all(p in (1, "big") for p in paths[1:]), paths


def test_fugue_left_child_of_a_node_with_left_children_falls_back(ctx, oracle):
    """A remote Fugue insert that makes a new left child of an old item which already has one
    (its place would need a search of the old left subtree) merges in full, and correctly; the
    next local edit is incremental again."""
    a = crdt_hip.OpLog(fugue=True)
    h = crdt_hip.OpLog(fugue=True)  # the host log fed the same (patched) updates
    r = crdt_hip.Replica(ctx, crdt_hip.OpLog(fugue=True))

    def ship(u):
        r.apply_updates([u])
        h.apply_update(u)

    a.insert(0, "abc")
    ship(a.encode_from(0))
    assert r.merge_inc(text=True)[3] == b"abc"
    v = a.version()
    a.insert(0, "x")  # a left child of 'a' (the leftmost node)
    ship(a.encode_from(v))
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == b"xabc"
    v = a.version()
    a.insert(0, "y")  # a left child of 'x' ...
    u = bytearray(a.encode_from(v))
    struct.pack_into("<I", u, 24, 1)  # ... re-parented under 'a' (id 1), which has 'x' already
    ship(bytes(u))
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 0 and text == oracle.merge_fugue(fugue_anchor(h.arrays())) == b"yxabc"
    v = h.version()
    h.insert(len(text), "!")
    r.apply_updates([h.encode_from(v)])
    cps, nb, path, text = r.merge_inc(text=True)
    assert path == 1 and text == oracle.merge_fugue(fugue_anchor(h.arrays())) == b"yxabc!"
