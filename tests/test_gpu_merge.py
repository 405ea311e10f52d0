"""GPU parity tests: device merge through the C ABI vs the oracle (bit-exact bytes / ids).

Every test runs the gfx950 kernels of libcrdt_hip.so; there is no CPU fallback in the product.
"""
import json
import os

import numpy as np
import pytest

import crdt_hip
from conftest import TESTS, TRACES, trace_path
from oracle_bind import AnchorLog

pytestmark = pytest.mark.gpu


def arrays_from_anchor(a: AnchorLog) -> crdt_hip.LogArrays:
    n = a.n
    return crdt_hip.LogArrays(a.parent[:n], a.lamport[:n], a.agent[:n], a.deleted[:n], a.cp[:n])


def to_anchor(arrs: crdt_hip.LogArrays) -> AnchorLog:
    a = AnchorLog(arrs.n)
    for f in ("parent", "lamport", "agent", "deleted", "cp"):
        getattr(a, f)[: arrs.n] = getattr(arrs, f)
    return a


_RESOLVED = {}


def resolved(name) -> crdt_hip.LogArrays:
    if name not in _RESOLVED:
        _RESOLVED[name] = crdt_hip.Trace(trace_path(name)).resolve().arrays()
    return _RESOLVED[name]


@pytest.mark.parametrize("name", TRACES)
def test_trace_merge_byte_exact(ctx, oracle, golden, name):
    """Config 2 for every trace: resolved anchor log -> one MI355X -> byte-exact endContent."""
    log = resolved(name)
    text, dig = ctx.merge(log)
    end_hash = golden[name]["sha256"]
    import hashlib
    assert hashlib.sha256(text).hexdigest() == end_hash
    assert text == oracle.merge(to_anchor(log))
    assert "%016x" % dig == golden[name]["tree_digest"]
    assert dig == oracle.tree_digest(text)


@pytest.mark.parametrize("scatter", [0, 1])
def test_repeated_text_merges_take_the_learnt_plan(golden, scatter):
    """The upstream closure of config 1 merges a document of the same shape again and again: from
    the second merge on the single wave runs on its learnt plan (no host wait inside the merge)
    and the text is copied back from the engine that ran it; the bytes stay endContent's, with
    the text from phase C or from the text kernel."""
    import hashlib
    c = crdt_hip.Context(0)
    c.set_param("text_scatter", scatter)
    for name in TRACES:
        log = resolved(name)
        for _ in range(3):
            text, dig = c.merge(log)
            assert hashlib.sha256(text).hexdigest() == golden[name]["sha256"], name
            assert "%016x" % dig == golden[name]["tree_digest"]
    c.close()


@pytest.mark.parametrize("name", ["sveltecomponent", "automerge-paper"])
def test_merge_order_matches_oracle_preorder(ctx, oracle, name):
    log = resolved(name)
    order = ctx.merge_order(log)
    _, ref = oracle.merge(to_anchor(log), want_order=True)
    assert np.array_equal(order, ref)


@pytest.mark.parametrize("name", TRACES)
def test_upstream_bench_loop_semantics(ctx, golden, py_trace, name):
    """The reference's upstream closure (main.rs:28-36) with HipMerge as R, every trace."""
    t = crdt_hip.Trace(trace_path(name))
    rope = crdt_hip.HipMerge.from_str(t.start_content)
    for i in range(len(t)):
        pos, dele, ins = t.patch(i)
        rope.replace(pos, pos + dele, ins)
    assert rope.len() == len(t.end_content)  # main.rs:35
    assert rope.text() == t.end_content


def test_downstream_bench_loop_semantics(golden, py_trace):
    """The reference's downstream closure (main.rs:60-69): clone + apply_update* + len()."""
    t = py_trace("sveltecomponent")
    patches = [(int(t.pos[i]), int(t.dele[i]),
                t.ins_cp[int(t.ins_off[i]): int(t.ins_off[i] + t.ins_len[i])].tobytes().decode("utf-32-le"))
               for i in range(len(t))]
    crdt0, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
    for _ in range(2):
        crdt = crdt0.clone()
        for u in updates:
            crdt.apply_update(u)
        assert crdt.len() == len(t.end_content)
        assert crdt.text() == t.end_content


def test_concurrent_fixtures_on_device(ctx):
    with open(os.path.join(TESTS, "golden", "concurrent.json")) as f:
        cases = json.load(f)
    for c in cases:
        log = crdt_hip.LogArrays(c["parent"], c["lamport"], c["agent"], c["deleted"], c["cp"])
        text, _ = ctx.merge(log)
        assert text.decode() == c["expected"], c["name"]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_synth_agents_vs_oracle(ctx, oracle, seed):
    log = crdt_hip.OpLog.synth_agents(200000, 64, 0x5EED0000 + seed).arrays()
    text, dig = ctx.merge(log)
    assert text == oracle.merge(to_anchor(log))
    order = ctx.merge_order(log)
    _, ref = oracle.merge(to_anchor(log), want_order=True)
    assert np.array_equal(order, ref)


def test_synth_agents_naive_prefix(ctx, oracle):
    """Causal prefix of the 64-agent log: device == tree oracle == O(n^2) integrator."""
    log = crdt_hip.OpLog.synth_agents(10000, 64, 0x5EED0001).arrays()
    text, _ = ctx.merge(log)
    a = to_anchor(log)
    assert text == oracle.merge(a) == oracle.merge_naive(a)


@pytest.mark.parametrize("p_chain", [90, 0])
def test_synth_tree_vs_oracle(ctx, oracle, p_chain):
    log = crdt_hip.OpLog.synth_tree(1_000_000, p_chain, 50, 0x5EED0002).arrays()
    text, dig = ctx.merge(log)
    ref = oracle.merge(to_anchor(log))
    assert text == ref
    assert dig == oracle.tree_digest(ref)


def fanout_log(n_children, depth_extra=0):
    """Every item anchored at the document start (typing backwards at position 0)."""
    n = n_children + depth_extra
    parent = np.zeros(n, np.uint32)
    if depth_extra:
        parent[n_children:] = np.arange(n_children, n, dtype=np.uint32)  # a chain under the last
    lam = np.arange(1, n + 1, dtype=np.uint32)
    rng = np.random.default_rng(n)
    cp = rng.integers(0x61, 0x7B, n).astype(np.uint32)
    deleted = (rng.random(n) < 0.2).astype(np.uint8)
    return crdt_hip.LogArrays(parent, lam, np.zeros(n, np.uint16), deleted, cp)


@pytest.mark.parametrize("k", [2, 3, 4, 8, 9, 17, 64, 65, 1000, 4096, 4097, 20000])
def test_sibling_groups_every_sort_path(ctx, oracle, k):
    """2 inline, 3..8 register network, 9..64 wave rank sort, 65..4096 LDS bitonic, >4096 global."""
    log = fanout_log(k, depth_extra=50)
    order = ctx.merge_order(log)
    _, ref = oracle.merge(to_anchor(log), want_order=True)
    assert np.array_equal(order, ref)
    text, _ = ctx.merge(log)
    assert text == oracle.merge(to_anchor(log))


def test_ragged_batch_with_edge_cases(ctx, oracle):
    rng = np.random.default_rng(7)
    logs = []
    logs.append(crdt_hip.LogArrays([], [], [], [], []))                   # empty document
    logs.append(crdt_hip.LogArrays([0], [1], [0], [0], [0x1F600]))         # one 4-byte char
    logs.append(crdt_hip.LogArrays([0, 1, 2], [1, 2, 3], [0, 0, 0], [1, 1, 1], [97, 98, 99]))  # all deleted
    logs.append(resolved("sveltecomponent"))
    for n in (63, 64, 65, 127, 128, 4095, 4097):
        logs.append(fanout_log(n // 2, n - n // 2))
    logs.append(crdt_hip.OpLog.synth_agents(50000, 64, 99).arrays())
    wide = crdt_hip.OpLog.synth_agents(3000, 8, 5).arrays()
    wide.cp[:] = rng.choice([0x41, 0xE9, 0x2019, 0x4E2D, 0x1F600], wide.n)  # every UTF-8 width
    logs.append(wide)
    dig, lens = ctx.merge_batch(logs)
    for i, lg in enumerate(logs):
        ref = oracle.merge(to_anchor(lg)) if lg.n else b""
        assert lens[i] == len(ref), i
        assert dig[i] == oracle.tree_digest(ref), i


@pytest.mark.parametrize("stride", [16, 256, 4096])
def test_splitter_stride_and_waves_do_not_change_results(oracle, stride):
    c = crdt_hip.Context(0)
    c.set_param("splitter_stride", stride)
    c.set_param("max_wave_slots", 1 << 20)  # forces several waves
    logs = [resolved(n) for n in TRACES]
    dig, lens = c.merge_batch(logs)
    for i, n in enumerate(TRACES):
        ref = oracle.merge(to_anchor(logs[i]))
        assert lens[i] == len(ref) and dig[i] == oracle.tree_digest(ref)
    c.close()


@pytest.mark.parametrize("lanes", [2, 3, 8])
@pytest.mark.parametrize("level1", [0, 1])
def test_concurrent_wave_lanes_do_not_change_results(golden, lanes, level1):
    """Waves of one merge run on `lanes` streams at once (Engine::merge_lanes): every replica's
    digest and length equal the one-lane merge's and the trace's, and every run is counted once."""
    bases = [resolved(n) for n in TRACES]
    out = {}
    for k in (1, lanes):
        c = crdt_hip.Context(0)
        c.set_param("lanes", k)
        c.set_param("level1", level1)
        c.set_param("max_wave_slots", 1 << 20)  # 3 replicas x 4 traces: several waves
        b = c.batch(bases, replicas=3, relabel="rotate", seed=77)
        for _ in range(2):  # the second merge reuses every lane's scratch
            dig, lens, st = b.merge()
        assert st["waves"] >= 3
        out[k] = (dig.copy(), lens.copy(), st["runs"], st["stage_launches"]["classify"])
        b.close()
        c.close()
    assert np.array_equal(out[1][0], out[lanes][0]) and np.array_equal(out[1][1], out[lanes][1])
    assert out[1][2:] == out[lanes][2:]
    for r in range(len(out[1][0])):
        name = TRACES[r % 4]
        assert "%016x" % out[lanes][0][r] == golden[name]["tree_digest"], r
        assert out[lanes][1][r] == golden[name]["end_bytes"], r


def test_concurrent_wave_lanes_report_a_malformed_wave():
    c = crdt_hip.Context(0)
    c.set_param("lanes", 4)
    c.set_param("max_wave_slots", 1 << 20)
    good = [resolved(n) for n in TRACES]
    bad = crdt_hip.LogArrays([0, 5], [1, 2], [0, 0], [0, 0], [97, 98])
    with pytest.raises(crdt_hip.CrdtHipError) as e:
        c.merge_batch(good + [bad] + good)
    assert e.value.code == -5
    dig, lens = c.merge_batch(good + good)  # every lane recovers
    assert np.array_equal(dig[:4], dig[4:]) and all(int(x) > 0 for x in lens)
    c.close()


@pytest.mark.parametrize("relabel", ["none", "rotate", "shuffle"])
def test_replica_batch_relabel_invariance(ctx, oracle, golden, relabel):
    """Config 3 shape at small scale: relabelled HBM replicas merge to the trace documents."""
    bases = [resolved(n) for n in TRACES]
    b = ctx.batch(bases, replicas=3, relabel=relabel, seed=1234)
    assert b.docs == 12
    dig, lens, st = b.merge()
    for r in range(b.docs):
        name = TRACES[r % 4]
        assert "%016x" % dig[r] == golden[name]["tree_digest"], (relabel, r)
        assert lens[r] == golden[name]["end_bytes"]
    assert st["items"] == 3 * sum(golden[n]["items"] for n in TRACES)


def _level1_cases():
    rng = np.random.default_rng(11)
    logs = [resolved(n) for n in TRACES]
    logs.append(crdt_hip.OpLog.synth_agents(20000, 64, 0x5EED0005).arrays())
    logs.append(crdt_hip.OpLog.synth_agents(4000, 3, 0x5EED0006).arrays())
    for k in (2, 5, 9, 40, 64, 65):
        logs.append(fanout_log(k, depth_extra=30))
    wide = crdt_hip.OpLog.synth_agents(3000, 8, 5).arrays()
    wide.cp[:] = rng.choice([0x41, 0xE9, 0x2019, 0x4E2D, 0x1F600], wide.n)
    logs.append(wide)
    big = crdt_hip.LogArrays(np.arange(70000, dtype=np.uint32), np.arange(1, 70001, dtype=np.uint32),
                             np.zeros(70000, np.uint16), np.zeros(70000, np.uint8),
                             np.full(70000, 0x4E2D, np.uint32))  # one run of 210,000 bytes
    logs.append(big)
    n = 40 * 22000  # 40 sibling runs of 66,000 bytes each: more heavy runs than the LDS table
    par = np.arange(n, dtype=np.uint32)
    par[::22000] = 0
    logs.append(crdt_hip.LogArrays(par, np.arange(1, n + 1, dtype=np.uint32), np.zeros(n, np.uint16),
                                   np.zeros(n, np.uint8), np.full(n, 0x4E2D, np.uint32)))
    logs.append(crdt_hip.LogArrays([], [], [], [], []))
    return logs


@pytest.mark.parametrize("slots", [16, 32, 64])
def test_runs_slots_per_thread_agree(oracle, golden, slots):
    """k_runs with 16, 32 (default) and 64 slots per thread (64: one wave per 4096-slot tile,
    64-bit slot masks): the level-1 cases against the oracle, a rotated trace batch (contracted,
    compact nsq list) and a shuffled one (no contraction) against the golden digests, with the
    synchronous merge and the learnt-plan merge."""
    c = crdt_hip.Context(0)
    c.set_param("runs_slots", slots)
    logs = _level1_cases()
    dig, lens = c.merge_batch(logs)
    for i, lg in enumerate(logs):
        ref = oracle.merge(to_anchor(lg)) if lg.n else b""
        assert lens[i] == len(ref), i
        assert dig[i] == oracle.tree_digest(ref), i
    bases = [resolved(n) for n in TRACES]
    for relabel in ("rotate", "shuffle"):
        b = c.batch(bases, replicas=2, relabel=relabel, seed=5)
        for _ in range(2):
            dig, lens, st = b.merge()
            for r in range(b.docs):
                name = TRACES[r % 4]
                assert "%016x" % dig[r] == golden[name]["tree_digest"], (relabel, r)
                assert lens[r] == golden[name]["end_bytes"], (relabel, r)
        b.close()
    c.close()


@pytest.mark.parametrize("level1,group,dbits", [(0, 0, 0), (1, 1, 0), (1, 2, 0), (1, 2, 10)])
def test_level1_paths_match_oracle(oracle, level1, group, dbits):
    """Per-document LDS level 1 (k_doctree, default) and the global level-1 kernels, with their
    sibling groups by counting (group 1) and by the two radix sorts (group 2; sort A with 8-bit
    or, dbits 10, 10-bit digits), must give the oracle's bytes and digests, including sibling
    groups of every sort width (> 64 makes the LDS path hand the wave to the global path) and a
    run heavier than 0xFFFF bytes."""
    c = crdt_hip.Context(0)
    c.set_param("level1", level1)
    c.set_param("l1_group", group)
    c.set_param("rs_digit_bits", dbits)
    logs = _level1_cases()
    dig, lens, st = c.merge_batch(logs, stats=True)
    for i, lg in enumerate(logs):
        ref = oracle.merge(to_anchor(lg)) if lg.n else b""
        assert lens[i] == len(ref), i
        assert dig[i] == oracle.tree_digest(ref), i
    for i in (0, 4, 6, 11, 12, 13, 14):  # one document per merge: the LDS path where it fits
        text, d1 = c.merge(logs[i])
        assert text == (oracle.merge(to_anchor(logs[i])) if logs[i].n else b""), i
        order = c.merge_order(logs[i])
        if logs[i].n:
            _, ref = oracle.merge(to_anchor(logs[i]), want_order=True)
            assert np.array_equal(order, ref), i
    c.close()


def test_level1_lds_path_is_taken_for_trace_batches(ctx):
    bases = [resolved(n) for n in TRACES]
    b = ctx.batch(bases, replicas=2, relabel="rotate", seed=5)
    _, _, st = b.merge()
    assert st["stage_launches"]["doctree"] == 2 and st["stage_launches"]["walk1"] == 0
    # the expansion runs inside k_doctree (the texts fit LDS)
    assert st["stage_launches"]["expand"] == 0
    # dead runs (no visible item, no child) are dropped at level 0: the four traces number
    # 44,844 runs without the drop and ~27,160 with it (the drop is conservative at wave
    # boundaries, so the exact count moves a little with each replica's relabelling shift), plus
    # at most one per 4096-slot tile (247 per replica of the four) since runs never cross tiles; a
    # regression that kept them would still merge correctly, so the count is checked here
    assert 2 * 27000 < st["runs"] < 2 * 27650


@pytest.mark.parametrize("lanes", [1, 3])
def test_grouped_batch_returns_results_in_the_callers_order(lanes):
    """group_docs places a replica batch base by base (each base in waves of its own); the
    digests and lengths still come back in the caller's replica-major order, equal to the
    ungrouped batch's, over several waves and lanes."""
    bases = [resolved(n) for n in TRACES]
    out = []
    for grp in (0, 1):
        c = crdt_hip.Context(0)
        c.set_param("lanes", lanes)
        c.set_param("group_docs", grp)
        c.set_param("max_wave_slots", 1 << 20)
        b = c.batch(bases, replicas=3, relabel="rotate", seed=8)
        for _ in range(2):
            dig, lens, st = b.merge()
        out.append((dig.copy(), lens.copy(), st["waves"]))
        b.close()
        c.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert out[1][2] >= 4


@pytest.mark.parametrize("shape", ["typing", "tree"])
def test_tiles_above_the_lds_text_stage(ctx, oracle, shape):
    """Tiles holding more than k_classify's 8 KiB LDS text stage (4-byte characters, nearly all
    visible) take the direct-store path; the document must still equal the oracle's."""
    rng = np.random.default_rng(7 if shape == "typing" else 8)
    n = 50_000
    ids = np.arange(1, n + 1, dtype=np.uint32)
    if shape == "typing":
        parent = ids - 1
        deleted = np.zeros(n, np.uint8)
    else:
        parent = np.where(rng.random(n) < 0.8, ids - 1, rng.integers(0, ids, dtype=np.uint32))
        deleted = (rng.random(n) < 0.05).astype(np.uint8)
    cp = rng.integers(0x10000, 0x110000, n, dtype=np.uint32)
    cp[::7] = rng.integers(0x800, 0xD800, len(cp[::7]), dtype=np.uint32)  # some 3-byte ones
    lg = crdt_hip.LogArrays(parent, ids, np.zeros(n, np.uint16), deleted, cp)
    text, dig = ctx.merge(lg)
    ref = oracle.merge(to_anchor(lg))
    assert len(ref) > 3 * n and text == ref and dig == oracle.tree_digest(ref)
    b = ctx.batch([lg], replicas=3, relabel="shuffle", seed=3)  # resident, relabelled
    d3, l3, _ = b.merge()
    assert all(int(x) == dig for x in d3) and all(int(x) == len(ref) for x in l3)
    b.close()


@pytest.mark.parametrize("level1", [0, 1])
def test_malformed_logs_are_rejected(level1):
    """Out-of-range parents, an item that is its own parent and parent cycles fail with EBADLOG on
    the per-document (LDS) and on the global level 1, as single merges and as resident batches
    (learnt plans on the second merge), and the engine merges a good log right after."""
    ctx = crdt_hip.Context(0)
    ctx.set_param("level1", level1)
    bad_parent = crdt_hip.LogArrays([0, 5], [1, 2], [0, 0], [0, 0], [97, 98])
    # item 2 is its own parent: k_runs must not give its row itself as parent (a self-loop the
    # global walks would follow), it clamps it to the document start and the merge is rejected
    self_parent = crdt_hip.LogArrays([0, 2], [1, 2], [0, 0], [0, 0], [97, 98])
    cycle = crdt_hip.LogArrays([0, 3, 2], [1, 2, 3], [0, 0, 0], [0, 0, 0], [97, 98, 99])
    # two runs that are each other's parent (neither reachable from the document start): their
    # up links never resolve, so the LDS path's pointer jumping has to give up, not spin
    cycle2 = crdt_hip.LogArrays([0, 4, 1, 2], [1, 2, 3, 4], [0, 0, 0, 0], [0, 0, 0, 0],
                                [97, 98, 99, 100])
    ok = crdt_hip.LogArrays([0, 1], [1, 2], [0, 0], [0, 0], [97, 98])
    for bad in (bad_parent, self_parent, cycle, cycle2):
        with pytest.raises(crdt_hip.CrdtHipError) as e:
            ctx.merge(bad)
        assert e.value.code == -5
        b = ctx.batch([ok, bad, ok], replicas=2, relabel="none")
        for _ in range(2):
            with pytest.raises(crdt_hip.CrdtHipError) as e:
                b.merge()
            assert e.value.code == -5
        b.close()
    assert ctx.merge(ok)[0] == b"ab"  # the engine recovers after an error
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("level1", [0, 1])
def test_parent_in_another_document_of_the_wave_is_rejected(level1):
    """A parent index past its document's items that lands on an item of the NEXT document of the
    same wave (documents are 64-slot aligned: index 70 of a 2-item document is slot 6 of the next
    one).  k_classify flags it; k_runs (which takes each word's document start from its head
    record and no longer clamps such a parent into its own document) then finds a run of the other
    document, which the level 1 must not follow into a wrong order or an endless walk.  The batch
    fails with EBADLOG on both level-1 paths, and the same engine merges a well-formed batch right
    after."""
    c = crdt_hip.Context(0)
    c.set_param("level1", level1)
    n = 10
    good = crdt_hip.LogArrays(list(range(n)), list(range(1, n + 1)), [0] * n, [0] * n,
                              [97 + i for i in range(n)])
    bad = crdt_hip.LogArrays([0, 70], [1, 2], [0, 0], [0, 0], [97, 98])
    with pytest.raises(crdt_hip.CrdtHipError) as e:
        c.merge_batch([bad, good])
    assert e.value.code == -5
    dig, lens = c.merge_batch([good, good])
    assert list(lens) == [n, n] and dig[0] == dig[1]
    c.close()


def test_repeated_merges_are_deterministic(ctx):
    log = crdt_hip.OpLog.synth_agents(300000, 64, 42).arrays()
    d0 = ctx.merge_digest(log)
    for _ in range(3):
        assert ctx.merge_digest(log) == d0


@pytest.mark.parametrize("p_chain", [90, 0])
def test_device_generated_config5_matches_host_log(ctx, oracle, p_chain):
    """crdt_hip_batch_synth_tree generates on the device exactly OpLog.synth_tree's log: its
    merge equals the oracle's merge of the host-generated log (same seed)."""
    n = 1_000_000
    b = crdt_hip.Batch.synth_tree(ctx, n, p_chain, 50, 0x5EED0002)
    assert b.docs == 1 and b.items == n
    dig, lens, _ = b.merge()
    host = crdt_hip.OpLog.synth_tree(n, p_chain, 50, 0x5EED0002).arrays()
    ref = oracle.merge(to_anchor(host))
    assert int(lens[0]) == len(ref) == int(np.count_nonzero(host.deleted == 0))
    assert int(dig[0]) == oracle.tree_digest(ref)


def test_document_above_16mib_digest(ctx, oracle):
    """20 MB of text (4,883 leaves > 4,096): the device hashes the leaf digests in groups."""
    n = 20_000_000
    par = np.arange(n, dtype=np.uint32)
    par[::1000] = np.arange(0, n, 1000, dtype=np.uint32) // 2  # some branching
    rng = np.random.default_rng(5)
    log = crdt_hip.LogArrays(par, np.arange(1, n + 1, dtype=np.uint32), np.zeros(n, np.uint16),
                             np.zeros(n, np.uint8), rng.integers(0x61, 0x7B, n).astype(np.uint32))
    dig, lens = ctx.merge_batch([log])
    ref = oracle.merge(to_anchor(log))
    assert int(lens[0]) == len(ref) == n
    assert int(dig[0]) == oracle.tree_digest(ref)


@pytest.mark.parametrize("lanes", [1, 2, 3])
def test_learnt_plan_merges_match_synchronous_ones(golden, lanes):
    """A second merge of the same batch enqueues every wave with the plan the first merge
    learnt (Engine::merge_async: no host wait after level 0); it must give the same digests,
    lengths, codepoints and run counts as the synchronous path, for one and several lanes."""
    bases = [resolved(n) for n in TRACES]
    out = {}
    for cache in (0, 1):
        c = crdt_hip.Context(0)
        c.set_param("text_scatter", 1)  # (the learnt-plan merges then take the text kernel)
        c.set_param("lanes", lanes)
        c.set_param("plan_cache", cache)
        c.set_param("max_wave_slots", 1 << 20)  # several waves
        b = c.batch(bases, replicas=3, relabel="rotate", seed=77)
        res = [b.merge() for _ in range(3)]
        for dig, lens, st in res:
            assert st["waves"] >= 3
            for r in range(b.docs):
                name = TRACES[r % 4]
                assert "%016x" % dig[r] == golden[name]["tree_digest"], (cache, r)
                assert lens[r] == golden[name]["end_bytes"], (cache, r)
        # (the learnt-plan merges write the text with k_tscatter, the synchronous ones in
        # k_doctree: the text stage's launches differ, every other stage's match)
        for i, (_, _, st) in enumerate(res):
            assert (st["stage_launches"]["text"] > 0) == (cache == 1 and i > 0)
        out[cache] = [(d.tolist(), l.tolist(), st["runs"],
                       {k: v for k, v in st["stage_launches"].items() if k != "text"})
                      for d, l, st in res]
        b.close()
        c.close()
    assert out[0] == out[1]


@pytest.mark.parametrize("l1_split,tail_div", [(0, 0), (1, 0), (1, 4), (1, 2)])
def test_scheduling_knobs_do_not_change_results(golden, l1_split, tail_div):
    """Level 1 on the lane's low-priority stream (l1_split) and the small trailing wave
    (tail_wave_div) only reorder work: digests, lengths and runs stay those of the traces, in the
    first (synchronous) merge and in the learnt-plan merges after it."""
    bases = [resolved(n) for n in TRACES]
    c = crdt_hip.Context(0)
    c.set_param("lanes", 2)
    c.set_param("l1_split", l1_split)
    c.set_param("tail_wave_div", tail_div)
    c.set_param("max_wave_slots", 1 << 20)
    b = c.batch(bases, replicas=3, relabel="rotate", seed=5)
    runs = set()
    for _ in range(3):
        dig, lens, st = b.merge()
        runs.add(st["runs"])
        for r in range(b.docs):
            name = TRACES[r % 4]
            assert "%016x" % dig[r] == golden[name]["tree_digest"], r
            assert lens[r] == golden[name]["end_bytes"], r
    assert len(runs) == 1
    waves = st["waves"]
    b.close()
    c.set_param("tail_wave_div", 0)
    b = c.batch(bases, replicas=3, relabel="rotate", seed=5)
    greedy = b.merge()[2]["waves"]
    b.close()
    c.close()
    # a separate trailing wave (its documents would otherwise have filled the last greedy wave)
    assert waves == greedy or (tail_div and waves == greedy + 1)


def test_plan_that_no_longer_fits_is_redone():
    """The device checks the enqueued plan (k_docmax flags C_REPLAN when the wave has more runs
    than planned) and the host merges such a wave again: forced here with a plan of half size."""
    bases = [resolved(n) for n in TRACES]
    c = crdt_hip.Context(0)
    c.set_param("max_wave_slots", 1 << 20)
    b = c.batch(bases, replicas=2, relabel="rotate", seed=3)
    d0, l0, s0 = b.merge()
    c.set_param("plan_shrink", 1)
    d1, l1, s1 = b.merge()
    c.set_param("plan_shrink", 0)
    d2, l2, s2 = b.merge()
    assert np.array_equal(d0, d1) and np.array_equal(d0, d2)
    assert np.array_equal(l0, l1) and np.array_equal(l0, l2)
    assert s0["runs"] == s1["runs"] == s2["runs"]
    b.close()
    c.close()


def test_merge_len_counts_codepoints_on_device(ctx, golden, py_trace):
    """Upstream::len (rope.rs:16-19, 133-136): codepoints of the merged text, counted on the
    device; multi-byte texts included."""
    for name in TRACES:
        cps, nbytes, dig = ctx.merge_len(resolved(name))
        end = py_trace(name).end_content
        assert (cps, nbytes) == (len(end), len(end.encode())), name
        assert "%016x" % dig == golden[name]["tree_digest"]
    rng = np.random.default_rng(3)
    wide = crdt_hip.OpLog.synth_agents(30000, 8, 5).arrays()
    wide.cp[:] = rng.choice([0x41, 0xE9, 0x2019, 0x4E2D, 0x1F600], wide.n)
    text, _ = ctx.merge(wide)
    cps, nbytes, _ = ctx.merge_len(wide)
    assert nbytes == len(text) and cps == len(text.decode("utf-8"))
    big = crdt_hip.LogArrays(np.arange(5_000_000, dtype=np.uint32),
                             np.arange(1, 5_000_001, dtype=np.uint32),
                             np.zeros(5_000_000, np.uint16), np.zeros(5_000_000, np.uint8),
                             np.full(5_000_000, 0x4E2D, np.uint32))  # 15 MB: many leaves
    cps, nbytes, _ = ctx.merge_len(big)
    assert (cps, nbytes) == (5_000_000, 15_000_000)


def test_rccl_single_rank_allgather(ctx):
    """The engine's RCCL communicator (crdt_hip_comm_init + crdt_hip_allgather_u64) on one rank:
    the digest / counter exchange bench.py runs after timing."""
    c = crdt_hip.Context(0)
    c.comm_init(1, 0, crdt_hip.Context.comm_unique_id())
    v = np.array([1, 2**63 + 5, 0xDEADBEEF, 7], np.uint64)
    out = c.allgather_u64(v, 1)
    assert np.array_equal(out, v)
    big = np.arange(16384, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    assert np.array_equal(c.allgather_u64(big, 1), big)
    c.close()


@pytest.mark.parametrize("relabel", ["rotate", "shuffle"])
def test_batch_mixed_ascii_and_escaped_codepoints(ctx, oracle, relabel):
    """Documents with a few multi-byte codepoints scattered among ASCII (2-, 3- and 4-byte UTF-8,
    some deleted), relabelled, as resident batches against the oracle: with the compact list of
    the non-seq items' parents and keys (Engine::build_nsq, the default) and without it (param
    nsq_list 0: the level-0 kernels gather the parent and key columns), the same digests."""
    rng = np.random.default_rng(11)
    logs = []
    for n, p_esc in ((30_000, 0.02), (5_000, 0.3), (20_000, 0.0005)):
        ids = np.arange(1, n + 1, dtype=np.uint32)
        parent = np.where(rng.random(n) < 0.9, ids - 1, rng.integers(0, ids, dtype=np.uint32))
        deleted = (rng.random(n) < 0.1).astype(np.uint8)
        cp = rng.integers(0x20, 0x7F, n, dtype=np.uint32)
        esc = rng.random(n) < p_esc
        cp[esc] = rng.choice([0xE9, 0x4E2D, 0x1F600, 0x7FF, 0x800, 0xFFFF, 0x10000],
                             int(esc.sum())).astype(np.uint32)
        logs.append(crdt_hip.LogArrays(parent, ids, np.zeros(n, np.uint16), deleted, cp))
    refs = [oracle.merge(to_anchor(lg)) for lg in logs]
    want = [oracle.tree_digest(r) for r in refs]
    digests = {}
    for nsq in (0, 1):
        ctx.set_param("nsq_list", nsq)
        try:
            b = ctx.batch(logs, replicas=3, relabel=relabel, seed=21)
            d, l, _ = b.merge()
            b.close()
        finally:
            ctx.set_param("nsq_list", 1)
        for i, (x, y) in enumerate(zip(d, l)):
            assert int(x) == want[i % 3] and int(y) == len(refs[i % 3]), (nsq, i)
        digests[nsq] = list(map(int, d))
    assert digests[0] == digests[1]


@pytest.mark.parametrize("relabel", ["rotate", "shuffle"])
def test_run_contraction_modes_agree(oracle, golden, relabel):
    """Run contraction by the input (0), always (1) and never (2: every item heads its own run,
    k_classify reads no parents, k_runs takes each run's parent from the column) give the same
    digests on relabelled trace batches; without contraction a wave numbers one run per item and
    document start.  By the input, the shuffled batch (no consecutive ids) goes uncontracted and
    the rotated one contracts."""
    bases = [resolved(n) for n in TRACES]
    runs = {}
    for mode in (0, 1, 2):
        c = crdt_hip.Context(0)
        c.set_param("contraction", mode)
        b = c.batch(bases, replicas=2, relabel=relabel, seed=77)
        for _ in range(2):  # (the synchronous merge, then the learnt-plan merge)
            dig, lens, st = b.merge()
            for r in range(b.docs):
                name = TRACES[r % 4]
                assert "%016x" % dig[r] == golden[name]["tree_digest"], (mode, r)
                assert lens[r] == golden[name]["end_bytes"], (mode, r)
        runs[mode] = st["runs"]
        assert (st["runs"] == st["items"] + b.docs) == (mode == 2) or mode == 0
        b.close()
        c.close()
    assert runs[0] == (runs[2] if relabel == "shuffle" else runs[1])
    assert runs[1] < runs[2]


@pytest.mark.parametrize("level1,group,stride,dbits", [(0, 0, 0, 0), (1, 1, 0, 0), (1, 2, 0, 0),
                                                        (1, 2, 0, 10), (1, 1, 4096, 0),
                                                        (1, 2, 4096, 0)])
def test_uncontracted_uploads_match_oracle_and_reject_bad_parents(oracle, level1, group, stride,
                                                                   dbits):
    """The same without contraction on uploaded logs (the level-1 cases: agents, wide sibling
    groups, heavy runs, multi-byte text), on the per-document and on the global level 1 (there
    the first walk stages each sublist's text, k_tcopy places it, and with 4096 runs per splitter
    most sublists hold more than the 128 staged bytes, whose rest k_walk_ovf writes), and a parent
    out of range is still reported."""
    c = crdt_hip.Context(0)
    c.set_param("contraction", 2)
    c.set_param("level1", level1)
    c.set_param("l1_group", group)
    c.set_param("rs_digit_bits", dbits)
    if stride:
        c.set_param("splitter_stride", stride)
    logs = _level1_cases()
    dig, lens, st = c.merge_batch(logs, stats=True)
    for i, lg in enumerate(logs):
        ref = oracle.merge(to_anchor(lg)) if lg.n else b""
        assert lens[i] == len(ref), i
        assert dig[i] == oracle.tree_digest(ref), i
    bad_parent = crdt_hip.LogArrays([0, 5], [1, 2], [0, 0], [0, 0], [97, 98])
    with pytest.raises(crdt_hip.CrdtHipError) as e:
        c.merge(bad_parent)
    assert e.value.code == -5
    c.close()


@pytest.mark.parametrize("knob", ["xcd_order", "stile_text"])
def test_level0_knobs_off_match_golden(golden, knob):
    """The XCD-aware tile order and the per-document text staged from the tile segments only
    change where work runs and where text is read from: off, the digests stay the traces'."""
    bases = [resolved(n) for n in TRACES]
    c = crdt_hip.Context(0)
    c.set_param(knob, 0)
    b = c.batch(bases, replicas=3, relabel="rotate", seed=9)
    for _ in range(2):
        dig, lens, st = b.merge()
        for r in range(b.docs):
            name = TRACES[r % 4]
            assert "%016x" % dig[r] == golden[name]["tree_digest"], (knob, r)
            assert lens[r] == golden[name]["end_bytes"], (knob, r)
    b.close()
    c.close()


def _mixed_logs(seed=11):
    """Documents with multi-byte codepoints among ASCII, some deleted, one spanning ~20 tiles
    (small enough in runs and text for k_doctree's LDS)."""
    rng = np.random.default_rng(seed)
    logs = []
    for n, p_esc, p_seq in ((30_000, 0.02, 0.9), (5_000, 0.3, 0.9), (80_000, 0.001, 0.97)):
        ids = np.arange(1, n + 1, dtype=np.uint32)
        parent = np.where(rng.random(n) < p_seq, ids - 1, rng.integers(0, ids, dtype=np.uint32))
        deleted = (rng.random(n) < 0.1).astype(np.uint8)
        cp = rng.integers(0x20, 0x7F, n, dtype=np.uint32)
        esc = rng.random(n) < p_esc
        cp[esc] = rng.choice([0xE9, 0x4E2D, 0x1F600, 0x7FF, 0x800, 0xFFFF, 0x10000],
                             int(esc.sum())).astype(np.uint32)
        logs.append(crdt_hip.LogArrays(parent, ids, np.zeros(n, np.uint16), deleted, cp))
    return logs


@pytest.mark.parametrize("scatter,stile,lanes", [(1, 2, 2), (1, 2, 1), (1, 1, 1), (0, 2, 2),
                                                  (0, 1, 1)])
def test_text_paths_match_golden(golden, scatter, stile, lanes):
    """The document text of the learnt-plan merges is written either by k_doctree itself
    (text_scatter 0: phase C, staged by loads and shifts or by LDS-DMA) or by k_tscatter from the
    tiles' text segments once k_doctree has left every run's place in roff (text_scatter 1): the
    same digests and lengths as the synchronous first merge and the traces', and
    the text stage runs exactly when scatter mode is on."""
    bases = [resolved(n) for n in TRACES]
    c = crdt_hip.Context(0)
    c.set_param("text_scatter", scatter)
    c.set_param("stile_text", stile)
    c.set_param("lanes", lanes)
    c.set_param("max_wave_slots", 1 << 21)  # several waves
    b = c.batch(bases, replicas=5, relabel="rotate", seed=13)
    for it in range(3):
        dig, lens, st = b.merge()
        for r in range(b.docs):
            name = TRACES[r % 4]
            assert "%016x" % dig[r] == golden[name]["tree_digest"], (it, r)
            assert lens[r] == golden[name]["end_bytes"], (it, r)
        if it:  # (learnt plans: stile staging, and the text kernel in scatter mode)
            assert (st["stage_launches"]["text"] > 0) == bool(scatter), st["stage_launches"]
            assert st["stage_launches"]["text"] in (0, st["waves"])
    b.close()
    c.close()


@pytest.mark.parametrize("scatter", [1, 0])
def test_text_paths_multibyte_match_oracle(oracle, scatter):
    """Multi-byte UTF-8 (2-4 bytes, escaped groups) in learnt-plan merges, both text paths, against
    the oracle's bytes and digests; one document spans ~20 tiles."""
    logs = _mixed_logs()
    refs = [oracle.merge(to_anchor(lg)) for lg in logs]
    c = crdt_hip.Context(0)
    c.set_param("text_scatter", scatter)
    b = c.batch(logs, replicas=4, relabel="rotate", seed=3)
    for it in range(3):
        d, l, st = b.merge()
        for i, (x, y) in enumerate(zip(d, l)):
            ref = refs[i % 3]
            assert int(y) == len(ref) and int(x) == oracle.tree_digest(ref), (it, i)
    assert (st["stage_launches"]["text"] > 0) == bool(scatter)
    b.close()
    c.close()


def test_glds_staging_wait_is_pinned(golden, oracle):
    """Guard of the s_waitcnt vmcnt(0) in front of k_doctree's text-output barrier (engine.hip
    doc_text): the LDS-DMA staging writes LDS as a global load, which a barrier does not wait for.
    With the glds_late hook every staging load is issued after the prefix and delta phases, right
    in front of that wait, so without it the output would read chunks still in flight; phase C
    (text_scatter 0) with LDS-DMA staging (stile_text 2) must still give the traces' digests and
    the oracle's for a document spanning more than 16 tiles."""
    bases = [resolved(n) for n in TRACES]
    logs = _mixed_logs(5)
    refs = [oracle.merge(to_anchor(lg)) for lg in logs]
    c = crdt_hip.Context(0)
    c.set_param("text_scatter", 0)
    c.set_param("stile_text", 2)
    c.set_param("glds_late", 1)
    b = c.batch(bases, replicas=3, relabel="rotate", seed=9)
    m = c.batch(logs, replicas=2, relabel="rotate", seed=9)
    for _ in range(3):
        dig, lens, st = b.merge()
        for r in range(b.docs):
            name = TRACES[r % 4]
            assert "%016x" % dig[r] == golden[name]["tree_digest"], r
            assert lens[r] == golden[name]["end_bytes"], r
        d, l, _ = m.merge()
        for i, (x, y) in enumerate(zip(d, l)):
            assert int(y) == len(refs[i % 3]) and int(x) == oracle.tree_digest(refs[i % 3]), i
    assert st["stage_launches"]["doctree"] > 0 and st["stage_launches"]["text"] == 0
    b.close()
    m.close()
    c.close()


@pytest.mark.parametrize("relabel", ["rotate", "shuffle"])
def test_raw_soa_mode_matches_encoded(golden, oracle, relabel):
    """Raw SoA mode (crdt_hip_batch_raw): every merge derives the key, the codepoint word with its
    tombstone and previous-slot flags and the compact nsq list on the device from the raw
    columns; the digests and lengths equal the encoded batch's and the golden / oracle ones, the
    encode stage runs, and leaving the mode merges the (now re-derived) encoded columns."""
    bases = [resolved(n) for n in TRACES]
    agents = crdt_hip.OpLog.synth_agents(50_000, 64, 0x5EED0007).arrays()  # (agent bits in keys)
    mixed = _mixed_logs(3)
    others = [agents] + mixed
    refs = [oracle.merge(to_anchor(lg)) for lg in others]
    c = crdt_hip.Context(0)
    for logs, check in ((bases, "golden"), (others, "oracle")):
        b = c.batch(logs, replicas=3, relabel=relabel, seed=17)
        d0, l0, _ = b.merge()
        b.set_raw(True)
        for it in range(3):
            d, l, st = b.merge()
            assert np.array_equal(d, d0) and np.array_equal(l, l0), it
            assert st["stage_launches"]["encode"] > 0 and st["stage_ns"]["encode"] > 0
        for r in range(b.docs):
            if check == "golden":
                name = TRACES[r % 4]
                assert "%016x" % d[r] == golden[name]["tree_digest"], r
                assert l[r] == golden[name]["end_bytes"], r
            else:
                ref = refs[r % len(others)]
                assert int(l[r]) == len(ref) and int(d[r]) == oracle.tree_digest(ref), r
        b.set_raw(False)
        d, l, st = b.merge()
        assert np.array_equal(d, d0) and st["stage_launches"]["encode"] == 0
        b.close()
    c.close()


def test_raw_soa_mode_rejects_fugue():
    c = crdt_hip.Context(0)
    lg = crdt_hip.Trace(trace_path("sveltecomponent")).resolve(fugue=True).arrays()
    b = c.batch([lg], replicas=2, relabel="rotate", seed=1)
    with pytest.raises(crdt_hip.CrdtHipError):
        b.set_raw(True)
    b.close()
    c.close()


def test_one_wave_uploads_back_to_back(ctx, oracle):
    """A one-wave upload is not waited for (Engine::upload): its merge runs behind the copies on
    the engine's stream, and the next upload waits for them before it rewrites the pinned staging,
    also when the staging grows and is reallocated.  Documents of different sizes, merged (text,
    then len()) back to back in an order that grows and shrinks the staging, match the oracle
    every time."""
    logs = _mixed_logs(23)
    refs = [oracle.merge(to_anchor(lg)) for lg in logs]
    order = [1, 0, 2, 0, 1, 2, 2, 0]
    for i in order:
        text, dig = ctx.merge(logs[i])
        assert text == refs[i] and dig == oracle.tree_digest(refs[i]), i
        cps, nb, dig2 = ctx.merge_len(logs[i])
        assert cps == len(refs[i].decode("utf-8")) and nb == len(refs[i]), i
        assert dig2 == oracle.tree_digest(refs[i]), i
