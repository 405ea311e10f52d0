"""GPU parity tests of the device-side Downstream path (crdt_hip_replica_*).

The reference's downstream bench (/root/reference/src/main.rs:63-69) clones an initial CRDT,
applies one encoded update per patch (rope.rs:210-216 encodes them, :222-224 decodes) and asks
for len().  Here the updates are decoded by the HIP kernels of replica.hip into a replica resident
in HBM and merged there.  Checked against: the trace's endContent (sha256 + tree digest from the
golden table), the host decoder (OpLog.apply_update, the sequential restatement of the same wire
format) and the CPU oracle's merge.
"""
import hashlib
import random
import struct

import numpy as np
import pytest

import crdt_hip
from conftest import TRACES, trace_path
from test_gpu_merge import to_anchor

pytestmark = pytest.mark.gpu

_UPD = {}


def trace_updates(name):
    """(patches, per-patch updates) of a trace, as Downstream::upstream_updates makes them."""
    if name not in _UPD:
        t = crdt_hip.Trace(trace_path(name))
        patches = [t.patch(i) for i in range(len(t))]
        _, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
        _UPD[name] = (t, patches, updates)
    return _UPD[name]


@pytest.mark.parametrize("name", TRACES)
def test_replica_decodes_every_trace_byte_exact(ctx, golden, name):
    t, patches, updates = trace_updates(name)
    r = crdt_hip.Replica(ctx)
    r.apply_updates(updates)
    text, dig = r.merge()
    assert hashlib.sha256(text).hexdigest() == golden[name]["sha256"]
    assert "%016x" % dig == golden[name]["tree_digest"]
    items, vis_cp, vis_b = r.info()
    assert vis_cp == len(t.end_content)       # Upstream::len in codepoints (rope.rs:16-19)
    assert vis_b == len(text)
    host = t.resolve()
    assert items == host.view().n


def test_replica_matches_host_decoder_in_random_batches(ctx, oracle):
    """Updates applied in random-sized batches, with a device clone taken midway, against the
    sequential host decoder fed the same updates one at a time."""
    t, patches, updates = trace_updates("sveltecomponent")
    rng = random.Random(7)
    r = crdt_hip.Replica(ctx)
    host = crdt_hip.OpLog()
    i, clone_at, snap = 0, len(updates) // 2, None
    while i < len(updates):
        k = rng.choice([1, 2, 3, 17, 100, 1000, 5000])
        batch = updates[i: i + k]
        r.apply_updates(batch)
        for u in batch:
            host.apply_update(u)
        i += len(batch)
        if snap is None and i >= clone_at:
            snap = (r.clone(), host.clone(), i)
    text, _ = r.merge()
    assert text.decode() == t.end_content
    assert text == oracle.merge(to_anchor(host.arrays()))
    # the clone is independent: finish it from where it was taken
    rc, hc, at = snap
    assert rc.merge()[0] == oracle.merge(to_anchor(hc.arrays()))
    rc.apply_updates(updates[at:])
    assert rc.merge()[0] == text
    assert r.merge()[0] == text


def test_replica_duplicates_are_idempotent(ctx):
    _, _, updates = trace_updates("sveltecomponent")
    r = crdt_hip.Replica(ctx)
    r.apply_updates(updates)
    ref = r.merge()
    info = r.info()
    rng = random.Random(3)
    again = rng.sample(updates, 500)
    r.apply_updates(again)                              # all known: nothing changes
    assert r.merge() == ref and r.info() == info
    r2 = crdt_hip.Replica(ctx)
    dup = []
    for u in updates:                                   # every update twice, in one batch
        dup += [u, u]
    r2.apply_updates(dup)
    assert r2.merge() == ref and r2.info() == info


def test_replica_concurrent_log_matches_oracle(ctx, oracle):
    """A 64-agent log (concurrent siblings) shipped as one update (encode_from(0))."""
    log = crdt_hip.OpLog.synth_agents(50_000, 64, 0x5EED0001)
    upd = log.encode_from(0)
    r = crdt_hip.Replica(ctx)
    r.apply_updates([upd])
    text, dig = r.merge()
    ref = oracle.merge(to_anchor(log.arrays()))
    assert text == ref
    assert (text, dig) == ctx.merge(log)


def test_replica_from_initial_log_and_empty(ctx):
    assert crdt_hip.Replica(ctx).merge()[0] == b""
    log = crdt_hip.Trace(trace_path("sveltecomponent")).resolve()
    r = crdt_hip.Replica(ctx, log)
    assert r.merge() == ctx.merge(log)
    assert r.info()[0] == log.view().n
    # a clone of a replica whose capacity is tight (uploaded, never grown) copies every slot
    # (k_rep_copy once stopped at the codepoint column's dword count, ~3/4 of the slots)
    c = r.clone()
    assert c.merge() == ctx.merge(log) and c.info() == r.info()


def _set_word(u: bytes, word: int, value: int) -> bytes:
    b = bytearray(u)
    struct.pack_into("<I", b, 4 * word, value)
    return bytes(b)


def test_replica_rejects_bad_batches_and_stays_unchanged(ctx):
    """Each malformed update is refused (EBADLOG) by the device decoder and by the host decoder
    (same condition); a refused batch leaves the replica as it was, even when it also holds
    good updates."""
    _, _, updates = trace_updates("sveltecomponent")

    def hdr(u):
        return struct.unpack_from("<6I", u, 0)  # magic, version, first, items, first_del, dels

    ins_i = next(i for i in range(1000, len(updates)) if hdr(updates[i])[3] > 0)
    del_i = next(i for i in range(1000, len(updates))
                 if hdr(updates[i])[3] == 0 and hdr(updates[i])[5] > 0)
    u, d = updates[ins_i], updates[del_i]
    first = hdr(u)[2]
    cases = [
        (ins_i, "magic", [_set_word(u, 0, 0x12345678)]),
        (ins_i, "version", [_set_word(u, 1, 99)]),
        (ins_i, "truncated", [u[:-4]]),
        (ins_i, "not ready", [_set_word(u, 2, first + 5)]),
        (ins_i, "first zero", [_set_word(u, 2, 0)]),
        (ins_i, "unknown parent", [_set_word(u, 6, first + 3)]),   # parent >= own id
        (del_i, "unknown delete", [_set_word(d, 6, 10 ** 9)]),     # items 0: dels at word 6
        (del_i, "delete id zero", [_set_word(d, 6, 0)]),
        (ins_i, "good then bad", [u, _set_word(updates[ins_i + 1], 0, 0)]),
    ]
    hosts = {}
    for i, what, batch in cases:
        r = crdt_hip.Replica(ctx)
        r.apply_updates(updates[:i])
        ref, info = r.merge(), r.info()
        with pytest.raises(crdt_hip.CrdtHipError) as e:
            r.apply_updates(batch)
        assert e.value.code == -5, what
        assert r.merge() == ref and r.info() == info, what
        if i not in hosts:
            hosts[i] = crdt_hip.OpLog()
            for x in updates[:i]:
                hosts[i].apply_update(x)
        host = hosts[i].clone()
        with pytest.raises(crdt_hip.CrdtHipError):
            for x in batch:
                host.apply_update(x)
        r.apply_updates([updates[i]])   # the good update still applies afterwards
        assert r.info()[0] >= info[0]
    # misaligned / out-of-range offsets
    r = crdt_hip.Replica(ctx)
    r.apply_updates(updates[:ins_i])
    ref = r.merge()
    buf, offs = crdt_hip.pack_updates([u])
    with pytest.raises(crdt_hip.CrdtHipError):
        r.apply_packed(np.concatenate([np.zeros(2, np.uint8), buf]), offs + 2)
    with pytest.raises(crdt_hip.CrdtHipError):
        r.apply_packed(buf, np.array([0, buf.size + 4], np.uint64))
    assert r.merge() == ref


def test_gap_in_deletes_host_rejects_device_accepts(ctx):
    """A delete-only update that arrives before the delete update preceding it.  The host log
    keeps the delete ops in order (encode_from re-sends them by index), so it refuses an update
    whose first delete index lies beyond the ones it holds ("missing deletes").  The device
    replica keeps no delete-op log, only tombstone bits: tombstoning a known item is state-based
    and order-free, so it accepts the update.  Once both have every update, the documents agree
    (documented divergence, crdt_hip.h crdt_hip_replica_apply)."""
    _, _, updates = trace_updates("sveltecomponent")

    def hdr(u):
        return struct.unpack_from("<6I", u, 0)

    i = next(i for i in range(1000, len(updates) - 1)
             if hdr(updates[i])[3] == 0 and hdr(updates[i])[5] > 0
             and hdr(updates[i + 1])[3] == 0 and hdr(updates[i + 1])[5] > 0)
    d1, d2 = updates[i], updates[i + 1]
    host = crdt_hip.OpLog()
    for x in updates[:i]:
        host.apply_update(x)
    with pytest.raises(crdt_hip.CrdtHipError):
        host.apply_update(d2)                 # first_del beyond the deletes it holds
    r = crdt_hip.Replica(ctx)
    r.apply_updates(updates[:i])
    r.apply_updates([d2])                     # accepted: its targets are known items
    r.apply_updates([d1])
    host.apply_update(d1)
    host.apply_update(d2)
    assert r.merge() == ctx.merge(host)
    assert r.info()[1] == host.arrays().deleted.size - int(host.arrays().deleted.sum())


def test_downstream_device_bench_loop(golden):
    """The reference's downstream closure (main.rs:63-69) with the device replica:
    clone the initial CRDT, apply every update, len() == endContent length."""
    name = "seph-blog1"
    t, patches, updates = trace_updates(name)
    crdt0 = crdt_hip.HipDownstream(crdt_hip.Replica(crdt_hip.HipMerge.context()))
    for _ in range(2):
        crdt = crdt0.clone()
        for u in updates:
            crdt.apply_update(u)
        assert crdt.len() == len(t.end_content)         # main.rs:68 (codepoints here)
        assert hashlib.sha256(crdt.text().encode()).hexdigest() == golden[name]["sha256"]


@pytest.mark.parametrize("name", TRACES)
def test_resident_update_batch_matches_host_batch(ctx, golden, name):
    """crdt_hip_replica_apply_resident: the update vector uploaded once, applied to fresh clones
    (main.rs:64-67 with the updates in HBM) gives the same replica as the host-buffer path."""
    t, patches, updates = trace_updates(name)
    buf, offs = crdt_hip.pack_updates(updates)
    ub = crdt_hip.UpdateBatch(ctx, buf, offs)
    init = crdt_hip.Replica(ctx)
    via_host = init.clone()
    via_host.apply_packed(buf, offs)
    for _ in range(2):  # the batch is reusable
        r = init.clone()
        r.apply_resident(ub)
        assert r.info() == via_host.info()
        n, dig = r.merge_digest()
        assert (n, "%016x" % dig) == (golden[name]["end_bytes"], golden[name]["tree_digest"])
        r.close()
    # applying it again is a no-op (every id already known)
    via_host.apply_resident(ub)
    assert via_host.merge_digest()[0] == golden[name]["end_bytes"]
    ub.close()


def test_resident_update_batch_rejects_bad_updates(ctx):
    t, patches, updates = trace_updates("sveltecomponent")
    buf, offs = crdt_hip.pack_updates(updates[1:50])  # update 0 missing: not causally ready
    ub = crdt_hip.UpdateBatch(ctx, buf, offs)
    r = crdt_hip.Replica(ctx)
    with pytest.raises(crdt_hip.CrdtHipError) as e:
        r.apply_resident(ub)
    assert e.value.code == -5 and r.info()[0] == 0
    ub.close()


@pytest.mark.parametrize("nsq", [2, 0])
@pytest.mark.parametrize("name", TRACES)
def test_replay_closure_matches_golden(ctx, golden, py_trace, name, nsq):
    """crdt_hip_replica_replay: the downstream closure (main.rs:63-69) in one call.  The first
    call learns the sizes, later ones merge right behind the decode (speculated sizes checked on
    the device); every call must give the trace's document, and init must stay unchanged.  With
    nsq_list 2 every merge rebuilds the replica's compact list of the non-seq items from the
    decoded contents (inside the captured closure; the default does so from 2^22 slots up), with
    0 level 0 gathers them."""
    ctx.set_param("nsq_list", nsq)
    try:
        _replay_closure(ctx, golden, py_trace, name)
    finally:
        ctx.set_param("nsq_list", 1)


def _replay_closure(ctx, golden, py_trace, name):
    t = crdt_hip.Trace(trace_path(name))
    patches = [t.patch(i) for i in range(len(t))]
    up, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
    init = crdt_hip.Replica(ctx, up.log if up.log.view().n else None)
    ub = crdt_hip.UpdateBatch(ctx, *crdt_hip.pack_updates(updates))
    end = py_trace(name).end_content
    want = (len(end), len(end.encode()), int(golden[name]["tree_digest"], 16))
    before = init.info()
    for _ in range(4):
        assert init.replay(ub) == want
    assert init.info() == before
    # the same closure as three calls agrees
    r = init.clone()
    r.apply_resident(ub)
    assert r.merge_len() == want
    r.close()
    ub.close()
    init.close()


@pytest.mark.parametrize("mode", [2, 1, 0])
def test_replica_merges_follow_the_contraction_knob(ctx, golden, py_trace, mode):
    """Replica merges (merge_len, the replay closure, the incremental state's full merge) honour
    "contraction": 2 merges without run contraction (every item its own run), 0 and 1 contract.
    Switching the knob between replays recaptures the closure (the graph key holds it); every
    result is the trace's document."""
    name = "sveltecomponent"
    t = crdt_hip.Trace(trace_path(name))
    patches = [t.patch(i) for i in range(len(t))]
    up, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
    end = py_trace(name).end_content
    want = (len(end), len(end.encode()), int(golden[name]["tree_digest"], 16))
    init = crdt_hip.Replica(ctx)
    ub = crdt_hip.UpdateBatch(ctx, *crdt_hip.pack_updates(updates))
    try:
        assert init.replay(ub) == want
        ctx.set_param("contraction", mode)
        for _ in range(3):
            assert init.replay(ub) == want
        r = init.clone()
        r.apply_resident(ub)
        assert r.merge_len() == want
        cps, nb, path, text = r.merge_inc(text=True)
        assert path == 0 and text.decode() == end
        r.close()
    finally:
        ctx.set_param("contraction", 0)
        ub.close()
        init.close()


def test_replay_falls_back_when_sizes_change(ctx, golden):
    """Speculated sizes that no longer hold (forced with the plan_shrink hook) are caught by the
    device check and the closure is merged again with the real ones; a changed init starts over."""
    name = "sveltecomponent"
    t = crdt_hip.Trace(trace_path(name))
    patches = [t.patch(i) for i in range(len(t))]
    up, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
    init = crdt_hip.Replica(ctx, None)
    half = len(updates) // 2
    ub = crdt_hip.UpdateBatch(ctx, *crdt_hip.pack_updates(updates))
    want = init.replay(ub)
    assert want[1] == golden[name]["end_bytes"]
    ctx.set_param("plan_shrink", 1)
    try:
        assert init.replay(ub) == want
    finally:
        ctx.set_param("plan_shrink", 0)
    assert init.replay(ub) == want
    # init receives the first half itself: the learnt sizes no longer apply, the result is the same
    init.apply_updates(updates[:half])
    assert init.replay(ub) == want
    assert init.replay(ub) == want
    ub.close()
    init.close()


def test_replay_rejects_a_bad_batch_and_keeps_init(ctx):
    log = crdt_hip.OpLog()
    log.insert(0, "hello")
    v0 = log.version()
    log.insert(5, " world")
    good = log.encode_from(v0)
    init = crdt_hip.Replica(ctx, None)
    bad = bytearray(good)
    bad[8:12] = (50).to_bytes(4, "little")  # first id far beyond the replica: not causally ready
    ub = crdt_hip.UpdateBatch(ctx, *crdt_hip.pack_updates([bytes(bad)]))
    with pytest.raises(crdt_hip.CrdtHipError) as e:
        init.replay(ub)
    assert e.value.code == -5
    assert init.info() == (0, 0, 0)
    ub.close()
    init.close()
