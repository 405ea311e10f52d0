"""Binary files of the merge path's inputs: the trace cache replaces
gunzip + JSON (load_testing_data, /root/reference/src/main.rs:19,52) and must load the same
TestData; the op-log file maps a resolved anchor log read-only as a zero-copy view."""
import os

import numpy as np
import pytest

import crdt_hip
from conftest import TRACES, trace_path
from oracle_bind import AnchorLog


def to_anchor(arrs) -> AnchorLog:
    a = AnchorLog(arrs.n)
    for f in ("parent", "lamport", "agent", "deleted", "cp"):
        getattr(a, f)[: arrs.n] = getattr(arrs, f)
    return a


def same_arrays(a, b) -> None:
    for f in crdt_hip.LogArrays.FIELDS:
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize("name", TRACES)
def test_trace_cache_loads_the_same_trace(tmp_path, name):
    gz = crdt_hip.Trace(trace_path(name))
    path = str(tmp_path / f"{name}.crdttrace")
    gz.save(path)
    b = crdt_hip.Trace(path)
    assert len(b) == len(gz) and b.txns == gz.txns
    assert b.start_content == gz.start_content and b.end_content == gz.end_content
    for i in list(range(0, len(gz), max(1, len(gz) // 500))) + [len(gz) - 1]:
        assert b.patch(i) == gz.patch(i)
    same_arrays(b.resolve().arrays(), gz.resolve().arrays())


def test_trace_cache_keeps_byte_offsets(tmp_path):
    t = crdt_hip.Trace(trace_path("seph-blog1"))
    t.chars_to_bytes()
    path = str(tmp_path / "s.crdttrace")
    t.save(path)
    b = crdt_hip.Trace(path)
    assert [b.patch(i) for i in range(len(b))] == [t.patch(i) for i in range(len(t))]
    with pytest.raises(crdt_hip.CrdtHipError):  # byte offsets cannot be resolved (rope.rs:16-19)
        b.resolve()


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode"])
def test_oplog_file_roundtrip_and_map(tmp_path, oracle, name, golden):
    log = crdt_hip.Trace(trace_path(name)).resolve()
    path = str(tmp_path / f"{name}.crdtlog")
    log.save(path)
    assert os.path.getsize(path) % 64 == 0
    f = crdt_hip.LogFile(path)
    same_arrays(f.arrays(), log.arrays())
    v = f.view()
    for field in ("parent", "lamport", "agent", "deleted", "cp", "origin_right"):
        assert C_addr(getattr(v, field)) % 64 == 0, field
    assert oracle.tree_digest(oracle.merge(to_anchor(f.arrays()))) == int(golden[name]["tree_digest"], 16)
    f.close()
    # an editable copy: the positional index is rebuilt, edits continue the log
    back = crdt_hip.OpLog.load(path)
    same_arrays(back.arrays(), log.arrays())
    assert back.visible_len() == log.visible_len()
    for L in (back, log):
        L.insert(7, "xyz€")
        L.remove(3, 5)
    same_arrays(back.arrays(), log.arrays())
    assert back.encode_from(0) == log.encode_from(0)


def C_addr(ptr) -> int:
    import ctypes
    return ctypes.cast(ptr, ctypes.c_void_p).value or 0


@pytest.mark.parametrize("name", ["sveltecomponent", "seph-blog1"])
def test_fugue_oplog_file_roundtrip(tmp_path, oracle, name):
    """A Fugue log's file (version 2) keeps the side column: mapped, loaded and edited on."""
    from test_fugue import to_anchor as fugue_anchor
    log = crdt_hip.Trace(trace_path(name)).resolve(fugue=True)
    path = str(tmp_path / f"{name}.fugue.crdtlog")
    log.save(path)
    assert open(path, "rb").read()[8:12] == b"\x02\0\0\0"
    f = crdt_hip.LogFile(path)
    a, b = f.arrays(), log.arrays()
    same_arrays(a, b)
    assert a.side is not None and np.array_equal(a.side, b.side) and a.side.any()
    assert C_addr(f.view().side) % 64 == 0
    f.close()
    back = crdt_hip.OpLog.load(path)
    assert np.array_equal(back.arrays().side, b.side)
    for L in (back, log):
        L.insert(11, "fugue€")
        L.remove(2, 6)
    same_arrays(back.arrays(), log.arrays())
    assert np.array_equal(back.arrays().side, log.arrays().side)
    assert back.encode_from(0) == log.encode_from(0)
    assert oracle.merge_fugue(fugue_anchor(back.arrays())) == oracle.merge_fugue(fugue_anchor(log.arrays()))
    empty = str(tmp_path / "e.fugue.crdtlog")
    crdt_hip.OpLog(fugue=True).save(empty)
    assert crdt_hip.LogFile(empty).view().side  # an empty Fugue file is still Fugue


def test_empty_log_file(tmp_path):
    path = str(tmp_path / "e.crdtlog")
    crdt_hip.OpLog().save(path)
    f = crdt_hip.LogFile(path)
    assert f.view().n == 0
    back = crdt_hip.OpLog.load(path)
    back.insert(0, "ab")
    assert back.visible_len() == 2


def test_bad_files_are_io_errors(tmp_path):
    log = crdt_hip.Trace(trace_path("sveltecomponent")).resolve()
    good = str(tmp_path / "g.crdtlog")
    log.save(good)
    raw = open(good, "rb").read()
    cases = {"missing": None, "truncated": raw[: len(raw) // 2], "magic": b"XXXX" + raw[4:],
             "short": raw[:40], "offsets": raw[:40] + b"\xff" * 8 + raw[48:]}
    for what, data in cases.items():
        p = str(tmp_path / f"{what}.crdtlog")
        if data is not None:
            open(p, "wb").write(data)
        for opener in (crdt_hip.LogFile, crdt_hip.OpLog.load):
            with pytest.raises(crdt_hip.CrdtHipError) as e:
                opener(p)
            assert e.value.code == -7, what
    t = crdt_hip.Trace(trace_path("sveltecomponent"))
    tp = str(tmp_path / "t.crdttrace")
    t.save(tp)
    traw = open(tp, "rb").read()
    for what, data in {"truncated": traw[:-3], "counts": traw[:16] + b"\xff" * 8 + traw[24:]}.items():
        p = str(tmp_path / f"{what}.crdttrace")
        open(p, "wb").write(data)
        with pytest.raises(crdt_hip.CrdtHipError) as e:
            crdt_hip.Trace(p)
        assert e.value.code == -7, what


@pytest.mark.gpu
def test_mapped_log_merges_on_device(tmp_path, golden):
    """A mapped op-log file is a view: merge and batch_create read it in place."""
    ctx = crdt_hip.Context(0)
    files = []
    for name in TRACES:
        p = str(tmp_path / f"{name}.crdtlog")
        crdt_hip.Trace(trace_path(name)).resolve().save(p)
        files.append(crdt_hip.LogFile(p))
    for name, f in zip(TRACES, files):
        text, dig = ctx.merge(f)
        assert len(text) == golden[name]["end_bytes"]
        assert dig == int(golden[name]["tree_digest"], 16)
    fp = str(tmp_path / "fugue.crdtlog")
    flog = crdt_hip.Trace(trace_path("rustcode")).resolve(fugue=True)
    flog.save(fp)
    ff = crdt_hip.LogFile(fp)
    assert ctx.merge(ff) == ctx.merge(flog)
    assert ctx.merge(ff)[1] == int(golden["rustcode"]["tree_digest"], 16)
    assert crdt_hip.Replica(ctx, ff).merge() == ctx.merge(flog)
    ff.close()
    b = ctx.batch(files, replicas=3, relabel=2, seed=5)
    digs, lens = b.merge()[:2]
    expect = [int(golden[n]["tree_digest"], 16) for n in TRACES] * 3
    assert [int(x) for x in digs] == expect
    b.close()
    ctx.close()
