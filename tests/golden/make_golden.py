#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (pure Python, no native code).

Pinning data (the reference's own fixtures): each trace's `endContent` is the text the
reference's length assert compares against (/root/reference/src/main.rs:35,68).  This script:
  1. replays every trace with naive str splicing (codepoint positions, remove-then-insert as in
     /root/reference/src/rope.rs:21-32) and asserts the result == endContent;
  2. records per-trace facts (patches, txns, items, tombstones, bytes, sha256, xxh64 and the
     4 KiB-leaf tree digest of endContent) into traces.json;
  3. resolves sveltecomponent into an anchor op log with a small pure-Python resolver (a third,
     independent restatement of the RGA anchor conventions), checks that a
     pure-Python RGA pre-order merge reproduces endContent, and stores the log as
     sveltecomponent_anchor.npz (allow_pickle-free arrays);
  4. writes concurrent.json: small hand-built multi-agent logs with their expected documents
     (RGA: siblings by (lamport, agent) descending).  Concurrent order is "parity unpinned":
     no reference test covers it; the expected strings follow the documented rule.

Run:  python tests/golden/make_golden.py   (about 10 s)
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import sys

import numpy as np
import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
TRACES = ["automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"]
LEAF = 4096


GROUP = 4096  # leaf digests per group (documents above 16 MiB hash their leaves in groups)


def tree_digest(b: bytes) -> int:
    leaves = b"".join(xxhash.xxh64(b[i:i + LEAF]).intdigest().to_bytes(8, "little")
                      for i in range(0, len(b), LEAF))
    if len(leaves) > 8 * GROUP:
        leaves = b"".join(xxhash.xxh64(leaves[o:o + 8 * GROUP], seed=k).intdigest().to_bytes(8, "little")
                          for k, o in enumerate(range(0, len(leaves), 8 * GROUP)))
    return xxhash.xxh64(leaves, seed=len(b)).intdigest()


def load(name):
    with gzip.open(os.path.join(ROOT, "traces", f"{name}.json.gz"), "rb") as f:
        return json.loads(f.read())


def replay(d) -> str:
    parts = list(d["startContent"])
    s = "".join(parts)
    for txn in d["txns"]:
        for pos, dele, ins in txn["patches"]:
            s = s[:pos] + ins + s[pos + dele:]
    return s


def resolve_py(d):
    """Pure-Python resolver: a list of item ids in document order (tombstones kept)."""
    seq = []          # ids in document order
    dead = [True]     # dead[0]: the start sentinel
    parent, lamport, cps = [], [], []
    deleted = []

    def nth_visible_index(p):  # index in seq of the p-th visible item (p >= 1)
        c = 0
        for i, x in enumerate(seq):
            if not dead[x]:
                c += 1
                if c == p:
                    return i
        raise ValueError("position out of range")

    def insert(pos, text):
        at = 0 if pos == 0 else nth_visible_index(pos) + 1
        left = 0 if pos == 0 else seq[at - 1]
        new = []
        for ch in text:
            nid = len(parent) + 1
            parent.append(left)
            lamport.append(nid)
            cps.append(ord(ch))
            deleted.append(0)
            dead.append(False)
            new.append(nid)
            left = nid
        seq[at:at] = new

    def remove(pos, n):
        i = nth_visible_index(pos + 1)
        while n:
            x = seq[i]
            if not dead[x]:
                dead[x] = True
                deleted[x - 1] = 1
                n -= 1
            i += 1

    if d["startContent"]:
        insert(0, d["startContent"])
    for txn in d["txns"]:
        for pos, dele, ins in txn["patches"]:
            if dele:
                remove(pos, dele)
            if ins:
                insert(pos, ins)
    return (np.array(parent, np.uint32), np.array(lamport, np.uint32),
            np.zeros(len(parent), np.uint16), np.array(deleted, np.uint8),
            np.array(cps, np.uint32))


def merge_py(parent, lamport, agent, deleted, cp) -> str:
    n = len(parent)
    kids = [[] for _ in range(n + 1)]
    for i in range(1, n + 1):
        kids[int(parent[i - 1])].append(i)
    for k in kids:
        k.sort(key=lambda x: (int(lamport[x - 1]), int(agent[x - 1])))  # ascending; stack pops newest
    out, stack = [], [0]
    while stack:
        v = stack.pop()
        if v and not deleted[v - 1]:
            out.append(chr(int(cp[v - 1])))
        stack.extend(kids[v])
    return "".join(out)


def concurrent_cases():
    """Hand-built multi-agent logs; expected text by the RGA rule (newest sibling first)."""
    cases = []
    # two agents insert concurrently at the document start with equal lamport: agent 1 first
    cases.append(dict(name="tie_on_lamport", parent=[0, 0], lamport=[1, 1], agent=[0, 1],
                      deleted=[0, 0], cp=[ord("a"), ord("b")], expected="ba"))
    # "ab" typed by agent 0; agents 1 and 2 concurrently insert after 'a' (lamport 3)
    cases.append(dict(name="concurrent_after_a", parent=[0, 1, 1, 1], lamport=[1, 2, 3, 3],
                      agent=[0, 0, 1, 2], deleted=[0, 0, 0, 0],
                      cp=[ord(c) for c in "abXY"], expected="aYXb"))
    # a run chained under a concurrent sibling keeps its subtree contiguous
    cases.append(dict(name="subtree_contiguous", parent=[0, 1, 1, 3, 4], lamport=[1, 2, 2, 3, 4],
                      agent=[0, 0, 1, 1, 1], deleted=[0, 0, 0, 0, 0],
                      cp=[ord(c) for c in "aBxyz"], expected="axyzB"))
    # tombstoned anchor still orders its children
    cases.append(dict(name="tombstone_anchor", parent=[0, 1, 1], lamport=[1, 2, 3],
                      agent=[0, 0, 0], deleted=[1, 0, 0], cp=[ord(c) for c in "abc"],
                      expected="cb"))
    # multi-byte codepoints
    cases.append(dict(name="utf8", parent=[0, 1, 2, 3], lamport=[1, 2, 3, 4], agent=[0, 0, 0, 0],
                      deleted=[0, 0, 1, 0], cp=[0xE9, 0x4E2D, 0x41, 0x1F600],
                      expected="é中\U0001F600"))
    for c in cases:
        got = merge_py(c["parent"], c["lamport"], c["agent"], c["deleted"], c["cp"])
        assert got == c["expected"], (c["name"], got)
    return cases


def main() -> int:
    facts = {}
    for name in TRACES:
        d = load(name)
        end = d["endContent"]
        got = replay(d)
        assert got == end, f"{name}: naive replay != endContent"
        patches = sum(len(t["patches"]) for t in d["txns"])
        items = len(d["startContent"]) + sum(len(p[2]) for t in d["txns"] for p in t["patches"])
        dels = sum(p[1] for t in d["txns"] for p in t["patches"])
        eb = end.encode("utf-8")
        facts[name] = dict(
            patches=patches, txns=len(d["txns"]), items=items, tombstones=dels,
            end_bytes=len(eb), end_chars=len(end), sha256=hashlib.sha256(eb).hexdigest(),
            xxh64="%016x" % xxhash.xxh64(eb).intdigest(),
            tree_digest="%016x" % tree_digest(eb),
        )
        print(name, facts[name])
    with open(os.path.join(HERE, "traces.json"), "w") as f:
        json.dump(facts, f, indent=1, sort_keys=True)

    d = load("sveltecomponent")
    parent, lamport, agent, deleted, cp = resolve_py(d)
    assert merge_py(parent, lamport, agent, deleted, cp) == d["endContent"]
    np.savez_compressed(os.path.join(HERE, "sveltecomponent_anchor.npz"), parent=parent,
                        lamport=lamport, agent=agent, deleted=deleted, cp=cp)
    with open(os.path.join(HERE, "concurrent.json"), "w") as f:
        json.dump(concurrent_cases(), f, indent=1)
    print("ok")
    return 0


if __name__ == "__main__":
    sys.exit(main())
