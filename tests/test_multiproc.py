"""Multi-rank path of bench.py on CPU: world_size 2 over gloo (127.0.0.1).

Each rank owns a shard of replicas (weak scaling: no data-path exchange), computes one digest
per document (here with the CPU oracle on small logs: the product path needs a GPU), all-gathers
the digests rank-major, and rank 0 checks every one against the golden vector with the same
helpers bench.py uses after its RCCL all-gather (`expected_digests`, `verify_gathered`,
`whole_job_rate`).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank: int, world: int, port: int, q) -> None:
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from oracle_bind import AnchorLog, Oracle
        from test_oracle import random_concurrent_log

        oracle = Oracle()
        bases = [random_concurrent_log(np.random.default_rng(s), 400 + 50 * s, 4) for s in range(4)]
        golden = [oracle.tree_digest(oracle.merge(b)) for b in bases]
        replicas = 3
        docs = replicas * len(bases)
        # this rank's shard: document r is a copy of base r % 4 (relabelling never changes text)
        local = np.array([oracle.tree_digest(oracle.merge(bases[r % 4])) for r in range(docs)],
                         np.uint64)
        gathered = [None] * world
        dist.all_gather_object(gathered, local.tolist())
        all_dig = np.array([x for part in gathered for x in part], np.uint64)
        expect = bench.expected_digests(golden, docs)
        ok = bench.verify_gathered(all_dig, expect, world)
        # a corrupted digest on the other rank must be caught
        bad = all_dig.copy()
        bad[-1] ^= np.uint64(1)
        caught = not bench.verify_gathered(bad, expect, world)
        rate = bench.whole_job_rate(1000, world, 0.5)
        dist.barrier()
        q.put((rank, ok, caught, rate))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), False, 0.0))


def test_two_rank_digest_gather_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, caught, rate in results:
        assert ok is True, (rank, ok)
        assert caught, rank
        assert rate == pytest.approx(4000.0)
