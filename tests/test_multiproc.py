"""Multi-rank path of bench.py on CPU: world_size 2 over gloo (127.0.0.1).

Each rank runs bench.py's own headline rank function (`bench.traces_rank`): its replica shard
seeded by rank (`bench.shard_seed`), the barriers around the timed merges, the exchange of every
rank's counters and per-document digests, the max-over-ranks time and the digest check against
the golden vector.  Only two pieces are stand-ins, because a CPU has no HIP device: the batch
(each document merged by the CPU oracle instead of the gfx950 kernels; the text, hence the
digest, of a relabelled replica equals its base's) and the data plane of `bench.Comm` (gloo
all_gather instead of the engine's RCCL all-gather, which tests/test_gpu_merge.py runs on the
GPU).  bench.spawn_ranks, which `bench.py --gpus N` uses without torchrun, is run as well.
"""
import argparse
import os
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)


class OracleBatch:
    """A replica shard merged by the oracle (test stand-in for crdt_hip.Batch)."""

    def __init__(self, oracle, bases, replicas, seed):
        self.oracle, self.bases, self.replicas, self.seed = oracle, bases, replicas, seed
        self.docs = len(bases) * replicas
        self.items = sum(b.n for b in bases) * replicas
        self.device_bytes = 0

    def merge(self):
        dig = np.zeros(self.docs, np.uint64)
        lens = np.zeros(self.docs, np.uint64)
        for r in range(self.docs):
            text = self.oracle.merge(self.bases[r % len(self.bases)])
            dig[r] = self.oracle.tree_digest(text)
            lens[r] = len(text)
        st = {"runs": self.items, "text_bytes": int(lens.sum()), "total_ns": 1, "waves": 1,
              "stage_ns": {}, "stage_launches": {}}
        return dig, lens, st

    def close(self):
        pass


def _rank_main(rank: int, world: int, port: int, corrupt: bool, q) -> None:
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import bench
        from oracle_bind import Oracle
        from test_oracle import random_concurrent_log

        oracle = Oracle()
        bases = [random_concurrent_log(np.random.default_rng(s), 300 + 50 * s, 4) for s in range(4)]
        golden = [oracle.tree_digest(oracle.merge(b)) for b in bases]
        survivors = [len(oracle.merge(b)) for b in bases]
        inputs = {"bases": bases, "patches": [100, 200, 300, 400], "items": [b.n for b in bases],
                  "survivors": survivors, "digests": golden}
        seeds = []

        def make_batch(b, replicas, relabel, seed):
            seeds.append(seed)
            batch = OracleBatch(oracle, b, replicas, seed)
            if corrupt and rank == 1:  # a wrong digest on the other rank must fail the job
                real = batch.merge

                def bad():
                    dig, lens, st = real()
                    dig[-1] ^= np.uint64(1)
                    return dig, lens, st
                batch.merge = bad
            return batch

        comm = bench.Comm(world, rank, data_plane="gloo")
        args = argparse.Namespace(replicas=3, relabel="rotate", warmup=1, steps=2)
        res = bench.traces_rank(args, comm, make_batch, inputs)
        comm.close()
        out = None
        if rank == 0:
            out = {"digests_ok": res["digests_ok"], "value": res["value"],
                   "elapsed": res["elapsed"], "per_rank": res["per_rank"]}
        q.put((rank, seeds, out))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None))


def _run(world: int, corrupt: bool):
    import bench
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, corrupt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, seeds, out = q.get(timeout=180)
        results[rank] = (seeds, out)
    for p in procs:
        p.join(timeout=60)
    return results


def test_two_rank_headline_path_gloo():
    import bench
    results = _run(2, corrupt=False)
    for rank in (0, 1):
        seeds, _ = results[rank]
        assert isinstance(seeds, list), seeds  # an exception string otherwise
        assert seeds == [bench.shard_seed(rank)]  # every rank's shard is its own relabelling
    out = results[0][1]
    assert out["digests_ok"] is True
    assert len(out["per_rank"]) == 2
    assert all(r["ok"] == 1 and r["docs"] == 12 for r in out["per_rank"])
    # value = every rank's patches per step over the slowest rank's step time
    step = out["elapsed"] / 2
    assert out["value"] == pytest.approx(2 * 3 * 1000 / step)
    assert out["elapsed"] * 1e9 == pytest.approx(max(r["elapsed_ns"] for r in out["per_rank"]))


def test_two_rank_headline_path_catches_a_bad_digest_on_another_rank():
    results = _run(2, corrupt=True)
    assert results[0][1]["digests_ok"] is False


def test_spawn_ranks_sets_rank_environment(tmp_path):
    """bench.py --gpus N without WORLD_SIZE: N children with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*
    (rendezvous on 127.0.0.1), the first failure is the exit status."""
    import bench
    out = tmp_path / "ranks"
    out.mkdir()
    prog = ("import os,sys;d=sys.argv[1];r=os.environ['RANK'];"
            "open(os.path.join(d,r),'w').write(' '.join(os.environ[k] for k in "
            "('RANK','LOCAL_RANK','WORLD_SIZE','MASTER_ADDR')))")
    assert bench.spawn_ranks(3, [sys.executable, "-c", prog, str(out)]) == 0
    got = sorted(p.read_text() for p in out.iterdir())
    assert got == [f"{r} {r} 3 127.0.0.1" for r in range(3)]
    fail = "import os,sys;sys.exit(3 if os.environ['RANK']=='1' else 0)"
    assert bench.spawn_ranks(2, [sys.executable, "-c", fail]) == 3


def test_bench_gpus_flag_spawns_ranks_before_the_gpu(tmp_path):
    """`bench.py --gpus 2` re-launches itself as 2 ranks; each rank sees WORLD_SIZE=2.  Run with
    an engine library that does not exist, so each rank fails loudly at its first engine call
    (no GPU here): the parent must report the failure, never run the workload itself."""
    env = dict(os.environ, CRDT_HIP_LIB="libcrdt_hip_missing.so")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert " of 2" in r.stderr and "libcrdt_hip_missing.so is not built" in r.stderr, \
        r.stderr[-2000:]
