#!/usr/bin/env python3
"""Headline benchmark: batched trace merge on MI355X.

A "step" = one merge pass of the hot path over every document resident on the GPU: the four
josephg traces (automerge-paper, rustcode, sveltecomponent, seph-blog1), resolved once on the
host into anchor op logs (untimed, like the reference's load at main.rs:19), materialised as
`--replicas` independent relabelled HBM copies each (4 x 4096 = 16,384 documents, 4.14 G items
per GPU by default), merged by the gfx950 kernels to per-document text + digest.

value = patches merged per second, whole job: sum over ranks of the patches each rank merged per
step / max-over-ranks step time; the reference's accounting unit is criterion's
Throughput::Elements(trace.len()) = patches (/root/reference/src/main.rs:25,58).

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) this process is one rank; with
`--gpus N` and no WORLD_SIZE it starts N rank processes itself (before any GPU call) and exits
with their status.  Replicas shard with no data-path collective (weak scaling).  After timing,
every rank's counters (patches, items, runs, text bytes, elapsed and device ns, digest check)
and its per-document digests are all-gathered over RCCL through the engine's C ABI
(crdt_hip_allgather_u64); rank 0 takes the max elapsed time and checks every digest against the
golden digest of the trace's endContent.  torch.distributed (gloo) is the control plane only:
the barriers around the timed region and the RCCL unique-id broadcast.

cpu_baseline (rank 0 of an N=1 run only): the oracle's sequential RGA merge (oracle/oracle.c
orc_merge_many), one document per thread over every CPU this process may run on, on a bounded
sample of the same documents.  config1 (likewise): the oracle's positional replay (orc_replay,
one core) of automerge-paper, timed like the reference's upstream closure (main.rs:28-36),
beside the engine's own upstream path (host resolve + device merge of the same trace).
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "crdt-benches_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

crdt_hip = None  # the engine binding, imported once this process knows it is a rank

TRACES = ["automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"]
# (experiments only: CRDT_BENCH_TRACES=a,b restricts the batch to those traces; bench lines
# use all four)
if os.environ.get("CRDT_BENCH_TRACES"):
    TRACES = [t for t in TRACES if t in os.environ["CRDT_BENCH_TRACES"].split(",")]
METRIC = "merged CRDT ops/sec (whole node) + achieved HBM GB/s, batched trace merge"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Minimum HBM traffic of the design (the §8(d) contract restated for the
# run-contraction pipeline over the device op-log format): every slot's 3-byte codepoint word
# (codepoint, tombstone, previous-slot flag) read once, the (lamport, agent) of every run head
# read once, the merged text written once.  (The parents of the non-seq items, 4 B each, are
# not counted: their number is not reported per step; they are ~4 % of the items.)
MIN_B_PER_SLOT = 3.0
MIN_B_PER_RUN = 6.0
MIN_B_PER_TEXT = 1.0
# Per-kernel algorithmic bytes: each kernel's declared inputs read once +
# outputs written once, as (bytes per item slot, bytes per run, bytes per visible UTF-8 byte).
KERNEL_BYTES = {
    # 3-byte cp|flags in; nsq + visible bits, jump bits, the escape word (1/128 B) out (weight
    # nibbles only for 16-slot groups with a visible multi-byte character: ~0 on the traces);
    # parents of the nsq items read + listed (counted per run); tile UTF-8 (stile) out
    "classify": (3.3828125, 8.0, 1.0),
    # head stage (k_heads: nsq, visible and jump bits in, head records out) and k_runs (head
    # records, visible and nsq bits in); per run: key + parent slot + rank lookup in, record
    # row out; the tile text moved to sbytes only when a later kernel reads it there (k_expand,
    # or stile_text 0): k_doctree's default staging reads the stile segments themselves
    "runs": (1.125, 38.0, 2.0),
    # global level 1, sibling groups by counting: parent in + child count (count), placement
    # (place), keys and links (link); the radix form is priced in level1_run_bytes below
    "count": (0.0, 4.0, 0.0),
    "scan": (0.0, 0.0, 0.0),
    "place": (0.0, 32.0, 0.0),
    "link": (0.0, 28.0, 0.0),
    "sortb": (0.0, 0.0, 0.0),
    "walk1": (0.0, 24.0, 0.0),       # the run record in; its sublist offset and sublist out
    "rank": (0.0, 0.5, 0.0),
    "walk2": (0.0, 0.0, 0.0),        # k_doctotals alone (per document; text mode: below)
    # run prefix/weight/head/offset (global level 1: {offset in sublist, sublist} + the sublist's
    # prefix, 20 B); slot-order text -> document
    "expand": (0.0, 16.0, 2.0),
    "digest": (0.0, 0.0, 1.0),
    "doctree": (0.0, 20.0, 2.0),     # parent run, weight, key in; slot-order text in, document out
    # k_tscatter (after k_doctree in scatter mode, which then moves no text and writes the run's
    # place, 4 B, inside its 20 B/run): per tile its {rows, weight} prefix (8 B per 4096 slots),
    # per run its weight prefix and place in, the tiles' text in and the documents out
    "text": (8.0 / 4096, 8.0, 2.0),
}


def level1_run_bytes(k: str, per_wave: dict, text_mode: bool):
    """Bytes per run of a global level-1 stage in its radix form, or None for the
    counting form (KERNEL_BYTES).  per_wave: the stage launches per wave (passes)."""
    if k == "count":      # k_rs_hist: parent in
        return 4.0
    if k == "place":      # sort A: first pass parent + key in, 16-B element out; then 16 in + 16 out
        return 28.0 + 32.0 * (per_wave["place"] - 1)
    if k == "link":       # k_rs_order: element in, pair + first child out
        return 28.0
    if k == "sortb":      # sort B passes (8 + 8), k_rs_place (8 in, 4 out), k_rs_records (16 in,
        #                   16 out; text mode: the second 16-B line and the run's bytes)
        return 16.0 * (per_wave["sortb"] - 2) + 12.0 + 32.0 + (17.0 if text_mode else 0.0)
    return None


STAGE_KERNEL = {"classify": "k_classify", "runs": "k_runs",
                "doctree": "k_doctree", "expand": "k_expand", "digest": "k_leafhash",
                "text": "k_tscatter"}
# HBM bytes per item of each kernel from rocprofv3 PMC passes of this build (FETCH_SIZE x2 for
# gfx950 wide reads + WRITE_SIZE, one pass each: tools/profile.sh + tools/pmc_summary.py).
PMC_FILE = "profiles/pmc_per_item.json"
# per-rank counters exchanged after timing (u64 each)
COUNTERS = ["patches", "items", "runs", "text_bytes", "docs", "elapsed_ns", "device_ns", "ok"]


# kernels whose PMC traffic makes up a stage's (the stage clock times them together, and the
# stage's algorithmic bytes in KERNEL_BYTES cover all of them)
STAGE_PMC_KERNELS = {
    "classify": ["k_clear", "k_classify"],
    "runs": ["k_heads", "k_tiles_reduce", "k_tiles_top", "k_tiles_apply", "k_runs", "k_docmax"],
    "doctree": ["k_doctotals", "k_doctree"],
    "digest": ["k_leafhash", "k_docdigest"],
}


def measured_traffic(stage: str, items_per_launch: float):
    """PMC-measured HBM bytes of one launch of the stage's kernels, or None."""
    try:
        with open(os.path.join(ROOT, PMC_FILE)) as f:
            ks = json.load(f)["kernels"]
        names = STAGE_PMC_KERNELS.get(stage, [STAGE_KERNEL[stage]])
        return sum(ks[n]["fetch_x2_per_item"] + ks[n]["write_per_item"] for n in names) * items_per_launch
    except (OSError, KeyError, ValueError):
        return None


def expected_digests(golden_dig, docs: int) -> np.ndarray:
    """Document r of a replica batch is a copy of trace r % 4."""
    return np.array([golden_dig[d % len(golden_dig)] for d in range(docs)], np.uint64)


def verify_gathered(all_dig: np.ndarray, expect: np.ndarray, world: int) -> bool:
    """Rank-major all-gathered digests: every rank's shard must equal the golden vector."""
    return bool(np.array_equal(np.asarray(all_dig, np.uint64), np.tile(expect, world)))


def whole_job_rate(units_per_rank: int, world: int, step_seconds: float) -> float:
    """Weak scaling: every rank processes its own shard; value = all units / max-rank time."""
    return units_per_rank * world / step_seconds


def shard_seed(rank: int) -> int:
    """Relabel seed of a rank's replica shard: every rank's HBM copies differ."""
    return 0x5EED0003 + 7919 * rank


def log(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------------------------
# ranks and communication
# ---------------------------------------------------------------------------------------------
def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list, env_extra: dict | None = None) -> int:
    """Start n rank processes of `argv` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, rendezvous on
    127.0.0.1) and wait for them; the first failure stops the others.  Called before this
    process touches the GPU, so only the children do."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update(env_extra or {})
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            st = p.poll()
            if st is None:
                continue
            live.remove(p)
            if st != 0 and rc == 0:
                rc = st
                for q in live:  # the exact children this call started
                    q.terminate()
        time.sleep(0.05)
    return rc


@contextlib.contextmanager
def native_stdout_to_stderr():
    """RCCL writes a version banner to stdout at communicator init; the bench's stdout is one
    JSON line, so native writes go to stderr while the engine's communicator is set up."""
    sys.stdout.flush()
    libc = ctypes.CDLL(None)
    libc.fflush(None)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


class Comm:
    """Control plane over torch.distributed (gloo: barriers, the RCCL unique-id broadcast) and
    the data collective over RCCL through the engine's C ABI (crdt_hip_comm_init /
    crdt_hip_allgather_u64).  With world 1 every call is local."""

    def __init__(self, world: int, rank: int, ctx=None, data_plane: str = "rccl"):
        self.world, self.rank, self.ctx, self.dist = world, rank, ctx, None
        self.data_plane = data_plane
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=rank, world_size=world)
            self.dist = dist
            if data_plane == "rccl":
                uid = [crdt_hip.Context.comm_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                with native_stdout_to_stderr():
                    ctx.comm_init(world, rank, uid[0])
        elif data_plane == "rccl" and ctx is not None:
            with native_stdout_to_stderr():
                ctx.comm_init(1, 0, crdt_hip.Context.comm_unique_id())

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def allgather_u64(self, values) -> np.ndarray:
        v = np.ascontiguousarray(values, dtype=np.uint64)
        if self.data_plane == "rccl":
            with native_stdout_to_stderr():
                return self.ctx.allgather_u64(v, self.world)
        if self.dist is None:
            return v.copy()
        import torch
        t = torch.from_numpy(v.view(np.int64).copy())
        parts = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return np.concatenate([p.numpy().view(np.uint64) for p in parts])

    def close(self) -> None:
        if self.dist is not None:
            self.dist.destroy_process_group()


def rank_env() -> tuple:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


# ---------------------------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------------------------
def load_bases(fugue: bool = False):
    """Resolve the four traces on the host (untimed setup, like the reference's load at
    main.rs:19): anchor logs + per-trace patches, items, end bytes, golden digest, resolve ms.
    `fugue`: Fugue anchors (left/right children, in-order document; same endContent)."""
    with open(os.path.join(ROOT, "tests", "golden", "traces.json")) as f:
        golden = json.load(f)
    bases, patches, items, survivors, digests, resolve_ms = [], [], [], [], [], []
    traces = [crdt_hip.Trace(os.path.join(ROOT, "traces", f"{name}.json.gz")) for name in TRACES]
    for name, t in zip(TRACES, traces):
        t0 = time.perf_counter()
        lg = t.resolve(fugue=fugue)
        resolve_ms.append((time.perf_counter() - t0) * 1e3)
        bases.append(lg.arrays())
        patches.append(len(t))
        items.append(bases[-1].n)
        survivors.append(golden[name]["end_bytes"])
        digests.append(int(golden[name]["tree_digest"], 16))
    # the same four documents resolved at once, one host thread each (crdt_hip_trace_resolve_many)
    t0 = time.perf_counter()
    crdt_hip.Trace.resolve_many(traces, len(traces))
    parallel_ms = (time.perf_counter() - t0) * 1e3
    return {"bases": bases, "patches": patches, "items": items, "survivors": survivors,
            "digests": digests, "resolve_ms": resolve_ms, "resolve_parallel_ms": parallel_ms}


def host_cpus() -> dict:
    """CPUs this process can actually use: the affinity mask (what hardware_concurrency honours)
    capped by the cgroup CPU quota (cpu.max; on the pool's boxes the mask shows the whole
    machine's 256 CPUs and the quota is 16).  `threads` = min(affinity, floor(quota)): more
    threads than the quota only time-slice the same CPUs."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                quota = round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    eff = n if quota is None else max(1, min(n, int(quota)))
    return {"threads": eff, "affinity_cpus": n, "cgroup_cpu_quota": quota}


def cpu_baseline(bases, patches, seconds: float, threads: int) -> dict:
    """Oracle RGA merge (orc_merge_many) over a bounded sample: rounds of `threads` x 4 docs."""
    from oracle_bind import AnchorLog, Oracle

    oracle = Oracle()
    logs = []
    for b in bases:
        a = AnchorLog(b.n)
        for f in ("parent", "lamport", "agent", "deleted", "cp"):
            getattr(a, f)[: b.n] = getattr(b, f)
        logs.append(a)
    batch = logs * threads
    per_round = sum(patches) * threads
    done, t0 = 0, time.perf_counter()
    rounds = 0
    while True:
        oracle.merge_many(batch, threads)
        rounds += 1
        done += per_round
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    cpus = host_cpus()
    return {"value": done / el, "unit": "patches/s", "cores": threads, "kind": "port",
            "affinity_cpus": cpus["affinity_cpus"], "cgroup_cpu_quota": cpus["cgroup_cpu_quota"],
            "sample": f"{rounds} rounds x {len(batch)} documents ({threads} copies of the 4 "
                      f"resolved traces), {el:.1f} s, oracle/oracle.c orc_merge_rga, one "
                      "document per thread, threads = min(affinity mask, cgroup CPU quota)"}


def config1(ctx, seconds: float) -> dict:
    """automerge-paper replayed from scratch per iteration, the reference's
    upstream closure (main.rs:28-36).  CPU: the oracle's positional replay (orc_replay, gap
    buffer, one core).  Engine: the native upstream loop (crdt_hip_trace_resolve: from_str +
    replace per patch) then len() = the device merge (crdt_hip_merge, PCIe included)."""
    from oracle_bind import Oracle, load_trace

    name = "automerge-paper"
    oracle = Oracle()
    td = load_trace(name)
    end = td.end_content.encode()
    n, t0 = 0, time.perf_counter()
    while True:
        out = oracle.replay(td)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    assert out == end, "oracle replay differs from endContent"
    cpu = {"value": len(td) * n / el, "unit": "patches/s", "cores": 1, "kind": "port",
           "sample": f"{n} replays of {name} ({len(td)} patches), {el:.1f} s, "
                     "oracle/oracle.c orc_replay"}
    t = crdt_hip.Trace(os.path.join(ROOT, "traces", f"{name}.json.gz"))
    with open(os.path.join(ROOT, "tests", "golden", "traces.json")) as f:
        want_dig = int(json.load(f)[name]["tree_digest"], 16)
    n_chars = len(td.end_content)
    res_s = mer_s = drop_s = 0.0
    k = 0
    ok = True
    while k < 3 or res_s + mer_s + drop_s < min(seconds, 3.0):
        a = time.perf_counter()
        lg = t.resolve()
        b = time.perf_counter()
        # r.len() (main.rs:35): the merged document's codepoints, counted on the device; the
        # digest of the merged text checks its bytes against endContent's
        cps, _, dig = ctx.merge_len(lg)
        c = time.perf_counter()
        # the log dropped inside the iteration, as the closure drops its rope (main.rs:27-36)
        del lg
        d = time.perf_counter()
        ok &= cps == n_chars and dig == want_dig
        res_s += b - a
        mer_s += c - b
        drop_s += d - c
        k += 1
    text, _ = ctx.merge(t.resolve())  # (once, outside the timing: the bytes themselves)
    ok &= text == end
    eng = {"value": len(t) * k / (res_s + mer_s + drop_s), "unit": "patches/s", "iterations": k,
           "resolve_ms": res_s / k * 1e3, "merge_ms": mer_s / k * 1e3,
           "drop_ms": drop_s / k * 1e3, "text_ok": bool(ok),
           "note": "host resolve (one core) + len() as a one-document device merge (upload of "
                   "the op log included; codepoints and digest back, as main.rs:35 asserts "
                   "len()) + the log dropped, as the closure drops its rope; the text itself "
                   "checked once outside the timing"}
    return {"trace": name, "patches": len(td), "cpu_replay": cpu, "engine_upstream": eng}


# ---------------------------------------------------------------------------------------------
# config 3: the headline
# ---------------------------------------------------------------------------------------------
def merge_steps(batch, comm, warmup: int, steps: int, on_warmup=None):
    for i in range(warmup):
        st = batch.merge()[2]
        if on_warmup:
            on_warmup(i, st)
    comm.barrier()
    t0 = time.perf_counter()
    stats = []
    for _ in range(steps):
        dig, lens, st = batch.merge()  # synchronous: returns after the device finished
        stats.append(st)
    comm.barrier()
    return dig, lens, stats, time.perf_counter() - t0


def traces_rank(args, comm, make_batch, inputs) -> dict | None:
    """One rank of the headline: its replica shard (seeded by rank), the timed merges, the counter
    and digest exchange, the whole-job figures.  Returns rank 0's result (None elsewhere)."""
    world, rank = comm.world, comm.rank
    t_enc = time.perf_counter()
    batch = make_batch(inputs["bases"], args.replicas, args.relabel, shard_seed(rank))
    enc_s = time.perf_counter() - t_enc  # (synchronous: upload + device encoding of every replica)
    if rank == 0:
        log(f"[bench] rank0: {batch.docs} docs, {batch.items} items, "
            f"{batch.device_bytes / 1e9:.1f} GB resident")

    def on_warmup(i, st):
        if rank == 0:
            log(f"[bench] warmup {i}: device {st['total_ns'] / 1e6:.1f} ms")

    dig, lens, stats, elapsed = merge_steps(batch, comm, args.warmup, args.steps, on_warmup)
    expect = expected_digests(inputs["digests"], batch.docs)
    surv = np.array([inputs["survivors"][d % len(TRACES)] for d in range(batch.docs)], np.uint64)
    ok_local = bool(np.array_equal(dig, expect)) and bool(np.array_equal(lens, surv))
    patches_rank = sum(inputs["patches"]) * args.replicas
    cnt = np.array([patches_rank, batch.items, stats[0]["runs"], stats[0]["text_bytes"],
                    batch.docs, int(elapsed * 1e9),
                    int(np.mean([s["total_ns"] for s in stats])), int(ok_local)], np.uint64)
    allc = comm.allgather_u64(cnt).reshape(world, len(COUNTERS))
    all_dig = comm.allgather_u64(dig)
    digests_ok = verify_gathered(all_dig, expect, world) and bool(np.all(allc[:, 7] == 1))
    el_max = float(allc[:, 5].max()) / 1e9
    step_s = el_max / args.steps
    res = {
        "batch": batch, "stats": stats, "elapsed": el_max, "step_s": step_s,
        "value": float(allc[:, 0].sum()) / step_s, "digests_ok": digests_ok,
        "per_rank": [{c: int(allc[r, i]) for i, c in enumerate(COUNTERS)} for r in range(world)],
        "items_per_s": float(allc[:, 1].sum()) / step_s,
        "encode_s": enc_s,
    }
    return res if rank == 0 else None


def roofline_fields(stats, batch, items_per_gpu, step_s, pmc: bool = True, stile_text: int = 2) -> dict:
    """Per-kernel algorithmic GB/s, the dominant kernel's roofline, the pipeline's fraction.
    pmc: the PMC traffic file describes this workload (the headline config); else traffic is
    null rather than another workload's bytes.  stile_text: the engine parameter (0: k_runs
    copies every tile's text to sbytes for k_doctree)."""
    stage_ns = {k: float(np.mean([s["stage_ns"][k] for s in stats])) for k in stats[0]["stage_ns"]}
    launches = stats[0]["stage_launches"]
    slots = items_per_gpu + batch.docs  # items + one document-start slot per document
    runs = stats[0]["runs"]
    text_bytes = stats[0]["text_bytes"]

    waves = max(1, stats[0]["waves"])
    per_wave = {k: launches[k] / waves for k in launches}
    radix = bool(launches.get("sortb"))
    # text mode (the global level 1's first walk stages the text): the re-walk stage is
    # k_tcopy + k_walk_ovf (+ k_doctotals), 4 launches per k_walk1 launch instead of 2
    text_mode = bool(launches.get("walk1")) and launches.get("walk2", 0) == 4 * launches["walk1"]
    # waves without run contraction: every live item is a run
    nocon = runs > 0.5 * slots

    def alg_bytes(k):
        per_slot, per_run, per_text = KERNEL_BYTES[k]
        if k == "doctree" and (launches.get("expand", 1) or launches.get("text")):
            per_text = 0.0  # text left to k_expand / k_tscatter: no text in or out of k_doctree
        if (k == "runs" and stile_text and launches.get("doctree") and not launches.get("expand")
                and not launches.get("walk1")):
            per_text = 0.0  # (k_doctree stages the text from the stile segments: no copy)
        if k == "expand" and launches.get("walk1"):
            per_run = 20.0
        if radix and level1_run_bytes(k, per_wave, text_mode) is not None:
            per_run = level1_run_bytes(k, per_wave, text_mode)
        if nocon:
            if k == "classify":
                per_run = 0.0   # no contraction: no parents read, no jump bits
            elif k == "runs":
                per_run = 32.0  # parent + key in; head, prefix, parent, key out
        if text_mode:
            if k == "walk1":
                # the 32-byte record line; the staged text out (+ in from the slot-order text
                # when runs are longer than the record carries)
                per_run, per_text = 32.0, 1.0 if nocon else 2.0
            elif k == "walk2":
                per_run, per_text = 0.5, 2.0   # splitter words; staged text in, document out
        return per_slot * slots + per_run * runs + per_text * text_bytes

    per_kernel = {k: {"ms": stage_ns[k] / 1e6, "launches": launches[k],
                      "alg_gbps": alg_bytes(k) / stage_ns[k] if stage_ns[k] and launches[k] else 0.0}
                  for k in stage_ns}

    # one launch of a stage's main kernel per wave (a stage's helper kernels, e.g. k_doctotals
    # beside k_doctree, are timed inside the stage: a few percent of it)

    def roof(k):
        ns = stage_ns[k] / waves
        b = alg_bytes(k) / waves
        return {"bound": "hbm", "kernel": STAGE_KERNEL.get(k, k), "achieved": b / ns,
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": b / ns / HBM_PEAK_GBPS,
                "traffic": measured_traffic(k, items_per_gpu / waves) if pmc else None,
                "alg_bytes_per_launch": b, "launch_us": ns / 1e3}

    # the dominant kernel = the stage with the most device time per step (HIP events, summed
    # over its launches; with lanes a stage's launches can overlap another lane's)
    timed = [k for k in stage_ns if launches[k] and stage_ns[k] > 0]
    dom = max(timed, key=lambda k: stage_ns[k])
    out = roof(dom)
    out["traffic_source"] = PMC_FILE if out["traffic"] is not None else None
    out["choice"] = "the stage with the most device time per step (one-lane HIP events)"
    # every stage's roofline (the dominant one can change from box to box when two stages are
    # within a few percent), and the batched-merge kernels together (north star: >= 50 %)
    rooflines = {k: roof(k) for k in timed}
    tot_b = sum(alg_bytes(k) for k in timed)
    tot_ns = sum(stage_ns[k] for k in timed)
    merge_all = {"bound": "hbm", "achieved": tot_b / tot_ns, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                 "frac": tot_b / tot_ns / HBM_PEAK_GBPS, "alg_bytes_per_step": tot_b,
                 "device_ms_per_step": tot_ns / 1e6, "stages": timed}
    min_bytes = MIN_B_PER_SLOT * slots + MIN_B_PER_RUN * runs + MIN_B_PER_TEXT * text_bytes
    pipeline = {"min_bytes_per_step": min_bytes,
                "contract_b_per_item": min_bytes / items_per_gpu,
                "gbps": min_bytes / step_s / 1e9, "frac": min_bytes / step_s / 1e9 / HBM_PEAK_GBPS,
                "note": "design minimum: 3 B/slot (codepoint word with tombstone and "
                        "previous-slot flags) + 6 B/run head (lamport, agent) + 1 B/merged byte, "
                        "over the wall time of a step"}
    return {"kernels": per_kernel, "roofline": out, "pipeline": pipeline,
            "rooflines": rooflines, "batched_merge": merge_all,
            "stream_kernel": roof("classify") if launches.get("classify") else None,
            "stage_ns": stage_ns, "launches": launches}


def traces_workload(args) -> int:
    world, rank, local = rank_env()
    ctx = crdt_hip.Context(local)
    comm = Comm(world, rank, ctx)
    t_setup = time.perf_counter()
    inputs = load_bases(args.order == "fugue")
    if args.splitter_stride:
        ctx.set_param("splitter_stride", args.splitter_stride)
    ctx.set_param("level1", args.level1)
    ctx.set_param("contraction", args.contraction)
    ctx.set_param("l1_group", args.l1_group)
    if not args.fuse_text:  # (the engine's default is 1; builds before the parameter lack it)
        ctx.set_param("fuse_text", 0)
    ctx.set_param("lanes", args.lanes)
    # (every knob the line reports is sent, defaults included: the JSON labels what ran)
    ctx.set_param("xcd_order", args.xcd_order)
    ctx.set_param("stile_text", args.stile_text)
    ctx.set_param("text_scatter", args.text_scatter)
    ctx.set_param("doctree_k32", args.doctree_k32)
    ctx.set_param("runs_slots", args.runs_slots)
    group = args.group_docs if args.group_docs >= 0 else int(args.order == "fugue")
    if group:
        ctx.set_param("group_docs", group)
    if args.nsq_list != 1:  # (likewise)
        ctx.set_param("nsq_list", args.nsq_list)
    ctx.set_param("lane_gate", args.lane_gate)
    ctx.set_param("max_wave_slots", 1 << args.wave_slots_log2)
    ctx.set_param("plan_cache", args.plan_cache)
    if args.l1_split != 0:  # (the engine's default; builds before the parameter lack it)
        ctx.set_param("l1_split", args.l1_split)
    if args.tail_wave_div != 0:  # (likewise)
        ctx.set_param("tail_wave_div", args.tail_wave_div)

    def make_batch(bases, replicas, relabel, seed):
        return ctx.batch(bases, replicas=replicas, relabel=relabel, seed=seed)

    if rank == 0:
        log(f"[bench] setup (load + resolve) {time.perf_counter() - t_setup:.1f} s")
    res = traces_rank(args, comm, make_batch, inputs)
    out = None
    if rank == 0:
        batch, stats = res["batch"], res["stats"]
        items_per_gpu = batch.items
        # Kernel times for the roofline come from merges with ONE lane (untimed, after the timed
        # region): with two lanes a wave's level 1 waits for CUs the other lane's level 0 holds,
        # so its HIP-event interval is not the kernel's own duration (a one-lane rocprofv3
        # kernel trace agrees with these).  The timed step itself ran with args.lanes lanes.
        iso_stats = stats
        if args.lanes > 1:
            ctx.set_param("lanes", 1)
            iso_stats = [batch.merge()[2] for _ in range(3)][1:]
            ctx.set_param("lanes", args.lanes)
        # (the committed PMC bytes per item were measured at the headline config)
        headline = (args.relabel == "rotate" and args.order != "fugue" and args.replicas == 4096
                    and args.nsq_list == 1)
        rf = roofline_fields(iso_stats, batch, items_per_gpu, res["step_s"], pmc=headline,
                             stile_text=args.stile_text)
        rf_lanes = None
        if args.lanes > 1:
            rf_lanes = {k: round(float(np.mean([s["stage_ns"][k] for s in stats])) / 1e6, 4)
                        for k in stats[0]["stage_ns"] if stats[0]["stage_launches"][k]}
        patches_per_gpu = sum(inputs["patches"]) * args.replicas
        out = {
            "metric": METRIC,
            "value": res["value"],
            "unit": "patches/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": res["step_s"] * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic replicas of the 4 real josephg traces (resolved on host, "
                    f"{args.order} anchors, relabel={args.relabel}, resident in HBM)",
            "config": {
                "workload": "config 3: 4 traces x %d replicas per GPU" % args.replicas,
                "docs_per_gpu": batch.docs,
                "items_per_gpu": items_per_gpu,
                "patches_per_gpu": patches_per_gpu,
                "relabel": args.relabel,
                "order": args.order,
                "waves": stats[0]["waves"],
                "lanes": min(args.lanes, stats[0]["waves"]),
                "parallelism": f"replicas x{world} (no data-path collective)",
            },
            "items_per_s": res["items_per_s"],
            "device_ms_per_step": float(np.mean([s["total_ns"] for s in stats])) / 1e6,
            "runs_per_gpu": stats[0]["runs"],
            "kernels": rf["kernels"],
            "kernels_source": "one-lane merges after the timed region (uncontended launches)"
                              if args.lanes > 1 else "the timed merges",
            "kernels_ms_with_lanes": rf_lanes,
            "ms_per_step_1_lane": float(np.mean([s["total_ns"] for s in iso_stats])) / 1e6,
            "roofline": rf["roofline"],
            "rooflines": rf["rooflines"],
            "batched_merge": rf["batched_merge"],
            "stream_kernel": rf["stream_kernel"],
            "pipeline": rf["pipeline"],
            "input_encoding": {
                "ms": res["encode_s"] * 1e3,
                "bytes_per_slot": 15,
                "note": "one-time, untimed: upload of the 4 resolved logs and the device build of "
                        "every replica's resident op log (relabelled parent u32, key u64 = lamport "
                        "<< 16 | agent, 3-byte codepoint word with the tombstone and previous-slot "
                        "flags: O(1) per item) and of the compact list of the items without the "
                        "previous-slot flag (parent u32 and key u64 each, slot order, a prefix "
                        "count per 64 slots; Engine::build_nsq); the traffic contract (DESIGN.md "
                        "section 7) prices the merge over this format"},
            "resolve": {"ms_per_trace": dict(zip(TRACES, inputs["resolve_ms"])),
                        "ms_total_one_core": sum(inputs["resolve_ms"]),
                        "ms_all_parallel": inputs["resolve_parallel_ms"],
                        "threads_parallel": len(TRACES),
                        "note": "host resolver (positional patches -> anchor log), untimed "
                                "setup of the batch; once per trace"},
            "per_rank": res["per_rank"],
            "digests_ok": res["digests_ok"],
        }
        res["batch"].close()  # free the headline shard before the companion's
        res = batch = stats = None
    # companion line: the same shard relabelled by a seeded random permutation per replica
    # (SURVEY §8(d) config 3's "seed-r permutation": runs no longer contract)
    if args.companion_replicas and args.relabel != "shuffle":
        ca = argparse.Namespace(replicas=args.companion_replicas, relabel="shuffle", warmup=1,
                                steps=2)
        cres = traces_rank(ca, comm, make_batch, inputs)
        if rank == 0:
            cb, cs = cres["batch"], cres["stats"]
            out["companion_shuffle"] = {
                "workload": "config 3, relabel=shuffle: 4 traces x %d replicas per GPU"
                            % ca.replicas,
                "value": cres["value"], "unit": "patches/s",
                "ms_per_step": cres["step_s"] * 1e3, "steps": ca.steps,
                "items_per_s": cres["items_per_s"], "runs_per_gpu": cs[0]["runs"],
                "waves": cs[0]["waves"], "digests_ok": cres["digests_ok"],
                "kernels_ms": {k: v / 1e6 for k, v in
                               {k: float(np.mean([s["stage_ns"][k] for s in cs]))
                                for k in cs[0]["stage_ns"]}.items() if v > 2e4},
            }
            crf = roofline_fields(cs, cb, cb.items, cres["step_s"], pmc=False, stile_text=args.stile_text)
            out["companion_shuffle"]["rooflines"] = {
                k: {"kernel": v["kernel"], "frac": v["frac"], "achieved_gbps": v["achieved"],
                    "launch_us": v["launch_us"]} for k, v in crf["rooflines"].items()}
            out["companion_shuffle"]["batched_merge"] = crf["batched_merge"]
            out["digests_ok"] = out["digests_ok"] and cres["digests_ok"]
            cb.close()
    # companion line: the same headline batch over the plain SoA (no compact list of the non-seq
    # items' parents and keys: the level-0 kernels gather them from the columns), so that the
    # headline's dependence on that one-time index is measured, not assumed
    if args.plain_companion:
        ctx.set_param("nsq_list", 0)
        pa = argparse.Namespace(replicas=args.replicas, relabel=args.relabel, warmup=1, steps=3)
        pres = traces_rank(pa, comm, make_batch, inputs)
        ctx.set_param("nsq_list", args.nsq_list)
        if rank == 0:
            pb, ps = pres["batch"], pres["stats"]
            out["companion_plain_soa"] = {
                "workload": "config 3 (%d replicas per GPU, relabel=%s) without the compact list "
                            "of the non-seq items' parents and keys (nsq_list 0)"
                            % (pa.replicas, pa.relabel),
                "value": pres["value"], "unit": "patches/s", "ms_per_step": pres["step_s"] * 1e3,
                "steps": pa.steps, "digests_ok": pres["digests_ok"],
                "input_encoding_ms": pres["encode_s"] * 1e3,
                "kernels_ms": {k: v / 1e6 for k, v in
                               {k: float(np.mean([s_["stage_ns"][k] for s_ in ps]))
                                for k in ps[0]["stage_ns"]}.items() if v > 2e4},
            }
            out["digests_ok"] = out["digests_ok"] and pres["digests_ok"]
        if rank == 0:
            pres["batch"].close()
    # companion line: the headline batch in raw SoA mode: every merge first
    # derives the key, the codepoint word with its flags and the compact nsq list on the device
    # from reference-shaped columns (lamport, agent, deleted, codepoint beside the parents), so
    # the step is priced over the raw SoA, the untimed input encoding included (RGA batches: the
    # raw columns carry no Fugue side)
    if args.raw_companion and args.order == "rga":
        def make_raw(bases, replicas, relabel, seed):
            b = make_batch(bases, replicas, relabel, seed)
            b.set_raw(True)
            return b
        ra = argparse.Namespace(replicas=args.replicas, relabel=args.relabel, warmup=1, steps=3)
        rres = traces_rank(ra, comm, make_raw, inputs)
        if rank == 0:
            rb, rs = rres["batch"], rres["stats"]
            kms = {k: float(np.mean([s_["stage_ns"][k] for s_ in rs])) / 1e6 for k in rs[0]["stage_ns"]}
            out["companion_raw_soa"] = {
                "workload": "config 3 (%d replicas per GPU, relabel=%s) over the raw SoA: the "
                            "input encoding (key, flags, nsq list) derived on the device inside "
                            "every timed merge" % (ra.replicas, ra.relabel),
                "value": rres["value"], "unit": "patches/s", "ms_per_step": rres["step_s"] * 1e3,
                "steps": ra.steps, "digests_ok": rres["digests_ok"],
                "encode_ms": kms.get("encode", 0.0),
                "raw_bytes_per_slot": 15, "encoded_bytes_per_slot_written": 11,
                "kernels_ms": {k: v for k, v in kms.items() if v > 0.02},
            }
            out["digests_ok"] = out["digests_ok"] and rres["digests_ok"]
        if rank == 0:
            rres["batch"].close()
    if rank == 0:
        if not args.no_cpu_baseline and world == 1:  # (the CPU lines belong to the N=1 run)
            threads = args.cpu_threads or host_cpus()["threads"]
            out["cpu_baseline"] = cpu_baseline(inputs["bases"], inputs["patches"],
                                               args.cpu_seconds, threads)
            out["config1"] = config1(ctx, args.config1_seconds)
        print(json.dumps(out), flush=True)
    ok = out["digests_ok"] if rank == 0 else True
    comm.close()
    return 0 if ok else 1


# ---------------------------------------------------------------------------------------------
# side workloads
# ---------------------------------------------------------------------------------------------
def side_workload(args) -> int:
    """one document per GPU, resident in HBM, merged `steps`
    times.  value = op-log items merged per second (every item is one insert op; config 2 also
    reports patches/s).  Multi-GPU: replicas only (each rank merges its own copy)."""
    world, rank, local = rank_env()
    ctx = crdt_hip.Context(local)
    comm = Comm(world, rank, ctx)
    ctx.set_param("level1", args.level1)
    ctx.set_param("contraction", args.contraction)
    ctx.set_param("l1_group", args.l1_group)
    ctx.set_param("stile_text", args.stile_text)
    ctx.set_param("text_scatter", args.text_scatter)
    if args.splitter_stride:
        ctx.set_param("splitter_stride", args.splitter_stride)
    t_setup = time.perf_counter()
    patches = None
    if args.workload == "seph":
        t = crdt_hip.Trace(os.path.join(ROOT, "traces", "seph-blog1.json.gz"))
        lg = t.resolve().arrays()
        patches = len(t)
        with open(os.path.join(ROOT, "tests", "golden", "traces.json")) as f:
            g = json.load(f)["seph-blog1"]
        expect = (int(g["tree_digest"], 16), g["end_bytes"])
        batch = ctx.batch([lg], replicas=1, relabel="none")
        desc = "config 2: seph-blog1 anchor log, one document"
    elif args.workload == "agents64":
        n = args.items or 10_000_000
        lg = crdt_hip.OpLog.synth_agents(n, 64, 0x5EED0001).arrays()
        # expected length = the UTF-8 bytes of the log's visible items (counted without merging);
        # the digest itself is checked against the oracle by tests/test_gpu_scale.py
        cp = lg.cp[lg.deleted == 0].astype(np.uint64)
        expect = (None, int(cp.size + np.count_nonzero(cp >= 0x80) + np.count_nonzero(cp >= 0x800)
                            + np.count_nonzero(cp >= 0x10000)))
        batch = ctx.batch([lg], replicas=1, relabel="none")
        desc = f"config 4: 64-agent concurrent log, {n} items, seed 0x5EED0001"
    else:
        n = args.items or 1_000_000_000
        batch = crdt_hip.Batch.synth_tree(ctx, n, args.p_chain, 50, 0x5EED0002)
        expect = (None, crdt_hip.synth_tree_visible(n, 50, 0x5EED0002))
        desc = (f"config 5: one document of {n} items (p_chain {args.p_chain / 100:.2f}, "
                "50% tombstones), generated on device")
    if rank == 0:
        log(f"[bench] {desc}: {batch.items} items, setup {time.perf_counter() - t_setup:.1f} s")
    dig, lens, stats, el = merge_steps(batch, comm, args.warmup, args.steps)
    ok = int(lens[0]) == expect[1] and (expect[0] is None or int(dig[0]) == expect[0])
    cnt = np.array([batch.items, int(el * 1e9), int(ok)], np.uint64)
    allc = comm.allgather_u64(cnt).reshape(world, 3)
    el = float(allc[:, 1].max()) / 1e9
    ok = bool(np.all(allc[:, 2] == 1))
    stage_ns = {k: float(np.mean([x["stage_ns"][k] for x in stats])) for k in stats[0]["stage_ns"]}
    if rank == 0:
        out = {
            "metric": METRIC, "value": float(allc[:, 0].sum()) / (el / args.steps),
            "unit": "items/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic" if patches is None else "trace",
            "config": {"workload": desc, "items_per_gpu": batch.items, "runs": stats[0]["runs"],
                       "parallelism": f"replicas x{world} (no data-path collective)"},
            "kernels_ms": {k: v / 1e6 for k, v in stage_ns.items() if v > 2e4},
            "device_ms_per_step": float(np.mean([x["total_ns"] for x in stats])) / 1e6,
            "text_bytes": int(lens[0]), "digest": "%016x" % int(dig[0]), "digests_ok": ok,
        }
        # every stage's roofline by its algorithmic bytes (DESIGN.md §7 pricing; no PMC here)
        rf = roofline_fields(stats, batch, batch.items, el / args.steps, pmc=False,
                             stile_text=args.stile_text)
        out["rooflines"] = {k: {"kernel": v["kernel"], "frac": v["frac"],
                                "achieved_gbps": v["achieved"], "launch_us": v["launch_us"]}
                            for k, v in rf["rooflines"].items()}
        out["batched_merge"] = rf["batched_merge"]
        if patches is not None:
            out["patches_per_s"] = patches * world / (el / args.steps)
        print(json.dumps(out), flush=True)
    comm.close()
    return 0 if ok else 1


def downstream_workload(args) -> int:
    """The reference's downstream group (main.rs:50-81) on the device: per trace, a step clones
    the initial replica (main.rs:64), applies every per-patch update (:65-67) and merges (:68).
    Updates are encoded on the host beforehand, as upstream_updates does (rope.rs:196-220), and
    packed into one buffer + offsets and uploaded to HBM once (crdt_hip_updates_upload; --pcie
    times the upload too); the timed region holds the clone, the device decode (replica.hip) and
    the merge, whose codepoint count is the len() the reference asserts (main.rs:68).
    value = patches/s over the 4 traces."""
    world, rank, local = rank_env()
    ctx = crdt_hip.Context(local)
    comm = Comm(world, rank, ctx)
    if args.nsq_list != 1:  # (each merge rebuilds the replica's compact nsq list; 0: gathers)
        ctx.set_param("nsq_list", args.nsq_list)
    with open(os.path.join(ROOT, "tests", "golden", "traces.json")) as f:
        golden = json.load(f)
    t_setup = time.perf_counter()
    work = []
    for name in TRACES:
        t = crdt_hip.Trace(os.path.join(ROOT, "traces", f"{name}.json.gz"))
        patches = [t.patch(i) for i in range(len(t))]
        if args.order == "fugue":  # a Fugue upstream: version-2 updates into a Fugue replica
            lg = crdt_hip.OpLog(fugue=True)
            if t.start_content:
                lg.insert(0, t.start_content)
            init = crdt_hip.Replica(ctx, lg)
            updates = []
            for pos, dele, ins in patches:
                v = lg.version()
                lg.replace(pos, pos + dele, ins)
                updates.append(lg.encode_from(v))
        else:
            up, updates = crdt_hip.HipMerge.upstream_updates(t.start_content, patches)
            init = crdt_hip.Replica(ctx, up.log if up.log.view().n else None)
        buf, offs = crdt_hip.pack_updates(updates)
        # the update vector (main.rs:58) resident in HBM, unless the PCIe upload is timed too
        src = (buf, offs) if args.pcie else crdt_hip.UpdateBatch(ctx, buf, offs)
        end = t.end_content
        work.append((name, len(t), init, src, buf.size, int(golden[name]["tree_digest"], 16),
                     golden[name]["end_bytes"], len(end)))
    if rank == 0:
        log(f"[bench] downstream: {sum(w[1] for w in work)} updates, "
            f"{sum(w[4] for w in work) / 2**20:.1f} MiB encoded, "
            f"setup {time.perf_counter() - t_setup:.1f} s")

    def step(per):
        ok = True
        for name, npatch, init, src, _, dig, nbytes, ncp in work:
            t0 = time.perf_counter()
            if args.stepwise or args.pcie:
                r = init.clone()
                if args.pcie:
                    r.apply_packed(*src)
                else:
                    r.apply_resident(src)
                res = r.merge_len()
                r.close()
            else:  # the closure as one device call (crdt_hip_replica_replay)
                res = init.replay(src)
            per[name] = per.get(name, 0.0) + time.perf_counter() - t0
            ok &= res == (ncp, nbytes, dig)
        return ok

    for _ in range(args.warmup):
        step({})
    comm.barrier()
    per: dict = {}
    t0 = time.perf_counter()
    ok = True
    for _ in range(args.steps):
        ok &= step(per)
    comm.barrier()
    el = time.perf_counter() - t0
    total_patches = sum(w[1] for w in work)
    allc = comm.allgather_u64(np.array([total_patches, int(el * 1e9), int(ok)], np.uint64))
    allc = allc.reshape(world, 3)
    el = float(allc[:, 1].max()) / 1e9
    ok = bool(np.all(allc[:, 2] == 1))
    if rank == 0:
        out = {
            "metric": METRIC, "value": float(allc[:, 0].sum()) / (el / args.steps),
            "unit": "patches/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "trace",
            "config": {"workload": "downstream (main.rs:63-69): clone + apply every update + len, "
                                   "device decode, 4 traces one after the other, "
                                   + ("clone / apply / merge_len calls" if args.stepwise or args.pcie
                                      else "one crdt_hip_replica_replay call per closure"),
                       "updates": total_patches, "order": args.order,
                       "nsq_list": args.nsq_list,
                       "encoded_bytes": int(sum(w[4] for w in work)),
                       "parallelism": f"replicas x{world} (no data-path collective)"},
            "per_trace": {w[0]: {"ms": per[w[0]] / args.steps * 1e3,
                                 "patches_per_s": w[1] / (per[w[0]] / args.steps)} for w in work},
            "pcie_included": bool(args.pcie), "digests_ok": bool(ok),
        }
        print(json.dumps(out), flush=True)
    comm.close()
    return 0 if ok else 1


def upstream_inc_workload(args) -> int:
    """the upstream loop (main.rs:28-36) with len() every K patches instead of
    once at the end.  The reference's len() (rope.rs:135, checkout_tip) materialises the whole
    document each time.  Per checkpoint the step applies the chunk's updates (encoded on the host
    beforehand, as upstream_updates does, rope.rs:196-220, resident in HBM) to a device replica
    and asks for the length, once with the incremental merge (crdt_hip_replica_merge_inc: only
    the appended items are ranked) and, in a second timed pass, with a full merge per checkpoint
    (crdt_hip_replica_merge_len).  Every checkpoint's codepoints are checked against the host
    log's visible length after the same patches.  value = patches/s of the incremental loop."""
    world, rank, local = rank_env()
    ctx = crdt_hip.Context(local)
    comm = Comm(world, rank, ctx)
    name, K = args.inc_trace, args.every
    t = crdt_hip.Trace(os.path.join(ROOT, "traces", f"{name}.json.gz"))
    patches = [t.patch(i) for i in range(len(t))]
    up = crdt_hip.HipMerge.from_str(t.start_content)
    chunks, expect = [], []
    for i in range(0, len(patches), K):
        v = up.log.version()
        for pos, dele, ins in patches[i:i + K]:
            up.replace(pos, pos + dele, ins)
        buf, offs = crdt_hip.pack_updates([up.log.encode_from(v)])
        chunks.append(crdt_hip.UpdateBatch(ctx, buf, offs))
        expect.append(up.log.visible_len())
    init = crdt_hip.HipMerge.from_str(t.start_content).log

    def loop(incremental, per_ck, check_text=False):
        r = crdt_hip.Replica(ctx, init if init.view().n else None)
        ok, paths = True, 0
        for c, ub in enumerate(chunks):
            r.apply_resident(ub)
            t0 = time.perf_counter()
            if incremental:
                cps, nb, path, _ = r.merge_inc()
                paths += path
            else:
                cps, nb, _ = r.merge_len()
            per_ck.append(time.perf_counter() - t0)
            ok &= cps == expect[c]
        if check_text:  # (untimed: the final document itself, not only its length)
            text = r.merge_inc(text=True)[3] if incremental else r.merge()[0]
            ok &= text == t.end_content.encode()
        r.close()
        return ok, paths

    res = {}
    text_ok = True
    for mode in ("incremental", "full"):
        for w in range(args.warmup):
            text_ok &= loop(mode != "full", [], check_text=(w == 0))[0]
        comm.barrier()
        per_ck: list = []
        t0 = time.perf_counter()
        ok, paths = True, 0
        for _ in range(args.steps):
            o, p = loop(mode != "full", per_ck)
            ok &= o
            paths += p
        comm.barrier()
        el = time.perf_counter() - t0
        res[mode] = {"ms_per_step": el / args.steps * 1e3, "ok": bool(ok),
                     "len_ms_mean": float(np.mean(per_ck)) * 1e3,
                     "len_ms_median": float(np.median(per_ck)) * 1e3,
                     "incremental_calls": paths // max(1, args.steps)}
    inc, full = res["incremental"], res["full"]
    ok = inc["ok"] and full["ok"] and (text_ok or not args.warmup)
    if rank == 0:
        out = {
            "metric": METRIC, "value": len(patches) / (inc["ms_per_step"] / 1e3),
            "unit": "patches/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": inc["ms_per_step"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "trace",
            "config": {"workload": f"extension workload (not in the reference, which asserts "
                                   f"len() once after the loop): upstream (main.rs:28-36) with "
                                   f"len() every {K} patches: apply the chunk's updates to a "
                                   "device replica + len()",
                       "trace": name, "patches": len(patches), "checkpoints": len(chunks),
                       "updates_resident": True},
            "incremental": inc, "full": full,
            "len_speedup_mean": full["len_ms_mean"] / inc["len_ms_mean"],
            "len_speedup_median": full["len_ms_median"] / inc["len_ms_median"],
            "lens_ok": bool(ok),
            "final_text_ok": bool(text_ok) if args.warmup else None,
        }
        print(json.dumps(out), flush=True)
    comm.close()
    return 0 if ok else 1


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; without WORLD_SIZE in the environment, bench.py "
                         "starts this many rank processes itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--replicas", type=int, default=4096, help="replicas of each trace per GPU")
    ap.add_argument("--relabel", default="rotate", choices=["none", "rotate", "shuffle"])
    ap.add_argument("--companion-replicas", type=int, default=1024,
                    help="replicas per trace of the relabel=shuffle companion line (0: none)")
    ap.add_argument("--splitter-stride", type=int, default=0)
    ap.add_argument("--wave-slots-log2", type=int, default=30,
                    help="slots per device wave (2^N; smaller waves pipeline better over lanes)")
    ap.add_argument("--pcie", action="store_true",
                    help="downstream: upload the encoded updates inside the timed region "
                         "(default: resident in HBM, as every other workload's inputs)")
    ap.add_argument("--stepwise", action="store_true",
                    help="downstream: clone, apply and merge as three calls (default: one "
                         "crdt_hip_replica_replay call per closure)")
    ap.add_argument("--lane-gate", type=int, default=1, choices=[0, 1],
                    help="1: lanes take turns at level 0 (the HBM stream)")
    ap.add_argument("--lanes", type=int, default=2,
                    help="waves merged concurrently, each on its own stream and scratch "
                         "(Engine::merge_lanes; 1 = one after the other)")
    ap.add_argument("--plan-cache", type=int, default=1, choices=[0, 1],
                    help="1: merges after the first enqueue every wave with its learnt launch "
                         "plan and wait once (Engine::merge_async); 0: wait after each level 0")
    ap.add_argument("--tail-wave-div", type=int, default=0,
                    help="the last wave of a multi-wave merge holds at most max_wave_slots / this "
                         "(its level 1 overlaps nothing); 0 = plain greedy waves")
    ap.add_argument("--l1-split", type=int, default=0, choices=[0, 1],
                    help="1: enqueued waves run level 1 on a low-priority stream of their lane "
                         "(level 0 of the next wave is favoured for the CUs); 0: one stream")
    ap.add_argument("--fuse-text", type=int, default=1, choices=[0, 1],
                    help="0: k_doctree leaves the text to k_expand (smaller LDS footprint)")
    ap.add_argument("--xcd-order", type=int, default=1, choices=[0, 1],
                    help="1: level-0 tiles in XCD-aware order (each XCD one contiguous range)")
    ap.add_argument("--stile-text", type=int, default=2, choices=[0, 1, 2],
                    help="fused level 1 stages text from the tile segments (k_runs skips the "
                         "slot-order copy): 1 by loads and shifts, 2 by LDS-DMA per tile")
    ap.add_argument("--raw-companion", type=int, default=1, choices=[0, 1],
                    help="1: also time the headline batch in raw SoA mode (the input encoding "
                         "derived on the device inside every merge)")
    ap.add_argument("--doctree-k32", type=int, default=0, choices=[0, 1],
                    help="1: every LDS level 1 on k_doctree_wide (32-bit sibling keys, 9 B of "
                         "LDS per run instead of 15)")
    ap.add_argument("--text-scatter", type=int, default=0, choices=[0, 1],
                    help="1: k_doctree stops at the run offsets and k_tscatter streams the tiles' "
                         "text to the documents; 0: k_doctree writes the text itself (phase C)")
    ap.add_argument("--group-docs", type=int, default=-1, choices=[-1, 0, 1],
                    help="replica batches placed base by base, each base in waves of its own "
                         "(-1: only for --order fugue, whose seph-blog1 rows exceed the LDS level 1)")
    ap.add_argument("--runs-slots", type=int, default=32, choices=[16, 32, 64],
                    help="k_runs slots per thread (16: 256 threads per tile, 32: 128, 64: one wave)")
    ap.add_argument("--nsq-list", type=int, default=1, choices=[0, 1, 2],
                    help="1: resident batches (input encoding) and replicas of 2^22+ slots (every "
                         "merge) carry the compact list of the non-seq items' parents and keys; "
                         "2: every replica too; 0: the level-0 kernels gather them")
    ap.add_argument("--plain-companion", type=int, default=1, choices=[0, 1],
                    help="1: a companion line of the headline batch without the compact nsq list")
    ap.add_argument("--l1-group", type=int, default=0, choices=[0, 1, 2],
                    help="global level-1 sibling grouping: 0 by the largest document, 1 counting, "
                         "2 radix sorts")
    ap.add_argument("--contraction", type=int, default=0, choices=[0, 1, 2],
                    help="run contraction of RGA waves: 0 by the input (none when most items lack "
                         "the previous-slot flag), 1 always, 2 never")
    ap.add_argument("--level1", type=int, default=0, choices=[0, 1],
                    help="0: per-document LDS level 1 where it fits (default), 1: global kernels")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--config1-seconds", type=float, default=4.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--order", default="rga", choices=["rga", "fugue"],
                    help="document order of the traces and downstream workloads (fugue: a "
                         "side line; the CPU baseline and the shuffle companion are RGA-only "
                         "and are skipped)")
    ap.add_argument("--workload", default="traces",
                    choices=["traces", "seph", "agents64", "big1b", "downstream", "upstream_inc"],
                    help="traces: config 3 (headline); seph: config 2; agents64: config 4; "
                         "big1b: config 5 (SURVEY.md §8(d)); downstream: the reference's "
                         "downstream group with device-side update decode (§8(f) row 2)")
    ap.add_argument("--items", type=int, default=0, help="items of the synthetic workloads")
    ap.add_argument("--every", type=int, default=1000,
                    help="upstream_inc: len() every this many patches")
    ap.add_argument("--inc-trace", default="automerge-paper", help="upstream_inc: the trace")
    ap.add_argument("--p-chain", type=int, default=90,
                    help="config 5: percent of items whose parent is the previous item "
                         "(0 = uniform random parents, the worst case for gathers)")
    args = ap.parse_args(argv)
    if args.order == "fugue":  # (the CPU baseline and the companion merge RGA logs)
        args.no_cpu_baseline = True
        args.companion_replicas = 0
    return args


def main() -> int:
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started before this process touches the GPU
        return spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if world > 1:
        log(f"[bench] rank {os.environ.get('RANK', '0')} of {world}")
    global crdt_hip
    import crdt_hip as _engine
    crdt_hip = _engine
    if args.workload == "downstream":
        return downstream_workload(args)
    if args.workload == "upstream_inc":
        return upstream_inc_workload(args)
    if args.workload != "traces":
        return side_workload(args)
    return traces_workload(args)


if __name__ == "__main__":
    sys.exit(main())
