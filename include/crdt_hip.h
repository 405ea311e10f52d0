/*
 * crdt_hip.h — C ABI of the MI355X-native merge engine (libcrdt_hip.so).
 *
 * This is the drop-in boundary for the replay-and-merge path of noib3/crdt-benches.  The
 * reference binds CRDT engines through two Rust traits:
 *   trait Upstream   /root/reference/src/rope.rs:6-33   (from_str, insert, remove, len, replace)
 *   trait Downstream /root/reference/src/rope.rs:185-191 (upstream_updates, apply_update)
 * and registers them in the bench at /root/reference/src/main.rs:43-46 and :78.  A Rust
 * `crdt-hip-sys` crate binds exactly the entry points below; the
 * `impl Upstream/Downstream for HipMerge` maps:
 *   from_str(s)          -> crdt_hip_oplog_new + crdt_hip_oplog_insert(0, s)   (rope.rs:113-121)
 *   insert(at, s)        -> crdt_hip_oplog_insert                               (rope.rs:124-126)
 *   remove(a..b)         -> crdt_hip_oplog_remove                               (rope.rs:129-131)
 *   len()                -> crdt_hip_merge  (replaces OpLog::checkout_tip().len(), rope.rs:134-136)
 *   upstream_updates     -> crdt_hip_oplog_version + crdt_hip_oplog_encode_from (rope.rs:196-220)
 *   apply_update(u)      -> crdt_hip_oplog_apply_update (replaces decode_and_add, rope.rs:222-224),
 *                           or on the device: crdt_hip_replica_apply_updates (batched)
 *   clone()              -> crdt_hip_oplog_clone (the device context is shared, never copied)
 *
 * Conventions
 *   - Every function returns int status: 0 = ok, < 0 = error (CRDT_HIP_E*).  Nothing throws or
 *     aborts across the ABI.  crdt_hip_last_error(ctx) returns the message of the last failure
 *     on that context (ctx == NULL: the last failure of a context-free call on this thread).
 *   - Host pointers are BORROWED for the duration of the call only.
 *   - Positions are Unicode codepoints (EDITS_USE_BYTE_OFFSETS = false, rope.rs:8,16-19).
 *   - A context is bound to one HIP device and must be used by one host thread at a time; calls
 *     are synchronous at the ABI (the work runs on the context's own HIP stream).
 *   - Op log ids: items are 1..n in creation order; id 0 is the document start (origin of an
 *     insert at position 0).
 */
#ifndef CRDT_HIP_H
#define CRDT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDT_HIP_ABI_VERSION 2

enum {
    CRDT_HIP_OK = 0,
    CRDT_HIP_EINVAL = -1,   /* bad argument */
    CRDT_HIP_ERANGE = -2,   /* position / id out of range */
    CRDT_HIP_ENOMEM = -3,   /* host or device allocation failed */
    CRDT_HIP_EDEVICE = -4,  /* HIP runtime error (no device, launch failure, ...) */
    CRDT_HIP_EBADLOG = -5,  /* malformed op log (bad parent, cycle) detected on device */
    CRDT_HIP_ESPACE = -6,   /* caller's output buffer too small (*out_len says how much) */
    CRDT_HIP_EIO = -7,      /* file / decompression / parse error */
    CRDT_HIP_ECOMM = -8     /* RCCL error */
};

typedef struct crdt_hip_ctx crdt_hip_ctx;
typedef struct crdt_hip_oplog crdt_hip_oplog;
typedef struct crdt_hip_trace crdt_hip_trace;
typedef struct crdt_hip_batch crdt_hip_batch;
typedef struct crdt_hip_replica crdt_hip_replica;
typedef struct crdt_hip_updates crdt_hip_updates;
typedef struct crdt_hip_logfile crdt_hip_logfile;

/* Anchor op log, structure of arrays (borrowed view).  Item k (0-based) has id k+1.
 * parent = origin_left id (0 = document start).  Document order (RGA): pre-order of the tree
 * parent -> children, siblings by (lamport, agent) descending.  cp = Unicode codepoint. */
typedef struct {
    uint32_t n;
    const uint32_t* parent;
    const uint32_t* origin_right; /* optional (may be NULL); not used by the RGA merge */
    const uint32_t* lamport;
    const uint16_t* agent;
    const uint8_t* deleted;
    const uint32_t* cp;
    /* optional (NULL: RGA).  Fugue order (SURVEY.md §8(a) s0 "side u8 (Fugue)"): side[k] != 0
     * makes item k a LEFT child of parent[k]; the document is then the in-order walk (left
     * children, the item, right children; each side by (lamport, agent) descending).  An RGA
     * log is the Fugue log without left children.  lamport must stay below 0xFFFFFFFF (a Fugue
     * log with lamport 0xFFFFFFFF, or with a left child of the document start, is malformed:
     * CRDT_HIP_EBADLOG on every path that takes a view).
     * ABI 2 added this field at the end of the struct: a caller written against ABI 1 must
     * zero-initialise the whole view (`crdt_hip_oplog_view v = {0};`) and check
     * crdt_hip_abi_version() == CRDT_HIP_ABI_VERSION, or a garbage `side` makes its log a Fugue
     * log. */
    const uint8_t* side;
} crdt_hip_oplog_view;

/* Per-stage device time of the last merge (HIP events on the context's stream), in ns,
 * summed over every wave of the call, plus work counters. */
typedef struct {
    uint64_t items;        /* op-log items merged */
    uint64_t docs;         /* documents merged */
    uint64_t text_bytes;   /* merged bytes produced */
    uint64_t runs;         /* runs (unary chains of consecutive items) the items collapsed to */
    uint32_t waves;        /* device waves the call was split into */
    uint32_t nstages;      /* valid entries in stage_ns / stage_launches */
    uint64_t stage_ns[16];
    uint32_t stage_launches[16];
    uint64_t total_ns;     /* first event to last event of the call */
} crdt_hip_stats;

/* Stage indices of crdt_hip_stats.stage_ns (one HIP-event interval per kernel group). */
enum {
    CRDT_HIP_STAGE_CLASSIFY = 0, /* level 0: seq/jump bits, weights, per-tile UTF-8           */
    CRDT_HIP_STAGE_RUNS = 1,     /* level 0: head bitvector, tile scan, run records, text     */
    CRDT_HIP_STAGE_SORTB = 2,    /* level 1 (radix): sort of the (run, next sibling) pairs by
                                    run id, and the run records in run order                  */
    CRDT_HIP_STAGE_COUNT = 3,    /* level 1: child counts (counting) or the digit histograms
                                    of the sort by parent run (radix)                         */
    CRDT_HIP_STAGE_SCAN = 4,     /* level 1: segment starts / radix bucket starts             */
    CRDT_HIP_STAGE_PLACE = 5,    /* level 1: runs grouped by parent run: placement (counting)
                                    or LDS-staged onesweep radix passes                       */
    CRDT_HIP_STAGE_LINK = 6,     /* level 1: sibling order of each group, first children      */
    CRDT_HIP_STAGE_WALK1 = 7,    /* level 1: Euler-tour sublist sums and each run's offset in
                                    its sublist (text mode: each sublist's text staged in walk
                                    order instead)                                            */
    CRDT_HIP_STAGE_RANK = 8,     /* level 1: ranking of the splitter lists                    */
    CRDT_HIP_STAGE_WALK2 = 9,    /* level 1: per-document totals (text mode: and the staged
                                    sublist texts copied to their documents)                  */
    CRDT_HIP_STAGE_EXPAND = 10,  /* runs copy their UTF-8 to their document offset (global
                                    level 1: offset in the sublist + the sublist's prefix)    */
    CRDT_HIP_STAGE_DIGEST = 11,  /* per-document tree digest                                  */
    CRDT_HIP_STAGE_DOCTREE = 12, /* level 1 in LDS: whole run tree of a document per workgroup
                                    (replaces stages 3-9 when every document fits)           */
    CRDT_HIP_STAGE_TEXT = 13,    /* text scatter after a k_doctree in scatter mode: the tiles'
                                    slot-order text to the documents (k_tscatter)            */
    CRDT_HIP_STAGE_ENCODE = 14,  /* raw SoA mode (crdt_hip_batch_raw): the input encoding derived
                                    from the raw columns inside the merge (k_raw_encode + the
                                    compact nsq list)                                        */
    CRDT_HIP_NSTAGES = 15
};

/* ---- library / context ----------------------------------------------------------------- */
int crdt_hip_abi_version(void);
int crdt_hip_device_count(int* out);
int crdt_hip_init(int device, crdt_hip_ctx** out);
int crdt_hip_destroy(crdt_hip_ctx* ctx);
const char* crdt_hip_last_error(const crdt_hip_ctx* ctx);
/* Tuning: "splitter_stride" of the global list ranking (power of two, 16..4096; default 16),
 * "max_wave_slots" per device wave (default 2^30), and "level1": 0 = per-document LDS merge of
 * the run tree whenever every document of a wave fits a workgroup's LDS (default), 1 = always
 * the global (multi-kernel) level-1 path, and "lanes" (1..8, default 2): waves of a multi-wave
 * merge run concurrently on that many streams, each with its own scratch (1 = one after the
 * other), "lane_gate" (default 1: lanes take turns at the HBM-bound level 0), "plan_cache"
 * (default 1: a merge of logs merged before enqueues every wave with the launch plan the earlier
 * merge learnt, checked on the device, and waits once instead of after each wave's level 0),
 * "l1_split" (default 0; 1: such enqueued waves run level 1 on a low-priority stream of their
 * lane, so that the next wave's level 0 is favoured when the two compete for the CUs),
 * "tail_wave_div" (default 0; k: a merge of several waves ends with a wave of at most
 * max_wave_slots / k slots), "xcd_order" (default 1: XCD-aware tile order in level 0),
 * "group_docs" (replica batches: 1 = documents placed in slots base by base, each base's
 * replicas in waves of their own, so that only the waves of a base whose run trees exceed the
 * per-document LDS level 1 take the global one; results stay in the caller's order; default 0),
 * "runs_slots" (k_runs slots per thread, 16, 32 or 64; default 32),
 * "stile_text" (default 2: the per-document merge stages text from the per-tile segments by
 * LDS-DMA, tile by tile; 1: by loads and shifts into one contiguous image; 0: from the slot-order
 * text k_runs then writes),
 * "nsq_list" (the compact list of the parents and keys of the items without the previous-slot
 * flag: 1 (default) = resident batches, and replicas of at least 2^22 slots, whose merges rebuild
 * it; 2 = every replica too; 0 = never), "contraction" (run contraction of RGA waves, decided
 * when a batch is built or logs are uploaded: 0 = by the input (default: no contraction when at
 * least 3/4 of a wave's items lack the previous-slot flag), 1 = always, 2 = never; replica
 * merges, which count no flags, contract under 0 and 1 and never under 2), "l1_group"
 * (sibling grouping of the global level 1: 0 = by counting when the wave's largest document has
 * at most 2^16 runs or the wave at most 2^23, else by radix sorts (default), 1 = always
 * counting, 2 = always radix sorts), "rs_digit_bits" (digit width of the radix sort by parent:
 * 0 = 10 bits where that takes fewer passes than 8 (default), 8, 10),
 * "fuse_text"
 * (default 1).  Results never depend on these. */
int crdt_hip_set_param(crdt_hip_ctx* ctx, const char* key, uint64_t value);

/* ---- op log: host-side resolver (positional patch -> anchor op) ---------------------------- */
int crdt_hip_oplog_new(crdt_hip_oplog** out);
/* Fugue anchors for every later insert (only on an empty log): an insert after left neighbour a
 * becomes a right child of a if a has none yet, else a left child of a's full-list successor.
 * A Fugue log's updates are wire version 2 (bit 31 of each cp word = left child); only Fugue
 * logs and Fugue replicas (crdt_hip_replica_new from a Fugue log's view, empty or not) take
 * them.  Version-1 (RGA) updates apply to either kind. */
int crdt_hip_oplog_set_fugue(crdt_hip_oplog* log, int on);
/* The agent id of this log's later local inserts (default 0).  Editors that exchange updates
 * need distinct agents: (lamport, agent) identifies an item. */
int crdt_hip_oplog_set_agent(crdt_hip_oplog* log, uint16_t agent);
int crdt_hip_oplog_clone(const crdt_hip_oplog* src, crdt_hip_oplog** out);
void crdt_hip_oplog_free(crdt_hip_oplog* log);
/* insert `nbytes` of UTF-8 at codepoint position `pos` (Upstream::insert). */
int crdt_hip_oplog_insert(crdt_hip_oplog* log, size_t pos, const char* utf8, size_t nbytes);
/* delete codepoints [start, end) (Upstream::remove). */
int crdt_hip_oplog_remove(crdt_hip_oplog* log, size_t start, size_t end);
/* Upstream::replace default (rope.rs:21-32): remove if end > start, then insert if non-empty. */
int crdt_hip_oplog_replace(crdt_hip_oplog* log, size_t start, size_t end, const char* utf8,
                           size_t nbytes);
/* Visible codepoints tracked by the resolver (host side; NOT the merged result). */
size_t crdt_hip_oplog_visible_len(const crdt_hip_oplog* log);
/* Borrowed SoA view, valid until the next mutation of `log`. */
int crdt_hip_oplog_get_view(const crdt_hip_oplog* log, crdt_hip_oplog_view* out);
/* Version token (items and delete ops so far) for encode_from. */
uint64_t crdt_hip_oplog_version(const crdt_hip_oplog* log);
/* Encode every op after `version` as one update (Downstream::upstream_updates, rope.rs:210-216).
 * If buf is NULL or cap too small, *out_len gets the needed size and ESPACE is returned. */
int crdt_hip_oplog_encode_from(const crdt_hip_oplog* log, uint64_t version, uint8_t* buf,
                               size_t cap, size_t* out_len);
/* Decode and append an update (Downstream::apply_update / decode_and_add, rope.rs:222-224). */
int crdt_hip_oplog_apply_update(crdt_hip_oplog* log, const uint8_t* buf, size_t len);

/* ---- trace loader (crdt-testdata load_testing_data / chars_to_bytes, main.rs:19-23) ---------- */
int crdt_hip_trace_load(const char* path, crdt_hip_trace** out);
void crdt_hip_trace_free(crdt_hip_trace* t);
/* Number of patches (TestData::len, main.rs:25) / txns. */
size_t crdt_hip_trace_len(const crdt_hip_trace* t);
size_t crdt_hip_trace_txns(const crdt_hip_trace* t);
/* Patch i: codepoint position, deleted codepoints, inserted UTF-8 (borrowed). */
int crdt_hip_trace_patch(const crdt_hip_trace* t, size_t i, size_t* pos, size_t* del,
                         const char** ins, size_t* ins_len);
int crdt_hip_trace_start_content(const crdt_hip_trace* t, const char** s, size_t* len);
int crdt_hip_trace_end_content(const crdt_hip_trace* t, const char** s, size_t* len);
/* Rewrite every patch from codepoint to UTF-8 byte offsets (TestData::chars_to_bytes). */
int crdt_hip_trace_chars_to_bytes(crdt_hip_trace* t);
/* Replay every patch into a fresh op log (the upstream loop body of main.rs:29-34). */
int crdt_hip_trace_resolve(const crdt_hip_trace* t, crdt_hip_oplog** out);
/* The same replay with Fugue anchors (crdt_hip_oplog_set_fugue). */
int crdt_hip_trace_resolve_fugue(const crdt_hip_trace* t, crdt_hip_oplog** out);
/* crdt_hip_trace_resolve of n traces on up to `threads` host threads (0: one per trace, capped
 * by the hardware), documents being independent.  out[i] receives trace
 * i's op log; on an error every out[i] is null and the first error is reported. */
int crdt_hip_trace_resolve_many(const crdt_hip_trace* const* traces, uint32_t n, uint32_t threads,
                                crdt_hip_oplog** out);

/* ---- binary files (skip gunzip + JSON; map resolved logs) ------------
 * Trace cache: the parsed trace in one flat file; crdt_hip_trace_load reads either format
 * (recognised by the file's magic), so a cache is a drop-in for the .json.gz path of
 * load_testing_data (main.rs:19,52).  Op-log file: the resolved anchor log as 64-byte-aligned
 * SoA arrays (a Fugue log's file is version 2 and adds its side column; its view has `side`).
 * Files are written to `path`.tmp and renamed. */
int crdt_hip_trace_save(const crdt_hip_trace* t, const char* path);
int crdt_hip_oplog_save(const crdt_hip_oplog* log, const char* path);
/* An editable op log read from a file (positional edits rebuild the resolver index first). */
int crdt_hip_oplog_load(const char* path, crdt_hip_oplog** out);
/* Map an op-log file read-only: *view points into the mapping (no copy) and stays valid until
 * crdt_hip_logfile_close.  The view can be passed to crdt_hip_merge*, crdt_hip_batch_create and
 * crdt_hip_replica_new. */
int crdt_hip_logfile_open(const char* path, crdt_hip_logfile** out, crdt_hip_oplog_view* view);
int crdt_hip_logfile_close(crdt_hip_logfile* f);

/* ---- synthetic op logs -------------------------------- */
/* 64-agent concurrent interleaved edits; `n_items` inserts, ~20% deletes, splitmix64 seed. */
int crdt_hip_synth_agents(uint32_t n_items, uint32_t agents, uint64_t seed, crdt_hip_oplog** out);
/* single document: parent of item i is i-1 with probability p_chain_pct/100, else uniform in
 * [0, i-1]; deleted ~ Bernoulli(del_pct/100); cp = 'a' + h % 26; lamport = i; agent = i % 64. */
int crdt_hip_synth_tree(uint32_t n_items, uint32_t p_chain_pct, uint32_t del_pct, uint64_t seed,
                        crdt_hip_oplog** out);
/* Visible items (= merged bytes) of that log, counted without building it. */
int crdt_hip_synth_tree_visible(uint32_t n_items, uint32_t del_pct, uint64_t seed, uint64_t* out);

/* ---- merge (device) --------------------------------------------------------------------- */
/* Merge one op log to its document: UTF-8 into out[0..cap), byte length in *out_len, tree
 * digest in *digest (either may be NULL).  If out is NULL only length/digest are produced. */
int crdt_hip_merge(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* log, uint8_t* out, size_t cap,
                   size_t* out_len, uint64_t* digest);
/* Upstream::len (rope.rs:16-19, 133-136) without copying the document back: merge one op log on
 * the device and return the merged text's codepoints (counted on the device from the merged
 * bytes), its UTF-8 length and its tree digest (each may be NULL). */
int crdt_hip_merge_len(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* log, uint64_t* codepoints,
                       uint64_t* bytes, uint64_t* digest);
/* Merge n independent op logs; digests[i], lens[i] per log.  stats may be NULL. */
int crdt_hip_merge_batch(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* logs, uint32_t n,
                         uint64_t* digests, uint64_t* lens, crdt_hip_stats* stats);
/* Pre-order of every item (tombstones included), ids 1..n, into order[0..n) (test hook for
 * the Euler-tour + list-ranking kernels). */
int crdt_hip_merge_order(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* log, uint32_t* order);

/* ---- device-resident replica batches (bench config 3) ------------------------------------- */
/* Upload `nbases` base logs once, then materialise `replicas` independent HBM copies of each
 * (document r uses base r % nbases).  relabel: 0 = ids kept, 1 = per-replica rotation of item
 * ids (locality kept), 2 = per-replica pseudo-random permutation of item ids (seeded by seed
 * and the replica index).  Parents are relabelled; lamport/agent kept, so every replica of a
 * base must merge to the base's document. */
int crdt_hip_batch_create(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* bases, uint32_t nbases,
                          uint32_t replicas, uint32_t relabel, uint64_t seed,
                          crdt_hip_batch** out);
/* A one-document batch generated on the device: crdt_hip_synth_tree's log (same parameters,
 * same items) without a host copy, for the 1 G-item config. */
int crdt_hip_batch_synth_tree(crdt_hip_ctx* ctx, uint32_t n_items, uint32_t p_chain_pct,
                              uint32_t del_pct, uint64_t seed, crdt_hip_batch** out);
int crdt_hip_batch_free(crdt_hip_batch* b);
int crdt_hip_batch_info(const crdt_hip_batch* b, uint64_t* docs, uint64_t* items,
                        uint64_t* device_bytes);
/* Merge every document of the batch (resident inputs); digests/lens sized to docs (may be
 * NULL). */
int crdt_hip_batch_merge(crdt_hip_ctx* ctx, crdt_hip_batch* b, uint64_t* digests,
                         uint64_t* lens, crdt_hip_stats* stats);
/* Raw SoA mode of a resident RGA batch (the companion line that prices the input encoding): keep
 * the reference-shaped columns (lamport u32, agent u16, deleted u8, codepoint u32 per item, beside
 * the parent column) and derive the engine's input format from them on the device at every
 * crdt_hip_batch_merge: the sibling key, the 3-byte codepoint word with its tombstone and
 * previous-slot flags, and the compact list of the items without that flag (stage
 * CRDT_HIP_STAGE_ENCODE).  on = 0 leaves the mode (the columns are kept until the batch is freed).
 * Replaces no reference interface: the reference's op log is its own in-memory format
 * (rope.rs:116-130 builds it). */
int crdt_hip_batch_raw(crdt_hip_ctx* ctx, crdt_hip_batch* b, int on);

/* ---- device-resident replicas: Downstream on the device ------------------------------------
 * A replica is an op log resident in HBM that receives encoded updates and is merged where it
 * lies.  Replaces diamond-types' decode_and_add (Dt Downstream, rope.rs:222-224) for the
 * downstream bench group (main.rs:63-69: clone the initial CRDT, apply every update, len()).
 * Updates are in the wire format of crdt_hip_oplog_encode_from; they are decoded on the device,
 * a whole batch per call, with crdt_hip_oplog_apply_update's semantics (ids already known are
 * skipped; an update must be causally ready: its first id <= known ids + 1).  Unlike the
 * host decoder, a batch that fails validation changes nothing.  A replica belongs to the
 * context that created it. */
/* New replica holding `init` (NULL: empty, = Downstream's from_str("")). */
int crdt_hip_replica_new(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* init,
                         crdt_hip_replica** out);
/* Device-to-device copy (Downstream: Clone, main.rs:64). */
int crdt_hip_replica_clone(crdt_hip_ctx* ctx, const crdt_hip_replica* src,
                           crdt_hip_replica** out);
int crdt_hip_replica_free(crdt_hip_replica* r);
/* Apply updates i = 0..n-1, update i = buf[offsets[i], offsets[i+1]) (n + 1 offsets, each a
 * multiple of 4, offsets[n] <= len < 4 GiB), in order (apply_update, rope.rs:222-224).
 * Same validation as crdt_hip_oplog_apply_update, with one documented difference: the device
 * replica keeps tombstone bits, not the host log's ordered list of delete ops (which
 * encode_from re-sends by index), so it does not refuse an update whose first delete index lies
 * beyond the deletes it has seen ("missing deletes" on the host).  Tombstoning a known item is
 * order-free, so the documents agree once both have every update
 * (tests/test_gpu_replica.py::test_gap_in_deletes_host_rejects_device_accepts). */
int crdt_hip_replica_apply_updates(crdt_hip_ctx* ctx, crdt_hip_replica* r, const uint8_t* buf,
                                   size_t len, const uint64_t* offsets, uint32_t n);
/* A batch of encoded updates (layout as crdt_hip_replica_apply_updates) uploaded to HBM once:
 * Downstream's `updates` vector held on the device (main.rs:58), so that applying it to a fresh
 * clone every iteration (main.rs:64-67) moves no bytes over PCIe. */
int crdt_hip_updates_upload(crdt_hip_ctx* ctx, const uint8_t* buf, size_t len,
                            const uint64_t* offsets, uint32_t n, crdt_hip_updates** out);
int crdt_hip_updates_free(crdt_hip_updates* u);
/* crdt_hip_replica_apply_updates with a resident batch (same semantics and validation). */
int crdt_hip_replica_apply_resident(crdt_hip_ctx* ctx, crdt_hip_replica* r,
                                    const crdt_hip_updates* u);
/* Items held, visible codepoints (Upstream::len, rope.rs:16-19) and visible UTF-8 bytes. */
int crdt_hip_replica_info(const crdt_hip_replica* r, uint64_t* items,
                          uint64_t* visible_codepoints, uint64_t* visible_bytes);
/* Merge the replica to its document (as crdt_hip_merge: out may be NULL). */
int crdt_hip_replica_merge(crdt_hip_ctx* ctx, crdt_hip_replica* r, uint8_t* out, size_t cap,
                           size_t* out_len, uint64_t* digest);

/* The downstream closure (main.rs:63-69) in one call: a copy of `init` (clone, :64) receives
 * every update of the resident batch `u` (apply_update, :65-67) and is merged (len(), :68).
 * Returns the merged text's codepoints, UTF-8 bytes and tree digest; `init` is unchanged.  The
 * context keeps a work replica per (init, u) and the sizes the last replay produced: the merge
 * is planned with them and enqueued right behind the decode (one host wait for the closure), a
 * device check compares them with the decode's counters, and on a mismatch the replica is merged
 * again with the real sizes.  A batch that fails validation returns EBADLOG. */
int crdt_hip_replica_replay(crdt_hip_ctx* ctx, const crdt_hip_replica* init,
                            const crdt_hip_updates* u, uint64_t* codepoints, uint64_t* bytes,
                            uint64_t* digest);
/* Downstream's len() (main.rs:68 asserts it; rope.rs:135 materialises): merge the replica and
 * return the merged text's codepoints (counted on the device), UTF-8 bytes and tree digest. */
int crdt_hip_replica_merge_len(crdt_hip_ctx* ctx, crdt_hip_replica* r, uint64_t* codepoints,
                               uint64_t* bytes, uint64_t* digest);

/* Incremental len(): the replica keeps its document order and text between
 * calls, and the items appended since the previous call are ranked alone when every one of them
 * with an old parent has a key (lamport, agent) above every older item's (local edits; updates
 * that race no older op), at most 4096 of them; deletes only re-weigh.  Anything else merges in
 * full (engine ORDER mode) and rebuilds the state.  Returns the merged text (out may be NULL),
 * its UTF-8 bytes and codepoints; *path = 1 for the incremental path, 0 for a full merge.
 * Replaces the from-scratch checkout_tip of Dt::len (rope.rs:135) for a caller that asks for the
 * length every K patches (main.rs:35 / :68 with len() inside the loop). */
int crdt_hip_replica_merge_inc(crdt_hip_ctx* ctx, crdt_hip_replica* r, uint8_t* out, size_t cap,
                               size_t* out_len, uint64_t* codepoints, uint32_t* path);

/* ---- multi-GPU (RCCL over xGMI): digest/counter exchange only ----------------------------- */
int crdt_hip_comm_unique_id(uint8_t id[128]);
int crdt_hip_comm_init(crdt_hip_ctx* ctx, int nranks, int rank, const uint8_t id[128]);
/* All-gather `count` u64 from every rank into recv[nranks * count] (rank-major). */
int crdt_hip_allgather_u64(crdt_hip_ctx* ctx, const uint64_t* send, size_t count,
                           uint64_t* recv);
int crdt_hip_comm_destroy(crdt_hip_ctx* ctx);

/* ---- helpers ------------------------------------------------------------------------------ */
uint64_t crdt_hip_xxh64(const void* data, size_t len, uint64_t seed);
uint64_t crdt_hip_tree_digest(const uint8_t* text, size_t len);

#ifdef __cplusplus
}
#endif
#endif
