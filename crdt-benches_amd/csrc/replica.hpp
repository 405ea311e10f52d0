// replica.hpp — Downstream on the device: an op log resident in HBM that receives encoded
// updates and is merged where it lies.
//
// Replaces diamond-types' OpLog::decode_and_add (the Dt Downstream adapter,
// /root/reference/src/rope.rs:222-224) for the bench's downstream group
// (/root/reference/src/main.rs:63-69: clone the initial replica, apply every update, len()).
// Updates use the wire format of OpLog::encode_from (oplog.cpp); a batch of them is decoded by
// the kernels in replica.hip straight into the replica's slot arrays, and the replica is then
// merged by the engine like any resident document (one document, slot k = item id k).
#pragma once
#include <cstdint>
#include <vector>

#include "engine.hpp"

namespace crdt {

// Incremental merge state of a replica (incr.hip, crdt_hip_replica_merge_inc): the document
// order of the items 0..n it covers (tombstones included; rank 0 = the document start), its
// inverse, and the merged text.
constexpr uint32_t kIncMax = 4096;  // most items a fast-path merge appends
struct IncState {
    bool valid = false;
    uint32_t n = 0;                  // items the order covers
    uint64_t cap = 0;                // entries of seq[0], seq[1], rank[0], rank[1]
    uint32_t* seq[2] = {nullptr, nullptr};  // rank -> slot (ping-pong: seq[cur] is current)
    int cur = 0;
    // slot -> rank, ping-pong like seq: a merge reads the old ranks of the new roots' parents in
    // every workgroup while the splices of other workgroups write the new ranks, so they are
    // two arrays (rank[cur] read, rank[cur ^ 1] written)
    uint32_t* rank[2] = {nullptr, nullptr};
    // (Fugue replicas) 1 bit per slot: the item has a left child (a new left child of an old
    // item goes right before it only while it has none)
    uint32_t* hasl = nullptr;
    // per new item (kIncMax): the anchor rank found by k_inc_search for a root whose key is not
    // above every old key (0xFFFFFFFF: the search ran out of range)
    uint64_t* hanc = nullptr;
    uint32_t* lb_flag = nullptr;     // per tile of the order: look-back status, aggregate and
    uint64_t* lb_agg = nullptr;      //   inclusive prefix of the text (incr.hip inc_lookback)
    uint64_t* lb_inc = nullptr;
    uint64_t lb_cap = 0;
    uint8_t* text = nullptr;
    uint64_t text_cap = 0;
    uint64_t* ctl = nullptr;         // device counters (incr.hip ICtl)
    uint64_t* hres = nullptr;        // host-mapped result block (written by the last phase)
    uint64_t* dres = nullptr;        //   (its device address)
    uint64_t calls = 0;              // calls made (stamps the result block)
    std::vector<uint32_t> hseq;      // (rebuild staging)
    // (CRDT_INC_PROFILE) this state's profile events and phase timestamps
    hipEvent_t pev[2] = {nullptr, nullptr};
    uint64_t* tsp = nullptr;
    IncState() = default;
    IncState(const IncState&) = delete;
    IncState& operator=(const IncState&) = delete;
    ~IncState();
};

struct Replica {
    DeviceLogs logs;          // one document: slot 0 = document start, slot k = item k
    uint32_t n = 0;           // items present (ids 1..n)
    uint64_t vis_cp = 0;      // visible codepoints (Upstream::len, rope.rs:16-19)
    uint64_t vis_bytes = 0;   // visible UTF-8 bytes (= merged length)
    // update staging, grown on demand
    uint8_t* ubuf = nullptr;
    uint64_t ubuf_cap = 0;
    uint64_t* uoff = nullptr;  // n + 1 byte offsets
    uint4* uhdr = nullptr;     // per update {first id, items, deletes, data word offset}
    uint4* uscan = nullptr;    // per update {item offset, delete offset, known before, known after}
    uint64_t ucap = 0;
    uint4* ublk = nullptr;     // per 256-update block aggregates
    uint64_t ublk_cap = 0;
    uint32_t* imap = nullptr;  // per flattened item / delete of a batch: its update
    uint32_t* dmap = nullptr;
    uint64_t imap_cap = 0, dmap_cap = 0;
    uint64_t* uctl = nullptr;  // device counters (see replica.hip)
    uint64_t* hctl = nullptr;  // pinned host copy
    bool pending = false;      // a decode was enqueued and its counters not yet applied
    uint64_t gen = 0;          // bumped by every (re)allocation of the replica's device arrays
    uint64_t version = 0;      // bumped by every change of the contents
    std::vector<void*> graveyard;  // arrays replaced by a regrow, freed at the next wait
    IncState inc;              // incremental merge state (invalid until the first merge_inc)

    Replica() = default;
    Replica(const Replica&) = delete;
    Replica& operator=(const Replica&) = delete;
    ~Replica();
};

// A batch of encoded updates resident in HBM (uploaded once, applied to any replica of the
// context without a PCIe transfer).
struct UpdateBatch {
    uint8_t* buf = nullptr;   // the updates, concatenated (each 4-aligned)
    uint64_t* off = nullptr;  // n + 1 byte offsets
    uint64_t len = 0;
    uint32_t n = 0;
    uint32_t max_id = 0;      // largest item id the batch carries (read from the headers on the
                              // host at upload; 0 = unknown): sizes a replica before the decode

    UpdateBatch() = default;
    UpdateBatch(const UpdateBatch&) = delete;
    UpdateBatch& operator=(const UpdateBatch&) = delete;
    ~UpdateBatch();
};

int updates_upload(Engine& E, UpdateBatch& ub, const uint8_t* buf, uint64_t len,
                   const uint64_t* offsets, uint32_t n);
// As replica_apply, with the batch already in HBM.
int replica_apply_resident(Engine& E, Replica& r, const UpdateBatch& ub);
// The decode itself: buf/offsets are host pointers (uploaded first) or, if resident, device ones.
int replica_decode(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                   const uint64_t* offsets, uint32_t n, bool resident);

// Room for ids 0..items (slot arrays grow by doubling; new slots are padding).
int replica_reserve(Engine& E, Replica& r, uint64_t items);
// Initial contents (Downstream's initial CRDT; may be empty).
int replica_upload(Engine& E, Replica& r, const crdt_hip_oplog_view* v);
// dst = src, device to device (Downstream: Clone, main.rs:64).
int replica_copy(Engine& E, const Replica& src, Replica& dst);
// Decode and apply updates i = 0..n-1, update i = buf[offsets[i], offsets[i+1]), in order, with
// OpLog::apply_update's semantics.  A batch that fails validation changes nothing.
int replica_apply(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                  const uint64_t* offsets, uint32_t n);
// The decode without the wait: counters are copied to r.hctl in stream order (copy_counters)
// and applied by replica_settle.  max_id: the batch's largest id if known (0: bound from len).
int replica_decode_enqueue(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                           const uint64_t* offsets, uint32_t n, bool resident, uint32_t max_id,
                           bool copy_counters);
// Wait for an enqueued decode and apply its counters (errors: the batch changed nothing).
int replica_settle(Engine& E, Replica& r);

// The downstream closure (main.rs:63-69: clone the initial replica, apply every update, len())
// in one call: `work` receives a copy of `init`, the resident batch is decoded into it and it is
// merged.  The merge is planned with the sizes the previous replay of the same init and batch
// produced, enqueued right behind the decode (one wait for the whole closure); a device check
// compares those sizes with the decode's counters, and on a mismatch the host merges again with
// the real ones.
// Once the sizes are known the whole closure (copy, decode, check, merge, result copies) is
// captured as a hipGraph and replayed while nothing it points to is reallocated.
struct ReplayState {
    Replica work;
    const Replica* init = nullptr;
    const UpdateBatch* ub = nullptr;
    uint64_t init_version = 0;
    bool known = false;
    uint32_t n_after = 0;
    uint64_t bytes_after = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    std::vector<uint64_t> key;  // what the graph was captured with
    ReplayState() = default;
    ReplayState(const ReplayState&) = delete;
    ReplayState& operator=(const ReplayState&) = delete;
    ~ReplayState();
};
int replica_replay(Engine& E, const Replica& init, const UpdateBatch& ub, ReplayState& st,
                   uint64_t* cps, uint64_t* bytes, uint64_t* digest);

// Merge the replica's document (text may be null: length and digest only; cps: codepoints of
// the merged text, counted on the device).
int replica_merge(Engine& E, Replica& r, std::vector<uint8_t>* text, uint64_t* len,
                  uint64_t* digest, crdt_hip_stats* st, uint64_t* cps = nullptr);

// Incremental merge (incr.hip): the merged text (may be null), its UTF-8 bytes and codepoints;
// *path = 1 when only the items appended since the previous merge_inc were ranked, 0 for a
// full merge (the first call, a concurrent update, more than kIncMax new items, Fugue).
int replica_merge_inc(Engine& E, Replica& r, std::vector<uint8_t>* text, uint64_t* bytes,
                      uint64_t* cps, uint32_t* path);

}  // namespace crdt
