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

#include "engine.hpp"

namespace crdt {

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
    uint64_t* uctl = nullptr;  // device counters (see replica.hip)
    uint64_t* hctl = nullptr;  // pinned host copy

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
// Merge the replica's document (text may be null: length and digest only; cps: codepoints of
// the merged text, counted on the device).
int replica_merge(Engine& E, Replica& r, std::vector<uint8_t>* text, uint64_t* len,
                  uint64_t* digest, crdt_hip_stats* st, uint64_t* cps = nullptr);

}  // namespace crdt
