// oplog.hpp — host-side resolver: positional patches -> anchor op log (SoA).
//
// Replaces the positional half of diamond-types' OpLog::add_insert / add_delete_without_content
// (called from the Dt adapter, /root/reference/src/rope.rs:116-131).  Conventions (SURVEY.md
// §4.2): an insert at visible codepoint position p is anchored to the p-th visible item
// (origin_left; id 0 = document start) and placed immediately after it, before any tombstones
// that follow it; origin_right = the item that followed origin_left (tombstones included, NIL
// at the end); char k > 0 of a multi-char insert is anchored to char k-1; every deleted
// codepoint is tombstoned exactly once.  lamport = max lamport seen + 1 per item, agent =
// the log's local agent.  With RGA ordering (siblings by (lamport, agent) descending) the
// resolver's sequence equals the merged document order at every step.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace crdt {

// Op-log columns: vectors whose growth leaves new elements default-initialised (uninitialised
// for these integer types) instead of zero-filled: the resolver sizes every column once to the
// trace's bound and writes each item by index (OpLog::replay), so a zero fill would be a second
// pass over the columns.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using Column = std::vector<T, DefaultInitAlloc<T>>;

// Update wire format (OpLog::encode_from / apply_update, decoded on the device by replica.hip).
constexpr uint32_t kUpdateMagic = 0x55445243u;  // "CRDU"
constexpr uint32_t kUpdateVersion = 1;
// A Fugue log's updates: the same layout, with bit 31 of cp[k] = side[k] (1: left child).
// Only Fugue logs and replicas accept them.
constexpr uint32_t kUpdateVersionFugue = 2;
constexpr uint32_t kUpdateSideBit = 0x80000000u;

class OpLog {
public:
    // ---- SoA (index k holds item id k+1) ----
    Column<uint32_t> parent, oright, lamport, cp;
    Column<uint16_t> agent;
    Column<uint8_t> deleted;
    Column<uint32_t> del_ops;  // target id of every delete op, in op order
    // Fugue mode (set on an empty log): side[k] = 1 if item k+1 is a LEFT child of parent[k].
    // An insert after left neighbour a (full-list successor b) is a right child of a when a has
    // no right child yet, else a left child of b (the leftmost node of a's right subtree): the
    // resolver's sequence is then the Fugue in-order at every step.  Empty in RGA mode.
    std::vector<uint8_t> side;
    bool fugue = false;
    uint16_t local_agent = 0;
    uint32_t max_lamport = 0;

    OpLog();
    uint32_t size() const { return (uint32_t)parent.size(); }
    uint64_t visible() const { return nvis_; }

    // Upstream::insert / remove (codepoint offsets).  Return "" or an error message.
    std::string insert(uint64_t pos, const uint32_t* cps, size_t k);
    std::string insert_utf8(uint64_t pos, const char* s, size_t nbytes);
    std::string remove(uint64_t start, uint64_t end);

    // The upstream loop of one editing trace (main.rs:28-36: replace = remove then insert per
    // patch, rope.rs:21-32) as one call: patches as (pos, del, ins_off, ins_len) in codepoints,
    // ins the concatenated inserted UTF-8 (ins_total bytes: every patch's text lies inside).
    // RGA logs run a fused loop over columns sized once; Fugue (or stale) logs take insert /
    // remove per patch.  "" or an error message.
    std::string replay(const uint64_t* patches, size_t n, const char* ins, size_t ins_total);

    // Downstream wire format (see oplog.cpp for the layout).
    uint64_t version() const { return ((uint64_t)size() << 32) | (uint32_t)del_ops.size(); }
    std::vector<uint8_t> encode_from(uint64_t version) const;
    std::string apply_update(const uint8_t* buf, size_t len);

    // Append a fully-specified item (synthetic generators / decoding); marks the positional
    // index stale.
    void push_item(uint32_t par, uint32_t orr, uint32_t lam, uint16_t ag, uint8_t del,
                   uint32_t c, uint8_t sd = 0);
    void mark_deleted(uint32_t id);
    // For bulk builders that fill the SoA directly.
    void mark_stale() { stale_ = true; }
    void reset_visible(uint64_t v) { nvis_ = v; }
    void reserve(size_t items, size_t dels = 0);

private:
    // RGA positional index: the visible items in document order as a gap buffer of spans (runs
    // of consecutive ids; typing extends the span before the gap), the gap at the last edit and
    // the visible items before it (gvis_), so an edit next to the previous one moves nothing and a
    // jump moves the spans in between, not the items; and the full-list successor of every item
    // (tombstones included; nxt_[0] = the first item) for origin_right.  Fugue logs use the span
    // index below: an insert there needs to know whether its left neighbour has a right child.
    struct GSpan {
        uint32_t id, len;
    };
    Column<GSpan> gb_;             // gap [g0_, g1_)
    size_t g0_ = 0, g1_ = 0;
    uint64_t gvis_ = 0;            // visible items in gb_[0, g0_)
    Column<uint32_t> nxt_;         // per id 0..n: next item in the full list (NIL: last)
    void gb_move(uint64_t pos);    // the gap at visible position pos (a span split if needed)
    void gb_reserve(size_t k);
    std::string insert_rga(uint64_t pos, const uint32_t* cps, size_t k);
    std::string remove_rga(uint64_t start, uint64_t end);
    std::string rebuild_index_rga(const std::vector<uint32_t>& order);

    // Positional index (Fugue): the document sequence (tombstones included) as spans of consecutive
    // item ids that are also consecutive in document order and share one deleted state, packed
    // into chunks of at most kSpanMax spans with a Fenwick tree over the chunks' visible counts.
    struct Span {
        uint32_t id;  // first item id
        uint32_t n;   // bit 31: deleted; low 31 bits: length
        uint32_t len() const { return n & 0x7FFFFFFFu; }
        bool del() const { return (n >> 31) != 0; }
    };
    struct Chunk {
        std::vector<Span> s;
        uint32_t vis = 0;
    };
    std::vector<Chunk> chunks_;
    // Fenwick tree over chunks_[i].vis; a chunk split shifts every later chunk, so the tree is
    // rebuilt lazily, at the next lookup that misses the hints (not at every split)
    mutable std::vector<int64_t> fen_;
    mutable bool fen_dirty_ = false;
    std::vector<uint32_t> cps_;  // scratch for insert_utf8
    std::vector<uint8_t> hasright_;  // Fugue: item (id) already has a right child
    uint64_t nvis_ = 0;
    // Chunk of the last lookup and the visible items before it.  Edits only change counts at or
    // after the chunk they start in and splits append after it, so the hint stays exact.
    mutable size_t hint_c_ = SIZE_MAX;
    mutable uint64_t hint_base_ = 0;
    // Span of the last lookup inside hint_c_ and the visible items of the chunk before it: edits
    // change spans only at or after it (tombstone spans merging into it count 0), so a lookup at
    // or after it scans on from there.  Dropped when a split moves it to another chunk.
    mutable size_t hint_si_ = SIZE_MAX;
    mutable uint64_t hint_vb_ = 0;
    bool stale_ = false;  // positional index must be rebuilt (after remote items arrived)

    void fen_build() const;
    void fen_add(size_t i, int64_t d);
    size_t fen_find(uint64_t& p) const;  // chunk holding the p-th visible item (p >= 1)
    Chunk new_chunk() const;
    bool split_chunk(size_t c);  // true if chunk c was split in two
    std::string rebuild_index();
    std::string rebuild_index_fugue();
    void index_append(uint32_t v);
    // p-th visible item (p >= 1): chunk c, span si, offset off inside the span.
    bool find_visible(uint64_t p, size_t& c, size_t& si, uint32_t& off) const;
    uint32_t first_id_from(size_t c, size_t si) const;  // first item at or after (c, si), or NIL
    size_t delete_in_span(Chunk& ch, size_t si, uint32_t off, uint32_t take);
};

}  // namespace crdt
