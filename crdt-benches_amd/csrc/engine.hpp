// engine.hpp — device merge engine: op logs resident in HBM in a slot layout, merged to their
// documents by the gfx950 kernels in engine.hip.
//
// Slot layout (DESIGN.md §Data layout): every document d owns slots [base_d, base_d + n_d + 1)
// of a wave, padded up to a multiple of 64: slot base_d is the document-start node (id 0), slot
// base_d + k holds item id k.  Input SoA arrays are indexed by slot.  Because every document
// starts on a multiple of 64, the chunk -> document table needs one entry per 64 slots.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "crdt_hip.h"

namespace crdt {

struct DocInfo {
    uint32_t n;          // items
    uint64_t text_cap;   // exact visible UTF-8 bytes (host-computed upper bound)
};

struct Wave {
    uint32_t first_doc, ndocs;
    uint64_t slot0;      // first slot of the wave
    uint32_t nslots;     // multiple of M
    uint32_t max_splitters_per_doc;
    uint64_t text_cap;   // bytes (docs aligned to 16)
    uint64_t leaf_cap;   // 4 KiB leaves
    uint64_t order_cap;  // u32 entries for ORDER mode
    uint64_t max_doc_text;  // largest document text bound of the wave
    uint64_t max_doc_slots = 0;  // largest document of the wave, in slots
    // Launch plan of the wave's level 1, learnt by a merge that waited for level 0 (run count,
    // runs of the largest document); valid until the logs are planned again.  A merge that
    // enqueues the wave with it does not wait for level 0: the device checks the plan (k_docmax
    // flags C_REPLAN if the wave outgrew it) and the host merges such a wave again.
    uint32_t hint_runs = 0, hint_rmax = 0;
    bool hint_lds = false;  // the wave took the per-document LDS level 1 with fused text
    // no run contraction (L0Args::nocon): most of the wave's items lack the previous-slot flag
    // (relabelled ids, uniformly random parents), so runs would not contract and level 0 skips
    // the parent scatter of the jump bits and the run-parent lookups; set with the wave's
    // encoding (Engine::build_nsq, Engine::upload) or forced by Engine::contraction
    bool nocon = false;
    uint64_t nsq_items = 0;  // items of the wave without the previous-slot flag (if known)
};

// Stage timing of one wave: an event at its start and after every stage that ran.
constexpr uint32_t kClockEvents = 24;
struct StageClock {
    hipEvent_t* ev = nullptr;              // kClockEvents events
    uint32_t n = 0;                        // events recorded
    uint8_t stage[kClockEvents] = {};      // stage timed by the interval ev[i] -> ev[i + 1]
};

// Level-1 launch configuration of a wave, from its run count and largest document.
struct L1Plan {
    uint32_t R = 0, rmax = 0;
    bool lds1 = false, fuse = false;
    bool wide = false;  // k_doctree_wide (32-bit keys, 14 runs per thread) instead of k_doctree
    // k_doctree stages each document's text from the per-tile segments k_classify wrote (stile),
    // so k_runs does not copy them into the slot-order text (sbytes): fused plans whose
    // documents span at most kDocTiles tiles
    bool stile_text = false;
    // k_doctree stops at the run offsets (wave-relative, in roff) and k_tscatter writes the text
    // from the tile segments: stile plans of waves with less than 4 GiB of text
    // (Engine::text_scatter); k_doctree then needs only the run tree's LDS (dyn_scatter)
    bool scatter = false;
    uint32_t rcap = 0, scap = 0;
    uint64_t dyn_bytes = 0, dyn_scatter = 0;
};

// The codepoint column: 3 bytes per slot, the codepoint (bits 0-20), the tombstone flag (bit 23)
// and a "parent is the previous slot" flag (bit 22) in one 24-bit value.  The level-0 stream
// reads this column and only the parents of slots without the flag: 3 + a few bytes per slot
// instead of 8.  The flag is a hint written with the parent: set only when the parent column
// holds the previous slot; a slot without it has its parent read and classified in full.
constexpr uint32_t kDelBit = 0x00800000u;
constexpr uint32_t kSeqBit = 0x00400000u;
// Fugue: the item is a LEFT child of its parent (bit 21; the previous-slot flag is then never
// set: a seq item is a right child of the slot before it)
constexpr uint32_t kLeftBit = 0x00200000u;
constexpr uint64_t kLeftKey = 1ull << 48;  // key bit of a left child (see engine.hip)
__host__ __device__ inline void cp3_put(uint8_t* b, uint64_t slot, uint32_t v) {
    b[3 * slot] = (uint8_t)v;
    b[3 * slot + 1] = (uint8_t)(v >> 8);
    b[3 * slot + 2] = (uint8_t)(v >> 16);
}
__host__ __device__ inline uint32_t cp3_get(const uint8_t* b, uint64_t slot) {
    return (uint32_t)b[3 * slot] | ((uint32_t)b[3 * slot + 1] << 8) | ((uint32_t)b[3 * slot + 2] << 16);
}
// bytes of the column for n slots (padded so that 16-byte loads of whole 16-slot groups and
// 16-byte copies stay inside it)
__host__ __device__ inline uint64_t cp3_bytes(uint64_t n) { return (3 * n + 63) & ~15ull; }

// Device-resident op logs in slot layout, planned into waves.
struct DeviceLogs {
    uint32_t log2m = 6;
    uint64_t total_slots = 0, cap_slots = 0;
    std::vector<DocInfo> docs;
    // (grouped replica batches) slot-order document -> the caller's document; empty: the same
    std::vector<uint32_t> api_doc;
    std::vector<uint64_t> doc_slot;  // global slot base per doc
    std::vector<Wave> waves;
    uint64_t items = 0;
    // device arrays (slot-indexed)
    uint32_t* parent = nullptr;
    uint64_t* key = nullptr;       // the item's id as a sibling key: lamport << 16 | agent
                                   //   (| 1 << 48 for a Fugue left child)
    bool fugue = false;            // some document has left children (Fugue logs)
    uint8_t* cp = nullptr;         // 3 bytes per slot: codepoint (bits 0-20) | tombstone (bit 23)
    uint2* docs_rel = nullptr;     // per doc {wave-relative base slot, n}
    uint32_t* doc_rank = nullptr;  // per document: its k_doctree workgroup within its wave
                                   //   (longest-processing-time order: costliest first)
    uint32_t* chunk_doc = nullptr; // per M-chunk of the whole slot space: wave-local doc index
    uint64_t cap_docs = 0, cap_chunks = 0;
    std::vector<uint64_t> tab_sig;  // the plan docs_rel / chunk_doc were last built for
    // Resident batches (Engine::build_nsq, part of the input encoding): the parents of the items
    // without the previous-slot flag, in slot order, and their prefix count per 64 slots
    // (nsq_pre[c] = such items in slots < 64 c).  k_classify streams a tile's range of it instead
    // of gathering the parent column.  Null for logs that change (uploads, replicas).
    uint32_t* nsq_par = nullptr;
    uint32_t* nsq_pre = nullptr;
    uint64_t* nsq_key = nullptr;   // beside nsq_par: the items' keys (k_runs reads a non-seq
                                   //   head's key there instead of gathering it)
    uint64_t nsq_items = 0;
    // the list matches the current slot layout and contents (plan() clears it; the arrays keep
    // their capacity, so that a replica rebuilds its list inside a captured replay)
    bool nsq_ok = false;
    uint64_t nsq_cap = 0, nsq_pre_cap = 0, nsq_sums_cap = 0;
    uint32_t* nsq_sums = nullptr;  // (scan scratch)
    uint64_t* nsq_mask = nullptr;  // (the nsq items of every 64-slot chunk, for the scatter)
    // Raw SoA mode (Engine::raw_keep, the companion line that prices the input encoding): the
    // reference-shaped columns beside the parent column, lamport u32, agent u16, deleted u8 and
    // codepoint u32 per slot; every merge first derives the key, the codepoint word with its
    // tombstone and previous-slot flags, and the compact nsq list from them on the device
    bool raw = false;
    uint32_t* raw_lam = nullptr;
    uint16_t* raw_agent = nullptr;
    uint8_t* raw_del = nullptr;
    uint32_t* raw_cp = nullptr;
    void release();
    ~DeviceLogs() { release(); }
};

class Engine {
public:
    Engine() = default;
    ~Engine();
    std::string init(int device);

    int device = 0;
    hipStream_t stream = nullptr;     // every launch of the engine (high priority)
    hipStream_t stream_l1 = nullptr;  // level 1 + tail of enqueued waves (low priority: l1_split)
    uint32_t log2m = 4;                    // level-1 splitter stride M = 2^log2m
    bool log2m_set = false;                // set by the caller; else chosen per wave from R
    uint64_t max_wave_slots = 1ull << 30;
    // last wave of a multi-wave merge <= max / div (0: off; off since the dead-run drop and the
    // smaller k_doctree: 12.37 -> 12.09 ms at the headline config, tools/sweep_sched.sh)
    uint32_t tail_wave_div = 0;
    bool level1_global = false;            // never use the per-document LDS level 1
    // Waves merged at once by a multi-wave merge, each on a lane of its own: a helper engine
    // (non-blocking stream + scratch) driven by its own host thread.  The latency-bound level 1
    // of one wave then overlaps the HBM-bound level 0 of another.
    uint32_t lanes = 2;
    bool l0_gated = true;  // lanes take turns at level 0 (see run_wave)
    // Enqueued waves (merge_async) run level 1 and the tail on stream_l1, created with the lowest
    // stream priority, so that when one wave's latency-bound level 1 and the next wave's HBM-bound
    // level 0 compete for the CUs, the dispatcher favours level 0 (the chain that bounds a merge).
    // (off by default since the round-2 level-0 work: 12.09 -> 12.05 ms, within noise; the
    // parameter stays for the A/B)
    bool l1_split = false;
    // Merges of logs merged before enqueue every wave with its learnt plan and wait once at the
    // end (merge_async) instead of after each wave's level 0.
    bool plan_cache = true;
    bool plan_shrink = false;  // test hook: enqueue with half the learnt plan (forces C_REPLAN)
    bool doctree_lds_max = false;  // experiment hook: k_doctree always takes the whole LDS
    bool fuse_text = true;         // k_doctree writes the text when it fits LDS (else k_expand)
    // the compact list of the non-seq items' parents and keys: 1 = resident batches (build_nsq)
    // and replicas of at least kNsqReplicaSlots slots (rebuilt by every merge: below that size
    // the rebuild's launches cost more than the gathers it saves, measured on the downstream
    // closures), 2 = every replica too, 0 = never (level 0 gathers the columns)
    uint32_t nsq_list = 1;
    static constexpr uint64_t kNsqReplicaSlots = 1ull << 22;
    // run contraction of RGA waves: 0 = by the wave's input (no contraction when at least
    // kNoconShare of its items lack the previous-slot flag), 1 = always, 2 = never
    uint32_t contraction = 0;
    // sibling grouping of the global level 1: 0 = by the largest document (counting up to
    // kCsrDocRuns runs, else radix sorts), 1 = always counting, 2 = always radix sorts
    uint32_t l1_group = 0;
    uint32_t rs_digit_bits = 0;  // sort A's digit width: 0 = 10 bits where that saves a pass, else 8
    std::string err;

    // Plan docs into waves and (re)allocate `L`'s arrays for them (contents undefined).
    // brk (optional, per document): 1 = start a new wave at this document
    int plan(DeviceLogs& L, const std::vector<DocInfo>& docs,
             const std::vector<uint8_t>* brk = nullptr);
    // Upload host views into `L` (plan first).  Synchronous.
    int upload(DeviceLogs& L, const crdt_hip_oplog_view* views, uint32_t n);
    // Build docs_rel / chunk_doc tables for L's plan.
    int upload_tables(DeviceLogs& L);

    enum Mode { TEXT = 0, ORDER = 1 };
    // Merge every wave of L.  digests/lens: per doc (host, may be null).  If text_out is set
    // (single-wave only), the merged bytes of the wave are copied back (docs concatenated,
    // each 16-aligned; offsets in text_offsets).
    // cps: per doc, codepoints of the merged text (counted on the device; may be null).
    int merge(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens, crdt_hip_stats* st,
              std::vector<uint8_t>* text_out = nullptr,
              std::vector<uint64_t>* text_offsets = nullptr, uint64_t* cps = nullptr);
    int merge_inner(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens,
                    crdt_hip_stats* st, std::vector<uint8_t>* text_out,
                    std::vector<uint64_t>* text_offsets, uint64_t* cps);

    // merge() of logs whose every wave has a learnt plan, in three phases so that the launches
    // can be captured in a graph: prepare (every allocation), enqueue (launches and copies only;
    // untimed: no events), then, after the caller waited for the stream, finish.
    struct AsyncMerge {
        uint32_t K = 1;
        bool timed = true;
        std::vector<Engine*> eng;
        std::vector<L1Plan> plans;
        std::vector<StageClock> clocks;
    };
    bool plans_known(const DeviceLogs& L) const {
        bool ok = plan_cache && !L.waves.empty();
        for (const Wave& w : L.waves) ok = ok && w.hint_lds;
        return ok;
    }
    int merge_async_prepare(DeviceLogs& L, AsyncMerge& m, bool timed);
    int merge_async_enqueue(DeviceLogs& L, AsyncMerge& m);
    int merge_async_finish(DeviceLogs& L, AsyncMerge& m, uint64_t* digests, uint64_t* lens,
                           uint64_t* cps, crdt_hip_stats* st);
    // bumped by every (re)allocation of scratch, this engine's or a lane engine's (a graph that
    // captured a multi-lane merge holds the lane engines' pointers too)
    bool xcd_order = true;  // XCD-aware tile order in k_classify / k_runs (engine.hip xcd_block)
    // fused plans stage text from the tile segments (L1Plan::stile_text): 1 by 16-byte loads and
    // funnel shifts into one contiguous image, 2 by LDS-DMA, tile by tile (engine.hip stage_glds)
    uint32_t stile_text = 2;
    // 1: stile plans leave the text to k_tscatter (L1Plan::scatter); 0: k_doctree phase C (the
    // default: the two measured equal on the RGA headline, 8.43 ms per step either way, and
    // phase C is 0.16 ms faster on the Fugue line)
    uint32_t text_scatter = 0;
    bool glds_late = false;  // test hook: k_doctree issues its LDS-DMA staging loads last
    // every LDS level 1 on k_doctree_wide (32-bit keys, 9 B of LDS per run instead of 15)
    bool doctree_k32 = false;
    // k_runs slots per thread: 16 (256 threads per tile), 32 (128) or 64 (one wave per tile,
    // 64-bit slot masks)
    uint32_t runs_slots = 32;
    bool group_docs = false;  // replicate(): documents in slots base by base (waves per base)
    uint64_t generation() const {
        uint64_t g = gen_;
        for (const auto& e : lane_eng_) g += e->generation() + 1;
        return g;
    }

    // One config-5 document generated on the device (synth.cpp synth_tree_item, item by item).
    int synth_tree(DeviceLogs& R, uint32_t n, uint32_t p_chain_pct, uint32_t del_pct,
                   uint64_t seed);

    // The compact nsq parent list of L (after its last plan; see DeviceLogs::nsq_par).
    int build_nsq(DeviceLogs& L);
    // raw SoA mode of resident logs (DeviceLogs::raw): keep the raw columns (once, untimed) /
    // derive the engine's input format from them (every merge, on the device)
    int raw_keep(DeviceLogs& L);
    int raw_encode(DeviceLogs& L);
    int nsq_reserve_prefix(DeviceLogs& L);
    void nsq_count_scan(DeviceLogs& L);
    void nsq_scan(DeviceLogs& L);
    void nsq_scatter(DeviceLogs& L);
    // Wave::nocon of every wave of L from its nsq_items and the contraction parameter.
    void set_contraction(DeviceLogs& L) const;
    // The compact nsq list of logs that change (replicas): room for every slot (nsq_reserve,
    // may allocate), then the list built by launches alone (nsq_launch, capturable).
    int nsq_reserve(DeviceLogs& L);
    int nsq_launch(DeviceLogs& L);
    void apply_shape_hints(DeviceLogs& L) const;
    static constexpr double kNoconShare = 0.75;

    // Materialise `replicas` relabelled copies of `bases` (already uploaded in B) into R.
    int replicate(DeviceLogs& B, DeviceLogs& R, uint32_t replicas, uint32_t relabel,
                  uint64_t seed);

private:
    // the stream the launch functions and the stage clock use (stream, or stream_l1 while an
    // enqueued wave's level 1 and tail are launched); events ordering the two streams
    hipStream_t cur_ = nullptr;
    hipEvent_t ev_l0_ = nullptr, ev_l1_ = nullptr;
    bool l1_pending_ = false;  // ev_l1_ marks this merge's last level 1 on stream_l1
    // level-0 scratch (per slot / per tile), grown on demand
    uint64_t cap_slots0_ = 0, cap_docs_ = 0, cap_text_ = 0, cap_leaves_ = 0;
    uint32_t* jbits_ = nullptr;
    uint16_t* nsqb_ = nullptr;
    uint64_t* wnib_ = nullptr;
    uint16_t* visb_ = nullptr;
    uint64_t* escm_ = nullptr;
    uint4* hrec_ = nullptr;
    uint8_t *stile_ = nullptr, *sbytes_ = nullptr;
    uint32_t* plist_ = nullptr;
    uint2 *tile_hw_ = nullptr, *tile_sums_ = nullptr;
    uint64_t cap_sbytes_ = 0;
    // per document
    uint32_t *doc_root_ = nullptr, *doc_p0_ = nullptr, *tlen_ = nullptr, *loff_ = nullptr;
    uint64_t *toff_ = nullptr, *leafh_ = nullptr, *ghash_ = nullptr;
    uint32_t *leafcp_ = nullptr, *gcp_ = nullptr;
    // result block of a wave: ctl (16 words) then one uint4 per document {bytes, codepoints,
    // digest lo, digest hi}; ctl_ and res_ point into it
    uint32_t* out_ = nullptr;
    uint4* res_ = nullptr;
    uint4* wgtab_ = nullptr;  // k_doctree workgroup descriptors (two uint4 per document)
    uint8_t* text_ = nullptr;
    uint8_t* doc_fused_ = nullptr;
    // level-1 scratch (per run / per splitter), grown on demand
    uint64_t cap_heads_ = 0, cap_runs_ = 0, cap_splitters_ = 0;
    uint32_t *r_head_ = nullptr, *r_pstart_ = nullptr, *r_parent_ = nullptr,
             *roff_ = nullptr;
    uint64_t* r_key_ = nullptr;
    uint32_t* ctl_ = nullptr;
    // radix-sort scratch of the global level 1 (engine.hip k_rs_*)
    uint64_t cap_rs_ = 0;
    uint4* rs_elem_[2] = {nullptr, nullptr};
    uint32_t *rs_status_ = nullptr, *rs_small_ = nullptr;
    uint2* rs_bigl_ = nullptr;
    uint32_t *deg_ = nullptr, *cstart_ = nullptr, *child_ = nullptr, *defer_ = nullptr,
             *bigl_ = nullptr, *scan_sums_ = nullptr;  // counting-path scratch (engine.hip k_count)
    uint64_t cap_csr_ = 0;
    bool l1_csr_ = false;      // the last global level 1 grouped siblings by counting
    uint8_t* wtmp_ = nullptr;  // text mode: the first 2^wtmp_log2_ bytes of every sublist's text
    uint64_t cap_wtmp_ = 0;    // (bytes)
    uint32_t wtmp_log2_ = 7;
    uint32_t tail_nspl_ = 0;   // splitters of the last global level 1 whose offsets are in rloc_
    bool tail_scatter_ = false;  // the last level 1 was k_doctree in scatter mode: k_tscatter
                                 //   next (0: k_expand reads roff_)
    hipEvent_t raw_ev_[2] = {nullptr, nullptr};  // (raw SoA mode: the encoding's interval)
    hipEvent_t up_ev_ = nullptr;  // after the copies of a one-wave upload (Engine::upload)
    bool up_pending_ = false;     //   not yet waited for: the staging is still being read
    uint32_t* ovf_ = nullptr;  // text mode: splitters whose sublist holds more than its slot
    uint64_t cap_ovf_ = 0;
    uint32_t rs_npass_ = 0, rs_npassB_ = 0;
    uint4* rec_ = nullptr;
    uint2* swn_ = nullptr;     // per splitter {sublist weight, next splitter}
    uint2* rloc_ = nullptr;    // per run: {offset in its sublist, the sublist} (global level 1)
    uint32_t* spref_ = nullptr;  // per splitter: exclusive prefix along its list
    uint2* sup_ = nullptr;     // super-splitters (engine.hip k_sup1): {weight, next}
    uint32_t* spred_ = nullptr;
    uint2* svp_[2] = {nullptr, nullptr};
    uint8_t* up_pin_ = nullptr;          // pinned staging of upload(): the encoded columns
    uint64_t cap_up_pin_ = 0;
    uint32_t* host_out_ = nullptr;       // pinned image of every wave's result block
    uint64_t cap_host_out_ = 0;          // bytes
    uint32_t probe_doc_ = 0;             // 1 + document whose k_doctree phases are printed
    uint64_t runs_ = 0;
    uint64_t gen_ = 0;
    std::vector<hipEvent_t> ev_;         // stage clock of a synchronous wave; merge start/end
    std::vector<hipEvent_t> wev_;        // stage clocks of every enqueued wave (merge_async)
    std::vector<std::unique_ptr<Engine>> lane_eng_;  // lanes 1..lanes-1 (lane 0 = this)
    std::mutex* l0_gate_ = nullptr;                  // set by merge_lanes

    // Launch plans learnt per wave shape (documents, slots, text bound, items): a new set of
    // logs of the same shape (the downstream loop merges a fresh clone every iteration) starts
    // from the plan an earlier merge learnt; the device checks it (C_REPLAN) as for any plan.
    struct WaveShape {
        uint32_t ndocs, nslots;
        uint64_t text_cap, order_cap, max_doc_text;
        bool nocon;
        bool operator==(const WaveShape& o) const {
            return ndocs == o.ndocs && nslots == o.nslots && text_cap == o.text_cap &&
                   order_cap == o.order_cap && max_doc_text == o.max_doc_text && nocon == o.nocon;
        }
    };
    struct ShapeHint {
        WaveShape shape;
        uint32_t runs, rmax;
    };
    std::vector<ShapeHint> shape_hints_;  // most recent first, at most kShapeHints
    static constexpr size_t kShapeHints = 64;
    static WaveShape shape_of(const Wave& w) {
        return WaveShape{w.ndocs, w.nslots, w.text_cap, w.order_cap, w.max_doc_text, w.nocon};
    }
    void learn_shape(const Wave& w);
    void forget_shape(const Wave& w);
    uint64_t* tab_slot_ = nullptr;   // upload_tables scratch (grown, never freed mid-merge)
    uint32_t* tab_local_ = nullptr;
    uint64_t cap_tab_ = 0;

    int merge_lanes(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens, uint64_t* cps,
                    crdt_hip_stats* st);
    int merge_async(DeviceLogs& L, uint64_t* digests, uint64_t* lens, uint64_t* cps,
                    crdt_hip_stats* st);
    int ensure_runs(uint64_t runs, uint64_t splitters);
    int ensure_radix(uint64_t runs);
    int ensure_csr(uint64_t runs);
    int ensure_splitters(uint64_t splitters);
    int ensure_scratch(const Wave& w);
    int ensure_host_out(const DeviceLogs& L);
    uint32_t* host_block(const DeviceLogs& L, uint32_t wi) const;
    int ensure_events(std::vector<hipEvent_t>& ev, size_t n);
    L1Plan plan_level1(const Wave& w, uint32_t R, uint32_t rmax, bool ord, bool force_global) const;
    // text written by the first walk (grid-wide level 1, TEXT mode: k_walk1 stages each sublist's
    // text, k_tcopy / k_walk_ovf place it) on waves without contraction; contracted waves keep
    // k_expand (their long runs and skewed sublist texts made the staged form 1.1-2.3x slower:
    // DESIGN.md §5b)
    static bool walk_text(const Wave& w, bool ord, const L1Plan& p) {
        return !p.lds1 && !ord && w.nocon;
    }
    int clock_mark(StageClock& c, int stage);
    // The launches of one wave, in stream order.
    int launch_runs(DeviceLogs& L, const Wave& w, bool ord);
    int launch_level0(DeviceLogs& L, const Wave& w, bool ord, bool copy_text, uint32_t cap_runs,
                      uint32_t cap_rmax,
                      StageClock& ck);
    // stile: k_doctree stages the text from the tile segments (k_runs did not copy it)
    int launch_lds_level1(DeviceLogs& L, const Wave& w, bool ord, const L1Plan& p, bool stile,
                          StageClock& ck);
    int launch_global_level1(DeviceLogs& L, const Wave& w, bool ord, const L1Plan& p,
                             StageClock& ck, uint32_t& rounds);
    int launch_tail(DeviceLogs& L, const Wave& w, bool ord, bool fused, StageClock& ck,
                    uint32_t* hblock);
    // After the wave's stream has drained: stage times, launch counts.
    int finish_wave(const Wave& w, bool ord, const L1Plan& p, uint32_t rounds, const StageClock& ck,
                    const uint32_t* hctl, std::vector<float>& stage_ms,
                    std::vector<uint32_t>& stage_launches);
    int run_wave(DeviceLogs& L, uint32_t wi, Mode mode, std::vector<float>& stage_ms,
                 std::vector<uint32_t>& stage_launches, bool force_global = false);
    void collect(const DeviceLogs& L, uint32_t wi, uint64_t* digests, uint64_t* lens,
                 uint64_t* cps, uint64_t& text_bytes) const;
    int fail(const char* what, hipError_t e);
};

}  // namespace crdt
