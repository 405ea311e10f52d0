// engine.hip — gfx950 kernels of the merge path and their host orchestration.
//
// Replaces diamond-types' OpLog::checkout_tip (/root/reference/src/rope.rs:134-136): anchor
// op log -> merged document.  Document order is the RGA order: pre-order of the tree
// item -> children (children = items whose origin_left is the item), siblings by (lamport,
// agent) descending.
//
// Two levels:
//  Level 0 streams over item slots in 4096-slot tiles.  A slot continues the run of the slot
//  before it iff its parent is that slot and that slot has no other child ("jump" child).  Such
//  runs are unary chains of the tree with consecutive ids, so their items are consecutive in
//  the document; on the josephg traces they hold 93-98 % of all items.  Run heads are recorded
//  in a rank bitvector (1 bit/slot + a u32 rank per 64 slots) and every run gets its parent run,
//  its key (lamport, agent of the head) and its weight (visible UTF-8 bytes).
//    k_classify    non-seq item bits (from the codepoint column's previous-slot flags), weight
//                  nibbles, each tile's UTF-8 compacted in slot order; jump bits and the
//                  tile's parent list from the parents of its non-seq items
//    k_heads       head bitvector words, per-tile head counts
//    k_tiles_*     exclusive scan of the per-tile (heads, weight) pairs
//    k_runs        run records (head slot, weight prefix, key, parent run by rank lookup),
//                  slot-order UTF-8
//  Level 1 merges the tree of runs:
//    k_rs_hist / k_rs_scan / k_rs_pass   LDS-staged LSD radix sort of (parent run, run id, key)
//                                        by parent run: sibling groups contiguous and keyed
//    k_rs_order / k_rs_big               sibling order: {run, next sibling} pairs, first children
//    k_rs_pass (sort B) / k_rs_records   the pairs by run id; the run records in run order
//    k_walk1 / k_sup1 / k_sup_step / k_sup2 (text mode: k_tcopy / k_walk_ovf)
//                                        Euler-tour list ranking (sublists from splitters
//                                        run id % M == 0, pointer jumping over the splitter
//                                        lists); weighted so the rank is each run's byte offset
//  Expansion and digest:
//    k_expand      runs copy their slot-order UTF-8 to run offset in the document
//    k_leafhash / k_docdigest  xxh64 tree digest per document
// The Euler tour is never materialised: succ(down v) = down(first_child v) or up v;
// succ(up v) = down(next_sibling v) or up(parent v).
#include "engine.hpp"

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>

#include "util.hpp"
#include "wave.hpp"

namespace crdt {

namespace {

constexpr uint32_t kNil = 0xFFFFFFFFu;
constexpr uint32_t kCpMask = 0x001FFFFFu;
constexpr int kBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;
constexpr uint32_t kDocAlignLog2 = 6;  // slot-level document alignment (chunk table: 1/64)
constexpr uint32_t kLeaf = 4096;
constexpr uint64_t kMaxWaveText = (1ull << 32) - (1ull << 20);  // weight prefixes are u32
constexpr int kBigGrid = 256;   // k_rs_big / k_sortbig workgroups
constexpr int kMidGrid = 4096;  // k_sortmid workgroups
// level-1 sibling grouping by counting (k_count ...) for waves whose largest document has at
// most this many runs (its child counts, placement and keys then stay within a few MB)
constexpr uint32_t kCsrDocRuns = 1u << 16;
constexpr uint32_t kCsrWaveRuns = 1u << 23;  // (or every wave this small: fewer launches)
constexpr int kBigThreads = 1024;

// ctl words (device, zeroed per wave)
enum Ctl {
    C_NBIGRUN = 0,  // (unused)
    C_NDEFER = 1,   // (CSR grouping) parents with 9 or more children
    C_ERR = 2,      // error bits: 1 bad parent, 2 walk overrun, 4 text overflow, 8 write out
                    //   of range, 16 unreachable runs (cycle)
    C_RTOTAL = 3,   // runs of the wave
    C_WTOTAL = 4,   // weight total of the wave
    C_RMAX = 5,     // most runs in one document
    C_VISITED = 6,  // runs passed by k_walk1
    C_UNFUSED = 7,  // documents whose text k_doctree left to k_expand
    C_NBIG = 9,     // (CSR grouping) parents with more than 64 children
    C_NOVF = 10,    // (text mode) sublists listed by k_tcopy for k_walk_ovf
    C_REPLAN = 8,   // the wave outgrew the launch plan it was enqueued with (runs / largest
                    //   document above the planned capacity): every later kernel of the wave
                    //   exits at once and the host merges the wave again with a fresh plan
};

// Level-0 scratch cleared in one launch: the wave's ctl words and its jump bitvector.
__global__ __launch_bounds__(256) void k_clear(uint32_t* __restrict__ ctl, uint4* __restrict__ bits,
                                               uint32_t nq) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < 16) ctl[i] = 0;
    for (uint32_t k = i; k < nq; k += gridDim.x * 256) bits[k] = make_uint4(0, 0, 0, 0);
}

// XCD-aware block order: the dispatcher hands consecutive workgroups to the 8 XCDs in turn, and
// each XCD has its own L2.  Block b of a grid of G is given item (b % 8) * ceil-share + b / 8, so
// that every XCD walks one contiguous range of tiles: the tiles of a document then share an L2,
// and the lookups k_runs makes into the head records of other tiles of the same document (and
// the jump bits k_classify sets there) stay inside it.  (A bijection for any G.)
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t G, uint32_t on) {
    if (!on) return b;
    const uint32_t q = G / kXcds, r = G % kXcds, x = b % kXcds, i = b / kXcds;
    return x < r ? x * (q + 1u) + i : r * (q + 1u) + (x - r) * q + i;
}

// Every kernel after level 0 starts with this: a wave whose plan was too small does nothing.
__device__ __forceinline__ bool replan(const uint32_t* ctl) { return ctl[C_REPLAN] != 0u; }

// Stages = event intervals of crdt_hip_stats (include/crdt_hip.h CRDT_HIP_STAGE_*).
enum Stage { S_CLASSIFY, S_RUNS, S_SORTB, S_COUNT, S_SCAN, S_PLACE, S_LINK, S_WALK1, S_RANK,
             S_WALK2, S_EXPAND, S_DIGEST, S_DOCTREE, S_TEXT, S_ENCODE, S_N };


// ---------------------------------------------------------------------------------------------
// Level 0: runs
// ---------------------------------------------------------------------------------------------
// Level 0 streams over 4096-slot tiles (one workgroup, 16 consecutive slots per thread; a
// thread's slots are always inside one document because documents start on 64-slot
// boundaries).  Runs are numbered by global head rank within the wave (run rho = number of
// heads before its head slot), so a run's weight is pstart[rho+1] - pstart[rho] and no
// per-document padding is needed: documents are contiguous ranges of runs from doc_root[d].
// There is no single-pass look-back: the three passes read 9.6, 0.2 and 0.7 bytes per slot.
struct L0Args {
    uint32_t nslots, log2m, ndocs, mode;  // mode: 0 text, 1 order
    uint32_t ntiles;
    const uint32_t* chunk_doc;  // per 64 slots: wave-local document
    const uint2* docs;          // per document {wave-relative base slot, n items}
    const uint32_t* in_parent;
    const uint64_t* in_key;     // lamport << 16 | agent (one gather per run head)
    const uint8_t* in_cp;       // 3 bytes per slot (cp3_get)
    uint32_t* jbits;            // per slot bit: has a non-consecutive child (a jump)
    uint16_t* nsqb;             // per slot bit, 16 per thread: an item whose parent is not the
                                //   previous slot (no previous-slot flag)
    uint64_t* wnib;             // per slot 4-bit weight (visible UTF-8 bytes / 1 per item), written
                                //   only for the 16-slot groups escm marks
    uint16_t* visb;             // per slot bit, 16 per thread: an item with a nonzero weight
    uint64_t* escm;             // per 1024 slots: bit i = the group of slots [16 i, 16 i + 16)
                                //   weighs other than its visible bits (a multi-byte character):
                                //   its weights are in wnib; every other group weighs 1 byte per
                                //   visible slot, so its nibbles are visb spread out
    uint32_t* lbits;            // Fugue: per slot bit, has a left child (its run gets a content
                                //   node; see k_runs)
    uint32_t fugue;             // the wave holds Fugue logs (left children)
    uint8_t* stile;             // per tile: its visible UTF-8 in slot order (kTileBytes each)
    uint32_t* plist;            // per tile (kScanTile each): the parents of its non-seq items in
                                //   slot order (k_classify reads them, k_runs reads them back)
    uint8_t* sbytes;            // the wave's visible UTF-8 in slot order (= weight order)
    uint64_t sbytes_cap;
    uint2* tile_hw;             // per tile {heads, weight}: totals, then exclusive prefixes
    uint2* tile_sums;           // per 4096 tiles: scan carries
    uint4* hrec;                // per 64 slots: run-head bits (x, y) and the heads before the
                                //   word inside its tile (z): a rank lookup is one 16-byte load
    uint32_t* r_head;           // per run: head slot
    uint32_t* r_pstart;         // per run: weight prefix at its head; [R] = the wave's weight
    uint32_t* r_parent;         // per run: parent run (kNil for a document start)
    uint64_t* r_key;            // per run: (lamport << 16 | agent) of the head
    uint32_t* doc_root;         // per document: its document-start run
    uint32_t* doc_p0;           // per document: weight prefix at its start
    uint32_t* ctl;
    uint32_t cap_runs, cap_rmax;  // capacity of the launch plan (k_docmax flags C_REPLAN above)
    uint32_t cap_rows;            // rows allocated in r_parent / r_key (more runs: not written)
    uint32_t xcd;                 // 1: XCD-aware tile order in k_classify / k_runs (xcd_block)
    uint32_t copy_text;           // k_runs copies the tile text into sbytes (0: k_doctree reads
                                  //   the tile segments itself, L1Plan::stile_text)
    // resident batches (Engine::build_nsq): the parents of the nsq items in slot order and their
    // prefix count per 64 slots (offset to the wave's first chunk); null: gather in_parent
    const uint32_t* nsq_par;
    const uint32_t* nsq_pre;
    const uint64_t* nsq_key;    // (beside nsq_par) the keys of the nsq items: every nsq item that
                                //   survives is a run head, whose key k_runs then need not gather
    // 1: no run contraction (Wave::nocon): every item heads its own run, so k_classify reads no
    // parents and sets no jump bits, k_heads marks every item, and k_runs reads each run's parent
    // and key from the columns in slot order (a run's parent run is its document start's run
    // plus the parent's item index).  RGA waves only.
    uint32_t nocon;
};

constexpr uint32_t kTileBytes = kScanTile * 4;  // worst case: every slot a 4-byte character
// Fugue (left children).  A run whose head has left children is numbered as two rows: a content
// row (the run's text, weight only) and then its tree row (no weight; its parent, key and every
// child: the head's left children, the content row, the last item's right children).  The
// content row sorts between the two sides: left children carry kLeftKey in their key (bit 48),
// the content row kMidKey, right children neither; siblings sort by key descending, so the
// weighted pre-order of the rows is the Fugue in-order (lamport < 0xFFFFFFFF).  The tree row is
// the last row of its run, so "the run of slot s" (a rank lookup) and "the previous run" of a seq
// head both land on it.
// (kLeftKey: engine.hpp)
// words of the jump bitvector of a wave (a multiple of 4: the left-child bits follow it aligned)
__host__ __device__ constexpr uint64_t jbits_words(uint64_t slots) { return (slots / 32 + 8 + 3) & ~3ull; }
constexpr uint64_t kMidKey = (1ull << 48) - 1ull;
constexpr uint32_t kRecTree = 1u << 31;  // k_runs record of a head with two rows

// 16 bits -> 16 nibbles (bit k to bit 4k), each half by three shift-or-mask steps
__device__ __forceinline__ uint64_t spread_nib16(uint32_t v) {
    uint32_t l8 = v & 0xFFu, h8 = (v >> 8) & 0xFFu;
    l8 = (l8 | (l8 << 12)) & 0x000F000Fu;
    h8 = (h8 | (h8 << 12)) & 0x000F000Fu;
    l8 = (l8 | (l8 << 6)) & 0x03030303u;
    h8 = (h8 | (h8 << 6)) & 0x03030303u;
    l8 = (l8 | (l8 << 3)) & 0x11111111u;
    h8 = (h8 | (h8 << 3)) & 0x11111111u;
    return ((uint64_t)h8 << 32) | l8;
}

// k_classify: the characters of 16 slots per thread (3 x 16-byte loads of the codepoint column:
// codepoint, tombstone, "parent is the previous slot" flag), then the parents of the tile's
// items without the flag (a few percent):
//  * "item whose parent is not the previous slot" (nsq) bits, one u16 store per thread;
//  * per-slot weights as nibbles, the tile's weight total, and the tile's visible UTF-8
//    compacted in slot order: assembled in LDS, stored to its stile segment in 16-byte pieces;
//  * the nsq items listed in LDS in slot order (the text stage's LDS, once stored) and their
//    parents read by the whole block, four loads per thread in flight at a time (the items
//    cluster; listing them spreads the loads over the block);
//  * the jump bit of every parent that has a non-consecutive child: parents inside the tile in
//    LDS (ORed into jbits word by word at the end), parents in other tiles by agent-scope
//    atomicOr on jbits;
//  * a parent out of range (or an item that is its own parent) is flagged; such an item becomes
//    a run head under the document start, and the merge reports CRDT_HIP_EBADLOG;
//  * the parents themselves (as wave slots), in slot order, to the tile's plist segment: every
//    nsq item is a run head, and k_runs reads its parent there (coalesced) instead of gathering it.
// The stream part reads 3 bytes per slot and waits for one round trip; the parent part is one
// more round trip at the end of the block, hidden behind the other blocks' streams.
__global__ __launch_bounds__(kBlock) void k_classify(L0Args a) {
    __shared__ uint32_t lds[kBlock / 64];
    __shared__ uint32_t jl[kScanTile / 32];
    __shared__ uint32_t ll[kScanTile / 32];  // (Fugue) the tile's own left-child bits
    __shared__ uint2 ldoc[kBlock];  // per thread: its document {base slot, items}
    // (+64: one sink byte per lane for the branch-free ASCII stores below)
    __shared__ __attribute__((aligned(16))) uint8_t sb[kTileBytes + 64];
    const uint32_t tile = xcd_block(blockIdx.x, gridDim.x, a.xcd);
    const uint32_t t0 = tile * kScanTile, gs = t0 + threadIdx.x * kScanItems;
    const bool live = gs < a.nslots;
    if (threadIdx.x < kScanTile / 32) {
        jl[threadIdx.x] = 0;
        ll[threadIdx.x] = 0;
    }
    // (resident batches) the tile's range of the compact nsq parent list, first: the loads of its
    // first entries are issued as soon as it arrives, behind the codepoint column, instead of a
    // gather round trip at the end of the block
    const bool cl = a.nsq_par != nullptr;
    uint32_t nlo = 0, nhi = 0;
    if (cl) {
        nlo = a.nsq_pre[t0 >> 6];
        nhi = a.nsq_pre[min(t0 + kScanTile, a.nslots) >> 6];
    }
    // the codepoint column first (its address does not wait for the document lookup); padding
    // slots hold junk and are masked below
    uint4 cq[3] = {};
    uint2 doc = make_uint2(0, 0);
    if (live) {
        const uint4* cv = reinterpret_cast<const uint4*>(a.in_cp + 3ull * gs);  // 48 B
#pragma unroll
        for (int q = 0; q < 3; ++q) cq[q] = cv[q];
        doc = a.docs[a.chunk_doc[gs >> a.log2m]];
    }

    const uint32_t n = doc.y, l0 = gs - doc.x;
    ldoc[threadIdx.x] = doc;
    uint32_t C[16];
    {
        // the 16 three-byte values from 12 dwords (constant shifts: value k at byte 3k)
        const uint32_t CW[13] = {cq[0].x, cq[0].y, cq[0].z, cq[0].w, cq[1].x, cq[1].y, cq[1].z,
                                 cq[1].w, cq[2].x, cq[2].y, cq[2].z, cq[2].w, 0u};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int byte = 3 * k, wd = byte >> 2, sh = 8 * (byte & 3);
            const uint32_t lo = CW[wd] >> sh, hi = sh > 8 ? CW[wd + 1] << (32 - sh) : 0u;
            C[k] = (lo | hi) & 0x00FFFFFFu;
        }
    }
    // classification of the 16 slots as bit masks.  The items are a contiguous range of them
    // (slot k is an item iff 0 <= l0 + k - 1 < n); the flags are gathered into masks, and a
    // thread whose codepoints are all ASCII (nearly every thread on the traces) weighs each
    // visible item 1 byte: its nibbles are its visible bits spread out.  Otherwise (or in ORDER
    // mode, where every item weighs 1) the weights are taken per slot.
    uint32_t itm = 0;
    if (live && l0 <= n) {
        const uint32_t k0 = l0 == 0u ? 1u : 0u, k1 = min(16u, n + 1u - l0);
        itm = k1 > k0 ? (((1u << k1) - 1u) & ~((1u << k0) - 1u)) : 0u;
    }
    uint32_t dm = 0, sm = 0, lfm = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        dm |= ((C[k] >> 23) & 1u) << k;
        sm |= ((C[k] >> 22) & 1u) << k;
        lfm |= ((C[k] >> 21) & 1u) << k;
        hi |= C[k] & (kCpMask & ~0x7Fu);
    }
    const uint32_t nsq0 = itm & ~sm, lm = itm & lfm;
    uint32_t nsq = nsq0, W, vis;
    uint64_t nib;
    if (a.mode || hi == 0u) {
        vis = a.mode ? itm : (itm & ~dm);
        W = (uint32_t)__popc(vis);
        nib = spread_nib16(vis);
    } else {
        W = 0;
        vis = 0;
        nib = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const bool it = (itm >> k) & 1u;
            const uint32_t w = it && !((dm >> k) & 1u) ? utf8_len(C[k] & kCpMask) : 0u;
            W += w;
            nib |= (uint64_t)w << (4 * k);
            vis |= (w ? 1u : 0u) << k;
        }
    }
    // the weight nibbles only of a group that weighs other than its visible bits (a visible
    // multi-byte character: rare), marked in the wave's escape word; k_runs spreads the visible
    // bits of every other group itself (the nibbles were 0.5 B per slot written and read back)
    const bool esc = live && W != (uint32_t)__popc(vis);
    const uint64_t em = __ballot(esc);
    if (live) {
        a.nsqb[gs >> 4] = (uint16_t)nsq;
        if (esc) a.wnib[gs >> 4] = nib;
        a.visb[gs >> 4] = (uint16_t)vis;
        if ((threadIdx.x & 63u) == 0u) a.escm[gs >> 10] = em;  // (a wave: 1024 aligned slots)
    }
    // one scan for both: nsq items << 16 | weight (a tile holds at most 4096 and 16,384)
    uint32_t tot;
    const uint32_t ex = block_excl_scan<kBlock / 64>(((uint32_t)__popc(nsq) << 16) | W, lds, tot);
    const uint32_t tw = tot & 0xFFFFu, T = tot >> 16;
    if (a.mode == 0 && W == (uint32_t)__popc(vis)) {
        // every visible character of the thread is one UTF-8 byte (nearly always on the traces):
        // 16 unconditional byte stores, a slot without a visible character into the lane's sink
        // byte, instead of a branch per slot and per byte
        uint8_t* o = sb + (ex & 0xFFFFu);
        uint8_t* sink = sb + kTileBytes + (threadIdx.x & 63u);
        uint32_t pos = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t v = (vis >> k) & 1u;
            *(v ? o + pos : sink) = (uint8_t)C[k];
            pos += v;
        }
    } else if (a.mode == 0 && W) {
        uint8_t* o = sb + (ex & 0xFFFFu);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t L = (uint32_t)(nib >> (4 * k)) & 15u, c = C[k] & kCpMask;
            if (L) {
                // UTF-8: lead byte = length prefix | top bits, then 6-bit continuation bytes
                const uint32_t s0 = 6u * (L - 1u);
                o[0] = (uint8_t)(L == 1u ? c : (((0xFF00u >> L) & 0xFFu) | (c >> s0)));
                if (L > 1u) o[1] = (uint8_t)(0x80u | ((c >> (s0 - 6u)) & 63u));
                if (L > 2u) o[2] = (uint8_t)(0x80u | ((c >> (s0 - 12u)) & 63u));
                if (L > 3u) o[3] = (uint8_t)(0x80u | (c & 63u));
            }
            o += L;
        }
    }
    __syncthreads();
    // (compact list) the tile's first list entries, loaded now that the slot words are dead: they
    // arrive while the text is copied out and the nsq items are listed
    uint32_t ppre[4] = {0u, 0u, 0u, 0u};  // list entries threadIdx.x + j kBlock of the tile
    if (cl) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = nlo + threadIdx.x + (uint32_t)j * kBlock;
            ppre[j] = q < nhi ? a.nsq_par[q] : 0u;
        }
    }
    if (threadIdx.x == 0) a.tile_hw[tile].y = tw;
    if (a.mode == 0) {
        uint4* dst = reinterpret_cast<uint4*>(a.stile + (uint64_t)tile * kTileBytes);
        const uint4* src = reinterpret_cast<const uint4*>(sb);
        for (uint32_t i = threadIdx.x; i < (tw + 15u) / 16u; i += kBlock) dst[i] = src[i];
    }
    if (cl && T != nhi - nlo && threadIdx.x == 0) atomicOr(&a.ctl[C_ERR], 1u);  // list != flags
    if (a.nocon) return;  // (no contraction: no jump bits; k_runs checks the parents)
    if (T == 0) return;  // (block-uniform) no nsq item: no jump bit from this tile
    __syncthreads();  // the text stage is stored: its LDS holds the list
    // list entries: tile-local slot, bit 15 = a left child (Fugue)
    uint16_t* lst = reinterpret_cast<uint16_t*>(sb);
    for (uint32_t i = ex >> 16; nsq; nsq &= nsq - 1u) {
        const uint32_t b = (uint32_t)__builtin_ctz(nsq);
        lst[i++] = (uint16_t)((threadIdx.x * kScanItems + b) | (((lm >> b) & 1u) << 15));
    }
    __syncthreads();
    uint32_t bad = 0;
    uint32_t* pl = a.plist + t0;
    for (uint32_t t = threadIdx.x; t < T; t += 4u * kBlock) {
        uint32_t o[4], p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = t + (uint32_t)j * kBlock;
            o[j] = q < T ? lst[q] : 0xFFFFu;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = t + (uint32_t)j * kBlock;
            p[j] = o[j] == 0xFFFFu             ? 0u
                   : !cl                       ? a.in_parent[t0 + (o[j] & 0x7FFFu)]
                   : t == threadIdx.x          ? ppre[j]
                   : nlo + q < nhi             ? a.nsq_par[nlo + q]
                                               : 0u;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (o[j] == 0xFFFFu) continue;
            const uint32_t oi = o[j] & 0x7FFFu;
            const uint2 d = ldoc[oi / kScanItems];
            // the parent's index in its document (the compact list holds wave slots); plist
            // gets the wave slot, as the list has it
            const uint32_t pj = cl ? p[j] - d.x : p[j];
            if (!cl) pl[t + (uint32_t)j * kBlock] = d.x + pj;
            const bool left = (o[j] >> 15) != 0u;
            if (pj > d.y || pj == t0 + oi - d.x || (left && pj == 0u)) {
                bad = 1u;  // (the document start has no left children)
            } else {
                const uint32_t ps = d.x + pj;
                if (left) {
                    // Fugue: the parent's run node holds its left children, so the parent must
                    // head its run (k_heads cuts before every slot with a left-child bit), and
                    // nothing more: the run goes on after it.  A parent inside the tile (most:
                    // text typed backwards) takes the bit in LDS
                    if (ps / kScanTile == tile)
                        atomicOr(&ll[(ps % kScanTile) >> 5], 1u << (ps & 31u));
                    else
                        atomicOr(&a.lbits[ps >> 5], 1u << (ps & 31u));
                } else if (ps / kScanTile == tile) {
                    atomicOr(&jl[(ps % kScanTile) >> 5], 1u << (ps & 31u));
                } else {
                    atomicOr(&a.jbits[ps >> 5], 1u << (ps & 31u));
                }
            }
        }
    }
    __syncthreads();
    // the tile's own jump words join the bits later tiles set, by one atomic OR per nonzero word
    // (a plain store could overwrite another tile's OR into the same word): k_heads then reads
    // a single jump bitvector
    if (threadIdx.x < kScanTile / 32 && jl[threadIdx.x])
        atomicOr(&a.jbits[tile * (kScanTile / 32) + threadIdx.x], jl[threadIdx.x]);
    if (threadIdx.x < kScanTile / 32 && ll[threadIdx.x])
        atomicOr(&a.lbits[tile * (kScanTile / 32) + threadIdx.x], ll[threadIdx.x]);
    if (bad) atomicOr(&a.ctl[C_ERR], 1u);
}

__device__ __forceinline__ uint64_t low_mask64(uint32_t b) {
    return b >= 64u ? ~0ull : ((1ull << b) - 1ull);
}

// k_heads: one thread per 64-slot word of the rank bitvector (a word is inside one document),
// one wave per tile.  head(g) = document start, or an item that does not continue the run of
// the slot before it: continue(g) = seq(g) && !jump(g-1) && g is not a tile's first slot (runs
// never cross tiles: +1 run per 4096 slots at most).  Besides the words: the heads before
// each word inside its tile (hrec .z), so that the run of any slot s is
// tile_hw[s / 4096].x + hrec[s / 64].z + popcount(bits of hrec[s / 64] up to s) - 1 once the tile
// prefixes are scanned.
// Dead runs are dropped here: a run none of whose items is visible and whose last item has no
// child adds nothing to the document and is nobody's parent (on the traces 40-50 % of the runs:
// typed-then-deleted text).  Its items are "live" neither by weight nor by a jump bit (inside a
// run only the last item can have a non-consecutive child, and a last item has a child at all
// only through its jump bit), so a head survives iff a live slot lies between it and the next
// head: a segmented OR, smeared down from every live slot to the head of its run in six
// shift steps.  A run that goes on into the next word takes that word's live slots before its
// first head (the next lane's word; the last lane of the wave, or a word without a head, keeps
// the run).  Without its head the dead run's items count as the previous run's, which changes
// nothing: they weigh nothing, and no parent lookup lands on them.  Nothing else moves: seq heads
// still follow their parent's run (rho - 1), whose last item is live by its jump bit.
// Fugue waves: a head with left children numbers two rows (see kRecTree), and hrec .z and the
// tile totals count rows, not heads.
__global__ __launch_bounds__(kBlock) void k_heads(L0Args a) {
    const uint32_t wi = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t gs = wi * 64u;
    uint64_t hw = 0, lv = 0, lb = 0, vs = 0, sqh = 0;
    uint32_t dbase = 0;  // the word's document start (hrec .w: k_runs reads it there)
    if (gs < a.nslots) {
        const uint2 doc = a.docs[a.chunk_doc[gs >> a.log2m]];
        dbase = doc.x;
        const uint32_t l0 = gs - doc.x, n = doc.y;
        if (l0 <= n) {
            const uint64_t nsq = *reinterpret_cast<const uint64_t*>(a.nsqb + (gs >> 4));
            const uint64_t vis = *reinterpret_cast<const uint64_t*>(a.visb + (gs >> 4));
            const uint64_t jw = *reinterpret_cast<const uint64_t*>(a.jbits + (gs >> 5));
            // (a tile's first slot always heads a run: no run crosses a tile, so the text of every
            // run lies inside one tile's stile segment, which k_doctree stages tile by tile)
            uint64_t pj = 0;
            if (l0 > 0)
                pj = (gs % kScanTile) == 0u
                         ? 1u
                         : (a.jbits[(gs >> 5) - 1] >> 31) & 1u;
            const uint64_t prevj = (jw << 1) | pj;  // bit k = jump(gs + k - 1)
            const uint64_t item = low_mask64(n + 1u - l0) & ~low_mask64(l0 == 0 ? 1u : 0u);
            const uint64_t root = l0 == 0 ? 1ull : 0ull;
            // (Fugue) a slot with left children heads its run and is live: its run node holds them
            if (a.fugue) lb = *reinterpret_cast<const uint64_t*>(a.lbits + (gs >> 5));
            hw = root | (item & (nsq | prevj | lb));
            lv = root | vis | (item & (jw | lb));
            vs = vis;
            // a head whose parent is the slot before it (a seq head) makes that slot live: it is
            // the last item of the head's parent run (RGA: that slot has a jump bit anyway)
            sqh = hw & item & ~nsq;
            lv |= sqh >> 1;
        }
    }
    const uint64_t hw0 = hw;  // the run boundaries (before the dead-run drop)
    if (a.nocon) {
        // no contraction: every item heads its own run, none is dropped
        hw = 0;
        if (gs < a.nslots) {
            const uint2 doc = a.docs[a.chunk_doc[gs >> a.log2m]];
            const uint32_t l0 = gs - doc.x, n = doc.y;
            if (l0 <= n) hw = low_mask64(n + 1u - l0);  // (the document start and its items)
        }
    } else {
        // the next word's live slots before its first head keep this word's last run, and so
        // does a seq head in its first slot
        const uint64_t hn = (uint64_t)__shfl_down((long long)hw, 1);
        const uint64_t ln = (uint64_t)__shfl_down((long long)lv, 1);
        lv |= (uint64_t)__shfl_down((long long)sqh, 1) << 63;
        const bool carry = (threadIdx.x & 63u) == 63u || hn == 0ull ||
                           (ln & low_mask64((uint32_t)__builtin_ctzll(hn))) != 0ull;
        uint64_t z = lv | (carry ? (1ull << 63) : 0ull);
        uint64_t pm = ~(hw >> 1);  // bit i: slot i + 1 is not a head (the OR may pass down)
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            z |= (z >> k) & pm;
            pm &= pm >> k;
        }
        hw &= z;
    }
    if (a.fugue) {
        // Fugue: a head with left children numbers two rows only if its run holds visible text;
        // a weightless content row is a leaf that adds nothing, so such a run keeps its tree row
        // alone (its left children, then the last item's right children).  The same segmented
        // OR over the visible bits alone (a run that goes on past the wave's words: kept), and
        // the left-child bits become the two-row bits k_runs reads.
        const uint64_t hn = (uint64_t)__shfl_down((long long)hw0, 1);
        const uint64_t vn = (uint64_t)__shfl_down((long long)vs, 1);
        const bool carry = (threadIdx.x & 63u) == 63u || hn == 0ull ||
                           (vn & low_mask64((uint32_t)__builtin_ctzll(hn))) != 0ull;
        uint64_t z = vs | (carry ? (1ull << 63) : 0ull);
        uint64_t pm = ~(hw0 >> 1);
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            z |= (z >> k) & pm;
            pm &= pm >> k;
        }
        lb &= z;
        if (gs < a.nslots) *reinterpret_cast<uint64_t*>(a.lbits + (gs >> 5)) = lb;
    }
    // Fugue: a head with left children numbers two run rows (k_runs)
    const uint32_t c = (uint32_t)__popcll(hw) + (uint32_t)__popcll(hw & lb);
    const uint32_t inc = wave_incl_scan(c);
    if (gs < a.nslots) a.hrec[wi] = make_uint4((uint32_t)hw, (uint32_t)(hw >> 32), inc - c, dbase);
    const uint32_t th = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    const uint32_t tile = wi >> 6;  // 64 words per tile: one wave
    if ((threadIdx.x & 63u) == 0 && tile < a.ntiles) a.tile_hw[tile].x = th;
}

// Exclusive scan of the tile {heads, weight} pairs: per-4096-tile sums, one workgroup over the
// sums (also the wave totals), then the in-place apply.
__global__ __launch_bounds__(kBlock) void k_tiles_reduce(L0Args a) {
    __shared__ uint32_t lh[kBlock / 64], lw[kBlock / 64];
    uint32_t h = 0, w = 0;
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
#pragma unroll 4
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < a.ntiles) {
            const uint2 v = a.tile_hw[base + k];
            h += v.x;
            w += v.y;
        }
    uint32_t th, tw;
    (void)block_excl_scan<kBlock / 64>(h, lh, th);
    (void)block_excl_scan<kBlock / 64>(w, lw, tw);
    if (threadIdx.x == 0) a.tile_sums[blockIdx.x] = make_uint2(th, tw);
}
__global__ __launch_bounds__(1024) void k_tiles_top(L0Args a, uint32_t nb) {
    __shared__ uint32_t lh[16], lw[16];
    uint32_t ch = 0, cw = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t b = b0 + threadIdx.x;
        const uint2 v = b < nb ? a.tile_sums[b] : make_uint2(0, 0);
        uint32_t th, tw;
        const uint32_t eh = block_excl_scan<16>(v.x, lh, th);
        const uint32_t ew = block_excl_scan<16>(v.y, lw, tw);
        if (b < nb) a.tile_sums[b] = make_uint2(ch + eh, cw + ew);
        ch += th;
        cw += tw;
    }
    if (threadIdx.x == 0) {
        a.ctl[C_RTOTAL] = ch;
        a.ctl[C_WTOTAL] = cw;
    }
}
__global__ __launch_bounds__(kBlock) void k_tiles_apply(L0Args a) {
    __shared__ uint32_t lh[kBlock / 64], lw[kBlock / 64];
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint2 v[kScanItems];
    uint32_t h = 0, w = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = base + k < a.ntiles ? a.tile_hw[base + k] : make_uint2(0, 0);
        h += v[k].x;
        w += v[k].y;
    }
    uint32_t th, tw;
    const uint2 c = a.tile_sums[blockIdx.x];
    uint32_t eh = c.x + block_excl_scan<kBlock / 64>(h, lh, th);
    uint32_t ew = c.y + block_excl_scan<kBlock / 64>(w, lw, tw);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < a.ntiles) {
            a.tile_hw[base + k] = make_uint2(eh, ew);
            eh += v[k].x;
            ew += v[k].y;
        }
}
// A wave of at most kScanTile tiles (16 M slots: single documents, replicas, the downstream
// closure) scans its tile pairs in one workgroup: the three launches above in one.
__global__ __launch_bounds__(kBlock) void k_tiles_one(L0Args a) {
    __shared__ uint32_t lh[kBlock / 64], lw[kBlock / 64];
    const uint32_t base = threadIdx.x * kScanItems;
    uint2 v[kScanItems];
    uint32_t h = 0, w = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = base + k < a.ntiles ? a.tile_hw[base + k] : make_uint2(0, 0);
        h += v[k].x;
        w += v[k].y;
    }
    uint32_t th, tw;
    uint32_t eh = block_excl_scan<kBlock / 64>(h, lh, th);
    uint32_t ew = block_excl_scan<kBlock / 64>(w, lw, tw);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < a.ntiles) {
            a.tile_hw[base + k] = make_uint2(eh, ew);
            eh += v[k].x;
            ew += v[k].y;
        }
    if (threadIdx.x == 0) {
        a.ctl[C_RTOTAL] = th;
        a.ctl[C_WTOTAL] = tw;
    }
}

// k_runs: one record per run head and the tile's UTF-8 moved from its stile segment to its place
// in sbytes.  One packed scan, heads << 16 | weight (a tile holds at most 4096 heads and 16,384
// bytes).  The run records are assembled in LDS (tile-local slot << 16 | tile-local weight
// prefix), then one thread per run of the tile writes its record row: head slot, weight prefix
// (r_pstart; the last tile adds the sentinel r_pstart[R] = the wave's weight, so a run's weight
// is always r_pstart[rho + 1] - r_pstart[rho]), key (lamport, agent of the head) and parent
// run.  A head whose parent is the slot before it (a seq head, cut by a jump) has the previous
// run as parent; any other head looks up the run of its parent slot in the head bitvector
// (tile prefix + hloc + popcount).  Storing the rows from the thread that found each head costs
// one vector store instruction per head position with lanes scattered over many lines (the
// address unit, not HBM, bounded that form); one thread per run stores them as contiguous rows.
// FUGUE: the wave has left children.  A head with left children then numbers two rows; the
// tile still keeps one record per head (kRecTree marks those heads) and the per-head loop finds
// each head's first row by a block scan of the rows per head.
// SL = slots per thread (16: 256 threads per tile; 32: 128 threads per tile).  With 32, a wave
// covers two 1024-slot stretches and a CU holds 16 tiles at once instead of 8 (32 waves per CU
// either way): the per-head phase is a chain of dependent gathers (list entry, then the parent's
// head record) with ~100 heads per tile on the traces, so the tiles a CU holds at once bound the
// gathers in flight.  The records are staged in an LDS window of kRunsWin heads (+1), filled and
// drained as often as the tile needs (nearly always once), which keeps the 128-thread block at
// ~6 KiB of LDS.
constexpr uint32_t kRunsWin = 1024;
__device__ __forceinline__ uint32_t mpop(uint32_t x) { return (uint32_t)__popc(x); }
__device__ __forceinline__ uint32_t mpop(uint64_t x) { return (uint32_t)__popcll(x); }
template <bool FUGUE, int SL>
__global__ __launch_bounds__(kScanTile / SL) __attribute__((amdgpu_waves_per_eu(8))) void k_runs(L0Args a) {
    static_assert(SL == 16 || SL == 32 || SL == 64, "slots per thread");
    using MT = typename std::conditional<SL == 64, uint64_t, uint32_t>::type;  // a thread's slot masks
    constexpr int NT = kScanTile / SL;  // threads per tile
    constexpr int NW = NT / 64;
    constexpr int NQ = SL / 16;         // weight-nibble words per thread
    constexpr uint32_t kWin = SL == 16 ? (uint32_t)kScanTile : SL == 32 ? kRunsWin : kRunsWin / 2;
    __shared__ uint32_t lsum[NW];
    __shared__ uint32_t lrow[NW];
    __shared__ uint32_t rec[kWin + 1];
    __shared__ MT lnsq[NT];            // nsq bits of every thread's slots
    __shared__ uint2 ldoc[NT];         // every thread's document {base slot, items}
    __shared__ uint32_t lsq[NW];
    __shared__ uint16_t lnpf[NT];      // non-seq items of the tile before every thread
    __shared__ uint16_t ldp[FUGUE ? NT : 1];  // Fugue: two-row heads before every thread
    __shared__ MT ldm[FUGUE ? NT : 1];        //   and every thread's two-row head bits
    const uint32_t tile = xcd_block(blockIdx.x, gridDim.x, a.xcd);
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t gs = tile * kScanTile + threadIdx.x * SL;
    MT hm = 0, nsq = 0, dm = 0;
    // weights: the visible bits (vw) of groups without a visible multi-byte character; a thread
    // holding an escaped group (e) takes its slots' nibbles: 8 slots per word nwd
    MT vw = 0;
    uint32_t e = 0;
    uint32_t nwd[2 * NQ];
#pragma unroll
    for (int q = 0; q < 2 * NQ; ++q) nwd[q] = 0;
    uint2 doc = make_uint2(0, 0);
    const uint2 pre = a.tile_hw[tile];
    // the parents of the tile's nsq items: the compact list of a resident batch, else the tile's
    // plist segment k_classify wrote
    const uint32_t nlo = a.nsq_par ? a.nsq_pre[tile * (kScanTile / 64)] : 0u;
    const uint32_t* pls = a.nsq_par ? a.nsq_par + nlo : a.plist + (uint64_t)tile * kScanTile;
    if (gs < a.nslots) {
        // the head bits and (.w) the document start from the word's head record; the document's
        // item count only where the parents are checked here (no contraction)
        const uint4 hb = a.hrec[gs >> 6];
        const uint32_t hw32 = (gs & 63u) < 32u ? hb.x : hb.y;
        doc = make_uint2(hb.w, 0xFFFFFFFFu);
        if (a.nocon) doc = a.docs[a.chunk_doc[gs >> a.log2m]];
        if constexpr (SL == 64) {
            hm = ((uint64_t)hb.y << 32) | hb.x;
            if (FUGUE) dm = hm & *reinterpret_cast<const uint64_t*>(a.lbits + (gs >> 5));
            vw = *reinterpret_cast<const uint64_t*>(a.visb + (gs >> 4));
        } else {
            hm = SL == 32 ? hw32 : (hw32 >> (gs & 31u)) & 0xFFFFu;
            if (FUGUE) dm = hm & (a.lbits[gs >> 5] >> (gs & 31u));
            vw = SL == 32 ? *reinterpret_cast<const uint32_t*>(a.visb + (gs >> 4)) : (uint32_t)a.visb[gs >> 4];
        }
        e = (uint32_t)(a.escm[gs >> 10] >> ((gs >> 4) & 63u)) & ((1u << NQ) - 1u);
        if (e) {  // (rare: the nibbles of the escaped groups, the visible bits spread for the rest)
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const uint64_t nb = (e >> q) & 1u ? a.wnib[(gs >> 4) + (uint32_t)q] : spread_nib16((uint32_t)(vw >> (16 * q)));
                nwd[2 * q] = (uint32_t)nb;
                nwd[2 * q + 1] = (uint32_t)(nb >> 32);
            }
        }
        if constexpr (SL == 64)
            nsq = *reinterpret_cast<const uint64_t*>(a.nsqb + (gs >> 4));
        else
            nsq = SL == 32 ? *reinterpret_cast<const uint32_t*>(a.nsqb + (gs >> 4)) : a.nsqb[gs >> 4];
    }
    lnsq[threadIdx.x] = nsq;
    ldoc[threadIdx.x] = doc;
    // The first 4*NT bytes of the tile's text are loaded with the rest, before the tile's
    // offset is known: thread t's destination dword needs source dwords t and t+1 whatever the
    // offset's alignment (the segment is kTileBytes long, so both are in bounds).
    const uint8_t* src = a.stile + (uint64_t)tile * kTileBytes;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    uint32_t w0 = 0, w1 = 0;
    const bool copy = a.mode == 0 && a.copy_text;
    if (copy) {
        w0 = s32[threadIdx.x];
        w1 = s32[threadIdx.x + 1];
    }
    // the weight before each nibble word (v_dot8 sums eight nibbles), and the thread's weight
    uint32_t nwc[2 * NQ];
    uint32_t W = 0;
#pragma unroll
    for (int q = 0; q < 2 * NQ; ++q) {
        nwc[q] = W;
        W = __builtin_amdgcn_udot8(nwd[q], 0x11111111u, W, false);
    }
    if (!e) W = mpop(vw);
    const uint32_t x = (mpop(hm) << 16) | W;  // heads (records) << 16 | weight
    const uint32_t inc = wave_incl_scan(x);
    const uint32_t cq = mpop(nsq), incq = wave_incl_scan(cq);
    const uint32_t cd = FUGUE ? mpop(dm) : 0u, incd = FUGUE ? wave_incl_scan(cd) : 0u;
    if (lane == 63u) {
        lsum[wv] = inc;
        lsq[wv] = incq;
        if (FUGUE) lrow[wv] = incd;
    }
    __syncthreads();
    uint32_t off = 0, tot = 0, offq = 0, offd = 0, totd = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const uint32_t v = lsum[i];
        off += (i < (int)wv) ? v : 0u;
        offq += (i < (int)wv) ? lsq[i] : 0u;
        tot += v;
        if (FUGUE) {
            offd += (i < (int)wv) ? lrow[i] : 0u;
            totd += lrow[i];
        }
    }
    lnpf[threadIdx.x] = (uint16_t)(offq + incq - cq);
    const uint32_t dpre = offd + incd - cd;  // (Fugue) two-row heads of the tile before the thread
    if (FUGUE) {
        ldp[threadIdx.x] = (uint16_t)dpre;
        ldm[threadIdx.x] = dm;
    }
    const uint32_t ex = off + inc - x;
    const uint32_t nh = tot >> 16;
    const uint32_t tw_all = tot & 0xFFFFu;
    uint32_t tw = tw_all;
    if (a.mode == 0 && tw && (uint64_t)pre.y + tw > a.sbytes_cap) {  // more text than the host bound
        if (threadIdx.x == 0) atomicOr(&a.ctl[C_ERR], 4u);
        tw = 0;
    }
    // text: the dwords of sbytes wholly inside [D, D + tw) are this tile's alone (funnel-shifted
    // from two source dwords); the partial dwords at either end are shared with the neighbouring
    // tiles and written bytewise.
    const uint32_t D = pre.y, lo = (D + 3u) & ~3u, hi = (D + tw) & ~3u, sh = (lo - D) & 3u;
    uint32_t m = lo + 4u * threadIdx.x;
    if ((hm & 1u) && (gs & 63u) == 0 && doc.x == gs) {  // document starts are 64-aligned
        const uint32_t d = a.chunk_doc[gs >> a.log2m];
        a.doc_root[d] = pre.x + (ex >> 16) + dpre;  // (rows: heads + two-row heads before)
        a.doc_p0[d] = pre.y + (ex & 0xFFFFu);
    }
    if (tile + 1u == a.ntiles && threadIdx.x == 0) a.r_pstart[pre.x + nh + totd] = pre.y + tw_all;
    if (copy) {
        uint32_t* d32 = reinterpret_cast<uint32_t*>(a.sbytes);
        if (m < hi) d32[m >> 2] = sh ? (uint32_t)((((uint64_t)w1 << 32) | w0) >> (8 * sh)) : w0;
        for (m += 4u * NT; m < hi; m += 4u * NT) {
            const uint32_t o = m - D;
            const uint32_t v0 = s32[o >> 2], v1 = sh ? s32[(o >> 2) + 1] : 0u;
            d32[m >> 2] = sh ? (uint32_t)((((uint64_t)v1 << 32) | v0) >> (8 * sh)) : v0;
        }
        if (tw && threadIdx.x == 0)
            for (uint32_t g = D; g < min(D + tw, lo); ++g) a.sbytes[g] = src[g - D];
        if (tw && threadIdx.x == 1)
            for (uint32_t g = max(hi, lo); g < D + tw; ++g) a.sbytes[g] = src[g - D];
    }
    const uint32_t tbase = tile * kScanTile;
    // the records of heads [h0, h0 + kWin] (the one past the window: a two-row head reads the
    // next head's weight prefix), then one thread per head of the window; block-uniform loop
    for (uint32_t h0 = 0;; h0 += kWin) {
        {
            // the thread's heads one by one (a lane holds ~1 on the traces), each record's weight
            // prefix = the thread's prefix + the weight of its slots below the head
            uint32_t r = ex >> 16;
            const uint32_t p0 = ex & 0xFFFFu;
            if (r <= h0 + kWin && r + mpop(hm) > h0) {
                for (MT m = hm; m; m &= m - 1u) {
                    const uint32_t j = SL == 64 ? (uint32_t)__builtin_ctzll((uint64_t)m) : (uint32_t)__builtin_ctz((uint32_t)m);
                    uint32_t p;
                    if (!e) {
                        p = mpop(vw & ((MT(1) << j) - 1u));
                    } else {
                        const uint32_t wi = j >> 3;
                        uint32_t xw = nwd[0], cw = nwc[0];
#pragma unroll
                        for (int q = 1; q < 2 * NQ; ++q)
                            if (wi == (uint32_t)q) {
                                xw = nwd[q];
                                cw = nwc[q];
                            }
                        p = __builtin_amdgcn_udot8(xw & ((1u << (4u * (j & 7u))) - 1u), 0x11111111u, cw, false);
                    }
                    if (r >= h0 && r - h0 <= kWin)
                        rec[r - h0] = ((threadIdx.x * SL + j) << 16) | (p0 + p) |
                                      ((dm >> j) & 1u ? kRecTree : 0u);  // (Fugue: two rows)
                    ++r;
                }
            }
        }
        __syncthreads();
        // one thread per head: every gather of a stage issued before any is used
        const uint32_t hend = min(nh, h0 + kWin);
        for (uint32_t i = h0 + threadIdx.x; i < hend; i += NT) {
            const uint32_t rv = rec[i - h0];
            const uint32_t li = (rv >> 16) & 0xFFFu, g = tbase + li;
            const uint32_t th = li / SL, bl = li % SL;
            const MT below = (MT(1) << bl) - 1u;
            const bool two = (rv & kRecTree) != 0u;  // Fugue: a content row, then the tree row
            // the head's first row: heads before it, plus (Fugue) the two-row heads before it
            const uint32_t rho =
                pre.x + i + (FUGUE ? ldp[th] + mpop(ldm[th] & below) : 0u);
            const uint32_t rt = rho + (two ? 1u : 0u);  // the row with the run's parent and key
            const uint2 dc = ldoc[th];
            const bool root = g == dc.x;
            const MT nw = lnsq[th];
            const bool sq = !root && !((nw >> bl) & 1u);
            // a non-seq head's parent from the tile's list: its index = the non-seq items before
            // it; (resident batches) its key from the same index of the key list, a seq head's
            // gathered
            const uint32_t lix = lnpf[th] + mpop(nw & below);
            const uint64_t key = (a.nsq_key && !sq && !root) ? a.nsq_key[nlo + lix] : a.in_key[g];
            if (!FUGUE && a.nocon) {
                // no contraction: the run's parent and key from the columns (heads are every
                // slot of the tile's items, so these reads are in slot order); parent run = the
                // document start's run + the parent's item index
                uint32_t pr = kNil;
                uint64_t k = 0;
                if (!root) {
                    uint32_t p = a.in_parent[g];
                    k = a.in_key[g];
                    if (p > dc.y || p == g - dc.x) {
                        atomicOr(&a.ctl[C_ERR], 1u);
                        p = 0;
                    }
                    pr = rho - (g - dc.x) + p;
                }
                a.r_head[rho] = g;
                a.r_pstart[rho] = pre.y + (rv & 0xFFFFu);
                if (rho < a.cap_rows) {
                    a.r_parent[rho] = pr;
                    a.r_key[rho] = k;
                }
                continue;
            }
            uint32_t ps = (!sq && !root) ? pls[lix] : 0u;  // (the parent as a wave slot)
            a.r_head[rho] = g;
            a.r_pstart[rho] = pre.y + (rv & 0xFFFFu);
            if (two) {
                // the tree row weighs nothing: its prefix is the next head's (the content row's
                // end)
                a.r_head[rt] = g;
                a.r_pstart[rt] = pre.y + (i + 1u < nh ? rec[i + 1u - h0] & 0xFFFFu : tw_all);
            }
            uint32_t pr = kNil;
            if (sq) {
                pr = rho - 1u;  // the parent is the slot before the head: the previous run's last row
            } else if (!root) {
                // (a bad parent, flagged by k_classify: out of range, or the item itself, whose
                // row would be its own parent, a self-loop for the global level 1; any in-range
                // read that names another row does)
                if (ps >= a.nslots || ps == g) ps = dc.x;
                const uint4 hr = a.hrec[ps >> 6];
                const uint64_t hb = ((uint64_t)hr.y << 32) | hr.x;
                const uint32_t hl = hr.z;
                const uint32_t tp = a.tile_hw[ps / kScanTile].x;
                const uint32_t b = ps & 63u;
                const uint64_t mask = (b == 63u) ? ~0ull : ((2ull << b) - 1ull);
                uint32_t rows = (uint32_t)__popcll(hb & mask);
                if (FUGUE) {  // (rows of the parent slot's run: its tree row is its last)
                    const uint64_t lw = *reinterpret_cast<const uint64_t*>(a.lbits + ((ps >> 5) & ~1u));
                    rows += (uint32_t)__popcll(hb & lw & mask);
                }
                pr = tp + hl + rows - 1u;
            }
            if (rt < a.cap_rows) {  // (beyond: the wave outgrew its plan, C_REPLAN follows)
                a.r_parent[rt] = pr;
                a.r_key[rt] = root ? 0ull : key;
                if (two) {
                    // the run's text: a child of its tree row between the left and the right
                    // children (kMidKey)
                    a.r_parent[rho] = rt;
                    a.r_key[rho] = kMidKey;
                }
            }
        }
        if (h0 + kWin >= nh) break;
        __syncthreads();  // (the window is read before the next one is written)
    }
}

// Single workgroup: the most runs any document of the wave has (sizes the pointer jumping).
__global__ __launch_bounds__(1024) void k_docmax(L0Args a) {
    __shared__ uint32_t mx;
    if (threadIdx.x == 0) mx = 0;
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t d = threadIdx.x; d < a.ndocs; d += 1024) {
        const uint32_t end = d + 1 < a.ndocs ? a.doc_root[d + 1] : a.ctl[C_RTOTAL];
        m = max(m, end - a.doc_root[d]);
    }
    atomicMax(&mx, m);
    __syncthreads();
    if (threadIdx.x == 0) {
        a.ctl[C_RMAX] = mx;
        if (a.ctl[C_RTOTAL] > a.cap_runs || mx > a.cap_rmax) a.ctl[C_REPLAN] = 1u;
    }
}

// Expansion, one wave per 64 consecutive runs.  Their bytes are contiguous in sbytes (runs are
// numbered in slot order), so the wave streams them with unit-stride loads and each byte goes
// to its run's place in the document: text[toff[d] + roff[run] + i].  ORDER mode writes the
// run's item ids instead (consecutive: a run is a chain of consecutive ids).
struct ExpandArgs {
    uint32_t mode, log2m;
    const uint32_t* chunk_doc;
    const uint2* docs;
    const uint32_t* r_head;
    const uint32_t* r_pstart;  // weight of run rho: r_pstart[rho + 1] - r_pstart[rho]
    const uint32_t* roff;
    const uint32_t* tlen;
    const uint64_t* toff;
    const uint8_t* sbytes;
    uint8_t* text;
    uint32_t* ctl;
    const uint8_t* fused;  // per document: text already written by k_doctree (or null)
    // global level 1 (non-null): a run's offset is {offset in its sublist, sublist} (k_walk1)
    // plus the sublist's prefix, read here instead of a separate pass writing roff
    const uint2* rloc;
    const uint32_t* spref;
    uint32_t nspl;         // splitters of the wave (bounds the sublist index)
};

// The grid strides over the wave's runs (their count comes from ctl).  After a fused k_doctree
// it only has work if some document did not fit that kernel's LDS (ctl C_UNFUSED), so it is
// launched unconditionally and exits at once in the common case.
__global__ __launch_bounds__(kBlock) void k_expand(ExpandArgs a) {
    if (replan(a.ctl) || (a.fused && a.ctl[C_UNFUSED] == 0u)) return;
    const uint32_t R = a.ctl[C_RTOTAL];
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t r0 = blockIdx.x * kBlock; r0 < R; r0 += gridDim.x * kBlock) {
        const uint32_t rho = r0 + threadIdx.x;
        uint32_t w = 0, src = 0, idb = 0;
        uint64_t dst = 0;
        if (rho < R) {
            src = a.r_pstart[rho];
            w = a.r_pstart[rho + 1] - src;
            if (w) {
                const uint32_t h = a.r_head[rho];
                const uint32_t d = a.chunk_doc[h >> a.log2m];
                const uint32_t base = a.docs[d].x;
                uint32_t ro = 0;
                bool bad = false;
                if (a.rloc) {
                    const uint2 l = a.rloc[rho];
                    bad = l.y >= a.nspl;  // (a run no walk reached: flagged by the totals too)
                    ro = bad ? 0u : l.x + a.spref[l.y];
                } else {
                    ro = a.roff[rho];
                }
                if (a.fused && a.fused[d]) {
                    dst = ~0ull;  // k_doctree wrote this document (w still counts: bytes stay aligned)
                } else if (bad || (uint64_t)ro + w > a.tlen[d]) {
                    atomicOr(&a.ctl[C_ERR], 8u);
                    dst = ~0ull;  // skipped below
                } else {
                    dst = a.toff[d] + ro;
                }
                idb = h - base + (h == base ? 1u : 0u);
            }
        }
        const uint32_t inc = wave_incl_scan(w);
        const uint32_t ex = inc - w;
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)src);
        for (uint32_t b = 0; b < T; b += 64) {
            const uint32_t x = b + lane;
            // the last lane whose run starts at or before byte x owns it
            uint32_t j = 0;
#pragma unroll
            for (uint32_t st = 32; st; st >>= 1) {
                const uint32_t e = (uint32_t)__shfl((int)ex, (int)(j + st));
                if (e <= x) j += st;
            }
            const uint32_t off = x - (uint32_t)__shfl((int)ex, (int)j);
            const uint64_t dj = ((uint64_t)(uint32_t)__shfl((int)(dst >> 32), (int)j) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)dst, (int)j);
            // (every shuffle above runs with the whole wave active: a ds_bpermute from an inactive
            // lane reads 0)
            const uint32_t ib = a.mode ? (uint32_t)__shfl((int)idb, (int)j) : 0u;
            if (x < T && dj != ~0ull) {
                if (a.mode == 0)
                    a.text[dj + off] = a.sbytes[s0 + x];
                else
                    reinterpret_cast<uint32_t*>(a.text)[dj + off] = ib + off;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Level 1: the tree of runs.  Runs 0..R-1 of the wave; r_parent = kNil marks a document start.
// ---------------------------------------------------------------------------------------------
struct TreeArgs {
    uint32_t R, log2m, ndocs, Sreg, S;
    uint32_t step_limit;
    const uint32_t* in_parent;   // parent run (kNil: document start)
    const uint64_t* key;         // sibling key: (lamport, agent) of the run's head
    const uint32_t* pstart;      // weight prefix per run (+ sentinel): weight = [g + 1] - [g]
    const uint32_t* doc_root;    // per document: its document-start run
    const uint32_t* doc_p0;      // per document: weight prefix at its start
    // per run two uint4 (one 32-byte line): {first_child, weight, next_sibling, parent} and
    // {weight prefix (its slot-order text), -, -, -}
    uint4* rec;
    uint32_t rsh;      // log2 of the uint4 per record (1: the second line, for walk-written text)
    uint32_t* ctl;
    uint2* swn;        // per splitter {sublist weight, next splitter}
    uint32_t* roff;
    uint2* rloc;       // per run with visible bytes: {offset in its sublist, the sublist}
    uint32_t* tlen;
    uint64_t* toff;
    uint32_t* loff;
    uint64_t* leafh;
    uint64_t* ghash;  // group digests of documents above 16 MiB (indexed like leafh)
    uint32_t* leafcp;  // per leaf: codepoints (UTF-8 bytes that are not continuation bytes)
    uint32_t* gcp;     // per group of a document above 16 MiB: codepoints
    uint4* res;        // per document {UTF-8 bytes, codepoints, digest lo, digest hi}: the wave's
                       // results, after ctl in one block, copied to the host in one transfer
    const uint32_t* rank;  // per document: its k_doctree workgroup
    uint4* wg;             // per k_doctree workgroup: its descriptor (DocArgs::wg)
    const uint2* docs;     // per document {wave-relative base slot, items}
    uint8_t* text;
    uint64_t text_cap;
    uint32_t align;  // per-document output alignment (16 for text, 1 for order)
    // text mode of the grid-wide level 1: the second line of a run's record holds its place in
    // the slot-order text (and its bytes, up to kWalkText of them), k_walk1 writes each sublist's
    // text in walk order to its splitter's 2^wtmp_log2-byte slot of wtmp, k_tcopy moves the slots
    // to the document once the splitters are ranked, and k_walk_ovf walks the few sublists with
    // more text again for the rest
    uint32_t walk_text, wtmp_log2;
    const uint8_t* sbytes;
    const uint32_t* r_head;
    const uint32_t* chunk_doc;
    uint32_t log2c;          // chunk_doc granularity (slots per entry, log2)
    uint8_t* wtmp;
    uint32_t* ovf;           // splitters whose sublists carry more text than their slot
};
constexpr uint32_t kWalkText = 4;  // (one codepoint: every run of a wave without contraction)

// The second line of a run record in text mode: {its place in the slot-order text, its bytes
// packed little-endian when there are at most kWalkText of them}.
__device__ __forceinline__ uint4 text_line(const TreeArgs& a, uint32_t p0, uint32_t w) {
    uint32_t b = 0;
    if (w <= kWalkText)
        for (uint32_t i = 0; i < w; ++i) b |= (uint32_t)a.sbytes[p0 + i] << (8u * i);
    return make_uint4(p0, b, 0u, 0u);
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t* __restrict__ in, uint32_t n,
                                                         uint32_t* __restrict__ sums) {
    __shared__ uint32_t lds[kBlock / 64];
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t s = 0;
    if (base + kScanItems <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; ++i) {
            uint4 v = p[i];
            s += v.x + v.y + v.z + v.w;
        }
    } else {
        for (int i = 0; i < kScanItems; ++i)
            if (base + i < n) s += in[base + i];
    }
    uint32_t total;
    block_excl_scan<kBlock / 64>(s, lds, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// Single workgroup: exclusive scan of the per-tile sums in place; out[n] = grand total.
__global__ __launch_bounds__(1024) void k_scan_top(uint32_t* sums, uint32_t nb, uint32_t* out,
                                                    uint32_t n) {
    __shared__ uint32_t lds[16];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        uint32_t v = i < nb ? sums[i] : 0u;
        uint32_t total;
        uint32_t ex = block_excl_scan<16>(v, lds, total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) out[n] = carry;
}

__global__ __launch_bounds__(kBlock) void k_scan_apply(const uint32_t* __restrict__ in, uint32_t n,
                                                        const uint32_t* __restrict__ sums,
                                                        uint32_t* __restrict__ out) {
    __shared__ uint32_t lds[kBlock / 64];
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    const bool full = base + kScanItems <= n;
    if (full) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; ++i) {
            uint4 q = p[i];
            v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) v[i] = (base + i < n) ? in[base + i] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) { uint32_t t = v[i]; v[i] = s; s += t; }
    uint32_t total;
    const uint32_t off = block_excl_scan<kBlock / 64>(s, lds, total) + sums[blockIdx.x];
    if (full) {
        uint4* p = reinterpret_cast<uint4*>(out + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; ++i)
            p[i] = make_uint4(v[4 * i] + off, v[4 * i + 1] + off, v[4 * i + 2] + off, v[4 * i + 3] + off);
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i)
            if (base + i < n) out[base + i] = v[i] + off;
    }
}

// Compare-exchange for a descending sort of (key, id) pairs held in registers (k_doctree).
__device__ __forceinline__ void cx(uint64_t& ka, uint32_t& ia, uint64_t& kb, uint32_t& ib) {
    if (ka < kb) {
        const uint64_t tk = ka; ka = kb; kb = tk;
        const uint32_t ti = ia; ia = ib; ib = ti;
    }
}

// ---------------------------------------------------------------------------------------------
// Level 1, grid-wide: the run records by two LDS-staged LSD radix sorts
// ---------------------------------------------------------------------------------------------
// The Euler-tour walks read one record per run: {first child, weight, next sibling, parent}.
// Children of a parent, ordered by sibling key, are found by sorting:
//  A. every run as a 16-byte element {parent run, run id, key lo, key hi} (a document start's
//     parent is R: those sort last and are nobody's child), by parent run, 8-bit digits, least
//     significant first, each pass stable.  A sibling group leaves it contiguous, in run-id
//     order, carrying its keys, so one streaming pass (k_rs_order) orders each group in
//     registers and emits, per run, the pair {run, next sibling}, and the first child of each
//     parent (parents ascend along the sorted array: those writes are monotone, not random);
//  B. the pairs by run id (a permutation of 0..R-1: its digit counts are known in closed form),
//     whose last pass writes the next siblings in run order.
// Both sorts replace random per-run accesses (a child-count atomic, a placement scatter, a key
// gather per child, a record scatter per child) with passes that read and write whole stretches.
// One launch per pass ("onesweep"): a workgroup claims the next tile from a counter, ranks its
// elements per wave and digit (ballot matching: stable within the wave), publishes the tile's
// digit counts, takes the counts of every earlier tile by decoupled look-back (one thread per
// digit), reorders the tile by digit in LDS and writes each digit's stretch contiguously.
// Tile shapes, measured on config 5 (750 M runs, tools/gpu_iter.sh A/B of builds): sort A
// 1024 threads x 8 elements (8192 x 16 B, one workgroup per CU) 25.3 ms for four passes against
// 28.5 for 512 x 8 and 35-38 for 2048-element tiles; sort B 512 x 16 (8192 x 8 B, two workgroups
// per CU) 21.6 against 24.8 for 1024 x 8 or 512 x 8.
#ifndef CRDT_RS_THREADS_A
#define CRDT_RS_THREADS_A 1024
#endif
#ifndef CRDT_RS_THREADS_B
#define CRDT_RS_THREADS_B 512
#endif
#ifndef CRDT_RS_ITEMS_A
#define CRDT_RS_ITEMS_A 8
#endif
#ifndef CRDT_RS_ITEMS_B
#define CRDT_RS_ITEMS_B 16
#endif
constexpr uint32_t kRsThreadsA = CRDT_RS_THREADS_A;
constexpr uint32_t kRsThreadsB = CRDT_RS_THREADS_B;
constexpr uint32_t kRsItemsA = CRDT_RS_ITEMS_A;
constexpr uint32_t kRsItemsB = CRDT_RS_ITEMS_B;
constexpr uint32_t kRsTileA = kRsThreadsA * kRsItemsA;   // sort A: 8192 x 16 B per tile
constexpr uint32_t kRsTileB = kRsThreadsB * kRsItemsB;   // sort B: 8192 x 8 B per tile
constexpr uint32_t kRsBins = 256;      // sort B's digits (8 bits); sort A's are 8 or 10 bits
constexpr uint32_t kRsBinsMax = 1024;
constexpr uint32_t kRsMaxPass = 4;
constexpr uint32_t kRsHistA = 3 * kRsBinsMax;  // sort A's bucket starts: 4 x 256 or 3 x 1024
constexpr uint32_t kRsAgg = 0x80000000u;  // look-back word: a tile's digit count (else prefix + 1)
constexpr uint32_t kRsLook = 16;          // look-back words read per round trip
// rs_small_: bucket starts of sort A [pass][bin], of sort B, then counters: tile counters of the
// passes of A (4) and B (4), the lengths of the deferred and the long group lists
constexpr uint32_t kRsHistB = kRsHistA;
constexpr uint32_t kRsCtl = kRsHistA + kRsMaxPass * kRsBins;
constexpr uint32_t kRsBig = 8;
constexpr uint32_t kRsSmall = kRsCtl + 16;
constexpr uint32_t kRsBigLds = 8192;  // groups of up to this many children sort in LDS
constexpr uint32_t kRsPlaceBits = 14;  // sort B: the low bits of the run id are placed in LDS

struct RsArgs {
    uint32_t R, pass, npass;
    uint32_t dbits;      // sort A's digit: 8 or 10 bits (sort B's: 8)
    uint32_t npassB;     // passes of sort B (the bits of the run id above kRsPlaceBits)
    uint32_t shift0;     // bit of the first digit (sort B sorts the bits above kRsPlaceBits)
    const void* in;      // the previous pass's output (or the order pass's pairs)
    void* out;
    uint32_t* hist;      // this sort's [pass][bins] bucket starts
    uint32_t* tctr;      // this sort's tile counter per pass
    uint32_t* rctl;      // the counters block
    uint32_t* status;    // [tiles][bins] look-back words (zeroed before every pass)
    uint2* bigl;         // {start, children} of each group of more than 64 children
    uint2* B;            // per element of A: {run, next sibling}
    uint32_t* fc;        // per run: its first child (kNil: a leaf)
};

// The parent run of run g in sort A (document starts and malformed parents: R).
__device__ __forceinline__ uint32_t rs_parent(const TreeArgs& a, uint32_t g, bool& bad) {
    const uint32_t p = a.in_parent[g];
    bad = p != kNil && (p >= a.R || p == g);
    return (p == kNil || bad) ? a.R : p;
}

// Digit histograms of every pass of sort A (LDS, then one global add per bin and block).  A wave
// whose 64 runs share a digit adds them with one LDS atomic: the high digits of the parents are
// nearly constant over a wave when documents are small (all parents of a document share them),
// and 64 per-lane atomics on one bin serialise.
__global__ __launch_bounds__(kBlock) void k_rs_hist(TreeArgs a, RsArgs r) {
    __shared__ uint32_t h[kRsHistA];
    const uint32_t db = r.dbits, bins = 1u << db, nb = r.npass * bins;
    for (uint32_t i = threadIdx.x; i < nb; i += kBlock) h[i] = 0;
    __syncthreads();
    uint32_t bad_any = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t end = (a.R + 63u) & ~63u;  // (whole waves in every round: the ballots below)
    for (uint32_t g = blockIdx.x * kBlock + threadIdx.x; g < end; g += gridDim.x * kBlock) {
        const bool valid = g < a.R;
        bool bad = false;
        const uint32_t pv = valid ? rs_parent(a, g, bad) : 0u;
        bad_any |= bad ? 1u : 0u;
        const uint64_t vm = __ballot(valid);
#pragma unroll
        for (int k = 0; k < (int)kRsMaxPass; ++k) {
            if ((uint32_t)k >= r.npass) break;
            const uint32_t d = (pv >> (db * k)) & (bins - 1u);
            const uint32_t d0 = (uint32_t)__shfl((int)d, 0);  // (lane 0 is valid when any lane is)
            if (__ballot(valid && d != d0) == 0ull) {
                if (lane == 0u && vm) atomicAdd(&h[k * bins + d0], (uint32_t)__popcll(vm));
            } else if (valid) {
                atomicAdd(&h[k * bins + d], 1u);
            }
        }
    }
    if (bad_any) atomicOr(&a.ctl[C_ERR], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += kBlock)
        if (h[i]) atomicAdd(&r.hist[i], h[i]);
}

// Single workgroup: bucket starts of every pass of both sorts.  Sort B sorts a permutation of
// 0..R-1: digit d of pass k is held by full * 256^k values of each complete cycle of 256^(k+1)
// and by the part of the last cycle's block of d.
__global__ __launch_bounds__(kRsBinsMax) void k_rs_scan(RsArgs r) {
    __shared__ uint32_t lds[kRsBinsMax / 64];
    const uint32_t d = threadIdx.x, bins = 1u << r.dbits;
    for (uint32_t k = 0; k < max(r.npass, r.npassB); ++k) {
        uint32_t tot;
        if (k < r.npass) {
            const uint32_t v = d < bins ? r.hist[k * bins + d] : 0u;
            const uint32_t e = block_excl_scan<kRsBinsMax / 64>(v, lds, tot);
            if (d < bins) r.hist[k * bins + d] = e;
        }
        const uint64_t P = 1ull << (kRsPlaceBits + 8u * k), Q = P << 8;
        const uint64_t rem = r.R % Q, lo = (uint64_t)d * P;
        const uint64_t cnt = d < kRsBins
            ? (r.R / Q) * P + (rem > lo ? std::min<uint64_t>(rem - lo, P) : 0ull) : 0ull;
        const uint32_t e = block_excl_scan<kRsBinsMax / 64>((uint32_t)cnt, lds, tot);
        if (d < kRsBins && k < r.npassB) r.hist[kRsHistB + k * kRsBins + d] = e;
    }
}

__device__ __forceinline__ uint32_t rs_lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One pass.  T: uint4 (sort A) or uint2 (sort B), the sort key in .x.  MODE 0: the first pass of
// A (elements built from r_parent / r_key); 1: elements from r.in to r.out.  DB: digit bits (8,
// or 10 for sort A when that saves a pass: 3 x 10 bits cover waves of up to 2^30 runs, where 8-bit
// digits need 4 passes).  The per-wave digit counts share LDS with the reordered tile: every
// element's tile position is taken from them before the tile is written.
template <class T, int MODE, int ITEMS, int THREADS, int DB>
__global__ __launch_bounds__(THREADS) void k_rs_pass(TreeArgs a, RsArgs r) {
    constexpr uint32_t kRsThreads = THREADS, kRsWaves = THREADS / 64;
    constexpr uint32_t TILE = kRsThreads * ITEMS;
    constexpr uint32_t BINS = 1u << DB;
    static_assert(BINS <= THREADS, "one thread per digit");
    constexpr uint32_t kBuf = sizeof(T) * TILE, kWc = 4u * kRsWaves * (BINS + 1u);
    // (the counts share the tile's LDS only where both would not fit: 10-bit digits of 16-byte
    // elements; elsewhere sharing costs a barrier and a pass over the positions)
    constexpr bool kAlias = kBuf + kWc + 8u * BINS > 156u * 1024u;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kAlias ? (kBuf > kWc ? kBuf : kWc) : kBuf + kWc];
    T* buf = reinterpret_cast<T*>(smem);
    // per wave and digit (+1: invalid elements)
    uint32_t (*wc)[BINS + 1] = reinterpret_cast<uint32_t (*)[BINS + 1]>(smem + (kAlias ? 0u : kBuf));
    __shared__ uint32_t dst[BINS];               // the tile's digit starts
    __shared__ uint32_t gof[BINS];               // bucket position of the tile's digit start
    __shared__ uint32_t red[kRsWaves];
    __shared__ uint32_t tsh;
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    if (t == 0) tsh = atomicAdd(&r.tctr[r.pass], 1u);
    for (uint32_t i = t; i < kRsWaves * (BINS + 1); i += kRsThreads) (&wc[0][0])[i] = 0;
    __syncthreads();
    const uint32_t tile = tsh, R = r.R, sh = r.shift0 + DB * r.pass;
    // wave wv takes elements [base, base + 64 ITEMS) of the tile, lane-striped
    const uint32_t base = tile * TILE + wv * (64u * ITEMS);
    T e[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t i = base + (uint32_t)j * 64u + lane;
        e[j] = T{};
        if (i < R) {
            if constexpr (MODE == 0) {
                bool bad;
                const uint64_t k = a.key[i];
                e[j] = make_uint4(rs_parent(a, i, bad), i, (uint32_t)k, (uint32_t)(k >> 32));
            } else {
                e[j] = reinterpret_cast<const T*>(r.in)[i];
            }
        }
    }
    // stable ranks per wave and digit: the lanes holding the same digit (DB ballots), the rank
    // among them, and the wave's running count of the digit in LDS (its leader adds them)
    uint32_t pos[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t i = base + (uint32_t)j * 64u + lane;
        const bool valid = i < R;
        const uint32_t d = valid ? (e[j].x >> sh) & (BINS - 1u) : BINS;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < DB; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t rk = rs_lanes_below(peers);
        const uint32_t old = wc[wv][d];
        if (valid && rk == 0u) wc[wv][d] = old + (uint32_t)__popcll(peers);
        pos[j] = (d << 16) | (old + rk);
    }
    __syncthreads();
    // per digit: the waves' counts -> exclusive prefixes over the waves, the tile's count
    uint32_t c = 0;
    if (t < BINS) {
#pragma unroll
        for (int w = 0; w < (int)kRsWaves; ++w) {
            const uint32_t x = wc[w][t];
            wc[w][t] = c;
            c += x;
        }
        // published at once (look-backs of later tiles wait for it); tile 0 is its own prefix
        __hip_atomic_store(&r.status[(uint64_t)tile * BINS + t], tile == 0 ? c + 1u : (kRsAgg | c),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint32_t nval;
    const uint32_t ds = block_excl_scan<kRsWaves>(c, red, nval);
    if (t < BINS) {
        dst[t] = ds;
        uint32_t ex = 0;
        if (tile > 0) {
            // decoupled look-back: earlier tiles' counts of this digit, nearest first, until one
            // that has published its inclusive prefix (tile 0 always has); kRsLook words per
            // round trip, consumed in order up to the first inclusive one or the first not yet
            // published (then read again from there)
            for (uint32_t j = tile - 1u;;) {
                uint32_t w[kRsLook];
#pragma unroll
                for (int q = 0; q < (int)kRsLook; ++q)
                    w[q] = (int)j - q >= 0 ? __hip_atomic_load(&r.status[(uint64_t)(j - q) * BINS + t],
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : 1u;
                uint32_t used = 0;
                bool done = false, stall = false;
#pragma unroll
                for (int q = 0; q < (int)kRsLook; ++q) {
                    if (done || stall) continue;
                    if (w[q] == 0u) {
                        stall = true;
                    } else if (w[q] & kRsAgg) {
                        ex += w[q] & ~kRsAgg;
                        ++used;
                    } else {
                        ex += w[q] - 1u;
                        done = true;
                    }
                }
                if (done) break;
                j -= used;
                if (stall) __builtin_amdgcn_s_sleep(1);
            }
            __hip_atomic_store(&r.status[(uint64_t)tile * BINS + t], ex + c + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        gof[t] = r.hist[r.pass * BINS + t] + ex - ds;  // (+ the element's tile position)
    }
    __syncthreads();
    // every element's place in the tile, then (where the counts' LDS is the tile's, after a
    // barrier) the tile in digit order in LDS
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t d = pos[j] >> 16;
        pos[j] = d < BINS ? dst[d] + wc[wv][d] + (pos[j] & 0xFFFFu) : 0u;
    }
    if constexpr (kAlias) __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t i = base + (uint32_t)j * 64u + lane;
        if (i < R) buf[pos[j]] = e[j];
    }
    __syncthreads();
    // out: each digit's stretch lands contiguously at its bucket position
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t i = (uint32_t)k * kRsThreads + t;
        if (i < nval) {
            const T x = buf[i];
            reinterpret_cast<T*>(r.out)[gof[(x.x >> sh) & (BINS - 1u)] + i] = x;
        }
    }
}

// Sibling order descending by (key, run id).
__device__ __forceinline__ bool rs_before(uint64_t ka, uint32_t ca, uint64_t kb, uint32_t cb) {
    return ka > kb || (ka == kb && ca > cb);
}

// One sibling group held by lanes [gs, ge] of a wave (lane l: child c, key k, element position
// j; on: the lane is in a group this wave orders): each child's rank among its siblings, the
// children by rank (ds_permute), next siblings by shuffle; the pair {c, next sibling} to B[j],
// and the group's first child to fc[p].
__device__ __forceinline__ void rs_order_lanes(const RsArgs& r, bool on, uint32_t gs, uint32_t ge,
                                               uint32_t p, uint32_t c, uint64_t k, uint32_t j,
                                               uint32_t maxlen) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t rank = 0;
    const uint32_t khi = (uint32_t)(k >> 32), klo = (uint32_t)k;
    for (uint32_t q = 0; q < maxlen; ++q) {
        const uint32_t l = min(gs + q, 63u);
        const uint32_t hj = (uint32_t)__shfl((int)khi, (int)l);
        const uint32_t lj = (uint32_t)__shfl((int)klo, (int)l);
        const uint32_t cj = (uint32_t)__shfl((int)c, (int)l);
        if (on && gs + q <= ge)
            rank += rs_before(((uint64_t)hj << 32) | lj, cj, k, c) ? 1u : 0u;
    }
    const uint32_t tgt = on ? gs + rank : lane;
    const uint32_t sorted = (uint32_t)__builtin_amdgcn_ds_permute((int)(tgt << 2), (int)c);
    const uint32_t nx = (uint32_t)__shfl((int)sorted, (int)min(tgt + 1u, 63u));
    if (on) {
        r.B[j] = make_uint2(c, tgt + 1u <= ge ? nx : kNil);
        if (rank == 0) r.fc[p] = c;
    }
}

// Streaming pass over sort A's output: one wave per 64 consecutive elements.  Groups wholly
// inside the window are ordered here; a group that starts in the window and runs past its end is
// ordered by the same wave from a second load at its start (up to 64 children; a longer one is
// listed for k_rs_big).  A group that started in an earlier window belongs to that window's
// wave.  Document starts have no sibling.
__global__ __launch_bounds__(kBlock) void k_rs_order(TreeArgs a, RsArgs r, const uint4* __restrict__ E) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x, lane = threadIdx.x & 63u;
    const uint32_t R = a.R;
    const bool valid = i < R;
    const uint4 e = valid ? E[i] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
    const uint32_t p = e.x;
    if (valid && p == R) r.B[i] = make_uint2(e.y, kNil);
    uint32_t pl = (uint32_t)__shfl_up((int)p, 1), pr = (uint32_t)__shfl_down((int)p, 1);
    if (lane == 0) pl = (valid && i > 0) ? E[i - 1].x : 0xFFFFFFFEu;
    if (lane == 63u) pr = (i + 1u < R) ? E[i + 1].x : 0xFFFFFFFDu;
    const bool st = valid && pl != p, en = valid && pr != p;
    const uint64_t SB = __ballot(st), EB = __ballot(en);
    const uint64_t below = SB & (lane == 63u ? ~0ull : ((2ull << lane) - 1ull));
    const uint64_t above = EB & ~((1ull << lane) - 1ull);
    const uint32_t gs = below ? 63u - (uint32_t)__clzll(below) : 64u;
    const uint32_t ge = above ? (uint32_t)__builtin_ctzll(above) : 64u;
    const bool on = valid && p != R && gs < 64u && ge < 64u;
    // the group that crosses the window's end (at most one): its start lane, if in this window
    const uint64_t cross = __ballot(valid && st && p != R && ge == 64u);
    uint32_t len = on ? ge - gs + 1u : 0u;
#pragma unroll
    for (int o = 32; o; o >>= 1) len = max(len, (uint32_t)__shfl_xor((int)len, o));
    if (len) rs_order_lanes(r, on, gs, ge, p, e.y, ((uint64_t)e.w << 32) | e.z, i, len);
    if (!cross) return;  // (wave-uniform)
    const uint32_t cl = (uint32_t)__builtin_ctzll(cross);
    const uint32_t s0 = (uint32_t)__shfl((int)i, (int)cl), cp = (uint32_t)__shfl((int)p, (int)cl);
    const uint32_t k = s0 + lane;
    const uint4 f = k < R ? E[k] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
    const uint64_t in = __ballot(f.x == cp);
    const uint32_t n = in == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~in);
    if (n == 64u && s0 + 64u < R && E[s0 + 64u].x == cp) {
        // more than 64 children: the group's length, then k_rs_big
        uint32_t m = 64;
        for (;;) {
            const uint32_t q = s0 + m + lane;
            const uint64_t b = __ballot(q < R && E[q].x == cp);
            if (b == ~0ull) {
                m += 64u;
                continue;
            }
            m += (uint32_t)__builtin_ctzll(~b);
            break;
        }
        if (lane == 0) r.bigl[atomicAdd(&r.rctl[kRsBig], 1u)] = make_uint2(s0, m);
        return;
    }
    rs_order_lanes(r, lane < n, 0u, n - 1u, cp, f.y, ((uint64_t)f.w << 32) | f.z, k, n);
}

// One workgroup per group of more than 64 children: bitonic sort (descending by key, run id;
// the "flip" formulation, so the padding to a power of two is never stored) in LDS, or in place
// in the element array beyond kRsBigLds children; then the pairs and the first child.
__global__ __launch_bounds__(kBigThreads) void k_rs_big(TreeArgs a, RsArgs r, uint4* __restrict__ E) {
    __shared__ uint64_t sk[kRsBigLds];
    __shared__ uint32_t sc[kRsBigLds];
    const uint32_t nb = r.rctl[kRsBig];
    for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
        const uint2 g = r.bigl[bi];
        const uint32_t s0 = g.x, cnt = g.y, p = E[s0].x;
        uint32_t P = 1;
        while (P < cnt) P <<= 1;
        const bool lds = P <= kRsBigLds;
        if (lds) {
            for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) {
                const uint4 e = E[s0 + i];
                sk[i] = ((uint64_t)e.w << 32) | e.z;
                sc[i] = e.y;
            }
            __syncthreads();
        }
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < P / 2; t += kBigThreads) {
                    const uint32_t i = (t / j) * 2 * j + (t % j);
                    const uint32_t l = (j == (k >> 1)) ? (i ^ (k - 1)) : (i ^ j);
                    if (l >= cnt) continue;
                    if (lds) {
                        if (rs_before(sk[l], sc[l], sk[i], sc[i])) {
                            const uint64_t tk = sk[i]; sk[i] = sk[l]; sk[l] = tk;
                            const uint32_t tc = sc[i]; sc[i] = sc[l]; sc[l] = tc;
                        }
                    } else {
                        const uint4 ei = E[s0 + i], el = E[s0 + l];
                        if (rs_before(((uint64_t)el.w << 32) | el.z, el.y, ((uint64_t)ei.w << 32) | ei.z, ei.y)) {
                            E[s0 + i] = el;
                            E[s0 + l] = ei;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) {
            const uint32_t c = lds ? sc[i] : E[s0 + i].y;
            const uint32_t nx = i + 1 < cnt ? (lds ? sc[i + 1] : E[s0 + i + 1].y) : kNil;
            r.B[s0 + i] = make_uint2(c, nx);
            if (i == 0) r.fc[p] = c;
        }
        __syncthreads();
    }
}

// Sort B's last step.  Its passes sorted the pairs by the run id's bits above kRsPlaceBits only;
// the ids are a permutation of 0..R-1, so block b of 2^kRsPlaceBits pairs holds exactly the ids
// [b 2^kRsPlaceBits, (b + 1) 2^kRsPlaceBits): one workgroup puts the next siblings in id order in
// LDS and writes them out as consecutive words.
__global__ __launch_bounds__(1024) void k_rs_place(TreeArgs a, const uint2* __restrict__ B,
                                                   uint32_t* __restrict__ ns) {
    __shared__ uint32_t buf[1u << kRsPlaceBits];
    const uint32_t base = blockIdx.x << kRsPlaceBits;
    const uint32_t n = min(1u << kRsPlaceBits, a.R - base);
    uint32_t bad = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 1024u) {
        const uint2 e = B[base + i];
        const uint32_t o = e.x - base;
        if (o < n) buf[o] = e.y;
        else bad = 1;
    }
    if (bad) atomicOr(&a.ctl[C_ERR], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += 1024u) ns[base + i] = buf[i];
}

// The run records in run order, every input coalesced: {first child, weight, next sibling,
// parent} (a document start, or a run with a malformed parent: no parent, no sibling).
__global__ __launch_bounds__(kBlock) void k_rs_records(TreeArgs a, const uint32_t* __restrict__ fc,
                                                       const uint32_t* __restrict__ ns) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.R) return;
    bool bad;
    const uint32_t p = rs_parent(a, g, bad);
    const uint32_t p0 = a.pstart[g];
    const uint32_t w = a.pstart[g + 1] - p0;
    a.rec[g << a.rsh] = make_uint4(fc[g], w, ns[g], p == a.R ? kNil : p);
    if (a.rsh) a.rec[(g << 1) + 1u] = text_line(a, p0, w);
}

// ---------------------------------------------------------------------------------------------
// Level 1, grid-wide, documents of up to kCsrDocRuns runs: sibling groups by counting
// ---------------------------------------------------------------------------------------------
// A child count per parent (one atomic per run, whose return value is the child's place in its
// parent's segment), an exclusive scan, a placement scatter, then the sibling order per parent
// (pairs inline, up to 8 by a register network, 9..64 one wave per group, wider one workgroup per
// group).  The atomics, the placement and the key reads land inside the run's own document, so
// when every document's runs span a few MB they hit the caches: measured faster than the radix
// sorts on such waves (the Fugue trace line: 7.3 against 19.4 ms of grouping per step); the
// radix sorts take waves with a larger document (config 5).
__global__ __launch_bounds__(kBlock) void k_count(TreeArgs a, uint32_t* __restrict__ deg) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.R) return;
    const uint32_t p = a.in_parent[g];
    if (p == kNil) return;
    if (p >= a.R || p == g) { atomicOr(&a.ctl[C_ERR], 1u); return; }
    // the child's place in its parent's segment comes with the count (roff is free until
    // k_walk1), so that k_place needs no second atomic
    a.roff[g] = atomicAdd(&deg[p], 1u);
}

__global__ __launch_bounds__(kBlock) void k_place(TreeArgs a, const uint32_t* __restrict__ cstart,
                                                  uint32_t* __restrict__ child) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.R) return;
    const uint32_t p = a.in_parent[g];
    if (p == kNil || p >= a.R || p == g) return;  // flagged by k_count
    child[cstart[p] + a.roff[g]] = g;  // (the place k_count's atomic handed out)
}

// Compare-exchange for a descending sort of (key, id) pairs held in registers.
__device__ __forceinline__ void cxi(uint64_t& ka, uint32_t& ia, uint64_t& kb, uint32_t& ib) {
    if (rs_before(kb, ib, ka, ia)) {
        const uint64_t tk = ka; ka = kb; kb = tk;
        const uint32_t ti = ia; ia = ib; ib = ti;
    }
}

struct CsrArgs {
    const uint32_t* cstart;  // per run: its children's segment start (cstart[R] = the total)
    uint32_t* child;         // children grouped by parent
    uint32_t* defer;         // parents with 9 or more children
    uint32_t* bigl;          // parents with more than 64 children
};

// Run records: {first child, weight} written by the run itself, {next sibling, parent} by
// whoever orders its sibling group (a.rsh: 1 when the records carry a second line).
__device__ __forceinline__ void set_dn(const TreeArgs& a, uint32_t g, uint32_t fc, uint32_t w) {
    reinterpret_cast<uint2*>(a.rec + (g << a.rsh))[0] = make_uint2(fc, w);
    if (a.rsh) a.rec[(g << 1) + 1u] = text_line(a, a.pstart[g], w);
}
__device__ __forceinline__ void set_upr(const TreeArgs& a, uint32_t c, uint32_t ns, uint32_t p) {
    reinterpret_cast<uint2*>(a.rec + (c << a.rsh))[1] = make_uint2(ns, p);
}
__device__ __forceinline__ void set_fcr(const TreeArgs& a, uint32_t p, uint32_t c) {
    reinterpret_cast<uint32_t*>(a.rec + (p << a.rsh))[0] = c;
}

// Up to 8 siblings: Batcher's 19-comparator odd-even merge network (padding key 0 sorts last:
// every child key has lamport >= 1).
__device__ __forceinline__ uint32_t link_small(const TreeArgs& a, const CsrArgs& c_, uint32_t g,
                                               uint32_t s0, uint32_t cnt) {
    uint64_t k[8];
    uint32_t c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = (uint32_t)i < cnt ? c_.child[s0 + i] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = (uint32_t)i < cnt ? a.key[c[i]] : 0ull;
    cxi(k[0], c[0], k[1], c[1]); cxi(k[2], c[2], k[3], c[3]);
    cxi(k[4], c[4], k[5], c[5]); cxi(k[6], c[6], k[7], c[7]);
    cxi(k[0], c[0], k[2], c[2]); cxi(k[1], c[1], k[3], c[3]);
    cxi(k[4], c[4], k[6], c[6]); cxi(k[5], c[5], k[7], c[7]);
    cxi(k[1], c[1], k[2], c[2]); cxi(k[5], c[5], k[6], c[6]);
    cxi(k[0], c[0], k[4], c[4]); cxi(k[1], c[1], k[5], c[5]);
    cxi(k[2], c[2], k[6], c[6]); cxi(k[3], c[3], k[7], c[7]);
    cxi(k[2], c[2], k[4], c[4]); cxi(k[3], c[3], k[5], c[5]);
    cxi(k[1], c[1], k[2], c[2]); cxi(k[3], c[3], k[4], c[4]); cxi(k[5], c[5], k[6], c[6]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if ((uint32_t)i < cnt) set_upr(a, c[i], (uint32_t)i + 1 < cnt ? c[i + 1 < 8 ? i + 1 : 7] : kNil, g);
    return c[0];
}

__global__ __launch_bounds__(kBlock) void k_link(TreeArgs a, CsrArgs c_) {
    __shared__ uint32_t nblk, bbase;
    if (threadIdx.x == 0) nblk = 0;
    __syncthreads();
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    bool defer = false;
    if (g < a.R) {
        const uint32_t w = a.pstart[g + 1] - a.pstart[g];
        if (a.in_parent[g] == kNil) set_upr(a, g, kNil, kNil);  // no sibling, no parent
        const uint32_t s0 = c_.cstart[g], cnt = c_.cstart[g + 1] - s0;
        uint32_t fc = kNil;
        if (cnt == 1) {
            const uint32_t c0 = c_.child[s0];
            fc = c0;
            set_upr(a, c0, kNil, g);
        } else if (cnt == 2) {
            uint32_t c0 = c_.child[s0], c1 = c_.child[s0 + 1];
            if (rs_before(a.key[c1], c1, a.key[c0], c0)) { const uint32_t t = c0; c0 = c1; c1 = t; }
            fc = c0;
            set_upr(a, c0, c1, g);
            set_upr(a, c1, kNil, g);
        } else if (cnt <= 8) {
            if (cnt) fc = link_small(a, c_, g, s0, cnt);
        } else {
            defer = true;  // first_child written by the sort kernels
        }
        set_dn(a, g, fc, w);
    }
    // deferred segments: one global atomic per block
    uint32_t slot = 0;
    if (defer) slot = atomicAdd(&nblk, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && nblk) bbase = atomicAdd(&a.ctl[C_NDEFER], nblk);
    __syncthreads();
    if (defer) c_.defer[bbase + slot] = g;
}

// One wave per deferred segment of 9..64 children: rank = #siblings before it, then ds_permute
// scatters ids into rank order and shuffles hand each lane its successor.
__global__ __launch_bounds__(kBlock) void k_sortmid(TreeArgs a, CsrArgs c_) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * kBlock) >> 6;
    const uint32_t nd = a.ctl[C_NDEFER];
    for (uint32_t i = (blockIdx.x * kBlock + threadIdx.x) >> 6; i < nd; i += nw) {
        const uint32_t p = c_.defer[i];
        const uint32_t s0 = c_.cstart[p], cnt = c_.cstart[p + 1] - s0;
        if (cnt > 64) {
            if (lane == 0) c_.bigl[atomicAdd(&a.ctl[C_NBIG], 1u)] = p;
            continue;
        }
        const bool on = lane < cnt;
        const uint32_t c = on ? c_.child[s0 + lane] : 0u;
        const uint64_t k = on ? a.key[c] : 0ull;
        const uint32_t khi = (uint32_t)(k >> 32), klo = (uint32_t)k;
        uint32_t rank = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t hj = (uint32_t)__shfl((int)khi, (int)j);
            const uint32_t lj = (uint32_t)__shfl((int)klo, (int)j);
            const uint32_t cj = (uint32_t)__shfl((int)c, (int)j);
            rank += rs_before(((uint64_t)hj << 32) | lj, cj, k, c) ? 1u : 0u;
        }
        // lane r <- id of rank r
        const uint32_t sorted =
            (uint32_t)__builtin_amdgcn_ds_permute((int)((on ? rank : lane) << 2), (int)c);
        const uint32_t succ = (uint32_t)__shfl((int)sorted, (int)((lane + 1) & 63));
        const uint32_t ns_of_rank = (lane + 1 < cnt) ? succ : kNil;
        const uint32_t ns = (uint32_t)__shfl((int)ns_of_rank, (int)(on ? rank : 0));
        if (on) {
            set_upr(a, c, ns, p);
            if (rank == 0) set_fcr(a, p, c);
        }
    }
}

// Bitonic sort (descending by key, run id) of one sibling segment of more than 64 children, in
// LDS up to kRsBigLds children, else in place in the child array ("flip" formulation: the
// padding to a power of two is never stored).
__global__ __launch_bounds__(kBigThreads) void k_sortbig(TreeArgs a, CsrArgs c_) {
    __shared__ uint64_t skey[kRsBigLds];
    __shared__ uint32_t sid[kRsBigLds];
    const uint32_t nb = a.ctl[C_NBIG];
    for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
        const uint32_t p = c_.bigl[bi];
        const uint32_t s0 = c_.cstart[p], cnt = c_.cstart[p + 1] - s0;
        uint32_t P = 1;
        while (P < cnt) P <<= 1;
        uint32_t* seg = c_.child + s0;
        const bool lds = P <= kRsBigLds;
        if (lds) {
            for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) {
                sid[i] = seg[i];
                skey[i] = a.key[seg[i]];
            }
            __syncthreads();
        }
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < P / 2; t += kBigThreads) {
                    const uint32_t i = (t / j) * 2 * j + (t % j);
                    const uint32_t l = (j == (k >> 1)) ? (i ^ (k - 1)) : (i ^ j);
                    if (l >= cnt) continue;
                    if (lds) {
                        if (rs_before(skey[l], sid[l], skey[i], sid[i])) {
                            const uint64_t tk = skey[i]; skey[i] = skey[l]; skey[l] = tk;
                            const uint32_t ti = sid[i]; sid[i] = sid[l]; sid[l] = ti;
                        }
                    } else {
                        const uint32_t ci = seg[i], cl = seg[l];
                        if (rs_before(a.key[cl], cl, a.key[ci], ci)) { seg[i] = cl; seg[l] = ci; }
                    }
                }
                __syncthreads();
            }
        }
        if (lds) {
            for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) seg[i] = sid[i];
            __syncthreads();
        }
        for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) {
            const uint32_t c = seg[i];
            set_upr(a, c, i + 1 < cnt ? seg[i + 1] : kNil, p);
        }
        if (threadIdx.x == 0) set_fcr(a, p, seg[0]);
        __syncthreads();
    }
}

// Euler-tour walks (sublist list ranking).  Regular splitters: both arcs of every run that is
// a multiple of M (splitter s <-> run (s>>1)<<log2m, arc s&1: 0 down, 1 up); plus one splitter
// per document for the down arc of its document-start run (index Sreg + d), the head of that
// document's list.  No arc leads into a document start's down arc, so walks only ever stop at
// regular splitters.  Returns false for an inactive splitter slot.
__device__ __forceinline__ bool splitter_arc(const TreeArgs& a, uint32_t s, uint32_t& v,
                                             bool& up) {
    if (s >= a.Sreg) {
        v = a.doc_root[s - a.Sreg];
        up = false;
        return true;
    }
    v = (s >> 1) << a.log2m;
    up = s & 1u;
    if (v >= a.R) return false;
    return up || a.in_parent[v] != kNil;  // a document start's down arc has its own splitter
}

// One step of a sublist walk from arc (v, up) with v's record r: the next arc, or false at the
// end of the sublist (the next arc is a splitter: *nxt = its index) or of the document's tour.
// A leaf's up arc follows its down arc from the same record.
__device__ __forceinline__ bool walk_next(const uint4& r, uint32_t m, uint32_t& v, bool& up,
                                          uint32_t& nxt) {
    const uint32_t mask = (1u << m) - 1u;
    uint32_t nv;
    bool nup;
    if (!up && r.x != kNil) {
        nv = r.x;
        nup = false;
    } else {
        if (!up && (v & mask) == 0) {  // a leaf whose up arc is a splitter
            nxt = ((v >> m) << 1) | 1u;
            return false;
        }
        if (r.z != kNil) { nv = r.z; nup = false; }
        else if (r.w != kNil) { nv = r.w; nup = true; }
        else return false;  // up arc of a document start: end of that document's tour
    }
    if ((nv & mask) == 0) {
        nxt = ((nv >> m) << 1) | (nup ? 1u : 0u);
        return false;
    }
    v = nv;
    up = nup;
    return true;
}

// Walks are chains of dependent random loads (one record per arc), so a thread can advance ILP
// sublists at once: that many loads in flight per thread instead of one.  Measured: 2 pays on
// waves without contraction (random trees, short sublists of single items), 1 on contracted
// waves (Fugue, config 4), whose walks diverge more.
// Text mode (TEXT): the walker also writes its sublist's text in walk order, the bytes of each
// run from its record's second line, into its splitter's kWalkTmp-byte slot of wtmp (a dword
// store per 4 bytes), and counts the runs it passes (reachability).
template <int ILP, bool TEXT>
__global__ __launch_bounds__(kBlock) void k_walk1(TreeArgs a) {
    const uint32_t base = (blockIdx.x * kBlock + threadIdx.x) * ILP;
    uint32_t v[ILP], sum[ILP], nxt[ILP], acc[ILP], live = 0, steps = 0, runs = 0;
    bool up[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
        const uint32_t s = base + q;
        sum[q] = 0;
        nxt[q] = kNil;
        v[q] = 0;
        up[q] = false;
        acc[q] = 0;
        if (s < a.S && splitter_arc(a, s, v[q], up[q])) live |= 1u << q;
    }
    while (live) {
        uint4 r[ILP], x[ILP];
#pragma unroll
        for (int q = 0; q < ILP; ++q)
            if ((live >> q) & 1u) {
                r[q] = a.rec[v[q] << (TEXT ? 1 : a.rsh)];
                if constexpr (TEXT) x[q] = a.rec[(v[q] << 1) + 1u];  // (the same 32-byte line)
            }
#pragma unroll
        for (int q = 0; q < ILP; ++q) {
            if (!((live >> q) & 1u)) continue;
            if (!up[q]) {
                const uint32_t w = r[q].y;
                if constexpr (!TEXT) {
                    // the run's offset inside its sublist and the sublist: k_expand adds the
                    // sublist's offset once the splitters are ranked (no second walk)
                    ++runs;
                    if (w) a.rloc[v[q]] = make_uint2(sum[q], base + q);  // (one 8-byte store)
                }
                if constexpr (TEXT) {
                    ++runs;
                    // append the run's bytes to the slot while they fit in it: up to kWalkText
                    // from the record, longer runs from the slot-order text
                    const uint32_t sb = 1u << a.wtmp_log2;
                    if (w && sum[q] < sb) {
                        uint32_t* slot = reinterpret_cast<uint32_t*>(
                            a.wtmp + ((uint64_t)(base + q) << a.wtmp_log2));
                        const uint32_t n = min(w, sb - sum[q]);
                        // (longer runs: the slot-order text a dword at a time)
                        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.sbytes);
                        uint32_t wd = x[q].y, sa = x[q].x;
                        for (uint32_t b = 0; b < n; ++b, ++sa) {
                            uint32_t c;
                            if (w <= kWalkText) {
                                c = (wd >> (8u * b)) & 255u;
                            } else {
                                if (b == 0 || (sa & 3u) == 0) wd = src[sa >> 2];
                                c = (wd >> (8u * (sa & 3u))) & 255u;
                            }
                            const uint32_t o = sum[q] + b;
                            acc[q] |= c << (8u * (o & 3u));
                            if ((o & 3u) == 3u) {
                                slot[o >> 2] = acc[q];
                                acc[q] = 0;
                            }
                        }
                    }
                }
                sum[q] += w;
            }
            if (!walk_next(r[q], a.log2m, v[q], up[q], nxt[q])) live &= ~(1u << q);
        }
        if (++steps > a.step_limit) {
            atomicOr(&a.ctl[C_ERR], 2u);
            break;
        }
    }
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
        if (base + q >= a.S) continue;
        a.swn[base + q] = make_uint2(sum[q], nxt[q]);
        // (the partial last dword of the slot; the bytes past the text are never copied)
        if (TEXT && (sum[q] & 3u) && sum[q] < (1u << a.wtmp_log2))
            reinterpret_cast<uint32_t*>(a.wtmp + ((uint64_t)(base + q) << a.wtmp_log2))[sum[q] >> 2] = acc[q];
    }
    // reachability: every run of the wave must be passed exactly once
    const uint32_t tot = wave_sum(runs);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&a.ctl[C_VISITED], tot);
}

// Ranking of the splitter lists (exclusive prefix of the sublist weights along each document's
// list), by sublists once more: every list head (a document start's splitter, s >= Sreg) and every
// regular splitter s = 0 mod kSup is a super-splitter; the supers' own lists are ranked by
// pointer jumping (kSup times fewer entries than the splitters), then every super walks its stretch
// of the splitter list once more writing the prefixes.  Two dependent gathers per splitter plus a
// few rounds over the supers, instead of log2(list length) rounds over all splitters.
// (kSup = 2^slog2: 64 on large waves, where the walks are throughput-bound; 8 on small ones,
// where a stretch walk is a chain of dependent loads that bounds the kernel)
__device__ __forceinline__ bool is_super(uint32_t s, uint32_t Sreg, uint32_t slog2) {
    return s >= Sreg || (s & ((1u << slog2) - 1u)) == 0u;
}
// compact index of a super: regular ones first, then one per document
__device__ __forceinline__ uint32_t super_idx(uint32_t s, uint32_t Sreg, uint32_t slog2) {
    return s >= Sreg ? ((Sreg + (1u << slog2) - 1u) >> slog2) + (s - Sreg) : s >> slog2;
}
__device__ __forceinline__ uint32_t super_of(uint32_t c, uint32_t Sreg, uint32_t slog2) {
    const uint32_t nr = (Sreg + (1u << slog2) - 1u) >> slog2;
    return c >= nr ? Sreg + (c - nr) : c << slog2;
}
struct SupArgs {
    uint32_t S, Sreg, Sc, step_limit, slog2;
    const uint2* swn;    // per splitter {weight, next}
    uint2* sup;          // per super {stretch weight, next super (compact, kNil: end)}
    uint32_t* pred;      // per super: its predecessor (kNil: a list head or unused)
    uint2* vp[2];        // pointer jumping {exclusive prefix, predecessor}
    uint32_t* spref;     // per splitter: its exclusive prefix along its list
    uint32_t* ctl;
};
__global__ __launch_bounds__(kBlock) void k_sup1(SupArgs a) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= a.Sc) return;
    uint32_t x = super_of(c, a.Sreg, a.slog2), sum = 0, nx = kNil, steps = 0;
    if (x < a.S) {
        for (;;) {
            const uint2 w = a.swn[x];
            sum += w.x;
            if (w.y == kNil) break;
            if (is_super(w.y, a.Sreg, a.slog2)) { nx = super_idx(w.y, a.Sreg, a.slog2); break; }
            x = w.y;
            if (++steps > a.step_limit) { atomicOr(&a.ctl[C_ERR], 2u); break; }
        }
    }
    a.sup[c] = make_uint2(sum, nx);
    if (nx != kNil) a.pred[nx] = c;  // (pred pre-filled with kNil)
}
__global__ __launch_bounds__(kBlock) void k_sup_init(SupArgs a) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= a.Sc) return;
    const uint32_t p = a.pred[c];
    a.vp[0][c] = make_uint2(p != kNil ? a.sup[p].x : 0u, p);
}
// One pointer-jumping round over the supers: {prefix so far, predecessor} packed, one gather.
__global__ __launch_bounds__(kBlock) void k_sup_step(const uint2* __restrict__ in, uint32_t n,
                                                     uint2* __restrict__ out) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= n) return;
    uint2 v = in[c];
    if (v.y != kNil) {
        const uint2 q = in[v.y];
        v = make_uint2(v.x + q.x, q.y);
    }
    out[c] = v;
}
__global__ __launch_bounds__(kBlock) void k_sup2(SupArgs a, const uint2* __restrict__ vp) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= a.Sc) return;
    uint32_t x = super_of(c, a.Sreg, a.slog2), steps = 0;
    if (x >= a.S) return;
    uint32_t pref = vp[c].x;
    for (;;) {
        const uint2 w = a.swn[x];
        a.spref[x] = pref;
        pref += w.x;
        if (w.y == kNil || is_super(w.y, a.Sreg, a.slog2)) break;
        x = w.y;
        if (++steps > a.step_limit) break;
    }
}

// Single workgroup: per-document length (weight between consecutive document starts), aligned
// output offsets, leaf offsets; for the LDS level 1 (wg != null) every k_doctree workgroup's
// descriptor (document, first run, runs, text prefix, text bytes, output offset), so that a
// k_doctree workgroup finds all of it in one round of loads.
__global__ __launch_bounds__(1024) void k_doctotals(TreeArgs a) {
    __shared__ uint64_t wt[16];  // per wave: its inclusive size total
    __shared__ uint32_t wl[16];  // (leaves)
    if (replan(a.ctl)) return;
    const uint32_t wtotal = a.ctl[C_WTOTAL];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint64_t carry_t = 0;
    uint32_t carry_l = 0;
    const uint64_t am = (uint64_t)a.align - 1u;
    for (uint32_t d0 = 0; d0 < a.ndocs; d0 += 1024) {
        const uint32_t d = d0 + threadIdx.x;
        uint32_t tl = 0, p0 = 0, r0 = 0, r1 = 0;
        if (d < a.ndocs) {
            const uint32_t end = d + 1 < a.ndocs ? a.doc_p0[d + 1] : wtotal;
            p0 = a.doc_p0[d];
            tl = end - p0;
            a.tlen[d] = tl;
            a.res[d] = make_uint4(tl, 0u, 0u, 0u);
            if (a.wg) {
                r0 = a.doc_root[d];
                r1 = d + 1 < a.ndocs ? a.doc_root[d + 1] : a.ctl[C_RTOTAL];
            }
        }
        const uint64_t sz = ((uint64_t)tl + am) & ~am;
        const uint32_t nl = a.align > 1 ? (tl + kLeaf - 1u) / kLeaf : 0u;
        // inclusive scans: the leaves by DPP, the 64-bit sizes by shuffles, then across the waves
        uint32_t il = wave_incl_scan(nl);
        uint64_t it = sz;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = ((uint64_t)(uint32_t)__shfl_up((int)(it >> 32), o) << 32) |
                               (uint32_t)__shfl_up((int)(uint32_t)it, o);
            if (lane >= (uint32_t)o) it += y;
        }
        if (lane == 63u) {
            wt[wv] = it;
            wl[wv] = il;
        }
        __syncthreads();
        uint64_t bt = 0, ct = 0;
        uint32_t bl = 0, cl = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            if (w < (int)wv) {
                bt += wt[w];
                bl += wl[w];
            }
            ct += wt[w];
            cl += wl[w];
        }
        __syncthreads();
        it += bt;
        il += bl;
        if (d < a.ndocs) {
            const uint64_t to = carry_t + it - sz;
            a.toff[d] = to;
            a.loff[d] = carry_l + il - nl;
            if (a.wg) {
                const uint32_t k = a.rank[d];
                const uint2 dr = a.docs[d];
                const uint32_t t0 = dr.x / kScanTile, t1 = (dr.x + dr.y) / kScanTile;
                a.wg[2u * k] = make_uint4(d, r0, r1 - r0, p0);
                a.wg[2u * k + 1u] = make_uint4(tl, (uint32_t)to, (uint32_t)(to >> 32),
                                               t0 | (min(t1 - t0, 0xFFFu) << 20));
            }
        }
        carry_t += ct;
        carry_l += cl;
    }
    if (threadIdx.x == 0) {
        a.toff[a.ndocs] = carry_t;
        a.loff[a.ndocs] = carry_l;
        if (carry_t > a.text_cap) atomicOr(&a.ctl[C_ERR], 4u);
    }
}

// The document of splitter s (whose first arc is v's).
__device__ __forceinline__ uint32_t splitter_doc(const TreeArgs& a, uint32_t s, uint32_t v) {
    return s >= a.Sreg ? s - a.Sreg : a.chunk_doc[a.r_head[v] >> a.log2c];
}

// Text mode, once the splitters are ranked: every sublist's staged text (up to its slot's bytes)
// to its place in its document, one thread per splitter, dword stores where the destination is
// aligned; sublists with more text are listed for k_walk_ovf.  The sublist's whole range is
// bounds-checked here (its weight is the walk's).
__global__ __launch_bounds__(kBlock) void k_tcopy(TreeArgs a, const uint32_t* __restrict__ spref) {
    if (replan(a.ctl)) return;
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    uint32_t v;
    bool up;
    if (s >= a.S || !splitter_arc(a, s, v, up)) return;
    const uint32_t n = a.swn[s].x;
    if (!n) return;
    const uint32_t d = splitter_doc(a, s, v), o = spref[s];
    if ((uint64_t)o + n > a.tlen[d]) {
        atomicOr(&a.ctl[C_ERR], 8u);
        return;
    }
    const uint32_t sb = 1u << a.wtmp_log2;
    if (n > sb) a.ovf[atomicAdd(&a.ctl[C_NOVF], 1u)] = s;  // (room for every splitter)
    const uint32_t m = min(n, sb);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.wtmp + ((uint64_t)s << a.wtmp_log2));
    uint8_t* dst = a.text + a.toff[d] + o;
    auto byte_at = [&](uint32_t i) { return (src[i >> 2] >> (8u * (i & 3u))) & 255u; };
    const uint32_t head = min(m, (4u - (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u);
    uint32_t i = 0;
    for (; i < head; ++i) dst[i] = (uint8_t)byte_at(i);
    const uint32_t sh = 8u * (i & 3u);
    for (; i + 4u <= m; i += 4u) {
        const uint32_t lo = src[i >> 2];
        const uint32_t wd = sh ? (lo >> sh) | (src[(i >> 2) + 1u] << (32u - sh)) : lo;
        *reinterpret_cast<uint32_t*>(dst + i) = wd;
    }
    for (; i < m; ++i) dst[i] = (uint8_t)byte_at(i);
}

// Text mode: the sublists k_tcopy listed, walked again; each writes the bytes past its slot.
__global__ __launch_bounds__(kBlock) void k_walk_ovf(TreeArgs a, const uint32_t* __restrict__ spref) {
    if (replan(a.ctl)) return;
    const uint32_t n = a.ctl[C_NOVF], sb = 1u << a.wtmp_log2;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const uint32_t s = a.ovf[i];
        uint32_t v, nxt, off = 0, steps = 0;
        bool up;
        if (!splitter_arc(a, s, v, up)) continue;
        uint8_t* out = a.text + a.toff[splitter_doc(a, s, v)] + spref[s];
        for (bool go = true; go;) {
            const uint4 r = a.rec[v << 1];
            if (!up) {
                const uint32_t w = r.y;
                if (w && off + w > sb) {
                    const uint32_t b0 = off >= sb ? 0u : sb - off;
                    const uint4 x = a.rec[(v << 1) + 1u];
                    const uint8_t* src = a.sbytes + x.x;
                    for (uint32_t b = b0; b < w; ++b)
                        out[off + b] = w <= kWalkText ? (uint8_t)(x.y >> (8u * b)) : src[b];
                }
                off += w;
            }
            go = walk_next(r, a.log2m, v, up, nxt);
            if (++steps > a.step_limit) break;  // (k_walk1 flagged it)
        }
    }
}

__device__ uint64_t xxh64_aligned(const uint8_t* __restrict__ p, uint32_t len, uint64_t seed);

// ---------------------------------------------------------------------------------------------
// Level 1 in LDS: the whole run tree of one document per workgroup (k_doctree)
// ---------------------------------------------------------------------------------------------
// Documents of the batched configs have at most ~10 k runs, so a document's run tree fits a
// workgroup's 160 KiB of LDS as four u16 arrays (8 B/run).  The count / scan / place / sort /
// Euler-tour ranking sequence of the global level-1 path then runs on LDS atomics and LDS
// gathers inside one 1024-thread workgroup, with barriers between phases, instead of 7+
// grid-wide kernels of HBM atomics and dependent HBM gathers.  From global memory it reads
// r_parent and r_w (coalesced) and r_key (sibling groups of two or more only); it writes the
// run offsets roff exactly as the global path's k_walk1 + sublist prefixes do.
//
// LDS image until the siblings are sorted (u16 arrays indexed by the local run v in [0, R); run 0
// is the document start):
//   D[v]   child count -> segment start (exclusive scan) -> segment end (after placement)
//   nx[v]  parent until placement, then the tour successor of v's up arc: the next sibling's
//          down arc, (parent | kUp16) = the parent's up arc, or kNil16 for the root
//   ch[]   children grouped by parent (segment of v = [D[v-1], D[v])), sorted by key desc
//   w[v]   the weight (0xFFFF: look it up in the LDS side table of big runs)
//   gl[]   the work list of sibling groups of two or more
// then one 8-byte record per run over the D / nx / ch / w arrays, so that a walk step is one
// LDS read:
//   rec[v] = {first child | nx << 16, weight | spare << 16}; once walk 1 has passed v's down
//            arc the second word holds v's offset inside its sublist (18 bits) and the sublist
//            (14 bits); 0xFFFFFFFF for weightless runs
// and the splitter records (u32 sublist sum << 14 | next splitter) in the gl region.
// Splitters are the down arcs of one run per block of 4 (splitter_run: block b, hashed offset).  Up arcs carry no
// weight and never split: pointer jumping over the last-child up links until none is left makes
// the tour a list of down arcs only (a leaf goes straight to the next sibling of its nearest
// ancestor-or-self that has one).  A walker that passes v's down arc leaves v's offset inside its
// sublist and the sublist's id in v's LDS entries, and once the splitter list is ranked (pointer
// jumping) one pass turns them into document offsets.
// Volatile LDS accesses through LDS-typed pointers: a volatile access through a generic pointer
// is not narrowed to the LDS aperture by the compiler and becomes a system-coherent flat access.
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) uint16_t lds_u16_t;
__device__ __forceinline__ uint32_t lds_ld32(uint32_t* p) { return *(volatile lds_u32_t*)p; }
__device__ __forceinline__ void lds_st32(uint32_t* p, uint32_t v) { *(volatile lds_u32_t*)p = v; }
__device__ __forceinline__ uint32_t lds_ld16(uint16_t* p) { return *(volatile lds_u16_t*)p; }
__device__ __forceinline__ void lds_st16(uint16_t* p, uint32_t v) { *(volatile lds_u16_t*)p = (uint16_t)v; }

constexpr int kDocThreads = 1024;
#ifndef CRDT_DOC_J
// 12,288 runs per document: the traces need at most 10,113 (seph-blog1) once dead runs are
// dropped.  Every per-run loop is unrolled kDocJ times (the per-thread arrays live in VGPRs), so
// kDocJ sets the code size: 20 made k_doctree 60 KB of code, 12 makes it 42 KB and the kernel
// ~8 % faster (A/B at the headline config; an instruction cache is shared by two CUs).
#define CRDT_DOC_J 17
#endif
constexpr int kDocJ = CRDT_DOC_J;  // runs per thread: documents of up to kDocJ * 1024 runs
#ifndef CRDT_DOC_LOG2S
#define CRDT_DOC_LOG2S 2
#endif
// splitters: one run per block of 2^kDocLog2S consecutive runs, at a hashed position inside the
// block (block 0: the document start), so that no chain of the tour whose run indices share a
// residue can miss every splitter; splitter b = block b; (J + S - 1) / S per thread
constexpr uint32_t kDocLog2S = CRDT_DOC_LOG2S;
#ifndef CRDT_DOC_HASHSPLIT
#define CRDT_DOC_HASHSPLIT 1
#endif
#ifndef CRDT_DOC_WALK_WAVES
#define CRDT_DOC_WALK_WAVES 16
#endif
// The offset is a Fibonacci hash of the block index (the top bits of the low 16 bits of its
// product with 2^16 / phi: one full-rate 24-bit multiply), so that the walk tests every node it
// reaches for being a splitter in three VALU ops.
__device__ __forceinline__ uint32_t splitter_off(uint32_t b) {
    if (!CRDT_DOC_HASHSPLIT) return 0u;
    return (__umul24(b, 0x9E37u) >> (16u - kDocLog2S)) & ((1u << kDocLog2S) - 1u);
}
__device__ __forceinline__ uint32_t splitter_run(uint32_t b) {
    return (b << kDocLog2S) | splitter_off(b);
}
constexpr uint32_t kDocLds = 163840 - 1024;  // dynamic LDS budget (static arrays use the rest)
constexpr uint16_t kNil16 = 0xFFFFu;
constexpr uint16_t kUp16 = 0x8000u;
constexpr uint32_t kNil14 = 0x3FFFu;   // no next splitter (splitter records: sum << 14 | next)
// Documents staged from the per-tile text segments span at most this many tiles (a tile prefix
// table of kDocTiles + 1 entries in LDS): documents of up to ~4 M slots
constexpr uint32_t kDocTiles = 1024;

struct DocArgs {
    uint32_t ndocs, rcap, scap, chbytes;
    uint32_t probe;  // 1 + document whose phase times are printed (0: none)
    const uint32_t* doc_root;
    // per workgroup (costliest document first), written by k_doctotals: {document, first run,
    // runs, text prefix}, {text bytes, output offset lo, hi, first tile | (tiles - 1) << 20}
    const uint4* wg;
    // stile_text: the slot-order text is read from the tiles' segments (k_classify's stile, one
    // kTileBytes segment per tile, tile_hw .y = the tile's weight prefix after the scan) instead
    // of sbytes, which k_runs then does not write
    uint32_t stile_text, ntiles;
    const uint8_t* stile;
    const uint2* tile_hw;
    uint32_t keyoff;  // LDS byte offset of the sibling keys
    const uint32_t* r_parent;
    const uint64_t* r_key;
    uint32_t* roff;
    uint32_t* ctl;
    // fused text (phase C): text == nullptr leaves the run offsets in roff for k_expand
    const uint32_t* r_pstart;
    const uint32_t* doc_p0;
    const uint32_t* tlen;
    const uint64_t* toff;
    const uint8_t* sbytes;
    uint8_t* text;
    uint8_t* fused;       // per document: 1 = text written by k_doctree
    uint32_t lds_bytes;   // dynamic LDS of the launch
    // scatter mode (text == nullptr): roff[run] = the run's place in the wave's text (its
    // document's output offset + its document offset, u32) for k_tscatter, which moves the text
    uint32_t scatter;
    uint32_t glds_late;  // test hook: LDS-DMA staging loads issued last (doc_text)
};

// LDS bytes of a document with up to rcap - 2 runs: D, nx, ch (2 B/run each), the sibling keys
// (4 B/run, doc_key32; the 8-byte run records later take D, nx, ch and the keys) and the gl
// region: the work list of sibling groups of three or more (at most one per three runs), later
// the splitter records (4 B per splitter).
__host__ __device__ constexpr uint32_t doctree_ch_bytes(uint32_t rcap, uint32_t) {
    return (2u * rcap + 15u) & ~15u;
}
// sibling groups of two or more: at most one per two runs
__host__ __device__ constexpr uint32_t doctree_defer_cap(uint32_t rcap) { return rcap / 2u + 8u; }
__host__ __device__ constexpr uint32_t doctree_gl_bytes(uint32_t rcap, uint32_t scap) {
    return ((2u * doctree_defer_cap(rcap) > 4u * scap ? 2u * doctree_defer_cap(rcap) : 4u * scap) +
            15u) & ~15u;
}
// k32 (k_doctree_wide): 4-byte keys, and no nx array of its own: a run's up-arc successor is
// written into its key slot once the key is dead (D, ch, keys: 8 B per run, + gl)
__host__ __device__ constexpr uint32_t doctree_key_off(uint32_t rcap, uint32_t scap, bool k32) {
    return ((k32 ? 2u : 4u) * rcap + doctree_ch_bytes(rcap, scap) + 15u) & ~15u;
}
__host__ __device__ constexpr uint64_t doctree_lds_bytes(uint32_t rcap, uint32_t scap, bool k32) {
    return (uint64_t)doctree_key_off(rcap, scap, k32) + (k32 ? 4ull : 8ull) * rcap +
           doctree_gl_bytes(rcap, scap);
}
// the nx array: its own u16 array, or (k32) the low half of every run's 4-byte key slot
struct NxRef {
    uint16_t* p;
    uint32_t stride;
    __device__ __forceinline__ uint16_t& operator[](uint32_t v) const { return p[stride * v]; }
};

// Sort key: the run head's (lamport, agent) (Fugue: and the left-child bit) compressed to 32
// bits for this document (doc_key32), and the local run index (15 bits), so that equal
// timestamps still order deterministically (greater run first, as the oracle does).  The keys
// were staged in LDS by the load phase.
template <bool K32>
__device__ __forceinline__ uint64_t doc_key(const void* keys, uint32_t v) {
    if (K32) return ((uint64_t) reinterpret_cast<const uint32_t*>(keys)[v] << 15) | v;
    return (reinterpret_cast<const uint64_t*>(keys)[v] << 15) | v;
}
// A run key (lamport << 16 | agent, bit 48 = a Fugue left child, kMidKey = a Fugue content row)
// as 32 bits that order siblings the same way: left children above everything (bit 31), then
// the content row (0x7FFFFFFF), then lamport << 8 | agent.  That holds for lamports below 2^23
// and agents below 256 (the traces: lamport < 2^20, one agent); a document with a wider key
// (key32_fits, checked in the load phase) goes to the global level 1, which sorts the 64-bit
// keys.  (A per-document layout from the document's largest lamport and agent cost k_doctree 6 %:
// the reduction kept every 64-bit key live across a barrier.)
constexpr uint32_t kKey32Agent = 8;
__device__ __forceinline__ bool key32_fits(uint64_t k) {  // (lamport < 2^23 - 1, agent < 256)
    return (k & 0xFF00u) == 0u && ((k >> 16) & 0xFFFFFFFFull) < (1ull << (31 - kKey32Agent)) - 1u;
}
__device__ __forceinline__ uint32_t doc_key32(uint64_t k) {
    if (k == kMidKey) return 0x7FFFFFFFu;
    const uint32_t c = ((uint32_t)(k >> 16) << kKey32Agent) | (uint32_t)(k & 0xFFu);
    return (k & kLeftKey) ? (c | 0x80000000u) : c;
}

// Phase C of k_doctree: expansion fused, when the document's text and its run-start index fit
// LDS.  1) The document's visible UTF-8 in slot order (one contiguous range of sbytes: runs are
// numbered in slot order) is staged in LDS with 16-byte loads.  2) Every run with visible bytes
// sets the bit of its document offset in a bitvector over the document; with u16 prefix counts
// per 32-bit word this gives the run its rank in document order, and it stores
// delta[rank] = staging offset - document offset.  3) The document is written in order, 4 bytes
// per lane (256-byte coalesced stores per wave): byte y belongs to the run of the last set bit
// at or before y.  Returns false (nothing written) when the document does not fit.
constexpr int kDocQ = 10;  // 16-byte pieces per thread: texts up to 160 KiB
// Staging from the tiles' text segments (DocArgs::stile_text): the document's text is the part
// [p0, p0 + tl) of the weight range of tiles t0 .. t0 + nt, each tile's share contiguous in its
// kTileBytes segment, staged at offset (weight position - p0 + sh).  tpx = the tiles' weight
// prefixes (the first nt + 2 lanes hold one each).  Work items are the 16-byte staging chunks each
// tile's share overlaps (a block scan of the per-tile counts, then a 10-step binary search per
// item over the table in LDS).  A chunk wholly inside one share is two aligned 16-byte loads from
// the segment, a funnel shift and one 16-byte LDS store; a chunk a share only partly covers (at
// most two per tile) stores its bytes one by one (the neighbouring tile stores the rest).
// First step of a power-of-two search over table entries 0..n (the steps sum to at least n):
// the document's tiles, not the kernel's 1024 at most
__device__ __forceinline__ uint32_t search_step0(uint32_t n) { return n ? 1u << (31 - __builtin_clz(n)) : 0u; }
__device__ __forceinline__ uint32_t funnel_byte(uint32_t lo, uint32_t hi, uint32_t b) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * b));
}
__device__ __forceinline__ void stage_from_tiles(const DocArgs& a, uint32_t p0, uint32_t tl,
                                                 uint32_t sh, uint32_t t0, uint32_t nt,
                                                 uint32_t tpx_reg, uint8_t* st, uint32_t* tab,
                                                 uint32_t* scan_lds) {
    const uint32_t t = threadIdx.x;
    uint32_t* tpx = tab;               // nt + 2 weight prefixes
    uint32_t* itp = tab + (nt + 2u);   // nt + 2 item prefixes
    if (t <= nt + 1u) tpx[t] = tpx_reg;
    __syncthreads();
    const uint32_t base = p0 - sh;  // weight position of staging byte 0
    uint32_t cnt = 0;
    if (t <= nt) {
        const uint32_t lo = max(tpx[t], p0), hi = min(tpx[t + 1u], p0 + tl);
        cnt = hi > lo ? ((hi - base + 15u) >> 4) - ((lo - base) >> 4) : 0u;
    }
    uint32_t total;
    const uint32_t ex = block_excl_scan<kDocThreads / 64>(cnt, scan_lds, total);
    if (t <= nt) itp[t] = ex;
    __syncthreads();
    constexpr int kE = 2;  // items per thread and round (registers: ro / ps are live here)
    for (uint32_t i0 = 0; i0 < total; i0 += kE * kDocThreads) {
        uint32_t kk[kE], ii[kE];
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            ii[e] = i0 + t + (uint32_t)e * kDocThreads;
            kk[e] = 0;
        }
        // the last tile whose first item is at or before the item (log2(nt) + 1 steps)
        for (uint32_t step = search_step0(nt); step; step >>= 1) {
#pragma unroll
            for (int e = 0; e < kE; ++e) {
                const uint32_t c = min(kk[e] + step, nt);  // (branch-free: reads issue together)
                kk[e] = itp[c] <= ii[e] ? c : kk[e];
            }
        }
        uint4 q0[kE], q1[kE];
        uint32_t cb[kE], slo[kE], shi[kE], u[kE];
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            const uint32_t x0 = tpx[kk[e]];
            const uint32_t lo = max(x0, p0) - base, hi = min(tpx[kk[e] + 1u], p0 + tl) - base;
            cb[e] = ((lo >> 4) + (ii[e] - itp[kk[e]])) << 4;  // the chunk (staging offset)
            slo[e] = lo;                                       // the share, in staging offsets
            shi[e] = ii[e] < total ? hi : 0u;
            // the chunk's first byte in the tile's segment, and the aligned pair covering it
            u[e] = cb[e] + base - x0;
            const uint4* src = reinterpret_cast<const uint4*>(
                a.stile + (uint64_t)(t0 + kk[e]) * kTileBytes + (u[e] & ~15u));
            q0[e] = make_uint4(0, 0, 0, 0);
            q1[e] = make_uint4(0, 0, 0, 0);
            if (ii[e] < total && cb[e] >= slo[e] && cb[e] + 16u <= shi[e]) {
                q0[e] = src[0];
                q1[e] = src[1];
            }
        }
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            if (ii[e] >= total) continue;
            if (cb[e] >= slo[e] && cb[e] + 16u <= shi[e]) {
                // wholly inside the share: 16 bytes from the aligned pair, shifted
                const uint32_t w[8] = {q0[e].x, q0[e].y, q0[e].z, q0[e].w,
                                       q1[e].x, q1[e].y, q1[e].z, q1[e].w};
                const uint32_t dw = (u[e] >> 2) & 3u, b = u[e] & 3u;
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // w[dw + k] and w[dw + k + 1] by selects (dw is per lane)
                    uint32_t lo = w[k], hi = w[k + 1];
#pragma unroll
                    for (uint32_t s2 = 1; s2 < 4; ++s2)
                        if (dw == s2) { lo = w[k + s2]; hi = w[k + s2 + 1]; }
                    o[k] = funnel_byte(lo, hi, b);
                }
                *reinterpret_cast<uint4*>(st + cb[e]) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
                // partly covered: the covered bytes one by one, from the segment directly
                const uint8_t* seg = a.stile + (uint64_t)(t0 + kk[e]) * kTileBytes;
                const uint32_t x0 = tpx[kk[e]];
                for (uint32_t j = max(cb[e], slo[e]); j < min(cb[e] + 16u, shi[e]); ++j)
                    st[j] = seg[j + base - x0];
            }
        }
    }
}

// Staging by LDS-DMA (DocArgs::stile_text == 2).  No run crosses a tile (k_heads), so the text
// need not be contiguous across tiles: tile k's share of the document is staged as the aligned
// 16-byte chunks of its segment that cover it, verbatim (chunks before it: cpx[k]; the first one at
// segment offset akt[k]).  Chunk c is one lane of a global_load_lds_dwordx4 (the LDS image of a
// wave instruction is lane-linear: 64 consecutive chunks); its tile comes from a binary search of
// cpx, four chunks per thread at once, and every load of the staging is in flight before the one
// wait at the barrier.  A run of tile k then reads its text at staging offset
// 16 cpx[k] + (ps - tpx[k]) - akt[k].  No register holds the bytes, no byte is shifted, and no
// chunk is partly copied.  Table: tpx, cpx, akt (nt + 2 u32 each) at `tab`.
// The table (returns the chunk count C); stage_glds_issue then issues the loads.
__device__ __forceinline__ uint32_t stage_glds_table(uint32_t p0, uint32_t tl, uint32_t nt,
                                                     uint32_t tpx_reg, uint32_t* tab,
                                                     uint32_t* scan_lds) {
    const uint32_t t = threadIdx.x;
    uint32_t* tpx = tab;
    uint32_t* cpx = tab + (nt + 2u);
    uint32_t* akt = cpx + (nt + 2u);
    if (t <= nt + 1u) tpx[t] = tpx_reg;
    __syncthreads();
    uint32_t nk = 0, ak = 0;
    if (t <= nt) {
        const uint32_t x0 = tpx[t];
        const uint32_t lo = max(x0, p0), hi = min(tpx[t + 1u], p0 + tl);
        if (hi > lo) {
            ak = (lo - x0) & ~15u;
            nk = ((hi - x0 + 15u) >> 4) - (ak >> 4);
        }
    }
    uint32_t C;
    const uint32_t ex = block_excl_scan<kDocThreads / 64>(nk, scan_lds, C);
    if (t <= nt) {
        cpx[t] = ex;
        akt[t] = ak;
    }
    __syncthreads();
    return C;
}
__device__ __forceinline__ void stage_glds_issue(const DocArgs& a, uint32_t C, uint32_t t0,
                                                 uint32_t nt, uint8_t* st, const uint32_t* tab) {
    const uint32_t t = threadIdx.x;
    const uint32_t* cpx = tab + (nt + 2u);
    const uint32_t* akt = cpx + (nt + 2u);
    const uint32_t lane = t & 63u, wv = t >> 6;
    constexpr int kG = 4;  // chunks per thread per round (their tile searches interleave)
    for (uint32_t c0 = 64u * wv; c0 < C; c0 += 64u * 16u * kG) {
        uint32_t k[kG];
#pragma unroll
        for (int e = 0; e < kG; ++e) k[e] = 0;
        // (branch-free: the clamped probe and a select, so that the kG reads of a step issue
        // together instead of one exec-masked read and wait each)
        for (uint32_t step = search_step0(nt); step; step >>= 1) {
#pragma unroll
            for (int e = 0; e < kG; ++e) {
                const uint32_t c = c0 + 1024u * (uint32_t)e + lane;
                const uint32_t q = min(k[e] + step, nt);
                k[e] = cpx[q] <= c ? q : k[e];
            }
        }
#pragma unroll
        for (int e = 0; e < kG; ++e) {
            const uint32_t cb = c0 + 1024u * (uint32_t)e;  // (wave-uniform: the LDS base)
            const uint32_t c = cb + lane;
            if (c < C) {
                const uint8_t* src = a.stile + (uint64_t)(t0 + k[e]) * kTileBytes + akt[k[e]] +
                                     16u * (c - cpx[k[e]]);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)src,
                    (__attribute__((address_space(3))) void*)(st + 16u * cb), 16, 0, 0);
            }
        }
    }
    // (the loads land while the run starts, prefix counts and deltas are computed; doc_text
    // waits for them before the barrier in front of the text output)
}

template <int J>
__device__ __forceinline__ bool doc_text(const DocArgs& a, uint32_t tl, uint32_t p0, uint64_t toff,
                                         uint32_t tiles, uint32_t tpx_reg,
                                         const uint32_t (&ro)[J], const uint32_t (&ps)[J],
                                         uint8_t* st, uint32_t* scan_lds, uint64_t* tprobe) {
    const uint32_t t = threadIdx.x;
    const bool glds = a.stile_text == 2u;
    const uint32_t sh = glds ? 0u : p0 & 15u;
    const uint32_t t0 = tiles & 0xFFFFFu, nt = tiles >> 20;
    // staged 16-byte pieces (glds: every tile share's covering chunks, at most two partly used
    // per tile)
    const uint32_t nq = glds ? ((tl + 15u) >> 4) + 2u * (nt + 1u) : (sh + tl + 15u) >> 4;
    const uint32_t nw = (tl + 31u) >> 5;       // bitvector words
    const uint32_t o_bits = 16u * nq + 16u, o_pref = o_bits + 4u * nw;
    const uint32_t o_delta = (o_pref + 2u * nw + 15u) & ~15u;
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) mine += ro[j] != kNil ? 1u : 0u;
    uint32_t Rw;
    (void)block_excl_scan<kDocThreads / 64>(mine, scan_lds, Rw);
    const uint32_t o_tab = (o_delta + 4u * Rw + 15u) & ~15u;
    if (o_tab + (a.stile_text ? (glds ? 12u : 8u) * (nt + 2u) : 0u) > a.lds_bytes ||
        (!glds && nq > (uint32_t)(kDocQ * kDocThreads)))
        return false;
    uint32_t* bits = reinterpret_cast<uint32_t*>(st + o_bits);
    uint16_t* pref = reinterpret_cast<uint16_t*>(st + o_pref);
    uint32_t* delta = reinterpret_cast<uint32_t*>(st + o_delta);
    uint32_t* tab = reinterpret_cast<uint32_t*>(st + o_tab);
    if (tprobe) tprobe[1] = wall_clock64();
    // 1) staging (every load first; the run prefixes ps were loaded before the offsets).  Test
    // hook glds_late: the LDS-DMA loads are issued after the deltas instead, right in front of
    // the wait and barrier before the output, so that the output reads chunks still in flight
    // unless that wait holds (tests/test_gpu_merge.py pins the engine.hip vmcnt wait with it)
    uint32_t gC = 0;
    if (a.stile_text) {
        for (uint32_t i = t; i < nw; i += kDocThreads) bits[i] = 0;
        if (glds) {
            gC = stage_glds_table(p0, tl, nt, tpx_reg, tab, scan_lds);
            if (!a.glds_late) stage_glds_issue(a, gC, t0, nt, st, tab);
        } else {
            stage_from_tiles(a, p0, tl, sh, t0, nt, tpx_reg, st, tab, scan_lds);
        }
    }
    {
        if (!a.stile_text) {
            const uint4* src = reinterpret_cast<const uint4*>(a.sbytes + (p0 - sh));
            uint4 q[kDocQ];
#pragma unroll
            for (int k = 0; k < kDocQ; ++k) {
                const uint32_t i = t + (uint32_t)k * kDocThreads;
                q[k] = i < nq ? src[i] : make_uint4(0, 0, 0, 0);
            }
            for (uint32_t i = t; i < nw; i += kDocThreads) bits[i] = 0;
            uint4* stq = reinterpret_cast<uint4*>(st);
#pragma unroll
            for (int k = 0; k < kDocQ; ++k) {
                const uint32_t i = t + (uint32_t)k * kDocThreads;
                if (i < nq) stq[i] = q[k];
            }
        }
        __syncthreads();
        if (tprobe) tprobe[2] = wall_clock64();
        // 2) run starts -> ranks in document order -> staging offset minus document offset
#pragma unroll
        for (int j = 0; j < J; ++j)
            if (ro[j] != kNil) atomicOr(&bits[ro[j] >> 5], 1u << (ro[j] & 31u));
        __syncthreads();
        if (tprobe) tprobe[3] = wall_clock64();
        {
            const uint32_t K = (nw + kDocThreads - 1) / kDocThreads;
            const uint32_t lo = min(nw, t * K), hi = min(nw, lo + K);
            uint32_t c = 0;
            for (uint32_t i = lo; i < hi; ++i) c += (uint32_t)__popc(bits[i]);
            uint32_t tot;
            uint32_t ex = block_excl_scan<kDocThreads / 64>(c, scan_lds, tot);
            for (uint32_t i = lo; i < hi; ++i) {
                pref[i] = (uint16_t)ex;
                ex += (uint32_t)__popc(bits[i]);
            }
        }
        __syncthreads();
        if (tprobe) tprobe[4] = wall_clock64();
        // (glds) the tile of every owned run's text: the last tile whose weight prefix is at or
        // below the run's (runs do not cross tiles), ten interleaved search steps
        // dv[j]: the run's staging offset minus its document offset (glds: the tile search
        // result first, then turned into the delta in place)
        uint32_t dv[J];
#pragma unroll
        for (int j = 0; j < J; ++j) dv[j] = 0;
        if (glds) {
            for (uint32_t step = search_step0(nt); step; step >>= 1) {
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const uint32_t q = min(dv[j] + step, nt);  // (branch-free, as in stage_glds)
                    dv[j] = tab[q] <= ps[j] ? q : dv[j];
                }
            }
#pragma unroll
            for (int j = 0; j < J; ++j)
                dv[j] = 16u * tab[nt + 2u + dv[j]] + (ps[j] - tab[dv[j]]) -
                        tab[2u * (nt + 2u) + dv[j]] - ro[j];
        } else {
#pragma unroll
            for (int j = 0; j < J; ++j) dv[j] = ps[j] - p0 + sh - ro[j];
        }
        uint32_t rk[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t y = ro[j] != kNil ? ro[j] : 0u;
            const uint32_t wd = y >> 5;
            rk[j] = pref[wd] + (uint32_t)__popc(bits[wd] & ((1u << (y & 31u)) - 1u));
        }
#pragma unroll
        for (int j = 0; j < J; ++j)
            if (ro[j] != kNil) delta[rk[j]] = dv[j];
    }
    if (glds && a.glds_late) stage_glds_issue(a, gC, t0, nt, st, tab);
    // (LDS-DMA staging) the DMA writes LDS as a global load, and a workgroup barrier waits only
    // for LDS operations (lgkmcnt): every wave waits for its own staging loads (vmcnt) before the
    // barrier after which any wave reads any staged chunk
    if (glds) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tprobe) *tprobe = wall_clock64();
    // 3) the document in order, 16 bytes per lane per step (one bitvector word covers them)
    uint4* out = reinterpret_cast<uint4*>(a.text + toff);  // 16-aligned
    // The run of the piece's first byte (the last start at or before it) comes from the bitvector
    // and its prefix count; every later start inside the piece (bit b of m) moves to the next run
    // in document order, whose delta is read then (an LDS read only in the lanes that have a
    // start at b: ~1 in 11 bytes on the traces, instead of one read per byte).  (A branch-free
    // form that reads the first four runs' deltas up front and picks one per byte by selects
    // made k_doctree 10 % slower: its per-byte VALU work costs more than the waits it saves.)
    for (uint32_t i = t; i < (tl + 15u) >> 4; i += kDocThreads) {
        const uint32_t y0 = 16u * i, wd = y0 >> 5, b0 = y0 & 31u;
        const uint32_t bw = bits[wd], pr = pref[wd];
        const uint32_t m = bw >> b0;  // bit b: a run starts at y0 + b
        uint32_t r = pr + (uint32_t)__popc(bw & ((2u << b0) - 1u)) - 1u;
        uint32_t dl = delta[r];
        uint32_t q[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b) {
            if (b && ((m >> b) & 1u)) dl = delta[++r];
            if (y0 + b < tl) q[b >> 2] |= (uint32_t)st[y0 + b + dl] << (8u * (b & 3u));
        }
        out[i] = make_uint4(q[0], q[1], q[2], q[3]);
    }
    return true;
}

// One document (workgroup descriptor widx); the kernel below runs it once per descriptor.  K32:
// the sibling keys are held in LDS as doc_key32 (4 bytes per run instead of 8).
template <int J, bool K32, bool PC>
__device__ __forceinline__ void doctree_doc(const DocArgs& a, uint32_t widx) {
    constexpr int KK = (J + (1 << kDocLog2S) - 1) >> kDocLog2S;
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    __shared__ uint32_t scan_lds[kDocThreads / 64];
    __shared__ uint32_t nwide, flags, visited_lds;
#ifdef CRDT_HIP_PROBE
    __shared__ uint32_t probe_max, probe_sum, probe_wave[48];
#endif
    const uint32_t t = threadIdx.x;
    // the plan check and the workgroup's document (written by k_doctotals in LPT order: document,
    // first run, runs, text offset / length) in one round of loads
#ifdef CRDT_HIP_PROBE
    const uint64_t tdesc = wall_clock64();  // (before the descriptor's round trip)
#endif
    const uint4 wg = a.wg[2u * widx], wg1 = a.wg[2u * widx + 1u];
    if (replan(a.ctl)) return;
    const uint32_t d = wg.x, base = wg.y, R = wg.z;
    (void)d;
    const uint32_t S = (R + (1u << kDocLog2S) - 1u) >> kDocLog2S;
    uint16_t* D = reinterpret_cast<uint16_t*>(dyn);
    uint8_t* keys = reinterpret_cast<uint8_t*>(dyn) + a.keyoff;
    const NxRef nx{K32 ? reinterpret_cast<uint16_t*>(keys) : D + a.rcap, K32 ? 2u : 1u};
    uint16_t* ch = D + (K32 ? 1u : 2u) * a.rcap;
    uint16_t* glist = reinterpret_cast<uint16_t*>(keys + (K32 ? 4u : 8u) * a.rcap);  // groups of 3..64
    uint32_t* srec = reinterpret_cast<uint32_t*>(glist);  // splitter records, once gl is dead
    uint2* rec = reinterpret_cast<uint2*>(dyn);           // run records, once D..keys are dead
    uint32_t* rec32 = dyn;
    uint32_t* D32 = dyn;
#ifdef CRDT_HIP_PROBE
    // phase timestamps of one document (probe build, CRDT_HIP_PROBE=<doc>)
    const bool probe = a.probe && d == a.probe - 1u && t == 0;
    uint64_t tp[20] = {};
    tp[0] = wall_clock64();
#define PROBE(i) if (probe) tp[i] = wall_clock64()
#else
#define PROBE(i) (void)0
#endif
    if (t == 0) {
        nwide = 0;
        flags = 0;
        visited_lds = 0;
#ifdef CRDT_HIP_PROBE
        probe_max = probe_sum = 0;
#endif
    }
    if (R + 2u > a.rcap || S > a.scap || R > (uint32_t)(J * kDocThreads)) {
        if (t == 0) atomicOr(&a.ctl[C_ERR], 32u);  // host sized rcap/scap from the largest document
        return;
    }
    // ---- parents and sibling keys (all loads first), cleared counts --------------------------
    // (weightless leaves are not pruned here: level 0 dropped 99 % of them, and walking the rest
    // costs less than a pass that finds them).  The keys go to LDS, so that no sibling sort waits
    // for a global gather; the weights are loaded later (doc_weights), beside the sorts.
    // pk[j]: the parent of run t + 1024 j (kNil16: none), then | its place among the parent's
    // children << 16 (from the count's atomic): the placement needs no second atomic
    uint32_t pk[J];
    // (stile_text) this lane's entry of the document's tile prefix table, used by phase C
    uint32_t tpx_reg = 0;
    if (PC && a.stile_text) {
        const uint32_t t0 = wg1.w & 0xFFFFFu, nt = wg1.w >> 20;
        if (t <= nt + 1u) tpx_reg = t0 + t < a.ntiles ? a.tile_hw[t0 + t].y : a.ctl[C_WTOTAL];
    }
    {
        uint32_t gp[J];
        uint64_t gk[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            gp[j] = v < R ? a.r_parent[base + v] : 0u;
            gk[j] = v < R ? a.r_key[base + v] : 0ull;
        }
        for (uint32_t i = t; i < (R + 2u) / 2u; i += kDocThreads) D32[i] = 0;
        uint32_t bad = 0, wide = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            uint32_t p = kNil16;
            if (v < R && v) {
                const uint32_t lp = gp[j] - base;
                if (lp >= R || lp == v) bad = 1;
                else p = lp;
            }
            pk[j] = p;
            if (v < R) {
                if (K32) {
                    reinterpret_cast<uint32_t*>(keys)[v] = doc_key32(gk[j]);
                    // (a key beyond the 32-bit layout: the document takes the global level 1)
                    if (v && gk[j] != kMidKey && !key32_fits(gk[j])) wide = 1;
                } else {
                    reinterpret_cast<uint64_t*>(keys)[v] = gk[j];
                }
            }
        }
        if (bad) atomicOr(&flags, 1u);
        if (wide) atomicOr(&flags, 2u);
    }
    __syncthreads();
    PROBE(1);
    // ---- child counts (u16 counters, two per LDS dword); each child keeps its place ----------
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const uint32_t p = pk[j];
        if (p != kNil16) {
            const uint32_t sh = 16u * (p & 1u);
            const uint32_t old = atomicAdd(&D32[p >> 1], 1u << sh);
            pk[j] = p | (((old >> sh) & 0xFFFFu) << 16);
        }
    }
    __syncthreads();
    PROBE(2);
    // ---- exclusive scan of the counts -> segment starts ------------------------------------
    {
        const uint32_t K = (R + kDocThreads - 1) / kDocThreads;
        const uint32_t lo = min(R, t * K), hi = min(R, lo + K);
        uint32_t s = 0;
        for (uint32_t v = lo; v < hi; ++v) s += D[v];
        uint32_t total;
        uint32_t ex = block_excl_scan<kDocThreads / 64>(s, scan_lds, total);
        for (uint32_t v = lo; v < hi; ++v) {
            const uint32_t c = D[v];
            D[v] = (uint16_t)ex;
            ex += c;
        }
        if (t == 0) D[R] = (uint16_t)total;  // (run p's children: [D[p], D[p + 1]))
    }
    __syncthreads();
    PROBE(3);
    // ---- placement: segment start + the place the count handed out ---------------------------
    // (every read first, unconditionally with a clamped index, then the stores: an LDS read
    // inside a per-run branch is waited for before the next run's; here and below)
    {
        uint32_t dp[J];
#pragma unroll
        for (int j = 0; j < J; ++j) dp[j] = D[min(pk[j] & 0xFFFFu, R)];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t p = pk[j] & 0xFFFFu;
            if (p != kNil16) ch[dp[j] + (pk[j] >> 16)] = (uint16_t)(t + (uint32_t)j * kDocThreads);
        }
    }
    __syncthreads();
    PROBE(4);
    // ---- sibling order + up-arc successors -------------------------------------------------
    // nx[] is written here: a child's entry by whoever orders its group.  Single children and
    // pairs (nearly every group on the traces) order themselves: every child reads its group's
    // bounds, an only child links up to its parent, a pair member reads its sibling and the
    // sibling's key and takes its rank (greater key first).  Every owned run is handled at once
    // (no branch per run), so the LDS round trips of all twelve overlap.  Groups of 3..64 go to
    // an LDS work list (by their parent's owner) and are sorted next: 3..8 by one register
    // network per thread, 9..64 by one wave per group; wider groups hand the wave to the global
    // path.  fcs[j]: 0x10000 | the segment start of run t + 1024 j's children (its first child
    // once they are ordered), or kNil16 for a leaf.
    uint32_t fcs[J];
    if (t == 0) nx[0] = kNil16;
    {
        // cw[j]: as a child, its group's start | (the pair's other member << 16); bit j of onlym /
        // pairm: an only child / a member of a pair (segment starts take 15 bits: up to 32 k runs)
        uint32_t cw[J], pw[J], onlym = 0, pairm = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t p = pk[j] & 0xFFFFu, v = t + (uint32_t)j * kDocThreads;
            const uint32_t q = p != kNil16 ? p : R, u = v < R ? v : R;  // (D[R] .. D[R + 1]: none)
            cw[j] = (uint32_t)D[q] | ((uint32_t)D[q + 1u] << 16);
            pw[j] = (uint32_t)D[u] | ((uint32_t)D[u + 1u] << 16);
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            // as a parent
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            const uint32_t b = pw[j] & 0xFFFFu, pc = (pw[j] >> 16) - b;
            fcs[j] = (v < R && pc) ? (0x10000u | b) : kNil16;
            if (v < R && pc > 2u) {
                if (pc > 64u) atomicOr(&flags, 2u);
                else glist[atomicAdd(&nwide, 1u)] = (uint16_t)v;
            }
            // as a child
            const uint32_t s0 = cw[j] & 0xFFFFu, cnt = (cw[j] >> 16) - s0;
            const bool child = (pk[j] & 0xFFFFu) != kNil16;
            const uint32_t oc = ch[min(s0 + ((pk[j] >> 16) ^ 1u), R)];
            const uint32_t o = (child && cnt == 2u) ? oc : 0u;
            cw[j] = s0 | (o << 16);
            onlym |= (child && cnt == 1u ? 1u : 0u) << j;
            pairm |= (child && cnt == 2u ? 1u : 0u) << j;
        }
        // (K32: nx lives in the key slots, so both members of every pair read both keys before
        // any nx is written)
        uint32_t firstm = 0;
        if (K32) {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const uint32_t v = t + (uint32_t)j * kDocThreads;
                if ((pairm >> j) & 1u)
                    firstm |= (doc_key<K32>(keys, v) > doc_key<K32>(keys, cw[j] >> 16) ? 1u : 0u) << j;
            }
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            const uint32_t up = (pk[j] & 0xFFFFu) | kUp16, s0 = cw[j] & 0xFFFFu;
            if ((onlym >> j) & 1u) {
                nx[v] = (uint16_t)up;
            } else if ((pairm >> j) & 1u) {
                const uint32_t o = cw[j] >> 16;
                const bool first = K32 ? ((firstm >> j) & 1u) != 0u
                                       : doc_key<K32>(keys, v) > doc_key<K32>(keys, o);
                ch[s0 + (first ? 0u : 1u)] = (uint16_t)v;
                nx[v] = (uint16_t)(first ? o : up);
            }
        }
    }
    __syncthreads();
    PROBE(12);
#ifdef CRDT_HIP_PROBE
    PROBE(11);
#endif
    // the weights of the owned runs (for the run records), loaded now so that the sorts of the
    // wider groups cover their latency: differences of consecutive weight prefixes, the next
    // run's prefix from the next lane (lane 63 loads it; v = R - 1 reads the next document's
    // first run or the sentinel)
    uint32_t wr[J];
    {
        uint32_t gn[J];
        const bool l63 = (t & 63u) == 63u;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            wr[j] = v <= R ? a.r_pstart[base + v] : 0u;  // (v = R: the next lane's successor)
            gn[j] = (l63 && v < R) ? a.r_pstart[base + v + 1] : 0u;
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            const uint32_t nxt = (uint32_t)__shfl_down((int)wr[j], 1);
            wr[j] = v < R ? (l63 ? gn[j] : nxt) - wr[j] : 0u;
        }
    }
    // 3..8 children: Batcher's 19-comparator network (padding key 0 sorts last)
    const uint32_t nw = nwide;
    for (uint32_t i0 = 0; i0 < nw; i0 += kDocThreads) {
        const uint32_t i = i0 + t;
        const uint32_t p = i < nw ? glist[i] : 0u;
        const uint32_t b = D[p], cnt = i < nw ? D[p + 1u] - b : 0u;
        if (cnt < 3u || cnt > 8u) continue;
        uint64_t k[8];
        uint32_t c[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) c[q] = (uint32_t)q < cnt ? ch[b + q] : 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q) k[q] = (uint32_t)q < cnt ? doc_key<K32>(keys, c[q]) : 0ull;
        cx(k[0], c[0], k[1], c[1]); cx(k[2], c[2], k[3], c[3]);
        cx(k[4], c[4], k[5], c[5]); cx(k[6], c[6], k[7], c[7]);
        cx(k[0], c[0], k[2], c[2]); cx(k[1], c[1], k[3], c[3]);
        cx(k[4], c[4], k[6], c[6]); cx(k[5], c[5], k[7], c[7]);
        cx(k[1], c[1], k[2], c[2]); cx(k[5], c[5], k[6], c[6]);
        cx(k[0], c[0], k[4], c[4]); cx(k[1], c[1], k[5], c[5]);
        cx(k[2], c[2], k[6], c[6]); cx(k[3], c[3], k[7], c[7]);
        cx(k[2], c[2], k[4], c[4]); cx(k[3], c[3], k[5], c[5]);
        cx(k[1], c[1], k[2], c[2]); cx(k[3], c[3], k[4], c[4]); cx(k[5], c[5], k[6], c[6]);
        const uint16_t up = (uint16_t)(p | kUp16);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if ((uint32_t)q < cnt) {
                ch[b + q] = (uint16_t)c[q];
                nx[c[q]] = (uint32_t)q + 1 < cnt ? (uint16_t)c[q + 1 < 8 ? q + 1 : 7] : up;
            }
        }
    }
    PROBE(5);
    // 9..64 siblings: one wave per group, rank = #siblings with a greater key
    {
        const uint32_t lane = t & 63u, wv = t >> 6;
        for (uint32_t i = wv; i < nw; i += kDocThreads / 64) {
            const uint32_t p = glist[i];
            const uint32_t s0 = D[p], cnt = D[p + 1u] - s0;
            if (cnt <= 8u) continue;  // wave-uniform
            const bool on = lane < cnt;
            const uint32_t c = on ? ch[s0 + lane] : 0u;
            const uint64_t k = on ? doc_key<K32>(keys, c) : 0ull;
            uint32_t rank = 0;
            for (uint32_t j = 0; j < cnt; ++j) {
                const uint64_t kj = ((uint64_t)(uint32_t)__shfl((int)(k >> 32), (int)j) << 32) |
                                    (uint32_t)__shfl((int)(uint32_t)k, (int)j);
                rank += kj > k;
            }
            const uint32_t sorted =
                (uint32_t)__builtin_amdgcn_ds_permute((int)((on ? rank : lane) << 2), (int)c);
            const uint32_t succ = (uint32_t)__shfl((int)sorted, (int)((lane + 1) & 63u));
            if (on) {
                ch[s0 + lane] = (uint16_t)sorted;  // lane r < cnt holds the rank-r child
                nx[sorted] = lane + 1 < cnt ? (uint16_t)succ : (uint16_t)(p | kUp16);
            }
        }
    }
    __syncthreads();
    PROBE(13);
    if (flags) {
        if (t == 0) atomicOr(&a.ctl[C_ERR], (flags & 1u) ? 1u : 32u);
        return;
    }
    // ---- first children of the sorted groups; the run records --------------------------------
    uint32_t act = 0;  // bit j: run t + 1024 j still has an up link (see below)
    {
        uint32_t fx[J], wx[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            const uint32_t fch = ch[min(fcs[j] & 0xFFFFu, R)], nn = nx[min(v, R)];
            uint32_t f = fcs[j], n = 0;
            if (v < R) {
                if (f & 0x10000u) f = fch;
                n = nn;
                if ((n & kUp16) && n != kNil16) act |= 1u << j;
            }
            fx[j] = (f & 0xFFFFu) | (n << 16);
            // the whole weight (below 2^18 on this path); bit 31: "not reached" until walk 1
            // passes v (then the word is v's sublist and offset, or ~0 for no weight)
            wx[j] = wr[j] | 0x80000000u;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            if (v < R) rec[v] = make_uint2(fx[j], wx[j]);
        }
        // record R: a leaf without weight at the tour's end, where walkers without a sublist
        // (and the splitter run of a last block beyond R) read and write harmlessly
        if (t == 0) rec[R] = make_uint2(0xFFFFFFFFu, 0x80000000u);
    }
    __syncthreads();
    PROBE(14);
    // ---- up links: a last child's up arc is followed by its parent's up arc (no weight, never a
    // splitter), so nx[v] = UP(p) may be replaced by nx[p].  In-place pointer jumping until no up
    // link is left: each thread keeps a bit per owned run still holding one and works only on
    // those.  A concurrent reader sees an old or a new link, both correct successors, so there
    // is no barrier at all until every thread's own links are resolved; every pass advances a
    // link by at least one level, so R passes bound it (more: a parent cycle, flagged).
    {
        uint16_t* vnx = reinterpret_cast<uint16_t*>(dyn) + 1;  // nx of v: [4 v]
        for (uint32_t pass = 0; act; ++pass) {
            if (pass > R) {
                atomicOr(&flags, 4u);
                break;
            }
            for (uint32_t m = act; m; m &= m - 1u) {
                const uint32_t j = (uint32_t)__ffs(m) - 1u;
                const uint32_t v = t + j * kDocThreads;
                // (the parent is an internal run: never dead)
                const uint32_t y = lds_ld16(vnx + 4u * (lds_ld16(vnx + 4u * v) & 0x7FFFu));
                lds_st16(vnx + 4u * v, y);
                if (!((y & kUp16) && y != kNil16)) act &= ~(1u << j);
            }
        }
    }
    __syncthreads();
    PROBE(6);
    // ---- walk 1: one walker per lane, each wave over its own range of splitters ---------------
    // A step at v's down arc reads v's record (first child, nx, weight: one 8-byte LDS read):
    // v's weight is added, v's offset inside the sublist and the sublist go to the record's
    // second word, and the walk goes to the first child, or for a leaf to nx (a down arc, or the
    // end of the tour).  The sublist ends at the next splitter (a node at its block's hashed
    // offset) or at the tour's end, and the lane takes the next splitter of its wave's range (a
    // wave-uniform cursor advanced by ballot).  The step is a short VALU chain with selects; a
    // lane without a splitter walks record R (a weightless leaf) with its stores masked off.
    uint32_t runs = 0;
    uint32_t lane_steps = 0;
    {
        constexpr uint32_t NWV = CRDT_DOC_WALK_WAVES;  // walking waves (the others wait)
        const uint32_t lane = t & 63u, wv = t >> 6;
        const uint32_t lo = wv < NWV ? (S * wv) / NWV : S, hi = wv < NWV ? (S * (wv + 1u)) / NWV : S;
        uint32_t cur = lo + 64u;  // the wave's next unassigned splitter (uniform over its lanes)
        uint32_t s = lo + lane < hi ? lo + lane : S;
        // (4 S >= R: the splitter run of splitter S, and of a last block beyond R, clamps to R)
        uint32_t V = min(splitter_run(s), R), SUM = 0, steps = 0;
        const uint32_t step_limit = R + S + 4u;
        constexpr uint32_t mm = (1u << kDocLog2S) - 1u;
#ifdef CRDT_HIP_PROBE
        const uint64_t wc0 = clock64(), ww0 = wall_clock64();
#endif
        while (__ballot(s < S)) {  // (steps: wave-uniform, the loop's trip count so far)
            if (++steps > step_limit) {
                if (lane == 0) atomicOr(&flags, 4u);
                break;
            }
            const uint2 r = rec[V];
            const uint32_t f = r.x & 0xFFFFu, n = r.x >> 16, wt = r.y & 0x3FFFFu;
            const bool act = s < S;
            // v's down arc is the last use of its record: the second word now holds v's offset
            // inside this sublist (18 bits) and the sublist (14 bits).  (The stores are exec-
            // masked, not sent to a dummy address: a wave's idle lanes all storing to one
            // address serialise on its bank.)
            const bool own = act & (V < R);
            if (own) rec32[2u * V + 1u] = wt ? (SUM | (s << 18)) : 0xFFFFFFFFu;
            SUM += wt;
            runs += own ? 1u : 0u;
            // the next down arc: the first child, or for a leaf nx (kNil16 at the tour's end; any
            // other value >= R is an up link a parent cycle left unresolved: the walk ends there
            // and the runs it misses are reported)
            const uint32_t go = f != kNil16 ? f : n;
            const uint32_t blk = go >> kDocLog2S;
            const bool end = go >= R;
            const bool split = ((go & mm) == splitter_off(blk)) & !end;
            const bool need = act & (end | split);
            if (need) srec[s] = (SUM << 14) | (split ? blk : kNil14);
            SUM = need ? 0u : SUM;
            const uint64_t m = __ballot(need);
            const uint32_t ns = cur + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            cur += (uint32_t)__popcll(m);
            const uint32_t s2 = ns < hi ? ns : S;
            const uint32_t v2 = min(splitter_run(s2), R);
            s = need ? s2 : s;
            V = need ? v2 : min(go, R);
        }
        lane_steps = steps;
#ifdef CRDT_HIP_PROBE
        if (lane == 0) {  // per wave: loop cycles, loop wall time (10 ns), iterations
            probe_wave[3 * (t >> 6)] = (uint32_t)(clock64() - wc0);
            probe_wave[3 * (t >> 6) + 1] = (uint32_t)(wall_clock64() - ww0);
            probe_wave[3 * (t >> 6) + 2] = steps;
        }
#endif
    }
    (void)lane_steps;
    __syncthreads();
    PROBE(7);
    // the slot-order text prefixes of the owned runs, for phase C: loaded now, so that the
    // pointer jumping and the offsets cover their latency
    uint32_t ps[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const uint32_t v = t + (uint32_t)j * kDocThreads;
        ps[j] = (PC && a.text && v < R) ? a.r_pstart[base + v] : 0u;
    }
    // ---- pointer jumping: record = (sum from the splitter to the end of the tour) << 14 | next.
    // A record always describes a valid stretch of the tour (sum up to its next splitter, read
    // and written as one dword), so joining it with an old or a new record of its successor is
    // equally right: the jumping runs without barriers, each thread until its own records reach
    // the end (every pass advances a record by at least one splitter: S passes bound it).
    {
        uint32_t x[KK], live = 0;
#pragma unroll
        for (int k = 0; k < KK; ++k) {
            const uint32_t s = t + (uint32_t)k * kDocThreads;
            x[k] = s < S ? srec[s] : kNil14;
            live |= ((x[k] & kNil14) != kNil14 ? 1u : 0u) << k;
        }
        for (uint32_t pass = 0; live; ++pass) {
            if (pass > S) {
                atomicOr(&flags, 4u);
                break;
            }
            uint32_t y[KK];
#pragma unroll
            for (int k = 0; k < KK; ++k) y[k] = ((live >> k) & 1u) ? lds_ld32(srec + (x[k] & kNil14)) : 0u;
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                if (!((live >> k) & 1u)) continue;
                x[k] = (x[k] & ~kNil14) + y[k];  // sums add, the link jumps
                lds_st32(srec + t + (uint32_t)k * kDocThreads, x[k]);
                if ((x[k] & kNil14) == kNil14) live &= ~(1u << k);
            }
        }
    }
    __syncthreads();
    PROBE(8);
    if (flags) {  // a walk or a jumping that did not end: a cycle (the log is malformed)
        if (t == 0) atomicOr(&a.ctl[C_ERR], 2u);
        return;
    }
    // ---- run offsets: sublist offset (total - suffix of its splitter) + offset inside ------
    uint32_t ro[J];  // document offset of every owned run with visible bytes, else kNil
    {
        const uint32_t total = srec[0] >> 14;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t v = t + (uint32_t)j * kDocThreads;
            const uint32_t pk = v < R ? rec32[2u * min(v, R) + 1u] : 0xFFFFFFFFu;
            const uint32_t sid = pk >> 18;
            const uint32_t sr = srec[min(sid, S - 1u)];
            // weightless (or never reached: flagged below)
            ro[j] = (pk != 0xFFFFFFFFu && sid < S) ? (pk & 0x3FFFFu) + total - (sr >> 14) : kNil;
        }
        if (!PC || !a.text) {  // offsets for k_expand (document-relative) or k_tscatter (wave-relative)
            const uint32_t ob = a.scatter ? wg1.y : 0u;  // (scatter: the wave's text is < 4 GiB)
#pragma unroll
            for (int j = 0; j < J; ++j)
                if (ro[j] != kNil) a.roff[base + t + (uint32_t)j * kDocThreads] = ob + ro[j];
        }
    }
    const uint32_t wsum = wave_sum(runs);
    if ((t & 63u) == 0 && wsum) atomicAdd(&visited_lds, wsum);
    __syncthreads();
    PROBE(9);
    if (PC && a.text) {
#ifdef CRDT_HIP_PROBE
        uint64_t* tprobe = probe ? &tp[15] : nullptr;
#else
        uint64_t* tprobe = nullptr;
#endif
        const uint64_t toff = ((uint64_t)wg1.z << 32) | wg1.y;
        const bool fused = doc_text(a, wg1.x, wg.w, toff, wg1.w, tpx_reg, ro, ps,
                                    reinterpret_cast<uint8_t*>(dyn), scan_lds, tprobe);
        if (!fused && a.stile_text) {
            // no slot-order text to copy from (k_runs skipped it): the host merges the wave
            // again on its synchronous path, which writes it
            if (t == 0) atomicOr(&a.ctl[C_ERR], 32u);
        } else if (!fused) {
            // the text did not fit LDS: every run copies its bytes from the slot-order text to
            // its document offset (byte stores; only documents above the LDS stage take this)
            uint8_t* out = a.text + toff;
            const uint32_t tl = wg1.x;
            bool oob = false;
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const uint32_t v = t + (uint32_t)j * kDocThreads;
                if (ro[j] == kNil) continue;
                const uint32_t wv = a.r_pstart[base + v + 1] - ps[j];
                if ((uint64_t)ro[j] + wv > tl) {
                    oob = true;
                    continue;
                }
                for (uint32_t b = 0; b < wv; ++b) out[ro[j] + b] = a.sbytes[ps[j] + b];
            }
            if (oob) atomicOr(&a.ctl[C_ERR], 8u);
            if (t == 0) atomicAdd(&a.ctl[C_UNFUSED], 1u);
        }
    }
    PROBE(10);
#ifdef CRDT_HIP_PROBE
    if (probe) {
        printf("[doctree] doc %u R %u S %u us: desc %.1f load %.1f count %.1f scan %.1f place %.1f "
               "glist %.1f pairs %.1f net3-8 %.1f wide9-64 %.1f fc %.1f uplinks %.1f walk1 %.1f "
               "jump %.1f offsets %.1f text-stage %.1f (scan %.1f load %.1f bits %.1f pref %.1f "
               "delta %.1f) text-out %.1f total %.1f | visited %u steps max %u sum %u\n", d, R, S,
               (tp[0] - tdesc) / 100.0, (tp[1] - tp[0]) / 100.0, (tp[2] - tp[1]) / 100.0, (tp[3] - tp[2]) / 100.0,
               (tp[4] - tp[3]) / 100.0, (tp[12] - tp[4]) / 100.0, (tp[11] - tp[12]) / 100.0,
               (tp[5] - tp[11]) / 100.0, (tp[13] - tp[5]) / 100.0, (tp[14] - tp[13]) / 100.0,
               (tp[6] - tp[14]) / 100.0, (tp[7] - tp[6]) / 100.0, (tp[8] - tp[7]) / 100.0,
               (tp[9] - tp[8]) / 100.0, (tp[15] - tp[9]) / 100.0, (tp[16] - tp[9]) / 100.0,
               (tp[17] - tp[16]) / 100.0, (tp[18] - tp[17]) / 100.0, (tp[19] - tp[18]) / 100.0,
               (tp[15] - tp[19]) / 100.0, (tp[10] - tp[15]) / 100.0,
               (tp[10] - tp[0]) / 100.0, visited_lds, probe_max, probe_sum);
    }
#endif
#ifdef CRDT_HIP_PROBE
    if (probe) {
        uint32_t cmax = 0, wmax = 0, imax = 0, csum = 0, isum = 0;
        for (int k = 0; k < 16; ++k) {
            cmax = max(cmax, probe_wave[3 * k]);
            wmax = max(wmax, probe_wave[3 * k + 1]);
            imax = max(imax, probe_wave[3 * k + 2]);
            csum += probe_wave[3 * k];
            isum += probe_wave[3 * k + 2];
        }
        printf("[walk] per wave: cycles max %u mean %u, wall max %.2f us, iterations max %u mean %.1f"
               " (%.0f cycles per iteration)\n", cmax, csum / 16, wmax / 100.0, imax, isum / 16.0,
               (double)csum / (isum ? isum : 1));
    }
#endif
#undef PROBE
    if (t == 0) {
        if (visited_lds) atomicAdd(&a.ctl[C_VISITED], visited_lds);
        if (flags & 4u) atomicOr(&a.ctl[C_ERR], 2u);
    }
}

// Level 1 in LDS: one workgroup per document descriptor (LPT order).  (A persistent form that
// walks several descriptors per workgroup spilled 34 VGPRs: not used.)
// The document's run count picks the instance: every per-run loop is unrolled J times, so a
// document of at most 4096 / 8192 runs skips the empty slots of the 12-run instance.
// Three kernels, so that the instance set of the common case stays small (every per-run loop is
// unrolled J times; one more instance in the same kernel made k_doctree 5 % slower on the traces,
// instruction fetch): k_doctree for documents of up to 12 runs per thread with 8-byte keys
// (instances 4 / 8 / 12: the RGA traces), k_doctree_wide for waves whose largest document does
// not fit those 15 bytes of LDS per run (32-bit keys and nx in the key slots: 9 bytes; instances
// 8 / 12: Fugue automerge-paper and rustcode, 11.8 k and 10.7 k rows), k_doctree_wide17 for up to
// 17 rows per thread (Fugue seph-blog1, 16.6 k rows; 8 VGPRs spill on its own, ~40 inside
// k_doctree_wide).
constexpr int kDocJNarrow = 12;
// PC: phase C (the document text written from LDS) compiled in.  The instances without it (the
// scatter mode, and the offsets left to k_expand) carry neither its code nor its registers.
template <int J, bool K32, bool PC>
__device__ __forceinline__ bool doctree_try(const DocArgs& a, uint32_t R) {
    if (R > (uint32_t)J * kDocThreads) return false;
    doctree_doc<J, K32, PC>(a, blockIdx.x);
    return true;
}
template <bool PC>
__global__ __launch_bounds__(kDocThreads) void k_doctree(DocArgs a) {
    const uint32_t R = a.wg[2u * blockIdx.x].z;
    if (doctree_try<4, false, PC>(a, R) || doctree_try<8, false, PC>(a, R)) return;
    doctree_doc<kDocJNarrow, false, PC>(a, blockIdx.x);
}
template <bool PC>
__global__ __launch_bounds__(kDocThreads) void k_doctree_wide(DocArgs a) {
    const uint32_t R = a.wg[2u * blockIdx.x].z;
    if (doctree_try<8, true, PC>(a, R)) return;
    doctree_doc<kDocJNarrow, true, PC>(a, blockIdx.x);
}
// (its own kernel: the 17 runs per thread spill ~40 VGPRs, which the 12-run instance beside them
// would pay for in scratch allocation and register pressure)
template <bool PC>
__global__ __launch_bounds__(kDocThreads) void k_doctree_wide17(DocArgs a) {
    doctree_doc<kDocJ, true, PC>(a, blockIdx.x);
}

// ---------------------------------------------------------------------------------------------
// Text scatter (k_tscatter): the documents of a wave whose k_doctree ran in scatter mode
// ---------------------------------------------------------------------------------------------
// k_doctree in scatter mode ends with the run offsets: every weighted row's place in the wave's
// text (its document's output offset + its offset in the document; u32, the host takes this mode
// only for waves with less than 4 GiB of text) goes to roff, and no text is staged in LDS.  This
// kernel then writes the text as a grid-wide stream, one wave per 4096-slot tile.  Runs never
// cross tiles (k_heads), so the tile's rows [tile_hw[k].x, tile_hw[k + 1].x) have their visible
// UTF-8 in row order in the tile's stile segment (k_classify), one contiguous range.  The wave
// takes the rows 64 at a time (a chunk): their bytes are one contiguous stretch of the segment.
// Per chunk one round of loads: the rows' weight prefixes and places, and (LDS-DMA, 16 B per lane)
// the first kScatterWin bytes of the stretch, whose start is the previous chunk's end; longer
// stretches take more windows.  Then 64 bytes per step, one per lane, each stored at its row's
// place.  The row of a byte: the starts of the chunk's weighted rows are bits of an LDS bitmap
// over the window (one ds_or each), a step reads its 64 bits with one broadcast read, and a
// lane's row is the starts at or before its byte (mbcnt) plus the starts of the earlier steps;
// the weighted rows' bases (place - start in the stretch) are compacted in LDS in start order.
// A step's 64 bytes land in the few rows they belong to (~9 bytes per row on the traces), each a
// contiguous destination range, so its stores touch a few lines.
#ifndef CRDT_TSC_WIN
#define CRDT_TSC_WIN 1024
#endif
#ifndef CRDT_TSC_RQ
#define CRDT_TSC_RQ 1
#endif
constexpr uint32_t kScatterWin = CRDT_TSC_WIN;  // stretch bytes staged per window (1 KiB per DMA)
static_assert(kScatterWin / 32 + 2 <= 64, "a window's bitmap words fit one VGPR of the wave");
constexpr uint32_t kScatterRows = 64 * CRDT_TSC_RQ;  // rows per round of loads
#ifndef CRDT_TSC_TPW
#define CRDT_TSC_TPW 1
#endif
constexpr uint32_t kScatterTiles = CRDT_TSC_TPW;  // consecutive tiles per wave (<= 63)
struct ScatterArgs {
    uint32_t ntiles, xcd;
    const uint2* tile_hw;      // per tile {rows before it, weight before it}
    const uint32_t* r_pstart;  // per row: weight prefix ([R] = the wave's weight)
    const uint32_t* roff;      // per weighted row: its place in the wave's text (k_doctree)
    const uint8_t* stile;      // per tile: its visible UTF-8 in row order (kTileBytes each)
    uint8_t* text;
    uint64_t text_cap;
    uint32_t* ctl;
};
// One window of the stretch: segment bytes [a0, min(a1, a0 + kScatterWin)) (a0 16-aligned) into
// buf, 16 B per lane and KiB, through registers: an LDS-DMA would leave a write to LDS pending on
// the vector-memory counter, and the compiler then waits for every outstanding store (the same
// counter) before each LDS read of the steps below.
__device__ __forceinline__ void scatter_window(const uint8_t* seg, uint32_t a0, uint32_t a1,
                                               uint8_t* buf, uint32_t lane) {
    uint4 v[kScatterWin / 1024u];
#pragma unroll
    for (uint32_t i = 0; i < kScatterWin / 1024u; ++i) {
        const uint32_t o = a0 + 1024u * i + 16u * lane;
        v[i] = o < a1 ? *reinterpret_cast<const uint4*>(seg + o) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t i = 0; i < kScatterWin / 1024u; ++i)
        *reinterpret_cast<uint4*>(buf + 1024u * i + 16u * lane) = v[i];
}
__device__ __forceinline__ uint32_t uni(uint32_t x) {  // (a wave-uniform value, as an SGPR)
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__global__ __launch_bounds__(kBlock) void k_tscatter(ScatterArgs a) {
    constexpr uint32_t NW = kBlock / 64;
    constexpr uint32_t BW = kScatterWin / 32 + 2;  // bitmap words (+2: a step's second word)
    constexpr int RQ = kScatterRows / 64;
    __shared__ __attribute__((aligned(16))) uint8_t tb[NW][kScatterWin];
    __shared__ uint32_t bm[NW][BW];
    __shared__ uint32_t lb[NW][kScatterRows];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    // (no barrier below: every wave works alone on its own LDS)
    if (replan(a.ctl) || a.ctl[C_ERR]) return;  // (an error: the host redoes or rejects the wave)
    const uint32_t tile0 = (xcd_block(blockIdx.x, gridDim.x, a.xcd) * NW + wv) * kScatterTiles;
    if (tile0 >= a.ntiles) return;
    uint8_t* buf = tb[wv];
    uint32_t* bmw = bm[wv];
    uint32_t* lbw = lb[wv];
    for (uint32_t i = lane; i < BW; i += 64u) bmw[i] = 0;
    // the {rows, weight} prefixes of the wave's tiles and of the one after them, one per lane
    // (the wave's last: ctl's totals)
    const uint2 hl = a.tile_hw[min(tile0 + lane, a.ntiles - 1u)];
    const uint2 hc = make_uint2(a.ctl[C_RTOTAL], a.ctl[C_WTOTAL]);
    const uint2 hv = tile0 + lane < a.ntiles ? hl : hc;
    bool oob = false;
    for (uint32_t tk = 0; tk < kScatterTiles && tile0 + tk < a.ntiles; ++tk) {
    const uint32_t tile = tile0 + tk;
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, (int)tk);
    const uint32_t h1 = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, (int)tk + 1);
    const uint32_t wt0 = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, (int)tk);
    // (the tile's text: segment bytes [0, te); no load reaches past it)
    const uint32_t te = min((uint32_t)__builtin_amdgcn_readlane((int)hv.y, (int)tk + 1) - wt0,
                            kTileBytes);
    const uint8_t* seg = a.stile + (uint64_t)tile * kTileBytes;
    uint32_t p0 = wt0;  // the rows' stretch start (weight position): the previous round's end
    for (uint32_t c = r0; c < h1; c += kScatterRows) {
        const uint32_t nr = min(kScatterRows, h1 - c);
        // one round of loads: prefixes, places, the stretch's first window
        const uint32_t sh = (p0 - wt0) & 15u, a0 = (p0 - wt0) & ~15u;
        uint32_t ps[RQ], ro[RQ];
        const uint32_t pe = a.r_pstart[c + nr];  // (the stretch's end)
#pragma unroll
        for (int i = 0; i < RQ; ++i) {
            const uint32_t r = lane + 64u * (uint32_t)i;
            ps[i] = r < nr ? a.r_pstart[c + r] : 0u;
            ro[i] = r < nr ? a.roff[c + r] : 0u;  // (weightless rows: unused)
        }
        scatter_window(seg, a0, te, buf, lane);  // (every load of the round issued before a use)
        const uint32_t pend = uni(pe);
#pragma unroll
        for (int i = 0; i < RQ; ++i) ps[i] = lane + 64u * (uint32_t)i < nr ? ps[i] : pend;
        const uint32_t T = pend - p0, U = T + sh;
        uint32_t w[RQ], u[RQ];
        bool bad = false;
#pragma unroll
        for (int i = 0; i < RQ; ++i) {
            const uint32_t nx = (uint32_t)__shfl_down((int)ps[i], 1);
            const uint32_t n63 = i + 1 < RQ ? uni(ps[i + 1 < RQ ? i + 1 : i]) : pend;
            w[i] = (lane == 63u ? n63 : nx) - ps[i];
            u[i] = ps[i] - p0 + sh;  // (the row's start in window coordinates)
            bad |= w[i] && (uint64_t)ro[i] + w[i] > a.text_cap;
        }
        // a place beyond the text buffer (only a malformed wave, which k_doctree flags): no store
        if (__ballot(bad)) {
            oob = true;
            p0 = pend;
            continue;
        }
        // compacted bases of the weighted rows, in start order: the byte at window coordinate x
        // goes to lbw[its row] + x
        uint32_t kb = 0;
#pragma unroll
        for (int i = 0; i < RQ; ++i) {
            const uint64_t wm = __ballot(w[i] != 0u);
            const uint32_t k = kb + __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u));
            if (w[i]) lbw[k] = ro[i] - u[i];
            kb += (uint32_t)__popcll(wm);
        }
        uint32_t cnt = 0;  // weighted starts before the step
        for (uint32_t w0 = 0; w0 < U; w0 += kScatterWin) {
            if (w0) scatter_window(seg, a0 + w0, te, buf, lane);  // (a longer stretch)
#pragma unroll
            for (int i = 0; i < RQ; ++i)
                if (w[i] && u[i] >= w0 && u[i] - w0 < kScatterWin)
                    atomicOr(&bmw[(u[i] - w0) >> 5], 1u << ((u[i] - w0) & 31u));
            __builtin_amdgcn_s_waitcnt(0xc07f);  // (lgkmcnt(0): the wave's bits are in)
            const uint32_t w1 = min(U, w0 + kScatterWin) - w0;
            // The window's bitmap in one VGPR (lane j: word j) and the starts before each word
            // (a wave scan): a lane's row is then pre[j] + the starts in word j at or before its
            // byte - 1, from two v_readlane pairs per step and no LDS round trip, and the steps
            // are independent of each other (no running count), so the unrolled steps' LDS reads
            // and stores overlap.
            const uint32_t bwd = lane < BW ? bmw[lane] : 0u;
            const uint32_t pc = (uint32_t)__popc(bwd);
            const uint32_t pinc = wave_incl_scan(pc);
            const uint32_t pre = cnt + pinc - pc - 1u;  // (- 1: rows are counted from 0)
            cnt += (uint32_t)__builtin_amdgcn_readlane((int)pinc, 63);
            const uint32_t lo = w0 ? 0u : sh;  // (the first window starts at sh)
            const bool hi = lane >= 32u;
            const uint32_t mle = (lane & 31u) == 31u ? ~0u : (2u << (lane & 31u)) - 1u;
            // Four steps at a time, their LDS reads issued unconditionally (clamped indices) so
            // that they overlap; only the stores are predicated.  (Four bytes per lane and step,
            // with four byte stores each, was slower: a store instruction then touches ~30 rows'
            // lines instead of ~8, and the store path is what this loop waits on.)
            constexpr uint32_t SU = 4;
            for (uint32_t b = 0; b < w1; b += 64u * SU) {
                uint32_t dst[SU], val[SU];
                bool ok[SU];
#pragma unroll
                for (uint32_t k = 0; k < SU; ++k) {
                    const uint32_t bk = b + 64u * k;
                    const int q = (int)min(bk >> 5, BW - 2u);
                    const uint32_t wlo = (uint32_t)__builtin_amdgcn_readlane((int)bwd, q);
                    const uint32_t whi = (uint32_t)__builtin_amdgcn_readlane((int)bwd, q + 1);
                    const uint32_t plo = (uint32_t)__builtin_amdgcn_readlane((int)pre, q);
                    const uint32_t phi = (uint32_t)__builtin_amdgcn_readlane((int)pre, q + 1);
                    const uint32_t own = (hi ? phi : plo) + (uint32_t)__popc((hi ? whi : wlo) & mle);
                    const uint32_t x = bk + lane;  // (this lane's byte, window coordinate)
                    ok[k] = x < w1 && x >= lo;
                    dst[k] = lbw[min(own, kScatterRows - 1u)] + w0 + x;
                    val[k] = buf[min(x, kScatterWin - 1u)];
                }
#pragma unroll
                for (uint32_t k = 0; k < SU; ++k) {
                    if (ok[k]) a.text[dst[k]] = (uint8_t)val[k];
                }
            }
            // (clear for the next window / round; the reads above are done first)
            __builtin_amdgcn_s_waitcnt(0xc07f);
            for (uint32_t i = lane; i < (w1 + 31u) / 32u + 2u && i < BW; i += 64u) bmw[i] = 0u;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        p0 = pend;
    }
    }
    if (oob) atomicOr(&a.ctl[C_ERR], 8u);
}

// ---------------------------------------------------------------------------------------------
// digest: xxh64 of 4 KiB leaves, then xxh64 of the leaf digests seeded with the length
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xr(uint64_t acc, uint64_t in) {
    return rotl(acc + in * 0xC2B2AE3D27D4EB4FULL, 31) * 0x9E3779B185EBCA87ULL;
}
__device__ __forceinline__ uint64_t xm(uint64_t acc, uint64_t v) {
    return (acc ^ xr(0, v)) * 0x9E3779B185EBCA87ULL + 0x85EBCA77C2B2AE63ULL;
}
// p must be 8-byte aligned.
__device__ uint64_t xxh64_aligned(const uint8_t* __restrict__ p, uint32_t len, uint64_t seed) {
    const uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL,
                   P3 = 0x165667B19E3779F9ULL, P4 = 0x85EBCA77C2B2AE63ULL,
                   P5 = 0x27D4EB2F165667C5ULL;
    const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
    uint32_t i = 0;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; i + 32 <= len; i += 32) {
            const uint64_t* q = w + i / 8;
            v1 = xr(v1, q[0]);
            v2 = xr(v2, q[1]);
            v3 = xr(v3, q[2]);
            v4 = xr(v4, q[3]);
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xm(h, v1); h = xm(h, v2); h = xm(h, v3); h = xm(h, v4);
    } else {
        h = seed + P5;
    }
    h += len;
    for (; i + 8 <= len; i += 8) {
        h ^= xr(0, w[i / 8]);
        h = rotl(h, 27) * P1 + P4;
    }
    if (i + 4 <= len) {
        h ^= (uint64_t)(*reinterpret_cast<const uint32_t*>(p + i)) * P1;
        h = rotl(h, 23) * P2 + P3;
        i += 4;
    }
    for (; i < len; ++i) {
        h ^= (uint64_t)p[i] * P5;
        h = rotl(h, 11) * P1;
    }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}

// One wave per 4 KiB leaf: the leaf is loaded into LDS with 16-byte loads (the whole wave, one
// round trip), then lanes 0-3 run xxh64's four stripe accumulators over it (lane i takes qword i
// of every 32-byte stripe), lane 0 merges them and hashes the tail, and every lane counts the
// codepoints of its 64 bytes.  The same digest as xxh64_aligned(leaf, len, 0), without a thread
// walking 4 KiB alone.
// Leaf digests, 16 leaves per wave: lanes 4g..4g+3 run the four stripe accumulators of leaf g
// (every lane of the wave busy in the 128 rounds, instead of 4 of 64 with a wave per leaf),
// reading their 8-byte words straight from the merged text (8 rounds of loads in flight), and
// counting the leaf's codepoints on the way; the first lane of each group adds the tail (< 32
// bytes), finalises and writes leafh / leafcp.  Leaf -> document by a binary search over loff.
constexpr uint32_t kLeafGroup = 16;  // leaves per wave
__device__ __forceinline__ uint32_t cont_bytes(uint64_t w, uint32_t n) {  // in the first n bytes
    const uint64_t m = n >= 8u ? ~0ull : ((1ull << (8u * n)) - 1ull);
    return (uint32_t)__popcll(w & ~(w << 1) & 0x8080808080808080ull & m);
}
__global__ __launch_bounds__(kBlock) void k_leafhash(TreeArgs a, uint32_t leaf_cap) {
    const uint32_t lane = threadIdx.x & 63u, g = lane >> 2, acc = lane & 3u;
    const uint32_t L = (blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * kLeafGroup + g;
    if (replan(a.ctl)) return;
    const uint32_t nleaves = min(leaf_cap, a.loff[a.ndocs]);
    const bool live = L < nleaves;
    uint32_t d = 0, j = 0, len = 0;
    if (live) {
        uint32_t lo = 0, hi = a.ndocs;  // last d with loff[d] <= L
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.loff[mid] <= L) lo = mid; else hi = mid;
        }
        d = lo;
        j = L - a.loff[d];
        len = min(kLeaf, a.tlen[d] - j * kLeaf);
    }
    const uint64_t* w = reinterpret_cast<const uint64_t*>(a.text + (live ? a.toff[d] : 0ull) +
                                                          (uint64_t)j * kLeaf);
    const uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL,
                   P3 = 0x165667B19E3779F9ULL, P4 = 0x85EBCA77C2B2AE63ULL,
                   P5 = 0x27D4EB2F165667C5ULL;
    const uint32_t nst = len / 32u;
    uint64_t v = acc == 0u ? P1 + P2 : acc == 1u ? P2 : acc == 2u ? 0ull : 0ull - P1;
    uint32_t cont = 0;
    uint32_t k = 0;
    for (; k + 8u <= nst; k += 8u) {
        uint64_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = w[4u * (k + u) + acc];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            v = xr(v, x[u]);
            cont += cont_bytes(x[u], 8u);
        }
    }
    for (; k < nst; ++k) {
        const uint64_t x = w[4u * k + acc];
        v = xr(v, x);
        cont += cont_bytes(x, 8u);
    }
    // the group's four accumulators and continuation counts (every lane takes part)
    const uint32_t b = lane & ~3u;
    uint64_t vv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        vv[q] = ((uint64_t)(uint32_t)__shfl((int)(v >> 32), (int)(b + q)) << 32) |
                (uint32_t)__shfl((int)(uint32_t)v, (int)(b + q));
    cont += (uint32_t)__shfl_xor((int)cont, 1);
    cont += (uint32_t)__shfl_xor((int)cont, 2);
    if (!live || acc != 0u) return;
    uint64_t h;
    if (len >= 32u) {
        h = rotl(vv[0], 1) + rotl(vv[1], 7) + rotl(vv[2], 12) + rotl(vv[3], 18);
        h = xm(h, vv[0]); h = xm(h, vv[1]); h = xm(h, vv[2]); h = xm(h, vv[3]);
    } else {
        h = P5;
    }
    h += len;
    const uint8_t* pb = reinterpret_cast<const uint8_t*>(w);
    uint32_t i = 32u * nst;
    for (; i + 8u <= len; i += 8u) {
        const uint64_t x = w[i / 8u];
        cont += cont_bytes(x, 8u);
        h ^= xr(0, x);
        h = rotl(h, 27) * P1 + P4;
    }
    if (i + 4u <= len) {
        const uint32_t x = *reinterpret_cast<const uint32_t*>(pb + i);
        cont += cont_bytes(x, 4u);
        h ^= (uint64_t)x * P1;
        h = rotl(h, 23) * P2 + P3;
        i += 4u;
    }
    for (; i < len; ++i) {
        const uint32_t x = pb[i];
        cont += (x & 0xC0u) == 0x80u ? 1u : 0u;
        h ^= (uint64_t)x * P5;
        h = rotl(h, 11) * P1;
    }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    a.leafh[L] = h;
    a.leafcp[L] = len - cont;
}

// Documents of more than kGroup leaves (16 MiB): leaf digests hashed in groups of kGroup (seed =
// group index) by one thread per group, into ghash[loff[d] + k].
constexpr uint32_t kGroup = 4096;
__global__ __launch_bounds__(kBlock) void k_grouphash(TreeArgs a, uint32_t leaf_cap) {
    const uint32_t L = blockIdx.x * kBlock + threadIdx.x;
    if (replan(a.ctl) || L >= leaf_cap || L >= a.loff[a.ndocs]) return;
    uint32_t lo = 0, hi = a.ndocs;  // last d with loff[d] <= L
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.loff[mid] <= L) lo = mid; else hi = mid;
    }
    const uint32_t l0 = a.loff[lo], nl = a.loff[lo + 1] - l0, j = L - l0;
    if (nl <= kGroup || j % kGroup) return;
    const uint32_t ng = min(kGroup, nl - j);
    a.ghash[l0 + j / kGroup] = xxh64_aligned(reinterpret_cast<const uint8_t*>(a.leafh + L),
                                             ng * 8u, j / kGroup);
    uint32_t cps = 0;
    for (uint32_t i = 0; i < ng; ++i) cps += a.leafcp[L + i];
    a.gcp[l0 + j / kGroup] = cps;
}

__global__ __launch_bounds__(kBlock) void k_docdigest(TreeArgs a) {
    const uint32_t d = blockIdx.x * kBlock + threadIdx.x;
    if (replan(a.ctl) || d >= a.ndocs) return;
    const uint32_t l0 = a.loff[d], nl = a.loff[d + 1] - l0;
    const uint64_t* h = nl > kGroup ? a.ghash + l0 : a.leafh + l0;
    const uint32_t* c = nl > kGroup ? a.gcp + l0 : a.leafcp + l0;
    const uint32_t nh = nl > kGroup ? (nl + kGroup - 1) / kGroup : nl;
    const uint64_t dig = xxh64_aligned(reinterpret_cast<const uint8_t*>(h), nh * 8u, a.tlen[d]);
    uint32_t cps = 0;
    for (uint32_t i = 0; i < nh; ++i) cps += c[i];
    a.res[d] = make_uint4(a.tlen[d], cps, (uint32_t)dig, (uint32_t)(dig >> 32));
}

// ---------------------------------------------------------------------------------------------
// batch materialisation
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_chunk_doc(const uint64_t* __restrict__ doc_slot,
                                                       const uint32_t* __restrict__ doc_local,
                                                       uint32_t ndocs, uint64_t nchunks,
                                                       uint32_t log2m, uint32_t* __restrict__ out) {
    const uint64_t c = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t slot = c << log2m;
    uint32_t lo = 0, hi = ndocs;  // last d with doc_slot[d] <= slot
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (doc_slot[mid] <= slot) lo = mid; else hi = mid;
    }
    out[c] = doc_local[lo];
}

struct Perm {
    uint32_t kind, n, bits;
    uint32_t shift;
    uint32_t mul[3], add[3];
};
__device__ __forceinline__ uint32_t perm_apply(const Perm& P, uint32_t id) {
    if (id == 0 || P.kind == 0) return id;
    if (P.kind == 1) {
        uint32_t x = id - 1 + P.shift;
        if (x >= P.n) x -= P.n;
        return x + 1;
    }
    const uint32_t mask = P.bits >= 32 ? 0xFFFFFFFFu : ((1u << P.bits) - 1u);
    const uint32_t sh = (P.bits + 1) / 2;
    uint32_t x = id - 1;
    do {  // cycle walking over a bijection of [0, 2^bits)
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            x = (x * P.mul[r] + P.add[r]) & mask;
            x ^= x >> sh;
        }
    } while (x >= P.n);
    return x + 1;
}

// The relabelling of replica r (of a base of n items): rotation (kind 1) or a seeded
// cycle-walking permutation (kind 2), parameters hashed from (seed, r) exactly as the host's
// mix64 would.
__device__ __forceinline__ Perm replica_perm(uint32_t kind, uint32_t n, uint64_t seed, uint64_t r) {
    Perm P{};
    P.kind = kind;
    P.n = n;
    uint32_t bits = 0;
    while ((1ull << bits) < n) ++bits;
    P.bits = bits < 2u ? 2u : bits;
    const uint64_t h = mix64(seed, r);
    P.shift = n ? (uint32_t)(h % n) : 0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        P.mul[k] = (uint32_t)mix64(h, 2 * k) | 1u;
        P.add[k] = (uint32_t)mix64(h, 2 * k + 1);
    }
    return P;
}

// Every replica of a batch in one launch: blockIdx.y strides over the replica documents,
// blockIdx.x x 256 threads over a document's items.  Replica r is a relabelled copy of base
// r % nb: item k goes to slot perm(k) and its parent is relabelled the same way.
// ---- the compact nsq parent list of a resident batch (Engine::build_nsq) ---------------------------
// The nsq items (items without the previous-slot flag) of every 64-slot chunk of a wave, the same
// classification as k_classify's: 16 slots per thread (three 16-byte loads, the lanes of a wave on
// 3 KiB of consecutive codepoint words), four lanes' 16-bit masks joined into the chunk's mask.
__global__ __launch_bounds__(kBlock) void k_nsq_count(L0Args a, uint32_t* cnt, uint64_t* mask) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;  // 16-slot group
    const uint32_t gs = t * 16u;
    uint32_t bits = 0;
    if (gs < a.nslots) {
        const uint2 doc = a.docs[a.chunk_doc[gs >> a.log2m]];
        const uint32_t l0 = gs - doc.x, n = doc.y;
        const uint4* cv = reinterpret_cast<const uint4*>(a.in_cp + 3ull * gs);  // 48 B, 16-aligned
        const uint4 q0 = cv[0], q1 = cv[1], q2 = cv[2];
        const uint32_t CW[13] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                 q2.x, q2.y, q2.z, q2.w, 0u};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int byte = 3 * k, wd = byte >> 2, sh = 8 * (byte & 3);
            const uint32_t lo = CW[wd] >> sh, hi = sh > 8 ? CW[wd + 1] << (32 - sh) : 0u;
            const uint32_t c = (lo | hi) & 0x00FFFFFFu;
            const bool it = (l0 + (uint32_t)k - 1u) < n;
            bits |= (it && !(c & kSeqBit) ? 1u : 0u) << k;
        }
    }
    // (every lane of the wave takes part in the shuffles; a chunk's four groups are lanes
    // 4i .. 4i + 3 of one wave)
    const uint32_t lane = threadIdx.x & 63u, l4 = lane & ~3u;
    const uint32_t b0 = (uint32_t)__shfl((int)bits, (int)l4), b1 = (uint32_t)__shfl((int)bits, (int)l4 + 1);
    const uint32_t b2 = (uint32_t)__shfl((int)bits, (int)l4 + 2), b3 = (uint32_t)__shfl((int)bits, (int)l4 + 3);
    if ((lane & 3u) == 0u && gs < a.nslots) {
        const uint64_t m = (uint64_t)(b0 | (b1 << 16)) | ((uint64_t)(b2 | (b3 << 16)) << 32);
        cnt[t >> 2] = (uint32_t)__popcll(m);
        mask[t >> 2] = m;
    }
}
// The list itself: one workgroup per 4096-slot tile (16 slots per thread, k_classify's layout):
// the tile's nsq items (k_nsq_count's masks) listed in LDS in slot order (a block scan of the
// per-thread counts), then their parents and keys read by the whole block and written to the
// tile's range of the list as consecutive words.
__global__ __launch_bounds__(kBlock) void k_nsq_scatter(L0Args a, const uint32_t* pre,
                                                        const uint64_t* mask, uint32_t* out,
                                                        uint64_t* kout) {
    __shared__ uint32_t lds[kBlock / 64];
    __shared__ uint16_t lst[kScanTile];
    const uint32_t tile = blockIdx.x, t0 = tile * kScanTile, gs = t0 + threadIdx.x * kScanItems;
    uint32_t nsq = 0;
    if (gs < a.nslots) nsq = (uint32_t)(mask[gs >> 6] >> (gs & 63u)) & 0xFFFFu;
    uint32_t T;
    uint32_t i = block_excl_scan<kBlock / 64>((uint32_t)__popc(nsq), lds, T);
    for (; nsq; nsq &= nsq - 1u) lst[i++] = (uint16_t)(threadIdx.x * kScanItems + __builtin_ctz(nsq));
    __syncthreads();
    const uint32_t o = pre[tile * (kScanTile / 64)];
    for (uint32_t k = threadIdx.x; k < T; k += kBlock) {
        const uint32_t g = t0 + lst[k];
        // the parent as a wave slot (its document's base + its index; the consumers recover the
        // index for their range checks)
        out[o + k] = a.docs[a.chunk_doc[g >> a.log2m]].x + a.in_parent[g];
        kout[o + k] = a.in_key[g];
    }
}

__global__ __launch_bounds__(kBlock) void k_replicate(
    const uint32_t* __restrict__ bp, const uint64_t* __restrict__ bk,
    const uint8_t* __restrict__ bc,
    const uint64_t* __restrict__ bslot, const uint32_t* __restrict__ bn, uint32_t nb,
    uint32_t* __restrict__ rp, uint64_t* __restrict__ rk,
    uint8_t* __restrict__ rc, const uint64_t* __restrict__ rslot, uint64_t ndocs,
    uint32_t kind, uint64_t seed) {
    for (uint64_t r = blockIdx.y; r < ndocs; r += gridDim.y) {
        const uint32_t b = (uint32_t)(r % nb);
        const uint32_t n = bn[b];
        if ((uint64_t)blockIdx.x * kBlock >= n) continue;  // block-uniform
        const Perm P = replica_perm(kind, n, seed, r);
        const uint64_t src = bslot[b], dst = rslot[r];
        for (uint32_t k = blockIdx.x * kBlock + threadIdx.x + 1; k <= n; k += gridDim.x * kBlock) {
            const uint32_t lk = perm_apply(P, k), pk = perm_apply(P, bp[src + k]);
            const uint64_t o = dst + lk;
            rp[o] = pk;
            rk[o] = bk[src + k];
            const uint32_t c = cp3_get(bc, src + k);
            cp3_put(rc, o, (c & ~kSeqBit) | (pk == lk - 1u && !(c & kLeftBit) ? kSeqBit : 0u));
        }
    }
}

// Config 5 generator, item by item on the device: exactly synth.cpp's synth_tree_item (the same
// counter-based hashes), so a device batch equals the host log of the same seed.  Slot 0 is the
// document start; padding slots are deleted, parentless.
__global__ __launch_bounds__(kBlock) void k_synth_tree(uint32_t* __restrict__ par,
                                                        uint64_t* __restrict__ key,
                                                        uint8_t* __restrict__ cp, uint32_t n,
                                                        uint64_t nslots, uint32_t p_chain_pct,
                                                        uint32_t del_pct, uint64_t seed) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= nslots) return;
    const uint32_t i = (uint32_t)g;
    uint32_t p = 0, l = 0, c = 0;
    uint16_t a = 0;
    uint8_t d = 1;
    if (i >= 1 && i <= n) {
        const uint64_t h0 = mix64(seed, i);
        const uint64_t h1 = mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL, i);
        const uint64_t h2 = mix64(seed ^ 0x5A5A5A5A5A5A5A5AULL, i);
        p = (h0 % 100 < p_chain_pct) ? i - 1 : (uint32_t)(h1 % i);
        d = (uint8_t)((h2 % 100) < del_pct);
        if (p == i - 1) c |= kSeqBit;
        c |= 'a' + (uint32_t)((h2 >> 32) % 26);
        l = i;
        a = (uint16_t)(i % 64);
    }
    par[g] = p;
    key[g] = ((uint64_t)l << 16) | a;
    cp3_put(cp, g, c | (d ? kDelBit : 0u));
}

inline uint32_t ceil_log2(uint64_t x) {
    uint32_t r = 0;
    while ((1ull << r) < x) ++r;
    return r;
}

}  // namespace

// =============================================================================================
// host side
// =============================================================================================
void DeviceLogs::release() {
    dfree(parent); dfree(key); dfree(cp);
    dfree(nsq_par); dfree(nsq_pre); dfree(nsq_key); dfree(nsq_sums); dfree(nsq_mask);
    nsq_items = 0;
    nsq_ok = false;
    nsq_cap = nsq_pre_cap = nsq_sums_cap = 0;
    dfree(docs_rel); dfree(doc_rank); dfree(chunk_doc);
    dfree(raw_lam); dfree(raw_agent); dfree(raw_del); dfree(raw_cp);
    raw = false;
    cap_slots = cap_docs = cap_chunks = 0;
    tab_sig.clear();
}

Engine::~Engine() {
    if (stream) (void)hipStreamSynchronize(stream);
    dfree(jbits_); dfree(nsqb_); dfree(visb_); dfree(wnib_); dfree(escm_); dfree(hrec_); dfree(stile_); dfree(plist_);
    dfree(tile_hw_); dfree(tile_sums_); dfree(sbytes_);
    dfree(doc_root_); dfree(doc_p0_); dfree(doc_fused_); dfree(wgtab_);
    dfree(r_head_); dfree(r_pstart_); dfree(r_parent_); dfree(roff_); dfree(rloc_); dfree(r_key_);
    dfree(rs_elem_[0]); dfree(rs_elem_[1]); dfree(rs_status_); dfree(rs_bigl_);
    dfree(rs_small_);
    dfree(wtmp_);
    dfree(ovf_);
    dfree(deg_); dfree(cstart_); dfree(child_); dfree(defer_); dfree(bigl_); dfree(scan_sums_);
    dfree(out_); dfree(rec_); dfree(swn_); dfree(spref_); dfree(sup_); dfree(spred_);
    dfree(svp_[0]); dfree(svp_[1]); dfree(tlen_); dfree(loff_); dfree(toff_);
    dfree(leafh_); dfree(ghash_); dfree(text_);
    dfree(leafcp_); dfree(gcp_); dfree(tab_slot_); dfree(tab_local_);
    if (host_out_) (void)hipHostFree(host_out_);
    if (up_pending_) (void)hipEventSynchronize(up_ev_);
    if (up_pin_) (void)hipHostFree(up_pin_);
    if (up_ev_) (void)hipEventDestroy(up_ev_);
    for (hipEvent_t e : ev_) (void)hipEventDestroy(e);
    for (hipEvent_t e : wev_) (void)hipEventDestroy(e);
    for (hipEvent_t e : raw_ev_)
        if (e) (void)hipEventDestroy(e);
    if (ev_l0_) (void)hipEventDestroy(ev_l0_);
    if (ev_l1_) (void)hipEventDestroy(ev_l1_);
    if (stream_l1) {
        (void)hipStreamSynchronize(stream_l1);
        (void)hipStreamDestroy(stream_l1);
    }
    if (stream) (void)hipStreamDestroy(stream);
}

int Engine::fail(const char* what, hipError_t e) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();
    return CRDT_HIP_EDEVICE;
}

#define HIPCHK(expr, what)                           \
    do {                                             \
        hipError_t _e = (expr);                      \
        if (_e != hipSuccess) return fail(what, _e); \
    } while (0)

std::string Engine::init(int dev) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return std::string("no HIP device: ") + hipGetErrorString(e);
    if (dev < 0 || dev >= n) return "device index out of range";
    device = dev;
    if ((e = hipSetDevice(dev)) != hipSuccess) return hipGetErrorString(e);
    int prio_lo = 0, prio_hi = 0;  // (numerically: least >= greatest)
    if ((e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi)) != hipSuccess)
        return hipGetErrorString(e);
    if ((e = hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, prio_hi)) != hipSuccess)
        return hipGetErrorString(e);
    if ((e = hipStreamCreateWithPriority(&stream_l1, hipStreamNonBlocking, prio_lo)) != hipSuccess)
        return hipGetErrorString(e);
    if ((e = hipEventCreateWithFlags(&ev_l0_, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ev_l1_, hipEventDisableTiming)) != hipSuccess)
        return hipGetErrorString(e);
    cur_ = stream;
    ev_.resize(2 * S_N + 4);
    for (hipEvent_t& x : ev_)
        if ((e = hipEventCreate(&x)) != hipSuccess) return hipGetErrorString(e);
    {
        const void* dk[6] = {reinterpret_cast<const void*>(&k_doctree<true>),
                             reinterpret_cast<const void*>(&k_doctree<false>),
                             reinterpret_cast<const void*>(&k_doctree_wide<true>),
                             reinterpret_cast<const void*>(&k_doctree_wide<false>),
                             reinterpret_cast<const void*>(&k_doctree_wide17<true>),
                             reinterpret_cast<const void*>(&k_doctree_wide17<false>)};
        for (const void* f : dk)
            if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)kDocLds)) != hipSuccess)
                return std::string("k_doctree LDS: ") + hipGetErrorString(e);
    }
    return "";
}

int Engine::plan(DeviceLogs& L, const std::vector<DocInfo>& docs,
                 const std::vector<uint8_t>* brk) {
    const uint64_t M = 1ull << kDocAlignLog2;  // documents start on 64-slot boundaries
    // (a new slot layout: the compact nsq list, if any, no longer matches it)
    L.nsq_ok = false;
    L.nsq_items = 0;
    L.log2m = kDocAlignLog2;
    L.docs = docs;
    L.api_doc.clear();  // (replicate sets it again for a grouped layout)
    L.doc_slot.resize(docs.size());
    L.waves.clear();
    L.items = 0;
    uint64_t slot = 0;
    const uint64_t hard_max = (1ull << 31) - M;
    // The last wave's level 1 overlaps nothing, so a merge of several waves ends with a small
    // one: the trailing documents that fit max_wave_slots / tail_wave_div go to a wave of their
    // own (from `tail0` on) when the whole merge needs more than one wave.
    uint64_t total = 0;
    for (const DocInfo& di : docs) total += (di.n + 1 + M - 1) / M * M;
    uint32_t tail0 = (uint32_t)docs.size();
    if (tail_wave_div && total > max_wave_slots) {
        uint64_t sfx = 0;
        while (tail0 > 1) {
            const uint64_t ds = (docs[tail0 - 1].n + 1 + M - 1) / M * M;
            if (sfx + ds > max_wave_slots / tail_wave_div && sfx) break;
            sfx += ds;
            --tail0;
        }
    }
    for (uint32_t d = 0; d < docs.size(); ++d) {
        const uint64_t ds = (docs[d].n + 1 + M - 1) / M * M;
        if (ds > hard_max) { err = "document too large for one wave"; return CRDT_HIP_ERANGE; }
        if (docs[d].text_cap >= (1ull << 32)) {
            err = "document text of 4 GiB or more is not supported";
            return CRDT_HIP_ERANGE;
        }
        const uint64_t dt = (docs[d].text_cap + 15) & ~15ull;
        if (L.waves.empty() || (uint64_t)L.waves.back().nslots + ds > max_wave_slots ||
            L.waves.back().text_cap + dt > kMaxWaveText || d == tail0 || (brk && (*brk)[d])) {
            Wave w{};
            w.first_doc = d;
            w.slot0 = slot;
            L.waves.push_back(w);
        }
        Wave& w = L.waves.back();
        L.doc_slot[d] = slot;
        w.ndocs++;
        w.nslots += (uint32_t)ds;
        w.max_splitters_per_doc = std::max<uint32_t>(w.max_splitters_per_doc, (uint32_t)(2 * ds / M));
        w.text_cap += dt;
        w.max_doc_text = std::max<uint64_t>(w.max_doc_text, docs[d].text_cap);
        w.max_doc_slots = std::max<uint64_t>(w.max_doc_slots, ds);
        w.leaf_cap += (docs[d].text_cap + kLeaf - 1) / kLeaf;
        w.order_cap += docs[d].n;
        L.items += docs[d].n;
        slot += ds;
    }
    L.total_slots = slot;
    // (replicas and single documents: the waves contract unless contraction is 2; uploads and
    // built batches decide per wave from their nsq counts afterwards, set_contraction)
    for (Wave& w : L.waves) w.nocon = !L.fugue && contraction == 2;
    apply_shape_hints(L);
    const uint64_t nchunks = slot / M;
    if (slot > L.cap_slots) {
        dfree(L.parent); dfree(L.key); dfree(L.cp);
        HIPCHK(dalloc(&L.parent, slot), "hipMalloc logs.parent");
        HIPCHK(dalloc(&L.key, slot), "hipMalloc logs.key");
        HIPCHK(dalloc(&L.cp, cp3_bytes(slot)), "hipMalloc logs.cp");
        L.cap_slots = slot;
        gen_++;
    }
    if (docs.size() > L.cap_docs) {
        L.tab_sig.clear();
        dfree(L.docs_rel);
        dfree(L.doc_rank);
        HIPCHK(dalloc(&L.docs_rel, docs.size()), "hipMalloc logs.docs");
        HIPCHK(dalloc(&L.doc_rank, docs.size()), "hipMalloc logs.doc_rank");
        gen_++;
        L.cap_docs = docs.size();
    }
    if (nchunks > L.cap_chunks) {
        L.tab_sig.clear();
        dfree(L.chunk_doc);
        HIPCHK(dalloc(&L.chunk_doc, nchunks), "hipMalloc logs.chunk_doc");
        gen_++;
        L.cap_chunks = nchunks;
    }
    return upload_tables(L);
}

int Engine::upload_tables(DeviceLogs& L) {
    const uint32_t nd = (uint32_t)L.docs.size();
    if (nd == 0) return CRDT_HIP_OK;
    // the same plan as the tables on the device (a replica merged again at the same size)
    std::vector<uint64_t> sig;
    sig.reserve(2 * nd + L.waves.size() + 1);
    sig.push_back(L.total_slots);
    for (uint32_t d = 0; d < nd; ++d) {
        sig.push_back(L.docs[d].n);
        sig.push_back(L.doc_slot[d]);
    }
    for (const Wave& w : L.waves) sig.push_back(w.first_doc);
    if (sig == L.tab_sig) return CRDT_HIP_OK;
    L.tab_sig.clear();
    std::vector<uint2> rel(nd);
    std::vector<uint32_t> local(nd), order(nd), rank(nd);
    for (const Wave& w : L.waves) {
        for (uint32_t k = 0; k < w.ndocs; ++k) {
            const uint32_t d = w.first_doc + k;
            rel[d] = make_uint2((uint32_t)(L.doc_slot[d] - w.slot0), L.docs[d].n);
            local[d] = k;
        }
        // k_doctree's workgroup order: the costliest documents first (longest-processing-time
        // order: the last workgroups of a launch are the short ones, so the CUs finish together);
        // the visible text stands in for the cost
        uint32_t* o = order.data() + w.first_doc;
        for (uint32_t k = 0; k < w.ndocs; ++k) o[k] = k;
        std::stable_sort(o, o + w.ndocs, [&](uint32_t x, uint32_t y) {
            return L.docs[w.first_doc + x].text_cap > L.docs[w.first_doc + y].text_cap;
        });
        for (uint32_t k = 0; k < w.ndocs; ++k) rank[w.first_doc + o[k]] = k;
    }
    // (pageable sources: hipMemcpyAsync has copied them when it returns; the tables are
    // consumed in stream order, so no wait here)
    HIPCHK(hipMemcpyAsync(L.docs_rel, rel.data(), nd * sizeof(uint2), hipMemcpyHostToDevice, stream),
           "upload docs");
    HIPCHK(hipMemcpyAsync(L.doc_rank, rank.data(), nd * 4ull, hipMemcpyHostToDevice, stream),
           "upload doc rank");
    const uint64_t nchunks = L.total_slots >> L.log2m;
    if (nd == 1) {  // one document: every chunk is document 0
        HIPCHK(hipMemsetAsync(L.chunk_doc, 0, nchunks * 4, stream), "chunk table");
        L.tab_sig = std::move(sig);
        return CRDT_HIP_OK;
    }
    if (nd > cap_tab_) {
        (void)hipStreamSynchronize(stream);
        dfree(tab_slot_);
        dfree(tab_local_);
        cap_tab_ = 0;
        HIPCHK(dalloc(&tab_slot_, nd), "hipMalloc doc_slot");
        HIPCHK(dalloc(&tab_local_, nd), "hipMalloc doc_local");
        cap_tab_ = nd;
    }
    HIPCHK(hipMemcpyAsync(tab_slot_, L.doc_slot.data(), nd * 8, hipMemcpyHostToDevice, stream),
           "upload doc slots");
    HIPCHK(hipMemcpyAsync(tab_local_, local.data(), nd * 4, hipMemcpyHostToDevice, stream),
           "upload doc index");
    k_chunk_doc<<<grid_for(nchunks), kBlock, 0, stream>>>(tab_slot_, tab_local_, nd, nchunks,
                                                          L.log2m, L.chunk_doc);
    HIPCHK(hipGetLastError(), "chunk table");
    L.tab_sig = std::move(sig);
    return CRDT_HIP_OK;
}

int Engine::upload(DeviceLogs& L, const crdt_hip_oplog_view* views, uint32_t n) {
    const uint64_t S = L.total_slots;
    // the encoded columns are written into a pinned staging buffer (kept and grown by the engine)
    // and copied by DMA: a pageable source is copied through the driver's own staging at a
    // fraction of the rate, and fresh host vectors cost a zero fill of every column (the upload
    // of a one-document merge, config 1's len(), was ~2/3 of that merge)
    if (up_pending_) {  // (the last upload's copies still read the staging)
        HIPCHK(hipEventSynchronize(up_ev_), "upload staging");
        up_pending_ = false;
    }
    const uint64_t need = S * 12ull + cp3_bytes(S) + 64;
    if (need > cap_up_pin_) {
        if (up_pin_) (void)hipHostFree(up_pin_);
        up_pin_ = nullptr;
        cap_up_pin_ = 0;
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&up_pin_), need), "pinned upload staging");
        cap_up_pin_ = need;
    }
    uint64_t* key = reinterpret_cast<uint64_t*>(up_pin_);
    uint32_t* par = reinterpret_cast<uint32_t*>(up_pin_ + S * 8ull);
    uint8_t* c = up_pin_ + S * 12ull;
    // the slots that hold no item (document starts, padding) before document d, and after the
    // last (d = n): parent 0, key 0, deleted
    auto gap = [&](uint32_t d, uint64_t& lo, uint64_t& hi) {
        lo = d ? L.doc_slot[d - 1] + 1 + views[d - 1].n : 0;
        hi = d < n ? L.doc_slot[d] + 1 : S;  // (through the start slot of doc d)
    };
    // Column by column, each copied (on the engine's stream: a null-stream copy does not wait
    // for the non-blocking streams the kernels run on, nor they for it) as soon as it is
    // written, so that the DMA of one column overlaps the encoding of the next.
    uint64_t lo, hi;
    for (uint32_t d = 0; d <= n; ++d) {
        gap(d, lo, hi);
        if (hi > lo) std::memset(par + lo, 0, (hi - lo) * 4);
        if (d < n && views[d].n) std::memcpy(par + L.doc_slot[d] + 1, views[d].parent, views[d].n * 4ull);
    }
    HIPCHK(hipMemcpyAsync(L.parent, par, S * 4, hipMemcpyHostToDevice, stream), "upload parent");
    L.fugue = false;
    for (uint32_t d = 0; d <= n; ++d) {
        gap(d, lo, hi);
        if (hi > lo) std::memset(key + lo, 0, (hi - lo) * 8);
        if (d == n) break;
        const crdt_hip_oplog_view& v = views[d];
        const uint64_t b = L.doc_slot[d] + 1;
        if (v.side) {  // Fugue: left children carry kLeftKey (and kLeftBit, never the seq flag)
            for (uint32_t i = 0; i < v.n; ++i) {
                const bool left = v.side[i] != 0;
                if (v.lamport[i] == 0xFFFFFFFFu) {  // (kMidKey sorts above every right child)
                    // a malformed log, as replica_upload reports it (one code on every path)
                    err = "invalid Fugue log (lamport 0xFFFFFFFF)";
                    (void)hipStreamSynchronize(stream);  // (the parent copy reads the staging)
                    return CRDT_HIP_EBADLOG;
                }
                L.fugue |= left;
                key[b + i] = ((uint64_t)v.lamport[i] << 16) | v.agent[i] | (left ? kLeftKey : 0ull);
            }
        } else {
            for (uint32_t i = 0; i < v.n; ++i) key[b + i] = ((uint64_t)v.lamport[i] << 16) | v.agent[i];
        }
    }
    HIPCHK(hipMemcpyAsync(L.key, key, S * 8, hipMemcpyHostToDevice, stream), "upload key");
    std::vector<uint64_t> nsq_doc(n, 0);
    for (uint32_t d = 0; d <= n; ++d) {
        gap(d, lo, hi);
        for (uint64_t g = lo; g < hi; ++g) cp3_put(c, g, kDelBit);
        if (d == n) break;
        const crdt_hip_oplog_view& v = views[d];
        const uint64_t b = L.doc_slot[d] + 1;
        if (v.side) {
            for (uint32_t i = 0; i < v.n; ++i) {
                const bool left = v.side[i] != 0;
                cp3_put(c, b + i, (v.cp[i] & kCpMask) | (v.deleted[i] ? kDelBit : 0u) |
                                      (left ? kLeftBit : (v.parent[i] == i ? kSeqBit : 0u)));
            }
            continue;
        }
        uint64_t q = 0;
        for (uint32_t i = 0; i < v.n; ++i) {
            cp3_put(c, b + i, (v.cp[i] & kCpMask) | (v.deleted[i] ? kDelBit : 0u) |
                                  (v.parent[i] == i ? kSeqBit : 0u));
            q += v.parent[i] != i;
        }
        nsq_doc[d] = q;
    }
    HIPCHK(hipMemcpyAsync(L.cp, c, cp3_bytes(S), hipMemcpyHostToDevice, stream), "upload cp");
    for (Wave& w : L.waves) {
        w.nsq_items = 0;
        for (uint32_t k = 0; k < w.ndocs; ++k) w.nsq_items += nsq_doc[w.first_doc + k];
    }
    set_contraction(L);
    // A one-wave upload (a single document: config 1's len()) is not waited for: its merge runs
    // on this stream behind the copies, and the next upload waits before it rewrites the staging
    // (up_ev_).  Merges of several waves may run on the lanes' streams: waited for here.
    if (L.waves.size() == 1) {
        if (!up_ev_) HIPCHK(hipEventCreateWithFlags(&up_ev_, hipEventDisableTiming), "event create");
        HIPCHK(hipEventRecord(up_ev_, stream), "upload event");
        up_pending_ = true;
    } else {
        HIPCHK(hipStreamSynchronize(stream), "upload sync");
    }
    return CRDT_HIP_OK;
}

int Engine::ensure_scratch(const Wave& w) {
    const uint64_t slots = w.nslots;
    if (slots > cap_slots0_) {
        dfree(jbits_); dfree(nsqb_); dfree(visb_); dfree(wnib_); dfree(escm_); dfree(hrec_); dfree(stile_); dfree(plist_);
        dfree(tile_hw_); dfree(tile_sums_);
        const uint64_t tiles = slots / kScanTile + 2;
        // jump bits, then (Fugue) the left-child bits: jbits_words(slots) words each
        HIPCHK(dalloc(&jbits_, 2 * jbits_words(slots)), "hipMalloc jump bits");
        HIPCHK(dalloc(&nsqb_, slots / 16 + 4), "hipMalloc seq bits");
        HIPCHK(dalloc(&wnib_, slots / 16 + 4), "hipMalloc weight nibbles");
        HIPCHK(dalloc(&visb_, slots / 16 + 4), "hipMalloc visible bits");
        HIPCHK(dalloc(&escm_, slots / 1024 + 4), "hipMalloc escape words");
        HIPCHK(dalloc(&hrec_, slots / 64 + 2), "hipMalloc head records");
        HIPCHK(dalloc(&stile_, tiles * kTileBytes), "hipMalloc tile text");
        HIPCHK(dalloc(&plist_, tiles * kScanTile), "hipMalloc parent lists");
        HIPCHK(dalloc(&tile_hw_, tiles), "hipMalloc tile totals");
        HIPCHK(dalloc(&tile_sums_, tiles / kScanTile + 2), "hipMalloc tile sums");
        cap_slots0_ = slots;
        gen_++;
    }
    if (w.text_cap + 64 > cap_sbytes_) {
        dfree(sbytes_);
        HIPCHK(dalloc(&sbytes_, w.text_cap + 64), "hipMalloc slot-order text");
        cap_sbytes_ = w.text_cap + 64;
        gen_++;
    }
    if (w.ndocs + 1 > cap_docs_) {
        dfree(tlen_); dfree(loff_); dfree(toff_); dfree(out_); dfree(doc_root_); dfree(doc_p0_);
        dfree(doc_fused_); dfree(wgtab_);
        const uint64_t nd = w.ndocs + 1;
        HIPCHK(dalloc(&out_, 16 + 4 * nd), "hipMalloc results");  // ctl + one uint4 per document
        ctl_ = out_;
        res_ = reinterpret_cast<uint4*>(out_ + 16);
        HIPCHK(dalloc(&tlen_, nd), "hipMalloc tlen");
        HIPCHK(dalloc(&loff_, nd), "hipMalloc loff");
        HIPCHK(dalloc(&toff_, nd), "hipMalloc toff");
        HIPCHK(dalloc(&doc_root_, nd), "hipMalloc doc_root");
        HIPCHK(dalloc(&doc_p0_, nd), "hipMalloc doc_p0");
        HIPCHK(dalloc(&doc_fused_, nd), "hipMalloc doc_fused");
        HIPCHK(dalloc(&wgtab_, 2 * nd), "hipMalloc workgroup descriptors");
        cap_docs_ = nd;
        gen_++;
    }
    const uint64_t tb = std::max<uint64_t>(w.text_cap, w.order_cap * 4) + 64;
    if (tb > cap_text_) {
        dfree(text_);
        HIPCHK(dalloc(&text_, tb), "hipMalloc text");
        cap_text_ = tb;
        gen_++;
    }
    if (w.leaf_cap + 1 > cap_leaves_) {
        dfree(leafh_);
        dfree(ghash_);
        dfree(leafcp_);
        dfree(gcp_);
        HIPCHK(dalloc(&leafh_, w.leaf_cap + 1), "hipMalloc leaf hashes");
        HIPCHK(dalloc(&ghash_, w.leaf_cap + 1), "hipMalloc group hashes");
        HIPCHK(dalloc(&leafcp_, w.leaf_cap + 1), "hipMalloc leaf codepoints");
        HIPCHK(dalloc(&gcp_, w.leaf_cap + 1), "hipMalloc group codepoints");
        cap_leaves_ = w.leaf_cap + 1;
        gen_++;
    }
    return CRDT_HIP_OK;
}

// Level-1 scratch, sized by the runs of the wave (known after level 0).
int Engine::ensure_runs(uint64_t R, uint64_t S) {
    if (R > cap_runs_) {
        dfree(r_parent_); dfree(roff_); dfree(rloc_); dfree(r_key_); dfree(rec_);
        const uint64_t r = R + (R >> 3) + 4096;  // headroom against regrowth
        HIPCHK(dalloc(&r_parent_, r), "hipMalloc r_parent");
        HIPCHK(dalloc(&r_key_, r), "hipMalloc r_key");
        HIPCHK(dalloc(&roff_, r), "hipMalloc roff");
        HIPCHK(dalloc(&rloc_, r), "hipMalloc run sublist offsets");
        HIPCHK(dalloc(&rec_, 2 * r), "hipMalloc run records");  // (two uint4 per run)
        cap_runs_ = r;
        gen_++;
    }
    return ensure_splitters(S);
}

// Counting-path scratch of the global level 1 (R runs): child counts, segment starts, children,
// the deferred and long group lists, scan sums.
int Engine::ensure_csr(uint64_t R) {
    if (R <= cap_csr_) return CRDT_HIP_OK;
    dfree(deg_); dfree(cstart_); dfree(child_); dfree(defer_); dfree(bigl_); dfree(scan_sums_);
    const uint64_t r = R + (R >> 3) + 4096;
    HIPCHK(dalloc(&deg_, r + 16), "hipMalloc child counts");
    HIPCHK(dalloc(&cstart_, r + 16), "hipMalloc segment starts");
    HIPCHK(dalloc(&child_, r), "hipMalloc children");
    HIPCHK(dalloc(&defer_, r / 9 + 64), "hipMalloc deferred groups");
    HIPCHK(dalloc(&bigl_, r / 65 + 64), "hipMalloc long groups");
    HIPCHK(dalloc(&scan_sums_, r / kScanTile + 2), "hipMalloc scan sums");
    cap_csr_ = r;
    gen_++;
    return CRDT_HIP_OK;
}

// Radix-sort scratch of the global level 1 (R runs): two element arrays, the look-back words
// (256 per tile), the histograms / counters, the lists of long sibling groups.
int Engine::ensure_radix(uint64_t R) {
    if (R > cap_rs_) {
        dfree(rs_elem_[0]); dfree(rs_elem_[1]); dfree(rs_status_); dfree(rs_bigl_);
        const uint64_t r = R + (R >> 3) + 4096;
        HIPCHK(dalloc(&rs_elem_[0], r), "hipMalloc radix elements");
        HIPCHK(dalloc(&rs_elem_[1], r), "hipMalloc radix elements");
        HIPCHK(dalloc(&rs_status_, (r / kRsTileA + 2) * kRsBinsMax), "hipMalloc radix look-back");
        HIPCHK(dalloc(&rs_bigl_, r / 65 + 64), "hipMalloc radix long groups");
        cap_rs_ = r;
        gen_++;
    }
    if (!rs_small_) {
        HIPCHK(dalloc(&rs_small_, (uint64_t)kRsSmall), "hipMalloc radix counters");
        gen_++;
    }
    return CRDT_HIP_OK;
}

int Engine::ensure_splitters(uint64_t S) {
    if (S > cap_splitters_) {
        dfree(swn_); dfree(spref_); dfree(sup_); dfree(spred_); dfree(svp_[0]); dfree(svp_[1]);
        const uint64_t sc = S + (S >> 3) + 1024;
        HIPCHK(dalloc(&swn_, sc), "hipMalloc splitter weights");
        HIPCHK(dalloc(&spref_, sc), "hipMalloc splitter prefixes");
        // (supers: one per kSup regular splitters and one per document: fewer than the splitters)
        HIPCHK(dalloc(&sup_, sc), "hipMalloc supers");
        HIPCHK(dalloc(&spred_, sc), "hipMalloc super links");
        HIPCHK(dalloc(&svp_[0], sc), "hipMalloc super ranks");
        HIPCHK(dalloc(&svp_[1], sc), "hipMalloc super ranks");
        cap_splitters_ = sc;
        gen_++;
    }
    return CRDT_HIP_OK;
}

// Pinned host image of every wave's result block: wave i's ctl (64 B) then one uint4 per
// document, at byte 64 i + 16 first_doc (one device-to-host copy per wave).
int Engine::ensure_host_out(const DeviceLogs& L) {
    const uint64_t need = 64ull * L.waves.size() + 16ull * L.docs.size() + 64;
    if (need <= cap_host_out_) return CRDT_HIP_OK;
    if (host_out_) (void)hipHostFree(host_out_);
    host_out_ = nullptr;
    cap_host_out_ = 0;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&host_out_), need), "pinned results");
    cap_host_out_ = need;
    gen_++;
    return CRDT_HIP_OK;
}

int Engine::ensure_events(std::vector<hipEvent_t>& ev, size_t n) {
    while (ev.size() < n) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e), "event create");
        ev.push_back(e);
    }
    return CRDT_HIP_OK;
}

// Level-1 path and LDS sizing of a wave with R runs whose largest document has rmax runs.
L1Plan Engine::plan_level1(const Wave& w, uint32_t R, uint32_t rmax, bool ord,
                           bool force_global) const {
    L1Plan p;
    p.R = R;
    p.rmax = rmax;
    p.rcap = (rmax + 2u + 7u) & ~7u;
    p.scap = (((rmax + (1u << kDocLog2S) - 1u) >> kDocLog2S) + 8u) & ~7u;
    // per-document LDS path when the largest document's run tree fits one workgroup (sublist
    // offsets are packed in 18 bits inside the walk: documents below 256 KiB of text):
    // k_doctree (8-byte keys, 12 runs per thread), else k_doctree_wide (32-bit keys, 14)
    uint64_t dbytes = doctree_lds_bytes(p.rcap, p.scap, false);
    p.wide = rmax > (uint32_t)(kDocJNarrow * kDocThreads) || dbytes > kDocLds || doctree_k32;
    if (p.wide) dbytes = doctree_lds_bytes(p.rcap, p.scap, true);
    p.lds1 = !level1_global && !force_global && rmax <= (uint32_t)(kDocJ * kDocThreads) &&
             dbytes <= kDocLds && w.max_doc_text < (1ull << 18);
    // expansion + digest fused into k_doctree when every document's text fits LDS: text staging
    // + run-start bitvector (tl/8 + tl/16) + one u32 per run
    p.fuse = fuse_text && p.lds1 && !ord && w.max_doc_text + 512u <= kDocLds;
    // (a document spans at most max_doc_slots / 4096 + 2 tiles)
    p.stile_text = p.fuse && stile_text && w.max_doc_slots / kScanTile + 2u <= kDocTiles;
    // (roff holds u32 places in the wave's text)
    p.scatter = p.stile_text && text_scatter && w.text_cap + 64u < (1ull << 32);
    p.dyn_scatter = dbytes;
    // (+ the glds staging's partly used chunks and tile table: 44 B per tile)
    p.dyn_bytes = p.fuse ? std::min<uint64_t>(kDocLds, std::max<uint64_t>(
                               dbytes, (w.max_doc_text * 5 / 4 + 4ull * rmax + 512u +
                                        44ull * (w.max_doc_slots / kScanTile + 3u) + 15u) & ~15ull))
                         : dbytes;
    if (doctree_lds_max && p.lds1) p.dyn_bytes = kDocLds;  // experiment: one workgroup per CU
    return p;
}

// Stage timing: an event at the start of the wave and after every stage that ran; a stage's time
// is the interval since the event before it.  (Two events per stage, recorded whether the stage
// ran or not, cost several microseconds of host time each on a one-document merge.)
int Engine::clock_mark(StageClock& c, int stage) {
    if (!c.ev || c.n >= kClockEvents) return CRDT_HIP_OK;  // untimed (a captured graph)
    if (c.n) c.stage[c.n - 1] = (uint8_t)stage;
    HIPCHK(hipEventRecord(c.ev[c.n], cur_), "event record");
    ++c.n;
    return CRDT_HIP_OK;
}
#define MARK(st)                                       \
    do {                                               \
        if (const int _rc = clock_mark(ck, (st))) return _rc; \
    } while (0)

// Level-0 argument block of a wave (device pointers of L and of this engine's scratch).
#define L0ARGS(a0)                                                  \
    L0Args a0{};                                                    \
    a0.nslots = w.nslots;                                           \
    a0.log2m = L.log2m;                                             \
    a0.ndocs = w.ndocs;                                             \
    a0.mode = ord ? 1u : 0u;                                        \
    a0.ntiles = (uint32_t)((w.nslots + kScanTile - 1) / kScanTile); \
    a0.chunk_doc = L.chunk_doc + (w.slot0 >> L.log2m);              \
    a0.docs = L.docs_rel + w.first_doc;                             \
    a0.in_parent = L.parent + w.slot0;                              \
    a0.in_key = L.key + w.slot0;                                    \
    a0.in_cp = L.cp + 3ull * w.slot0;                               \
    a0.jbits = jbits_;                                              \
    a0.nsqb = nsqb_;                                                \
    a0.wnib = wnib_;                                                \
    a0.visb = visb_;                                                \
    a0.escm = escm_;                                                \
    a0.lbits = jbits_ + jbits_words(w.nslots);                      \
    a0.fugue = L.fugue ? 1u : 0u;                                   \
    a0.stile = stile_;                                              \
    a0.plist = plist_;                                              \
    a0.sbytes = sbytes_;                                            \
    a0.sbytes_cap = cap_sbytes_ - 64;                               \
    a0.tile_hw = tile_hw_;                                          \
    a0.tile_sums = tile_sums_;                                      \
    a0.hrec = hrec_;                                                \
    a0.doc_root = doc_root_;                                        \
    a0.doc_p0 = doc_p0_;                                            \
    a0.ctl = ctl_;                                                  \
    a0.r_head = r_head_;                                            \
    a0.r_pstart = r_pstart_;                                        \
    a0.r_parent = r_parent_;                                        \
    a0.r_key = r_key_;                                              \
    a0.cap_runs = 0xFFFFFFFFu;                                      \
    a0.cap_rmax = 0xFFFFFFFFu;                                      \
    a0.cap_rows = (uint32_t)std::min<uint64_t>(cap_runs_, 0xFFFFFFFFull);  \
    a0.xcd = xcd_order ? 1u : 0u;                                  \
    a0.nsq_par = L.nsq_ok ? L.nsq_par : nullptr;                    \
    a0.nsq_key = L.nsq_ok ? L.nsq_key : nullptr;                    \
    a0.nsq_pre = L.nsq_ok ? L.nsq_pre + (w.slot0 >> 6) : nullptr;   \
    a0.nocon = w.nocon ? 1u : 0u;                                   \
    a0.copy_text = 1u

// Tree / digest argument block (run counts come from ctl where the kernels need them).
#define TREEARGS(a)                                                                   \
    TreeArgs a{};                                                                     \
    a.ndocs = w.ndocs;                                                                \
    a.in_parent = r_parent_;                                                          \
    a.key = r_key_;                                                                   \
    a.pstart = r_pstart_;                                                             \
    a.doc_root = doc_root_;                                                           \
    a.doc_p0 = doc_p0_;                                                               \
    a.rec = rec_; a.ctl = ctl_; a.swn = swn_;                                         \
    a.roff = roff_;                                                                   \
    a.rloc = rloc_;                                                                   \
    a.tlen = tlen_; a.toff = toff_; a.loff = loff_; a.leafh = leafh_; a.ghash = ghash_; \
    a.leafcp = leafcp_; a.gcp = gcp_; a.res = res_;                                   \
    a.rank = L.doc_rank + w.first_doc; a.wg = nullptr;                                \
    a.docs = L.docs_rel + w.first_doc;                                                \
    a.text = text_;                                                                   \
    a.text_cap = ord ? w.order_cap : cap_text_ - 64;                                  \
    a.align = ord ? 1u : 16u;                                                         \
    a.walk_text = 0;                                                                  \
    a.rsh = 0;                                                                        \
    a.sbytes = sbytes_;                                                               \
    a.r_head = r_head_;                                                               \
    a.chunk_doc = L.chunk_doc + (w.slot0 >> L.log2m);                                 \
    a.log2c = L.log2m;                                                                \
    a.wtmp = wtmp_;                                                                   \
    a.ovf = ovf_

// k_runs with 16, 32 or 64 slots per thread (Engine::runs_slots)
void launch_k_runs(const L0Args& a0, uint32_t ntiles, hipStream_t s, uint32_t slots) {
    if (a0.fugue) {
        if (slots == 64)
            k_runs<true, 64><<<ntiles, kScanTile / 64, 0, s>>>(a0);
        else if (slots == 32)
            k_runs<true, 32><<<ntiles, kScanTile / 32, 0, s>>>(a0);
        else
            k_runs<true, 16><<<ntiles, kScanTile / 16, 0, s>>>(a0);
    } else {
        if (slots == 64)
            k_runs<false, 64><<<ntiles, kScanTile / 64, 0, s>>>(a0);
        else if (slots == 32)
            k_runs<false, 32><<<ntiles, kScanTile / 32, 0, s>>>(a0);
        else
            k_runs<false, 16><<<ntiles, kScanTile / 16, 0, s>>>(a0);
    }
}

int Engine::launch_level0(DeviceLogs& L, const Wave& w, bool ord, bool copy_text,
                          uint32_t cap_runs, uint32_t cap_rmax, StageClock& ck) {
    hipStream_t s = cur_;
    L0ARGS(a0);
    a0.copy_text = copy_text ? 1u : 0u;
    a0.cap_runs = cap_runs;
    a0.cap_rmax = cap_rmax;
    const uint32_t ntiles = a0.ntiles;
    const uint32_t nsums = (ntiles + kScanTile - 1) / kScanTile;
    // jump-bit words (and the left-child bits right after them), in uint4
    const uint32_t nq = (uint32_t)(jbits_words(w.nslots) / 4) * (L.fugue ? 2u : 1u);
    k_clear<<<std::min<uint32_t>(grid_for(nq), 2048u), 256, 0, s>>>(ctl_, reinterpret_cast<uint4*>(jbits_), nq);
    MARK(-1);
    k_classify<<<ntiles, kBlock, 0, s>>>(a0);
    MARK(S_CLASSIFY);
    k_heads<<<grid_for(w.nslots / 64), kBlock, 0, s>>>(a0);
    if (nsums == 1) {
        k_tiles_one<<<1, kBlock, 0, s>>>(a0);
    } else {
        k_tiles_reduce<<<nsums, kBlock, 0, s>>>(a0);
        k_tiles_top<<<1, 1024, 0, s>>>(a0, nsums);
        k_tiles_apply<<<nsums, kBlock, 0, s>>>(a0);
    }
    launch_k_runs(a0, ntiles, s, runs_slots);
    k_docmax<<<1, 1024, 0, s>>>(a0);
    MARK(S_RUNS);
    HIPCHK(hipGetLastError(), "level-0 launch");
    return CRDT_HIP_OK;
}

// k_runs alone (run_wave: the run rows did not fit the rows allocated when level 0 ran).
int Engine::launch_runs(DeviceLogs& L, const Wave& w, bool ord) {
    L0ARGS(a0);
    launch_k_runs(a0, a0.ntiles, cur_, runs_slots);
    HIPCHK(hipGetLastError(), "k_runs launch");
    return CRDT_HIP_OK;
}

// k_doctotals, k_doctree (k_expand for documents whose text did not fit runs in the tail).
int Engine::launch_lds_level1(DeviceLogs& L, const Wave& w, bool ord, const L1Plan& p,
                              bool stile, StageClock& ck) {
    hipStream_t s = cur_;
    TREEARGS(a);
    tail_nspl_ = 0;  // (k_doctree leaves any offsets k_expand needs in roff)
    const bool scatter = stile && p.scatter;
    tail_scatter_ = scatter;
    DocArgs da{};
    da.ndocs = w.ndocs;
    da.rcap = p.rcap;
    da.scap = p.scap;
    da.chbytes = doctree_ch_bytes(p.rcap, p.scap);
    da.doc_root = doc_root_;
    da.r_parent = r_parent_;
    da.r_key = r_key_;
    da.roff = roff_;
    da.ctl = ctl_;
    da.r_pstart = r_pstart_;
    da.doc_p0 = doc_p0_;
    da.tlen = tlen_;
    da.toff = toff_;
    da.sbytes = sbytes_;
    da.text = p.fuse && !scatter ? text_ : nullptr;
    da.fused = doc_fused_;
    da.scatter = scatter ? 1u : 0u;
    da.glds_late = glds_late ? 1u : 0u;
    da.lds_bytes = (uint32_t)(scatter ? p.dyn_scatter : p.dyn_bytes);
    da.probe = probe_doc_;
    da.wg = wgtab_;
    da.keyoff = doctree_key_off(p.rcap, p.scap, p.wide);
    da.stile_text = stile && !scatter ? (stile_text == 2u ? 2u : 1u) : 0u;
    da.ntiles = (uint32_t)((w.nslots + kScanTile - 1) / kScanTile);
    da.stile = stile_;
    da.tile_hw = tile_hw_;
    a.wg = wgtab_;  // (k_doctotals writes the k_doctree workgroup descriptors)
    k_doctotals<<<1, 1024, 0, s>>>(a);
    const bool pc = da.text != nullptr;  // (phase C: the instances that write the text)
    if (p.wide && p.rmax > (uint32_t)(kDocJNarrow * kDocThreads)) {
        if (pc) k_doctree_wide17<true><<<w.ndocs, kDocThreads, da.lds_bytes, s>>>(da);
        else k_doctree_wide17<false><<<w.ndocs, kDocThreads, da.lds_bytes, s>>>(da);
    } else if (p.wide) {
        if (pc) k_doctree_wide<true><<<w.ndocs, kDocThreads, da.lds_bytes, s>>>(da);
        else k_doctree_wide<false><<<w.ndocs, kDocThreads, da.lds_bytes, s>>>(da);
    } else {
        if (pc) k_doctree<true><<<w.ndocs, kDocThreads, da.lds_bytes, s>>>(da);
        else k_doctree<false><<<w.ndocs, kDocThreads, da.lds_bytes, s>>>(da);
    }
    MARK(S_DOCTREE);
    HIPCHK(hipGetLastError(), "level-1 launch");
    return CRDT_HIP_OK;
}

// The global (grid-wide) level 1, for waves whose documents do not fit the LDS path.  Grids are
// sized by the exact run count (the caller waited for level 0).
int Engine::launch_global_level1(DeviceLogs& L, const Wave& w, bool ord, const L1Plan& p,
                                 StageClock& ck, uint32_t& rounds) {
    hipStream_t s = cur_;
    TREEARGS(a);
    tail_scatter_ = false;
    const uint32_t R = p.R;
    // splitter stride: longer sublists once the pointer jumping over the splitter lists
    // dominates (measured on config 5: 182 M runs, stride 16 -> 64 took 72 -> 59 ms)
    const uint32_t log2m_w = log2m_set ? this->log2m : (R > (1u << 24) ? 6u : 4u);
    const uint32_t Sreg = 2 * ((R + (1u << log2m_w) - 1) >> log2m_w);
    const uint32_t S = Sreg + w.ndocs;
    a.R = R;
    a.log2m = log2m_w;
    a.Sreg = Sreg;
    a.S = S;
    a.step_limit = 2u * R + 4u;
    const uint32_t gR = grid_for(R);
    // text mode of a wave without run contraction: the walkers write the text (runs are single
    // items), from records that carry their place in the slot-order text (two lines per run)
    a.walk_text = walk_text(w, ord, p) ? 1u : 0u;
    a.rsh = a.walk_text;
    a.wtmp_log2 = wtmp_log2_;
    if (l1_csr_) {  // (chosen by run_wave, which sized the scratch)
        CsrArgs c_{cstart_, child_, defer_, bigl_};
        const uint32_t nb = (uint32_t)((R + kScanTile - 1) / kScanTile);
        HIPCHK(hipMemsetAsync(deg_, 0, (R + 1ull) * 4ull, s), "clear child counts");
        k_count<<<gR, kBlock, 0, s>>>(a, deg_);
        MARK(S_COUNT);
        k_scan_reduce<<<nb, kBlock, 0, s>>>(deg_, R, scan_sums_);
        k_scan_top<<<1, 1024, 0, s>>>(scan_sums_, nb, cstart_, R);
        k_scan_apply<<<nb, kBlock, 0, s>>>(deg_, R, scan_sums_, cstart_);
        MARK(S_SCAN);
        k_place<<<gR, kBlock, 0, s>>>(a, cstart_, child_);
        MARK(S_PLACE);
        k_link<<<gR, kBlock, 0, s>>>(a, c_);
        k_sortmid<<<kMidGrid, kBlock, 0, s>>>(a, c_);
        k_sortbig<<<kBigGrid, kBigThreads, 0, s>>>(a, c_);
        MARK(S_LINK);
    } else {
        // sort A by parent run (document starts: R), 8-bit digits or 10-bit ones where they save a
        // pass (waves of 2^24..2^30 runs: 3 passes instead of 4); sort B by run id, 8 bits per pass
        const uint32_t bitsA = std::max<uint32_t>(1u, ceil_log2((uint64_t)R + 1u));
        const uint32_t p8 = (bitsA + 7u) / 8u, p10 = (bitsA + 9u) / 10u;
        const uint32_t dbA = rs_digit_bits ? (p10 <= 3u ? rs_digit_bits : 8u)  // (kRsHistA)
                                           : (p10 < p8 ? 10u : 8u);
        const uint32_t npass = dbA == 10u ? p10 : p8;
        const uint64_t tilesA = ((uint64_t)R + kRsTileA - 1) / kRsTileA;
        const uint64_t tilesB = ((uint64_t)R + kRsTileB - 1) / kRsTileB;
        rs_npass_ = npass;
        RsArgs r{};
        r.R = R;
        r.npass = npass;
        r.dbits = dbA;
        {
            const uint32_t bits = ceil_log2((uint64_t)R);  // (run ids < R)
            r.npassB = bits > kRsPlaceBits ? (bits - kRsPlaceBits + 7u) / 8u : 0u;
        }
        rs_npassB_ = r.npassB;
        r.shift0 = 0;
        r.rctl = rs_small_ + kRsCtl;
        r.status = rs_status_;
        r.bigl = rs_bigl_;
        r.fc = roff_;  // (free until k_walk1)
        HIPCHK(hipMemsetAsync(rs_small_, 0, kRsSmall * 4ull, s), "clear radix counters");
        HIPCHK(hipMemsetAsync(roff_, 0xFF, R * 4ull, s), "clear first children");
        r.hist = rs_small_;
        k_rs_hist<<<std::min<uint32_t>(gR, 2048u), kBlock, 0, s>>>(a, r);
        MARK(S_COUNT);
        k_rs_scan<<<1, kRsBinsMax, 0, s>>>(r);
        MARK(S_SCAN);
        r.tctr = r.rctl;
        for (uint32_t k = 0; k < npass; ++k) {
            r.pass = k;
            r.in = k ? rs_elem_[(k - 1) & 1] : nullptr;
            r.out = rs_elem_[k & 1];
            HIPCHK(hipMemsetAsync(rs_status_, 0, tilesA * (1ull << dbA) * 4ull, s), "clear look-back");
            const dim3 g((uint32_t)tilesA), b(kRsThreadsA);
            if (dbA == 10u) {
                if (k == 0) k_rs_pass<uint4, 0, kRsItemsA, kRsThreadsA, 10><<<g, b, 0, s>>>(a, r);
                else k_rs_pass<uint4, 1, kRsItemsA, kRsThreadsA, 10><<<g, b, 0, s>>>(a, r);
            } else {
                if (k == 0) k_rs_pass<uint4, 0, kRsItemsA, kRsThreadsA, 8><<<g, b, 0, s>>>(a, r);
                else k_rs_pass<uint4, 1, kRsItemsA, kRsThreadsA, 8><<<g, b, 0, s>>>(a, r);
            }
        }
        MARK(S_PLACE);
        uint4* E = rs_elem_[(npass - 1) & 1];
        uint2* B0 = reinterpret_cast<uint2*>(rs_elem_[npass & 1]);  // (the other element array:
        uint2* B1 = B0 + cap_rs_;                                     //  room for two pair arrays)
        r.B = B0;
        k_rs_order<<<gR, kBlock, 0, s>>>(a, r, E);
        k_rs_big<<<kBigGrid, kBigThreads, 0, s>>>(a, r, E);
        MARK(S_LINK);
        // sort B: the pairs by the run id's bits above kRsPlaceBits, then k_rs_place puts each
        // block's next siblings in run order (over the element array of sort A: dead once the
        // pairs are out)
        uint32_t* ns = reinterpret_cast<uint32_t*>(E);
        r.hist = rs_small_ + kRsHistB;
        r.tctr = r.rctl + kRsMaxPass;
        r.shift0 = kRsPlaceBits;
        r.dbits = 8;
        const uint2* Bf = B0;
        for (uint32_t k = 0; k < r.npassB; ++k) {
            r.pass = k;
            r.in = (k & 1) ? B1 : B0;
            r.out = (k & 1) ? B0 : B1;
            Bf = (k & 1) ? B0 : B1;
            HIPCHK(hipMemsetAsync(rs_status_, 0, tilesB * kRsBins * 4ull, s), "clear look-back");
            k_rs_pass<uint2, 1, kRsItemsB, kRsThreadsB, 8><<<(uint32_t)tilesB, kRsThreadsB, 0, s>>>(a, r);
        }
        k_rs_place<<<(uint32_t)(((uint64_t)R + (1u << kRsPlaceBits) - 1) >> kRsPlaceBits), 1024, 0, s>>>(a, Bf, ns);
        k_rs_records<<<gR, kBlock, 0, s>>>(a, roff_, ns);
        MARK(S_SORTB);
    }
    // two walkers per thread on waves without contraction in text mode, else one (§5b; the
    // grids of both walks are sized by it)
    const uint32_t ilp = a.walk_text && w.nocon ? 2u : 1u;
    const uint32_t gW = grid_for(((uint64_t)S + ilp - 1) / ilp);
    if (a.walk_text) HIPCHK(hipMemsetAsync(ctl_ + C_NOVF, 0, 4, s), "clear overflow count");
    if (a.walk_text && ilp == 2)
        k_walk1<2, true><<<gW, kBlock, 0, s>>>(a);
    else if (a.walk_text)
        k_walk1<1, true><<<gW, kBlock, 0, s>>>(a);
    else
        k_walk1<1, false><<<gW, kBlock, 0, s>>>(a);
    MARK(S_WALK1);
    SupArgs sa{};
    sa.S = S;
    sa.Sreg = Sreg;
    sa.slog2 = S >= (1u << 22) ? 6u : 3u;
    sa.Sc = ((Sreg + (1u << sa.slog2) - 1u) >> sa.slog2) + w.ndocs;
    sa.step_limit = S + 4u;
    sa.swn = swn_;
    sa.sup = sup_;
    sa.pred = spred_;
    sa.vp[0] = svp_[0];
    sa.vp[1] = svp_[1];
    sa.spref = spref_;
    sa.ctl = ctl_;
    const uint32_t gC = grid_for(sa.Sc);
    HIPCHK(hipMemsetAsync(spred_, 0xFF, sa.Sc * 4ull, s), "memset pred");
    k_sup1<<<gC, kBlock, 0, s>>>(sa);
    k_sup_init<<<gC, kBlock, 0, s>>>(sa);
    // a document's list holds at most 2 * (ceil(runs / M) + 1) + 1 splitters, of which at most
    // that / kSup + 2 are supers
    rounds = ceil_log2((2ull * ((p.rmax + (1u << log2m_w) - 1) >> log2m_w) >> sa.slog2) + 8);
    for (uint32_t k = 0; k < rounds; ++k)
        k_sup_step<<<gC, kBlock, 0, s>>>(svp_[k & 1], sa.Sc, svp_[(k + 1) & 1]);
    k_sup2<<<gC, kBlock, 0, s>>>(sa, svp_[rounds & 1]);
    const uint32_t* spref = spref_;
    MARK(S_RANK);
    k_doctotals<<<1, 1024, 0, s>>>(a);
    if (a.walk_text) {
        // the staged sublist texts out, then the rest of the longer sublists
        k_tcopy<<<grid_for(S), kBlock, 0, s>>>(a, spref);
        k_walk_ovf<<<1024, kBlock, 0, s>>>(a, spref);
    }
    // (otherwise k_expand adds the sublist prefixes to k_walk1's offsets as it copies the text)
    tail_nspl_ = a.walk_text ? 0u : S;
    MARK(S_WALK2);
    HIPCHK(hipGetLastError(), "level-1 launch");
    return CRDT_HIP_OK;
}

// Expansion (documents k_doctree did not write), digest, and one copy of the wave's result block
// (ctl + a {bytes, codepoints, digest} record per document) into the pinned host image.
int Engine::launch_tail(DeviceLogs& L, const Wave& w, bool ord, bool fused, StageClock& ck,
                        uint32_t* hblock) {
    hipStream_t s = cur_;
    L0ARGS(a0);
    TREEARGS(a);
    ExpandArgs ea{};
    ea.mode = a0.mode;
    ea.log2m = L.log2m;
    ea.chunk_doc = a0.chunk_doc;
    ea.docs = a0.docs;
    ea.r_head = r_head_;
    ea.r_pstart = r_pstart_;
    ea.roff = roff_;
    ea.tlen = tlen_;
    ea.toff = toff_;
    ea.sbytes = sbytes_;
    ea.text = text_;
    ea.ctl = ctl_;
    ea.fused = nullptr;
    ea.rloc = tail_nspl_ ? rloc_ : nullptr;
    ea.spref = spref_;
    ea.nspl = tail_nspl_;
    if (!fused) {  // (a fused k_doctree writes every document itself)
        k_expand<<<4096, kBlock, 0, s>>>(ea);
        MARK(S_EXPAND);
    }
    if (tail_scatter_) {  // (k_doctree in scatter mode left the text to k_tscatter)
        ScatterArgs sa{};
        sa.ntiles = a0.ntiles;
        sa.xcd = a0.xcd;
        sa.tile_hw = tile_hw_;
        sa.r_pstart = r_pstart_;
        sa.roff = roff_;
        sa.stile = stile_;
        sa.text = text_;
        sa.text_cap = cap_text_ - 64;
        sa.ctl = ctl_;
        k_tscatter<<<grid_for(sa.ntiles, (kBlock / 64) * kScatterTiles), kBlock, 0, s>>>(sa);
        MARK(S_TEXT);
    }
    if (!ord) {
        k_leafhash<<<grid_for(w.leaf_cap + 1, (kBlock / 64) * kLeafGroup), kBlock, 0, s>>>(
            a, (uint32_t)(w.leaf_cap + 1));
        if (w.max_doc_text > (uint64_t)kLeaf * kGroup)
            k_grouphash<<<grid_for(w.leaf_cap + 1), kBlock, 0, s>>>(a, (uint32_t)(w.leaf_cap + 1));
        k_docdigest<<<grid_for(w.ndocs), kBlock, 0, s>>>(a);
        MARK(S_DIGEST);
    }
    HIPCHK(hipGetLastError(), "kernel launch");
    HIPCHK(hipMemcpyAsync(hblock, out_, 64 + 16ull * w.ndocs, hipMemcpyDeviceToHost, s),
           "copy results");
    return CRDT_HIP_OK;
}
#undef MARK
#undef TREEARGS

int Engine::finish_wave(const Wave& w, bool ord, const L1Plan& p, uint32_t rounds,
                        const StageClock& ck, const uint32_t* hctl, std::vector<float>& stage_ms,
                        std::vector<uint32_t>& stage_launches) {
    const uint32_t g1 = p.lds1 ? 0u : 1u;
    const bool wt = walk_text(w, ord, p);
    const bool expand_run = !p.fuse && !wt;
    const uint32_t rs = l1_csr_ ? 0u : 1u;
    // (the runs stage: k_heads, the tile scan in one launch or three, k_runs, k_docmax)
    const uint64_t ntiles = (w.nslots + kScanTile - 1) / kScanTile;
    const uint32_t runs_launches = ntiles <= (uint64_t)kScanTile ? 4u : 6u;
    const uint32_t launches[S_N] = {1, runs_launches, (rs_npassB_ + 2) * g1 * rs, g1, (rs ? 1u : 3u) * g1,
                                    (rs ? rs_npass_ : 1u) * g1, (rs ? 2u : 3u) * g1, g1,
                                    (3 + rounds) * g1, (wt ? 4u : 1u) * g1,
                                    expand_run ? 1u : 0u,
                                    ord ? 0u : (w.max_doc_text > (uint64_t)kLeaf * kGroup ? 3u : 2u),
                                    p.lds1 ? 2u : 0u, p.lds1 && p.scatter ? 1u : 0u, 0u};
    for (uint32_t i = 0; i + 1 < ck.n; ++i) {
        if (ck.stage[i] >= S_N) continue;  // not a stage (a host wait between two launches)
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ck.ev[i], ck.ev[i + 1]), "event time");
        stage_ms[ck.stage[i]] += ms;
    }
    for (int i = 0; i < S_N; ++i) stage_launches[i] += launches[i];
    return CRDT_HIP_OK;
}

uint32_t* Engine::host_block(const DeviceLogs& L, uint32_t wi) const {
    return host_out_ + (64ull * wi + 16ull * L.waves[wi].first_doc) / 4;
}

// One wave, waiting for level 0 to learn its run counts (the first merge of a set of logs, the
// global level-1 path, ORDER mode).  Records the wave's launch plan for later merges.
int Engine::run_wave(DeviceLogs& L, uint32_t wi, Mode mode, std::vector<float>& stage_ms,
                     std::vector<uint32_t>& stage_launches, bool force_global) {
    Wave& w = L.waves[wi];
    hipStream_t s = stream;
    const bool ord = mode == ORDER;
    StageClock ck{ev_.data(), 0, {}};
    uint32_t* hctl = host_block(L, wi);
    // run records are written before the run count is known: runs <= slots (Fugue: rows <=
    // 2 slots, a content and a tree row per head with left children)
    const uint64_t hrows = w.nslots * (L.fugue ? 2ull : 1ull);
    if (hrows > cap_heads_) {
        dfree(r_head_); dfree(r_pstart_);
        HIPCHK(dalloc(&r_head_, hrows + 64ull), "hipMalloc r_head");
        HIPCHK(dalloc(&r_pstart_, hrows + 64ull), "hipMalloc r_pstart");
        cap_heads_ = hrows;
    }
    // ---- level 0: runs.  Lanes take turns here (an HBM stream): the gate is held from the first
    // level-0 launch to the level-0 sync, so one lane's level 0 overlaps the others' latency-bound
    // level 1.
    std::unique_lock<std::mutex> gate;
    if (l0_gate_) gate = std::unique_lock<std::mutex>(*l0_gate_);
    // (the plan is not known yet: k_runs writes the slot-order text)
    int rc = launch_level0(L, w, ord, true, 0xFFFFFFFFu, 0xFFFFFFFFu, ck);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(hctl, ctl_, 64, hipMemcpyDeviceToHost, s), "copy ctl");
    HIPCHK(hipStreamSynchronize(s), "level-0 sync");
    if (gate.owns_lock()) gate.unlock();
    if (hctl[C_ERR]) {
        err = hctl[C_ERR] & 4u ? "op log holds more text than planned"
                               : "malformed op log: parent id out of range";
        return CRDT_HIP_EBADLOG;
    }
    L1Plan p = plan_level1(w, hctl[C_RTOTAL], hctl[C_RMAX], ord, force_global);
    p.scatter = false;  // (no stile here: k_runs writes the slot-order text, k_doctree stages it)
    const uint32_t lg = log2m_set ? log2m : (p.R > (1u << 24) ? 6u : 4u);
    const uint32_t Sreg = 2 * ((p.R + (1u << lg) - 1) >> lg);
    const uint64_t rows = cap_runs_;  // run rows k_runs could write
    rc = ensure_runs(p.R, Sreg + w.ndocs);
    if (rc) return rc;
    // sibling grouping of the global level 1: by counting when every document's runs stay within
    // a few MB (the atomics and gathers land in cache), else by the two radix sorts
    l1_csr_ = l1_group == 1 || (l1_group == 0 && (p.rmax <= kCsrDocRuns || p.R <= kCsrWaveRuns));
    if (!p.lds1 && !l1_csr_ && (rc = ensure_radix(p.R))) return rc;
    if (!p.lds1 && l1_csr_ && (rc = ensure_csr(p.R))) return rc;
    if (walk_text(w, ord, p)) {
        // a text slot per splitter of ~4x the mean sublist text (128 B .. 4 KiB; + slack for
        // k_tcopy's dword reads) and the overflow list
        const uint64_t ns = (uint64_t)Sreg + w.ndocs;
        wtmp_log2_ = std::min<uint32_t>(12u, std::max<uint32_t>(
                         7u, ceil_log2(4ull * hctl[C_WTOTAL] / std::max<uint64_t>(1, ns) + 1)));
        if ((ns << wtmp_log2_) + 64 > cap_wtmp_) {
            dfree(wtmp_);
            cap_wtmp_ = 0;
            HIPCHK(dalloc(&wtmp_, (ns << wtmp_log2_) + 64), "hipMalloc sublist text");
            cap_wtmp_ = (ns << wtmp_log2_) + 64;
            gen_++;
        }
        if (ns > cap_ovf_) {
            dfree(ovf_);
            cap_ovf_ = 0;
            HIPCHK(dalloc(&ovf_, ns), "hipMalloc sublist overflow list");
            cap_ovf_ = ns;
            gen_++;
        }
    }
    if (p.R > rows) {
        // more runs than rows: the run records again, now that they fit (k_runs only reads
        // level-0 outputs, so it can run twice)
        if ((rc = launch_runs(L, w, ord))) return rc;
    }
    if ((rc = clock_mark(ck, 0xFF))) return rc;  // the host wait above is no stage's time
    uint32_t rounds = 0;
    // (k_runs wrote the slot-order text here: the plan was not known when level 0 ran)
    rc = p.lds1 ? launch_lds_level1(L, w, ord, p, false, ck)
                : launch_global_level1(L, w, ord, p, ck, rounds);
    if (rc) return rc;
    // (text mode of the global level 1 without run contraction: k_tcopy and k_walk_ovf wrote
    // the text)
    rc = launch_tail(L, w, ord, p.fuse || walk_text(w, ord, p), ck, hctl);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s), "merge wave");
    uint32_t errs = hctl[C_ERR];
    if (p.lds1 && (errs & 32u)) {
        // a sibling group wider than the LDS path sorts: redo the wave on the global path
        return run_wave(L, wi, mode, stage_ms, stage_launches, true);
    }
    rc = finish_wave(w, ord, p, rounds, ck, hctl, stage_ms, stage_launches);
    if (rc) return rc;
    runs_ += p.R;
    if (!errs && hctl[C_VISITED] != p.R) errs |= 16u;  // unreachable runs: a cycle
    if (errs) {
        (void)hipStreamSynchronize(stream);
        err = "malformed op log detected on device (flags " + std::to_string(errs) + ")";
        return CRDT_HIP_EBADLOG;
    }
    w.hint_runs = p.R;
    w.hint_rmax = p.rmax;
    w.hint_lds = p.lds1 && (p.fuse || !fuse_text) && !ord;
    if (w.hint_lds) learn_shape(w);
    return CRDT_HIP_OK;
}

void Engine::learn_shape(const Wave& w) {
    const WaveShape sh = shape_of(w);
    forget_shape(w);
    shape_hints_.insert(shape_hints_.begin(), ShapeHint{sh, w.hint_runs, w.hint_rmax});
    if (shape_hints_.size() > kShapeHints) shape_hints_.pop_back();
}

void Engine::forget_shape(const Wave& w) {
    const WaveShape sh = shape_of(w);
    for (size_t i = 0; i < shape_hints_.size(); ++i)
        if (shape_hints_[i].shape == sh) {
            shape_hints_.erase(shape_hints_.begin() + (long)i);
            return;
        }
}

void Engine::collect(const DeviceLogs& L, uint32_t wi, uint64_t* digests, uint64_t* lens,
                     uint64_t* cps, uint64_t& text_bytes) const {
    const Wave& w = L.waves[wi];
    const uint4* r = reinterpret_cast<const uint4*>(host_block(L, wi) + 16);
    for (uint32_t k = 0; k < w.ndocs; ++k) {
        // (a grouped replica batch: the caller's document of slot-order document first_doc + k)
        const uint32_t d = L.api_doc.empty() ? w.first_doc + k : L.api_doc[w.first_doc + k];
        if (lens) lens[d] = r[k].x;
        if (cps) cps[d] = r[k].y;
        if (digests) digests[d] = ((uint64_t)r[k].w << 32) | r[k].z;
        text_bytes += r[k].x;
    }
}

int Engine::merge(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens, crdt_hip_stats* st,
                  std::vector<uint8_t>* text_out, std::vector<uint64_t>* text_offsets,
                  uint64_t* cps) {
    HIPCHK(hipSetDevice(device), "hipSetDevice");
    if ((text_out || text_offsets) && L.waves.size() > 1) {
        err = "text output needs a single-wave merge";
        return CRDT_HIP_EINVAL;
    }
    if (const char* pe = getenv("CRDT_HIP_PROBE")) probe_doc_ = 1u + (uint32_t)atoi(pe);
    if (L.raw) {  // (raw SoA mode: the input encoding is part of every merge)
        if (!raw_ev_[0]) {
            HIPCHK(hipEventCreate(&raw_ev_[0]), "event create");
            HIPCHK(hipEventCreate(&raw_ev_[1]), "event create");
        }
        HIPCHK(hipEventRecord(raw_ev_[0], stream), "event record");
        if (const int rc = raw_encode(L)) return rc;
        HIPCHK(hipEventRecord(raw_ev_[1], stream), "event record");
        const int rc = merge_inner(L, mode, digests, lens, st, text_out, text_offsets, cps);
        if (rc || !st) return rc;
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, raw_ev_[0], raw_ev_[1]), "event time");
        st->stage_ns[S_ENCODE] += (uint64_t)((double)ms * 1e6);
        st->stage_launches[S_ENCODE] += (uint32_t)L.waves.size() + (L.nsq_ok ? 3u + (uint32_t)L.waves.size() : 0u);
        st->total_ns += (uint64_t)((double)ms * 1e6);
        return rc;
    }
    return merge_inner(L, mode, digests, lens, st, text_out, text_offsets, cps);
}

int Engine::merge_inner(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens,
                        crdt_hip_stats* st, std::vector<uint8_t>* text_out,
                        std::vector<uint64_t>* text_offsets, uint64_t* cps) {
    // learnt plans: every wave enqueued without a host wait; with text out for a one-wave merge
    // too (a document merged again and again, the upstream closure of config 1), the text then
    // copied back from this engine, which ran the one wave
    const bool want_text = text_out || text_offsets;
    bool hinted = plan_cache && mode == TEXT && !L.waves.empty() && (!want_text || L.waves.size() == 1);
    for (const Wave& w : L.waves) hinted = hinted && w.hint_lds;
    if (hinted) {
        const int rc = merge_async(L, digests, lens, cps, st);
        if (rc || !want_text) return rc;
        const Wave& w = L.waves[0];
        std::vector<uint64_t> offs(w.ndocs + 1);
        HIPCHK(hipMemcpyAsync(offs.data(), toff_, (w.ndocs + 1) * 8ull, hipMemcpyDeviceToHost, stream),
               "copy offsets");
        HIPCHK(hipStreamSynchronize(stream), "copy offsets");
        if (text_out) {
            text_out->resize(offs[w.ndocs]);
            if (offs[w.ndocs]) {
                HIPCHK(hipMemcpyAsync(text_out->data(), text_, offs[w.ndocs], hipMemcpyDeviceToHost,
                                      stream), "copy text");
                HIPCHK(hipStreamSynchronize(stream), "copy text");
            }
        }
        if (text_offsets) *text_offsets = offs;
        return CRDT_HIP_OK;
    }
    if (lanes > 1 && L.waves.size() > 1 && !text_out) return merge_lanes(L, mode, digests, lens, cps, st);
    std::vector<float> stage_ms(S_N, 0.f);
    std::vector<uint32_t> stage_launches(S_N, 0);
    const uint32_t ndocs = (uint32_t)L.docs.size();
    runs_ = 0;
    if (const int rc = ensure_host_out(L)) return rc;
    HIPCHK(hipEventRecord(ev_[2 * S_N + 1], stream), "event record");
    uint64_t text_bytes = 0;
    for (uint32_t wi = 0; wi < L.waves.size(); ++wi) {
        const Wave& w = L.waves[wi];
        int rc = ensure_scratch(w);
        if (rc) return rc;
        rc = run_wave(L, wi, mode, stage_ms, stage_launches);
        if (rc) return rc;
        collect(L, wi, digests, lens, cps, text_bytes);
        if (text_out) {
            std::vector<uint64_t> offs(w.ndocs + 1);
            HIPCHK(hipMemcpyAsync(offs.data(), toff_, (w.ndocs + 1) * 8ull, hipMemcpyDeviceToHost,
                                  stream), "copy offsets");
            HIPCHK(hipStreamSynchronize(stream), "copy offsets");
            const uint64_t total = offs[w.ndocs] * (mode == ORDER ? 4 : 1);
            text_out->resize(total);
            if (total) {
                HIPCHK(hipMemcpyAsync(text_out->data(), text_, total, hipMemcpyDeviceToHost, stream),
                       "copy text");
                HIPCHK(hipStreamSynchronize(stream), "copy text");
            }
            if (text_offsets) *text_offsets = offs;
        }
    }
    HIPCHK(hipEventRecord(ev_[2 * S_N + 2], stream), "event record");
    HIPCHK(hipEventSynchronize(ev_[2 * S_N + 2]), "event sync");
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->items = L.items;
        st->docs = ndocs;
        st->text_bytes = text_bytes;
        st->runs = runs_;
        st->waves = (uint32_t)L.waves.size();
        st->nstages = S_N;
        for (int i = 0; i < S_N; ++i) {
            st->stage_ns[i] = (uint64_t)((double)stage_ms[i] * 1e6);
            st->stage_launches[i] = stage_launches[i];
        }
        float tot = 0;
        HIPCHK(hipEventElapsedTime(&tot, ev_[2 * S_N + 1], ev_[2 * S_N + 2]), "event time");
        st->total_ns = (uint64_t)((double)tot * 1e6);
    }
    return CRDT_HIP_OK;
}

// Every wave of a merge whose launch plans are known (an earlier merge of the same logs, or of
// logs of the same shape, learnt them), enqueued without waiting: wave i goes to lane i % K (this
// engine or a helper engine: own stream and scratch), one host thread enqueues them all.  With
// the level-0 gate, a wave's level 0 waits (hipStreamWaitEvent) for the previous wave's level 0
// to end, so level 0 of one wave runs beside the latency-bound level 1 of another, as
// merge_lanes' mutex does.  The host waits once, at the end; a wave whose device check failed
// (C_REPLAN, or a sibling group too wide for the LDS path) is merged again synchronously.
// Three phases, so that a caller can capture the launches in a graph: prepare (lanes, plans,
// every allocation), enqueue (launches and copies only), finish (after the wait: errors, redo,
// results).
int Engine::merge_async_prepare(DeviceLogs& L, AsyncMerge& m, bool timed) {
    const uint32_t nw = (uint32_t)L.waves.size();
    m.K = std::max<uint32_t>(1, std::min<uint32_t>(lanes, nw));
    m.timed = timed;
    while (lane_eng_.size() + 1 < m.K) {
        auto e = std::make_unique<Engine>();
        const std::string msg = e->init(device);
        if (!msg.empty()) {
            err = "lane engine: " + msg;
            return CRDT_HIP_EDEVICE;
        }
        lane_eng_.push_back(std::move(e));
    }
    m.eng.assign(m.K, this);
    for (uint32_t i = 1; i < m.K; ++i) {
        m.eng[i] = lane_eng_[i - 1].get();
        m.eng[i]->log2m = log2m;
        m.eng[i]->log2m_set = log2m_set;
        m.eng[i]->level1_global = level1_global;
        m.eng[i]->fuse_text = fuse_text;
        m.eng[i]->xcd_order = xcd_order;
        m.eng[i]->stile_text = stile_text;
        m.eng[i]->text_scatter = text_scatter;
        m.eng[i]->glds_late = glds_late;
        m.eng[i]->doctree_k32 = doctree_k32;
        m.eng[i]->runs_slots = runs_slots;
        m.eng[i]->l1_split = l1_split;
        m.eng[i]->probe_doc_ = probe_doc_;
    }
    // every allocation before the first launch (a pool free waits for the device)
    const uint32_t per_lane = (nw + m.K - 1) / m.K;
    m.plans.assign(nw, L1Plan{});
    for (uint32_t wi = 0; wi < nw; ++wi) {
        Engine& E = *m.eng[wi % m.K];
        Wave& w = L.waves[wi];
        // test hook: a plan too small for the wave (the device must flag it, the host redo it)
        const uint32_t cr = plan_shrink ? w.hint_runs / 2 : w.hint_runs;
        const uint32_t cm = plan_shrink ? w.hint_rmax / 2 : w.hint_rmax;
        m.plans[wi] = E.plan_level1(w, cr, cm, false, false);
        int rc = E.ensure_scratch(w);
        if (rc) return rc;
        rc = E.ensure_runs(cr, 0);
        if (rc) return rc;
        const uint64_t hrows = w.nslots * (L.fugue ? 2ull : 1ull);  // (see run_wave)
        if (hrows > E.cap_heads_) {
            dfree(E.r_head_); dfree(E.r_pstart_);
            HIPCHK(dalloc(&E.r_head_, hrows + 64ull), "hipMalloc r_head");
            HIPCHK(dalloc(&E.r_pstart_, hrows + 64ull), "hipMalloc r_pstart");
            E.cap_heads_ = hrows;
            E.gen_++;
        }
    }
    for (uint32_t i = 0; i < m.K; ++i) {
        int rc = m.eng[i]->ensure_host_out(L);
        if (rc) return rc;
        rc = m.eng[i]->ensure_events(m.eng[i]->wev_, per_lane * (size_t)kClockEvents);
        if (rc) return rc;
        m.eng[i]->runs_ = 0;
    }
    m.clocks.assign(nw, StageClock{});
    return CRDT_HIP_OK;
}

int Engine::merge_async_enqueue(DeviceLogs& L, AsyncMerge& m) {
    const uint32_t nw = (uint32_t)L.waves.size();
    const uint32_t K = m.K;
    if (m.timed || K > 1) HIPCHK(hipEventRecord(ev_[2 * S_N + 1], stream), "event record");
    // the other lanes start after the merge's start event
    for (uint32_t i = 1; i < K; ++i)
        HIPCHK(hipStreamWaitEvent(m.eng[i]->stream, ev_[2 * S_N + 1], 0), "stream wait");
    hipEvent_t prev_l0 = nullptr;
    const bool split = l1_split;
    for (uint32_t i = 0; i < K; ++i) m.eng[i]->l1_pending_ = false;
    for (uint32_t wi = 0; wi < nw; ++wi) {
        Engine& E = *m.eng[wi % K];
        const Wave& w = L.waves[wi];
        StageClock& ck = m.clocks[wi];
        ck.ev = m.timed || K > 1 ? E.wev_.data() + (size_t)(wi / K) * kClockEvents : nullptr;
        if (l0_gated && prev_l0 && K > 1)
            HIPCHK(hipStreamWaitEvent(E.stream, prev_l0, 0), "stream wait");
        // level 0 overwrites the lane's scratch: after the lane's previous level 1
        if (E.l1_pending_) HIPCHK(hipStreamWaitEvent(E.stream, E.ev_l1_, 0), "stream wait");
        E.cur_ = E.stream;
        int rc = E.launch_level0(L, w, false, !m.plans[wi].stile_text, m.plans[wi].R,
                                 m.plans[wi].rmax, ck);
        if (rc) return rc;
        prev_l0 = ck.ev ? ck.ev[ck.n - 1] : nullptr;  // the end of level 0
        if (split) {
            HIPCHK(hipEventRecord(E.ev_l0_, E.stream), "event record");
            HIPCHK(hipStreamWaitEvent(E.stream_l1, E.ev_l0_, 0), "stream wait");
            E.cur_ = E.stream_l1;
        }
        rc = E.launch_lds_level1(L, w, false, m.plans[wi], m.plans[wi].stile_text, ck);
        if (!rc) rc = E.launch_tail(L, w, false, m.plans[wi].fuse, ck, E.host_block(L, wi));
        if (split) {
            E.cur_ = E.stream;
            if (!rc) {
                HIPCHK(hipEventRecord(E.ev_l1_, E.stream_l1), "event record");
                E.l1_pending_ = true;
            }
        }
        if (rc) return rc;
    }
    // join: the merge's end event on this stream after every lane's last launch
    for (uint32_t i = 0; i < K; ++i) {
        Engine& E = *m.eng[i];
        if (E.l1_pending_) {
            HIPCHK(hipStreamWaitEvent(E.stream, E.ev_l1_, 0), "stream wait");
            E.l1_pending_ = false;
        }
        if (i == 0) continue;
        hipEvent_t done = E.ev_[2 * S_N + 3];
        HIPCHK(hipEventRecord(done, E.stream), "event record");
        HIPCHK(hipStreamWaitEvent(stream, done, 0), "stream wait");
    }
    if (m.timed) HIPCHK(hipEventRecord(ev_[2 * S_N + 2], stream), "event record");
    return CRDT_HIP_OK;
}

int Engine::merge_async_finish(DeviceLogs& L, AsyncMerge& m, uint64_t* digests, uint64_t* lens,
                               uint64_t* cps, crdt_hip_stats* st) {
    const uint32_t nw = (uint32_t)L.waves.size();
    const uint32_t ndocs = (uint32_t)L.docs.size();
    std::vector<float> stage_ms(S_N, 0.f);
    std::vector<uint32_t> stage_launches(S_N, 0);
    uint64_t text_bytes = 0, runs = 0;
    std::vector<uint32_t> redo;
    uint32_t bad = 0;
    for (uint32_t wi = 0; wi < nw; ++wi) {
        Engine& E = *m.eng[wi % m.K];
        const uint32_t* hctl = E.host_block(L, wi);
        const Wave& w = L.waves[wi];
        uint32_t errs = hctl[C_ERR];
        if (hctl[C_REPLAN] || (errs & 32u)) {
            redo.push_back(wi);
            continue;
        }
        if (!errs && hctl[C_VISITED] != hctl[C_RTOTAL]) errs |= 16u;
        if (errs) {
            bad |= errs;
            continue;
        }
        StageClock ck = m.clocks[wi];
        if (!m.timed) ck.n = 0;
        int rc = E.finish_wave(w, false, m.plans[wi], 0, ck, hctl, stage_ms, stage_launches);
        if (rc) return rc;
        runs += hctl[C_RTOTAL];
        E.collect(L, wi, digests, lens, cps, text_bytes);
    }
    if (bad) {
        err = "malformed op log detected on device (flags " + std::to_string(bad) + ")";
        return CRDT_HIP_EBADLOG;
    }
    for (uint32_t wi : redo) {  // the logs changed under the plan: learn it again
        L.waves[wi].hint_lds = false;
        forget_shape(L.waves[wi]);
        runs_ = 0;
        int rc = ensure_scratch(L.waves[wi]);
        if (rc) return rc;
        rc = run_wave(L, wi, TEXT, stage_ms, stage_launches);
        if (rc) return rc;
        runs += runs_;
        collect(L, wi, digests, lens, cps, text_bytes);
    }
    runs_ = runs;
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->items = L.items;
        st->docs = ndocs;
        st->text_bytes = text_bytes;
        st->runs = runs;
        st->waves = nw;
        st->nstages = S_N;
        for (int i = 0; i < S_N; ++i) {
            st->stage_ns[i] = (uint64_t)((double)stage_ms[i] * 1e6);
            st->stage_launches[i] = stage_launches[i];
        }
        if (m.timed) {
            float tot = 0;
            HIPCHK(hipEventElapsedTime(&tot, ev_[2 * S_N + 1], ev_[2 * S_N + 2]), "event time");
            st->total_ns = (uint64_t)((double)tot * 1e6);
        }
    }
    return CRDT_HIP_OK;
}

int Engine::merge_async(DeviceLogs& L, uint64_t* digests, uint64_t* lens, uint64_t* cps,
                        crdt_hip_stats* st) {
    AsyncMerge m;
    int rc = merge_async_prepare(L, m, true);
    if (rc) return rc;
    rc = merge_async_enqueue(L, m);
    if (rc) return rc;
    HIPCHK(hipEventSynchronize(ev_[2 * S_N + 2]), "event sync");
    return merge_async_finish(L, m, digests, lens, cps, st);
}

// Multi-wave merge over lanes, synchronous per wave: wave i runs on lane i % K, every lane in its
// own host thread on its own stream and scratch (run_wave waits for each wave's level 0).  Stage
// times are summed over the lanes (kernel time, which can exceed the wall time); total_ns is the
// host wall time.
int Engine::merge_lanes(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens,
                        uint64_t* cps, crdt_hip_stats* st) {
    const uint32_t nw = (uint32_t)L.waves.size();
    const uint32_t K = std::min<uint32_t>(lanes, nw);
    // the lanes' streams do not wait for this one: let its queued table uploads finish
    HIPCHK(hipStreamSynchronize(stream), "table sync");
    while (lane_eng_.size() + 1 < K) {
        auto e = std::make_unique<Engine>();
        const std::string m = e->init(device);
        if (!m.empty()) {
            err = "lane engine: " + m;
            return CRDT_HIP_EDEVICE;
        }
        lane_eng_.push_back(std::move(e));
    }
    std::vector<Engine*> eng(K, this);
    std::mutex gate;
    for (uint32_t i = 1; i < K; ++i) {
        eng[i] = lane_eng_[i - 1].get();
        eng[i]->log2m = log2m;
        eng[i]->log2m_set = log2m_set;
        eng[i]->level1_global = level1_global;
        eng[i]->fuse_text = fuse_text;
        eng[i]->xcd_order = xcd_order;
        eng[i]->stile_text = stile_text;
        eng[i]->text_scatter = text_scatter;
        eng[i]->glds_late = glds_late;
        eng[i]->doctree_k32 = doctree_k32;
        eng[i]->runs_slots = runs_slots;
        eng[i]->probe_doc_ = probe_doc_;
    }
    std::vector<int> rc(K, CRDT_HIP_OK);
    std::vector<std::vector<float>> ms(K, std::vector<float>(S_N, 0.f));
    std::vector<std::vector<uint32_t>> nl(K, std::vector<uint32_t>(S_N, 0));
    for (uint32_t i = 0; i < K; ++i)
        if ((rc[0] = eng[i]->ensure_host_out(L))) return rc[0];
    auto lane = [&](uint32_t i) {
        Engine& E = *eng[i];
        const hipError_t e = hipSetDevice(device);  // the current device is per host thread
        if (e != hipSuccess) {
            rc[i] = E.fail("hipSetDevice", e);
            return;
        }
        E.runs_ = 0;
        E.l0_gate_ = l0_gated ? &gate : nullptr;
        for (uint32_t wi = i; wi < nw && rc[i] == CRDT_HIP_OK; wi += K) {
            rc[i] = E.ensure_scratch(L.waves[wi]);
            if (rc[i] == CRDT_HIP_OK) rc[i] = E.run_wave(L, wi, mode, ms[i], nl[i]);
        }
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    th.reserve(K - 1);
    for (uint32_t i = 1; i < K; ++i) th.emplace_back(lane, i);
    lane(0);
    for (std::thread& t : th) t.join();
    for (uint32_t i = 0; i < K; ++i) eng[i]->l0_gate_ = nullptr;
    const double wall_ns =
        std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t i = 0; i < K; ++i)
        if (rc[i] != CRDT_HIP_OK) {
            if (i) err = eng[i]->err;
            return rc[i];
        }
    const uint32_t ndocs = (uint32_t)L.docs.size();
    uint64_t text_bytes = 0, runs = 0;
    for (uint32_t wi = 0; wi < nw; ++wi) eng[wi % K]->collect(L, wi, digests, lens, cps, text_bytes);
    for (uint32_t i = 0; i < K; ++i) runs += eng[i]->runs_;
    runs_ = runs;
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->items = L.items;
        st->docs = ndocs;
        st->text_bytes = text_bytes;
        st->runs = runs;
        st->waves = nw;
        st->nstages = S_N;
        for (int s = 0; s < S_N; ++s) {
            double t = 0;
            uint32_t n = 0;
            for (uint32_t i = 0; i < K; ++i) {
                t += ms[i][s];
                n += nl[i][s];
            }
            st->stage_ns[s] = (uint64_t)(t * 1e6);
            st->stage_launches[s] = n;
        }
        st->total_ns = (uint64_t)wall_ns;
    }
    return CRDT_HIP_OK;
}

int Engine::synth_tree(DeviceLogs& R, uint32_t n, uint32_t p_chain_pct, uint32_t del_pct,
                       uint64_t seed) {
    std::vector<DocInfo> docs(1);
    docs[0].n = n;
    docs[0].text_cap = n;  // one byte per visible item at most ('a'..'z')
    int rc = plan(R, docs);
    R.fugue = false;
    if (rc) return rc;
    k_synth_tree<<<grid_for(R.total_slots), kBlock, 0, stream>>>(
        R.parent, R.key, R.cp, n, R.total_slots, p_chain_pct, del_pct, seed);
    HIPCHK(hipGetLastError(), "synth launch");
    HIPCHK(hipStreamSynchronize(stream), "synth");
    const int rc2 = build_nsq(R);
    return rc2;
}

int Engine::replicate(DeviceLogs& B, DeviceLogs& R, uint32_t replicas, uint32_t relabel,
                      uint64_t seed) {
    const uint32_t nb = (uint32_t)B.docs.size();
    if (nb == 0) { err = "no base logs"; return CRDT_HIP_EINVAL; }
    std::vector<DocInfo> docs;
    const uint64_t total = (uint64_t)nb * replicas;
    if (total > 0xFFFFFFFFull) { err = "too many documents"; return CRDT_HIP_ERANGE; }
    docs.reserve(total);
    uint32_t nmax = 0;
    // Replica r of base r % nb is the caller's document r.  Grouped (group_docs): the documents
    // lie in slots base by base, each base's replicas in waves of their own, so that a base whose
    // run trees do not fit the per-document LDS level 1 (Fugue seph-blog1) sends only its own
    // waves to the global level 1; results still come back in the caller's order (api_doc).
    const bool grp = group_docs && nb > 1 && replicas > 1;
    std::vector<uint32_t> order;  // slot-order document k -> the caller's document
    std::vector<uint8_t> brk;
    if (grp) {
        order.reserve(total);
        brk.assign(total, 0);
        for (uint32_t b = 0; b < nb; ++b) {
            brk[order.size()] = 1;
            for (uint32_t q = 0; q < replicas; ++q) order.push_back(q * nb + b);
        }
    }
    for (uint64_t k = 0; k < total; ++k) docs.push_back(B.docs[(grp ? order[k] : k) % nb]);
    for (uint32_t b = 0; b < nb; ++b) nmax = std::max(nmax, B.docs[b].n);
    int rc = plan(R, docs, grp ? &brk : nullptr);
    if (rc) return rc;
    R.fugue = B.fugue;
    std::vector<uint64_t> rslot(R.doc_slot);  // (by the caller's document)
    if (grp) {
        R.api_doc = order;
        for (uint64_t k = 0; k < total; ++k) rslot[order[k]] = R.doc_slot[k];
    }
    std::vector<uint32_t> bn(nb);
    for (uint32_t b = 0; b < nb; ++b) bn[b] = B.docs[b].n;
    uint64_t *dbslot = nullptr, *drslot = nullptr;
    uint32_t* dbn = nullptr;
    HIPCHK(dalloc(&dbslot, nb), "hipMalloc base slots");
    HIPCHK(dalloc(&dbn, nb), "hipMalloc base sizes");
    HIPCHK(dalloc(&drslot, total), "hipMalloc replica slots");
    hipError_t e = hipMemcpyAsync(dbslot, B.doc_slot.data(), nb * 8ull, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dbn, bn.data(), nb * 4ull, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(drslot, rslot.data(), total * 8ull, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess && nmax) {
        // one launch for the whole batch (a launch per replica made setup, and a profiler
        // serialising every dispatch, slow at 16,384 replicas)
        const dim3 grid(std::min<uint32_t>(grid_for(nmax), 1024u),
                        (uint32_t)std::min<uint64_t>(total, 65535u));
        k_replicate<<<grid, kBlock, 0, stream>>>(B.parent, B.key, B.cp, dbslot, dbn,
                                                 nb, R.parent, R.key, R.cp, drslot,
                                                 total, relabel, seed);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    dfree(dbslot);
    dfree(dbn);
    dfree(drslot);
    if (e != hipSuccess) return fail("replicate", e);
    const int rc2 = build_nsq(R);
    return rc2;
}

// The compact nsq parent list of resident logs (input encoding, once per batch): count the nsq
// items per 64-slot chunk, scan, scatter their parents in slot order.  k_classify then streams
// each tile's range of it (4 bytes per nsq item) instead of gathering the parent column (a 64-byte
// sector per nsq item), and k_runs reads the parents of its nsq heads there.
int Engine::build_nsq(DeviceLogs& L) {
    HIPCHK(hipStreamSynchronize(stream), "nsq list");
    L.nsq_ok = false;
    L.nsq_items = 0;
    if (!L.total_slots || !nsq_list) {
        set_contraction(L);
        return CRDT_HIP_OK;
    }
    const uint64_t nch = L.total_slots / 64 + 64;  // (a last tile's range ends within)
    if (nch >= (1ull << 32)) return CRDT_HIP_OK;
    if (int rc = nsq_reserve_prefix(L)) return rc;
    nsq_count_scan(L);
    const uint32_t n = (uint32_t)nch;
    uint32_t total = 0;
    hipError_t e = hipMemcpyAsync(&total, L.nsq_pre + n, 4, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return fail("nsq scan", e);
    if ((uint64_t)total + 1 > L.nsq_cap) {
        dfree(L.nsq_par);
        dfree(L.nsq_key);
        L.nsq_cap = 0;
        HIPCHK(dalloc(&L.nsq_par, (uint64_t)total + 1), "hipMalloc nsq list");
        HIPCHK(dalloc(&L.nsq_key, (uint64_t)total + 1), "hipMalloc nsq keys");
        L.nsq_cap = (uint64_t)total + 1;
    }
    nsq_scatter(L);
    HIPCHK(hipGetLastError(), "nsq list launch");
    // every wave's count of items without the previous-slot flag (its run contraction)
    for (Wave& w : L.waves) {
        uint32_t b[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(&b[0], L.nsq_pre + (w.slot0 >> 6), 4, hipMemcpyDeviceToHost, stream), "nsq counts");
        HIPCHK(hipMemcpyAsync(&b[1], L.nsq_pre + ((w.slot0 + w.nslots) >> 6), 4, hipMemcpyDeviceToHost, stream),
               "nsq counts");
        HIPCHK(hipStreamSynchronize(stream), "nsq counts");
        w.nsq_items = b[1] - b[0];
    }
    HIPCHK(hipStreamSynchronize(stream), "nsq list");
    L.nsq_items = total;
    L.nsq_ok = true;
    set_contraction(L);
    return CRDT_HIP_OK;
}

// Room for the nsq prefix counts and their scan scratch of L's slot layout.
int Engine::nsq_reserve_prefix(DeviceLogs& L) {
    const uint64_t nch = L.total_slots / 64 + 64;
    if (nch + 1 > L.nsq_pre_cap) {
        dfree(L.nsq_pre);
        dfree(L.nsq_mask);
        L.nsq_pre_cap = 0;
        HIPCHK(dalloc(&L.nsq_mask, nch + 1), "hipMalloc nsq masks");
        HIPCHK(dalloc(&L.nsq_pre, nch + 1), "hipMalloc nsq prefix");
        L.nsq_pre_cap = nch + 1;
        gen_++;  // (captured replays point at the old arrays)
    }
    const uint64_t nb = (nch + kScanTile - 1) / kScanTile;
    if (nb > L.nsq_sums_cap) {
        dfree(L.nsq_sums);
        L.nsq_sums_cap = 0;
        HIPCHK(dalloc(&L.nsq_sums, nb), "hipMalloc nsq scan");
        L.nsq_sums_cap = nb;
        gen_++;
    }
    return CRDT_HIP_OK;
}

// Counts of the nsq items per 64-slot chunk, scanned in place into L.nsq_pre (launches only).
void Engine::nsq_count_scan(DeviceLogs& L) {
    const bool ord = false;  // (L0ARGS)
    const uint32_t n = (uint32_t)(L.total_slots / 64 + 64);
    (void)hipMemsetAsync(L.nsq_pre, 0, (n + 1ull) * 4, stream);
    for (const Wave& w : L.waves) {
        L0ARGS(a0);
        k_nsq_count<<<grid_for((w.nslots + 15) / 16), kBlock, 0, stream>>>(a0, L.nsq_pre + (w.slot0 >> 6),
                                                                   L.nsq_mask + (w.slot0 >> 6));
    }
    nsq_scan(L);
}
void Engine::nsq_scan(DeviceLogs& L) {
    const uint32_t n = (uint32_t)(L.total_slots / 64 + 64), nb = (n + kScanTile - 1) / kScanTile;
    k_scan_reduce<<<nb, kBlock, 0, stream>>>(L.nsq_pre, n, L.nsq_sums);
    k_scan_top<<<1, 1024, 0, stream>>>(L.nsq_sums, nb, L.nsq_pre, n);
    k_scan_apply<<<nb, kBlock, 0, stream>>>(L.nsq_pre, n, L.nsq_sums, L.nsq_pre);
}

// Raw SoA mode (DeviceLogs::raw).  k_raw_fill keeps the reference-shaped columns of resident logs
// once (lamport, agent, deleted, codepoint per slot, from the encoded key and codepoint word);
// k_raw_encode derives the encoded input from them and the parent column at every merge: 4
// slots per thread, the key (lamport << 16 | agent), the 3-byte codepoint word with the tombstone
// and the previous-slot flag (parent == index - 1), and the nsq count and mask of each 64-slot
// chunk (what k_nsq_count reads back from the codepoint words otherwise).  Item slots only: a
// document start and the padding keep their words.  RGA logs.
__global__ __launch_bounds__(kBlock) void k_raw_fill(L0Args a, uint32_t* __restrict__ lam,
                                                     uint16_t* __restrict__ agent,
                                                     uint8_t* __restrict__ del,
                                                     uint32_t* __restrict__ cpw) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.nslots) return;
    const uint64_t k = a.in_key[g];
    const uint32_t c = cp3_get(a.in_cp, g);
    lam[g] = (uint32_t)(k >> 16);
    agent[g] = (uint16_t)k;
    del[g] = (c & kDelBit) ? 1u : 0u;
    cpw[g] = c & 0x1FFFFFu;
}
__global__ __launch_bounds__(kBlock) void k_raw_encode(L0Args a, const uint32_t* __restrict__ lam,
                                                       const uint16_t* __restrict__ agent,
                                                       const uint8_t* __restrict__ del,
                                                       const uint32_t* __restrict__ cpw,
                                                       uint64_t* __restrict__ key,
                                                       uint8_t* __restrict__ cp3,
                                                       uint32_t* __restrict__ cnt,
                                                       uint64_t* __restrict__ mask) {
    // four slots per lane (every column read with one vector load, the keys written as two
    // 16-byte stores); a wave = four 64-slot chunks, 16 lanes each (their nsq masks joined by
    // shuffles); the block's 1024 codepoint words are assembled in LDS and stored as 192 16-byte
    // pieces.  Wave slot counts are multiples of 64 (documents start 64-aligned).
    __shared__ __attribute__((aligned(16))) uint32_t cb[3 * kBlock];
    const uint32_t g0 = (blockIdx.x * kBlock + threadIdx.x) * 4u;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t nsq = 0, c[4] = {0u, 0u, 0u, 0u};
    const bool live = g0 < a.nslots;
    uint4 lm = make_uint4(0, 0, 0, 0);
    uint2 ag2 = make_uint2(0, 0);
    if (live) lm = *reinterpret_cast<const uint4*>(lam + g0);
    if (live) ag2 = *reinterpret_cast<const uint2*>(agent + g0);
    if (live) {
        const uint2 doc = a.docs[a.chunk_doc[g0 >> a.log2m]];  // (the four slots share a chunk)
        const uint4 p4 = *reinterpret_cast<const uint4*>(a.in_parent + g0);
        const uint4 cw4 = *reinterpret_cast<const uint4*>(cpw + g0);
        const uint32_t dl4 = *reinterpret_cast<const uint32_t*>(del + g0);
        const uint32_t P[4] = {p4.x, p4.y, p4.z, p4.w}, CW[4] = {cw4.x, cw4.y, cw4.z, cw4.w};
        const uint32_t LM[4] = {lm.x, lm.y, lm.z, lm.w};
        const uint32_t AG[4] = {ag2.x & 0xFFFFu, ag2.x >> 16, ag2.y & 0xFFFFu, ag2.y >> 16};
        uint64_t K[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t l = g0 + (uint32_t)k - doc.x;  // (item index + 1; 0: the document start)
            K[k] = ((uint64_t)LM[k] << 16) | AG[k];
            if (l - 1u < doc.y) {
                const bool sq = P[k] == l - 1u;
                nsq |= (sq ? 0u : 1u) << k;
                c[k] = (CW[k] & 0x1FFFFFu) | ((dl4 >> (8 * k)) & 0xFFu ? kDelBit : 0u) | (sq ? kSeqBit : 0u);
            } else {
                c[k] = cp3_get(a.in_cp, g0 + (uint32_t)k);  // (a document start or padding keeps its word)
                K[k] = a.in_key[g0 + (uint32_t)k];
            }
        }
        uint4* kd = reinterpret_cast<uint4*>(key + g0);
        kd[0] = make_uint4((uint32_t)K[0], (uint32_t)(K[0] >> 32), (uint32_t)K[1], (uint32_t)(K[1] >> 32));
        kd[1] = make_uint4((uint32_t)K[2], (uint32_t)(K[2] >> 32), (uint32_t)K[3], (uint32_t)(K[3] >> 32));
    }
    // the four 3-byte words as three dwords at the lane's 12 bytes
    cb[3 * threadIdx.x] = c[0] | (c[1] << 24);
    cb[3 * threadIdx.x + 1] = (c[1] >> 8) | (c[2] << 16);
    cb[3 * threadIdx.x + 2] = (c[2] >> 16) | (c[3] << 8);
    // the chunk's mask: 16 lanes' nibbles
    uint64_t m = (uint64_t)nsq << (4u * (lane & 15u));
#pragma unroll
    for (int x = 1; x < 16; x <<= 1) m |= (uint64_t)__shfl_xor((long long)m, x);
    if ((lane & 15u) == 0u && live && cnt) {
        cnt[g0 >> 6] = (uint32_t)__popcll(m);
        mask[g0 >> 6] = m;
    }
    __syncthreads();
    const uint32_t b0 = blockIdx.x * kBlock * 4u;
    for (uint32_t i = threadIdx.x; i < 3u * kBlock * 4u / 16u; i += kBlock)
        if (b0 + 16u * i / 3u < a.nslots)
            reinterpret_cast<uint4*>(cp3 + 3ull * b0)[i] = reinterpret_cast<const uint4*>(cb)[i];
}

int Engine::raw_keep(DeviceLogs& L) {
    if (L.fugue) {
        err = "raw SoA mode needs RGA logs";
        return CRDT_HIP_EINVAL;
    }
    if (L.raw) return CRDT_HIP_OK;
    const uint64_t n = L.total_slots + 64;
    HIPCHK(dalloc(&L.raw_lam, n), "hipMalloc raw lamport");
    HIPCHK(dalloc(&L.raw_agent, n), "hipMalloc raw agent");
    HIPCHK(dalloc(&L.raw_del, n), "hipMalloc raw deleted");
    HIPCHK(dalloc(&L.raw_cp, n), "hipMalloc raw codepoint");
    const bool ord = false;  // (L0ARGS)
    for (const Wave& w : L.waves) {
        L0ARGS(a0);
        k_raw_fill<<<grid_for(w.nslots), kBlock, 0, stream>>>(a0, L.raw_lam + w.slot0,
                                                               L.raw_agent + w.slot0,
                                                               L.raw_del + w.slot0,
                                                               L.raw_cp + w.slot0);
    }
    HIPCHK(hipGetLastError(), "raw fill launch");
    HIPCHK(hipStreamSynchronize(stream), "raw fill");
    L.raw = true;
    gen_++;
    return CRDT_HIP_OK;
}

// The merge's input encoding from the raw columns (launches only, on the engine's stream): keys,
// codepoint words and nsq counts per wave, then the nsq scan and list (when the batch keeps one).
int Engine::raw_encode(DeviceLogs& L) {
    const bool ord = false;  // (L0ARGS)
    const bool nsq = L.nsq_ok && L.nsq_pre;
    if (nsq) (void)hipMemsetAsync(L.nsq_pre, 0, (L.total_slots / 64 + 65) * 4ull, stream);
    for (const Wave& w : L.waves) {
        L0ARGS(a0);
        k_raw_encode<<<grid_for((w.nslots + 3) / 4), kBlock, 0, stream>>>(
            a0, L.raw_lam + w.slot0, L.raw_agent + w.slot0, L.raw_del + w.slot0,
            L.raw_cp + w.slot0, L.key + w.slot0, L.cp + 3ull * w.slot0,
            nsq ? L.nsq_pre + (w.slot0 >> 6) : nullptr, nsq ? L.nsq_mask + (w.slot0 >> 6) : nullptr);
    }
    if (nsq) {
        nsq_scan(L);
        nsq_scatter(L);
    }
    HIPCHK(hipGetLastError(), "raw encode launch");
    return CRDT_HIP_OK;
}

// The list itself, every wave's tiles (launches only).
void Engine::nsq_scatter(DeviceLogs& L) {
    const bool ord = false;  // (L0ARGS)
    for (const Wave& w : L.waves) {
        L0ARGS(a0);
        k_nsq_scatter<<<(uint32_t)((w.nslots + kScanTile - 1) / kScanTile), kBlock, 0, stream>>>(
            a0, L.nsq_pre + (w.slot0 >> 6), L.nsq_mask + (w.slot0 >> 6), L.nsq_par, L.nsq_key);
    }
}

int Engine::nsq_reserve(DeviceLogs& L) {
    L.nsq_ok = false;
    if (!nsq_list || (nsq_list == 1 && L.total_slots < kNsqReplicaSlots) || !L.total_slots ||
        L.total_slots / 64 + 64 >= (1ull << 32))
        return CRDT_HIP_OK;
    if (int rc = nsq_reserve_prefix(L)) return rc;
    if (L.total_slots + 1 > L.nsq_cap) {  // (every slot an nsq item, at most)
        dfree(L.nsq_par);
        dfree(L.nsq_key);
        L.nsq_cap = 0;
        HIPCHK(dalloc(&L.nsq_par, L.total_slots + 1), "hipMalloc nsq list");
        HIPCHK(dalloc(&L.nsq_key, L.total_slots + 1), "hipMalloc nsq keys");
        L.nsq_cap = L.total_slots + 1;
        gen_++;
    }
    return CRDT_HIP_OK;
}

int Engine::nsq_launch(DeviceLogs& L) {
    if (!nsq_list || (nsq_list == 1 && L.total_slots < kNsqReplicaSlots) || !L.nsq_pre ||
        L.nsq_cap < L.total_slots + 1 ||
        L.nsq_pre_cap < L.total_slots / 64 + 65)
        return CRDT_HIP_OK;  // (nsq_reserve found no room: the merge gathers from the columns)
    nsq_count_scan(L);
    nsq_scatter(L);
    HIPCHK(hipGetLastError(), "nsq list launch");
    L.nsq_ok = true;
    return CRDT_HIP_OK;
}

// Run contraction per wave (Wave::nocon) from its count of items without the previous-slot flag;
// the plans learnt for the shape (which includes the mode) then apply again.
void Engine::set_contraction(DeviceLogs& L) const {
    for (Wave& w : L.waves) {
        uint64_t items = 0;
        for (uint32_t k = 0; k < w.ndocs; ++k) items += L.docs[w.first_doc + k].n;
        // (Fugue logs always contract: level 0 has no uncontracted form of the two-row heads, and
        // their items never carry the previous-slot flag)
        w.nocon = !L.fugue && (contraction == 2 ||
                               (contraction == 0 && items &&
                                (double)w.nsq_items >= kNoconShare * (double)items));
    }
    apply_shape_hints(L);
}

// Every wave of L takes the launch plan learnt on logs of its shape, if any.
void Engine::apply_shape_hints(DeviceLogs& L) const {
    for (Wave& w : L.waves) {
        const WaveShape sh = shape_of(w);
        w.hint_lds = false;
        for (const ShapeHint& h : shape_hints_)
            if (h.shape == sh) {
                w.hint_runs = h.runs;
                w.hint_rmax = h.rmax;
                w.hint_lds = true;
                break;
            }
    }
}

}  // namespace crdt
