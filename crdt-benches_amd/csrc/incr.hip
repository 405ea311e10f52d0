// incr.hip — incremental merge of a device replica.
//
// The reference's len() (Dt::len -> checkout_tip, /root/reference/src/rope.rs:135) materialises
// the whole document every time it is called; the upstream loop (/root/reference/src/main.rs:
// 28-36) and the downstream loop (:63-69) call it once per iteration.  A caller that asks for the
// length every K patches pays a full merge each time.  Here a replica keeps the document ORDER of
// every item it holds (tombstones included: a dense permutation `seq`, rank 0 = the document
// start, and its inverse `rank`) together with the merged text, and a later merge re-ranks only
// what the appended items touch:
//
//   new items with an old parent p (the roots of the new forest) go right after p, ahead of p's
//   old children, when their sibling key (lamport, agent) is above every old item's key — the
//   case of every local edit (the resolver's lamport = max + 1) and of any update that does not
//   race an older one.  One launch (k_inc), one workgroup per tile of 4096 old ranks:
//   - every workgroup orders the new forest (at most kIncMax items) in LDS (inc_forest): children
//     grouped by parent and ranked among their siblings (roots by (anchor rank asc, key desc),
//     other groups by key desc), an Euler tour of the forest ranked by barrier-free pointer
//     jumping, every item's place and the old rank its subtree follows;
//   - it splices its tile (an old rank k moves to k + #new items anchored before it, the new items
//     anchored inside the tile go in between) and rewrites `rank`;
//   - it takes its text offset from the tiles before it by decoupled look-back and writes its
//     text.  Deletes change no order: the tombstone bits the decode set make those items weigh
//     nothing.
//
// A root whose key is not above every old key (a concurrent update) takes its place from a search
// of its parent's old subtree.  Fugue replicas (in-order: left children, the item, right children)
// take the same path: a new right child of an old item goes right after it, a new left child right
// before it while it has no left child (the resolver's local edits: a left child is only ever given
// to the leftmost node of a right subtree), the forest's tour carries an item's place on the up arc
// of its last left child, and runs are not contracted.  Anything else — more than kIncMax new
// items, a Fugue root that needs a search — falls back to a full merge (engine ORDER mode), which
// also rebuilds the state.  Every fast-path merge is checked against the decode's counters (bytes
// and codepoints of the visible text) by the host.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "engine.hpp"
#include "replica.hpp"
#include "util.hpp"
#include "wave.hpp"

namespace crdt {
namespace {

#ifndef CRDT_INC_THREADS
#define CRDT_INC_THREADS 1024
#endif
constexpr uint32_t kIncThreads = CRDT_INC_THREADS;
constexpr uint32_t kSpliceRanks = 4;                                // old ranks per thread
constexpr uint32_t kSpliceTile = kIncThreads * kSpliceRanks;        // old ranks per tile
constexpr uint32_t kIncGroupMax = 1024;  // largest sibling group ranked in inc_forest
constexpr uint32_t kIncThinGroup = 32;   // more roots than this: ranked one wave per root
// Roots that do not sort above every old item (a concurrent insert) take their place from a
// search of their parent's old subtree (inc_search, by k_inc's first kIncSearchers workgroups):
// at most kIncHard of them per call, each search over at most kIncScan ranks (else the call
// merges in full)
constexpr uint32_t kIncHard = 256;
constexpr uint32_t kIncSearchers = 16;
constexpr uint32_t kIncScan = 1u << 16;
#ifndef CRDT_INC_RUNS
#define CRDT_INC_RUNS 1
#endif
constexpr bool kIncRuns = CRDT_INC_RUNS;  // contract runs of new items before the tour
constexpr uint32_t kCpMaskI = 0x001FFFFFu;
constexpr uint32_t kDelBitI = 0x00800000u;
constexpr uint32_t kLeftBitI = 0x00200000u;  // (Fugue) a left child
constexpr uint64_t kLeftKeyI = 1ull << 48;   // (Fugue) the key bit of a left child

// device counters (u64)
enum ICtl { I_MAXKEY = 0, I_MAXKEY_B, I_N };  // the largest key, two slots (calls alternate)
// flag bits (the result block): the fast path does not apply (the host merges in full)
constexpr uint64_t F_KEY = 1, F_ORDER = 2, F_GROUP = 4, F_TEXT = 8;  // (F_KEY: too many searches)

struct IncArgs {
    uint32_t n0, m;             // items the order covers, items appended since
    const uint32_t* parent;     // replica slot arrays (slot = id)
    const uint64_t* key;
    const uint8_t* cp;
    const uint32_t* rank;       // slot -> rank (the order of n0 items)
    uint32_t* rank2;            // slot -> rank in the new order (every slot 0..n0 + m written)
    const uint32_t* seq;        // rank -> slot (n0 + 1 entries)
    uint32_t* seq2;             // the new order (n0 + 1 + m entries)
    uint32_t* lb_flag;          // per tile: look-back status (call epoch << 2 | state)
    uint64_t* lb_agg;           //   its aggregate and its inclusive prefix {bytes | cps << 32}
    uint64_t* lb_inc;
    uint32_t nblk;
    uint8_t* text;
    uint64_t text_cap;
    uint64_t* ctl;
    uint64_t* hres;             // host-mapped result {flag, bytes, codepoints, call number}
    uint64_t* tsp;              // (CRDT_INC_PROFILE) phase timestamps of the forest, or null
    uint64_t call;              // this call's number (a stale result block is detected)
    const uint32_t* hasl;       // (Fugue) 1 bit per old slot: it has a left child
    uint64_t* hanc;             // per new item: a searched root's anchor rank | call << 32
    uint32_t nsearch;           // leading workgroups of k_inc that search (0: none, Fugue)
};

typedef __attribute__((address_space(3))) uint32_t lds_u32i_t;
__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) { return *(volatile lds_u32i_t*)p; }
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) { *(volatile lds_u32i_t*)p = v; }

__device__ __forceinline__ uint32_t cp_word(const uint8_t* cp, uint32_t s) {
    return (uint32_t)cp[3ull * s] | ((uint32_t)cp[3ull * s + 1] << 8) |
           ((uint32_t)cp[3ull * s + 2] << 16);
}
// The codepoint word of slot s (the document start: a tombstone, it has no text)
__device__ __forceinline__ uint32_t slot_word(const uint8_t* cp, uint32_t s) {
    return s ? cp_word(cp, s) : kDelBitI;
}
// UTF-8 bytes of a codepoint word in the text (0: a tombstone)
__device__ __forceinline__ uint32_t word_bytes(uint32_t c) {
    return (c & kDelBitI) ? 0u : utf8_len(c & kCpMaskI);
}


// ---- inc_forest: the order of the appended items (in each workgroup) ---------------------------
// Items i = 0..m-1 are slots n0 + 1 + i.  Local node m is a virtual root V whose children are
// the items with an old parent.  LDS (dynamic): see the carve-up below.
__host__ __device__ constexpr uint32_t inc_forest_lds(uint32_t mmax) {
    return 2u * (mmax + 2u)          // lp: local parent (u16)
           + 4u * (mmax + 2u)        // start: child count -> segment start (u32)
           + 2u * (mmax + 2u)        // ch: children by segment, then sorted (u16)
           + 8u * mmax               // keys (u64), later the output pairs
           + 4u * mmax               // A: anchor rank of a root (u32)
           + 4u * (2u * mmax + 4u)   // tour successor (u16) and suffix sum (u16), packed u32
           + 2u * mmax               // vrk: ranks among many roots, then run heads (u16)
           + 2u * mmax               // rend: the last item of each run (u16)
           + 2u * (mmax + 2u)        // cs: children by segment, sorted (u16)
           + 4u * mmax               // PR: a root's parent's old rank (u32)
           + 64u;
}

// Order of the new items in one sibling group: the roots (children of the virtual root) by anchor
// rank, then among roots at the same anchor the one whose parent ranks later first (the anchor
// item's own new children come before those of its ancestors, whose old subtrees end there), then
// by key descending, ties by the greater index; other groups have A = PR = 0: key order.
__device__ __forceinline__ bool root_before(uint32_t aj, uint32_t pj, uint64_t kj, uint32_t j,
                                            uint32_t ai, uint32_t pi, uint64_t ki, uint32_t i) {
    if (aj != ai) return aj < ai;
    if (pj != pi) return pj > pi;
    return kj > ki || (kj == ki && j > i);
}

#define INC_TS(i) \
    if (a.tsp && threadIdx.x == 0) a.tsp[i] = wall_clock64()
// (sl / cwq: the splice's old order of this tile and its codepoint words, gathered here beside
// the forest's own dependent loads so that the splice does not wait for them)
// Q: items per thread (m <= Q * kIncThreads); the caller picks the smallest instance that holds
// the batch, so that no per-item loop runs over empty slots
template <uint32_t Q, bool FG>
__device__ __forceinline__ void inc_forest(const IncArgs& a, uint8_t* lds, uint32_t* red,
                                           uint32_t& flag, uint32_t& nhard,
                                           const uint32_t (&sl)[kSpliceRanks],
                                           uint32_t (&cwq)[kSpliceRanks]) {
    static_assert(Q * kIncThreads <= kIncMax, "items per thread");
    const uint32_t t = threadIdx.x, m = a.m, n0 = a.n0;
    uint64_t* keys = reinterpret_cast<uint64_t*>(lds);
    uint32_t* A = reinterpret_cast<uint32_t*>(keys + kIncMax);
    uint32_t* start = A + kIncMax;                          // kIncMax + 2
    uint32_t* tour = start + (kIncMax + 2u);                // 2 kIncMax + 4: succ | sum << 16
    uint16_t* lp = reinterpret_cast<uint16_t*>(tour + (2u * kIncMax + 4u));  // kIncMax + 2
    uint16_t* ch = lp + (kIncMax + 2u);                     // kIncMax + 2
    uint16_t* vrk = ch + (kIncMax + 2u);                    // kIncMax: ranks among the roots
    uint16_t* rend = vrk + kIncMax;                         // kIncMax: the last item of a run
    uint16_t* cs = rend + kIncMax;                          // kIncMax + 2: ch sorted
    uint32_t* PR = reinterpret_cast<uint32_t*>(cs + (kIncMax + 2u));  // kIncMax
    if (t == 0) {
        flag = 0;
        nhard = 0;
    }
    INC_TS(0);
    const uint64_t maxkey0 = a.ctl[I_MAXKEY + ((a.call & 1u) ^ 1u)];
    // ---- load: parents, keys, anchors; child counts (each child keeps its place among its
    // parent's children).  The counts are cleared while the loads are in flight ----
    uint32_t plc[Q];
    uint64_t kmax = 0;
    uint32_t hq = 0;  // (RGA) this thread's roots whose place a search gives
    {
        uint32_t pp[Q];
        uint64_t kk[Q];
#pragma unroll
        for (int q = 0; q < (int)Q; ++q) {
            const uint32_t i = t + (uint32_t)q * kIncThreads;
            pp[q] = i < m ? a.parent[n0 + 1u + i] : 0u;
            kk[q] = i < m ? a.key[n0 + 1u + i] : 0ull;
        }
        uint32_t bad = 0;
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) cwq[q] = slot_word(a.cp, sl[q]);
        for (uint32_t x = t; x <= m + 1u; x += kIncThreads) start[x] = 0;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < (int)Q; ++q) {
            const uint32_t i = t + (uint32_t)q * kIncThreads;
            plc[q] = 0;
            if (i >= m) continue;
            keys[i] = kk[q];
            const uint64_t kv = kk[q] & ~kLeftKeyI;  // (the key without the Fugue side bit)
            kmax = max(kmax, kv);
            uint32_t li;
            if (FG && pp[q] <= n0) {
                // a Fugue root: a right child goes right after its old parent, a left child right
                // before it (the parent must have no old left child); right roots first at a
                // shared anchor (PR 1 before 0), each side by key; a root that an old sibling may
                // precede is not searched for (F_KEY: the full merge)
                li = m;
                const bool left = (kk[q] & kLeftKeyI) != 0ull;
                const uint32_t rp = a.rank[pp[q]];
                A[i] = left ? rp - 1u : rp;
                PR[i] = left ? 0u : 1u;
                if (kv <= maxkey0 || (left && (rp == 0u || ((a.hasl[pp[q] >> 5] >> (pp[q] & 31u)) & 1u))))
                    bad |= (uint32_t)F_KEY;
            } else if (pp[q] <= n0) {  // a root: after its old parent, ahead of the parent's old children
                li = m;
                A[i] = PR[i] = a.rank[pp[q]];
                if (kk[q] <= maxkey0) {
                    // some old sibling may sort above it: its place comes from the search
                    // workgroups (taken below, once every such root is counted)
                    hq |= 1u << q;
                    atomicAdd(&nhard, 1u);
                }
            } else {
                const uint32_t l = pp[q] - (n0 + 1u);
                if (l >= i) bad |= (uint32_t)F_ORDER;  // (parents precede their children)
                li = l < i ? l : m;
                A[i] = 0;
                PR[i] = 0;
            }
            lp[i] = (uint16_t)li;
            plc[q] = atomicAdd(&start[li], 1u);
        }
        if (bad) atomicOr(&flag, bad);
    }
    INC_TS(1);
    __syncthreads();
    if (!FG && nhard) {
        // the searched anchors (published by the leading workgroups, stamped with the call);
        // more roots than kIncHard: none was searched, the call merges in full
        if (nhard > kIncHard) {
            if (t == 0) atomicOr(&flag, (uint32_t)F_KEY);
        } else {
#pragma unroll
            for (int q = 0; q < (int)Q; ++q) {
                if (!((hq >> q) & 1u)) continue;
                const uint32_t i = t + (uint32_t)q * kIncThreads;
                // (bounded: the searchers lead the grid and are dispatched first, so they are
                // resident or done; should they not be, the wait gives up after ~50 ms and the
                // call merges in full instead of hanging on the dispatch order)
                uint64_t v;
                uint32_t spins = 0;
                while ((uint32_t)((v = __hip_atomic_load(&a.hanc[i], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)) >> 32) != (uint32_t)a.call) {
                    if (++spins > (1u << 20)) {
                        v = 0xFFFFFFFFull;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if ((uint32_t)v != 0xFFFFFFFFu)
                    A[i] = (uint32_t)v;
                else
                    atomicOr(&flag, (uint32_t)F_KEY);
            }
        }
    }
    INC_TS(2);
    // ---- segment starts: exclusive scan over nodes 0..m (m + 1 <= kIncMax + 1 counts) ----
    {
        constexpr uint32_t P = (Q * kIncThreads + 1u + kIncThreads - 1u) / kIncThreads + 1u;
        const uint32_t lo = min(m + 1u, t * P), hi = min(m + 1u, lo + P);
        uint32_t s = 0;
        for (uint32_t x = lo; x < hi; ++x) s += start[x];
        uint32_t tot;
        uint32_t ex = block_excl_scan<kIncThreads / 64>(s, red, tot);
        for (uint32_t x = lo; x < hi; ++x) {
            const uint32_t c = start[x];
            start[x] = ex;
            ex += c;
        }
        if (t == 0) start[m + 1u] = tot;  // (= m)
    }
    INC_TS(3);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t i = t + (uint32_t)q * kIncThreads;
        if (i < m) ch[start[lp[i]] + plc[q]] = (uint16_t)i;
    }
    INC_TS(4);
    __syncthreads();
    // ---- rank among siblings: roots by (anchor asc, key desc), other groups by key desc (the
    // anchors of non-roots are all 0); ties by the greater index, as the full merge does ----
    uint32_t rk[Q];
    // the roots (children of V) when there are many of them: one wave per root, its lanes over
    // the other roots (a thread walking all of them alone is an r-long chain of LDS reads)
    const uint32_t v0 = start[m], nv = start[m + 1u] - v0;
    const bool wide_v = nv > kIncThinGroup;
    if (wide_v) {
        const uint32_t lane = t & 63u;
        for (uint32_t idx = t >> 6; idx < nv; idx += kIncThreads / 64) {
            const uint32_t i = ch[v0 + idx];
            const uint32_t ai = A[i], pi = PR[i];
            const uint64_t ki = keys[i];
            uint32_t r = 0;
            for (uint32_t s = lane; s < nv; s += 64) {
                const uint32_t j = ch[v0 + s];
                r += root_before(A[j], PR[j], keys[j], j, ai, pi, ki, i) ? 1u : 0u;
            }
            r = wave_sum(r);
            if (lane == 0) vrk[i] = (uint16_t)r;
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t i = t + (uint32_t)q * kIncThreads;
        rk[q] = 0;
        if (i >= m) continue;
        if (wide_v && lp[i] == m) {
            rk[q] = vrk[i];
            continue;
        }
        const uint32_t g0 = start[lp[i]], g1 = start[lp[i] + 1u];
        if (g1 - g0 > kIncGroupMax) {
            atomicOr(&flag, (uint32_t)F_GROUP);
            continue;
        }
        const uint32_t ai = A[i], pi = PR[i];
        const uint64_t ki = keys[i];
        uint32_t r = 0;
        for (uint32_t s = g0; s < g1; ++s) {
            const uint32_t j = ch[s];
            r += root_before(A[j], PR[j], keys[j], j, ai, pi, ki, i) ? 1u : 0u;
        }
        rk[q] = r;
    }
    // (sorted into a second array: ch is still being read by other threads)
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t i = t + (uint32_t)q * kIncThreads;
        if (i < m) cs[start[lp[i]] + rk[q]] = (uint16_t)i;
    }
    INC_TS(5);
    INC_TS(6);
    __syncthreads();
    if (flag) return;  // (block-uniform after the barrier)
    // ---- runs: item i continues i - 1 when i - 1 is its parent and i its only child (typing),
    // so a run is a range of consecutive items whose places are consecutive; only run heads
    // enter the tour (run i's weight = its length).  hd[i] = the head of i's run (a max-scan in
    // item order, four consecutive items per thread), rend[h] = the last item of run h ----
    uint16_t* hd = vrk;  // (the root ranks are dead)
    {
        const uint32_t i0 = Q * t;
        uint32_t h[Q], mx = 0;
#pragma unroll
        for (int k = 0; k < (int)Q; ++k) {
            const uint32_t i = i0 + (uint32_t)k;
            const bool cont = kIncRuns && !FG && i < m && i > 0 && lp[i] == i - 1u &&
                              start[i] - start[i - 1u] == 1u;
            h[k] = (i < m && !cont) ? i : 0u;
            mx = max(mx, h[k]);
        }
        uint32_t inc = mx;
        const uint32_t lane = t & 63u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= (uint32_t)o) inc = max(inc, y);
        }
        if (lane == 63u) red[t >> 6] = inc;
        __syncthreads();
        uint32_t run = 0;
        for (uint32_t w = 0; w < (t >> 6); ++w) run = max(run, red[w]);
        const uint32_t prev = (uint32_t)__shfl_up((int)inc, 1);
        run = max(run, lane ? prev : 0u);
#pragma unroll
        for (int k = 0; k < (int)Q; ++k) {
            const uint32_t i = i0 + (uint32_t)k;
            run = max(run, h[k]);
            if (i >= m) continue;
            hd[i] = (uint16_t)run;
            const bool next_cont = kIncRuns && !FG && i + 1u < m && lp[i + 1u] == i &&
                                   start[i + 1u] - start[i] == 1u;
            if (!next_cont) rend[run] = (uint16_t)i;
        }
    }
    __syncthreads();
    // ---- Euler tour of the run forest: down(h) = 2h, up(h) = 2h + 1 (h a run head or V = m),
    // end E; succ in the low 16 bits, the arc's weight (a run's length on its down arc) high ----
    // (Fugue: an item's place is on its down arc when it has no left child, else on the up arc of
    // its last left child; fl[q] bit 0: x has a left child, bit 1: x is its parent's last one)
    const uint32_t E = 2u * m + 2u, V = m;
    uint32_t fl[Q];
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t x = t + (uint32_t)q * kIncThreads;
        fl[q] = 0;
        if (x >= m || hd[x] != x) continue;
        const uint32_t e = rend[x];
        const uint32_t c0 = start[e], c1 = start[e + 1u];
        const uint32_t sd = c1 > c0 ? 2u * cs[c0] : 2u * x + 1u;
        const uint32_t p = lp[x], pos = start[p] + rk[q];
        const uint32_t pr = p == V ? V : hd[p];  // (a parent is always the last item of its run)
        const bool more = pos + 1u < start[p + 1u];
        const uint32_t su = more ? 2u * cs[pos + 1u] : 2u * pr + 1u;
        if (FG) {
            const bool hasl = c1 > c0 && (keys[cs[c0]] & kLeftKeyI);
            const bool lastl = p != V && (keys[x] & kLeftKeyI) && !(more && (keys[cs[pos + 1u]] & kLeftKeyI));
            fl[q] = (hasl ? 1u : 0u) | (lastl ? 2u : 0u);
            tour[2u * x] = sd | ((hasl ? 0u : 1u) << 16);
            tour[2u * x + 1u] = su | ((lastl ? 1u : 0u) << 16);
        } else {
            tour[2u * x] = sd | ((e - x + 1u) << 16);
            tour[2u * x + 1u] = su;
        }
    }
    if (t == 0) {
        const uint32_t c0 = start[V], c1 = start[V + 1u];
        tour[2u * V] = c1 > c0 ? 2u * cs[c0] : 2u * V + 1u;
        tour[2u * V + 1u] = E;
        tour[E] = E;
    }
    INC_TS(7);
    __syncthreads();
    // ---- pointer jumping without barriers: a record (succ | weight of [arc, succ) << 16) is a
    // valid stretch of the tour at all times, so joining it with an old or a new record of its
    // successor is equally right; each thread jumps its own arcs (those of run heads and V) until
    // they reach the end (every pass extends a record by at least one arc: E passes bound it) ----
    {
        constexpr int NA = (int)((2u * Q * kIncThreads + 4u + kIncThreads - 1u) / kIncThreads);
        static_assert(NA <= 32, "arcs per thread");
        uint32_t live = 0;
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            const uint32_t arc = t + (uint32_t)q * kIncThreads, x = arc >> 1;
            live |= (arc < E && (x == V || hd[x] == x) ? 1u : 0u) << q;
        }
        for (uint32_t pass = 0; live && pass <= E; ++pass) {
#pragma unroll
            for (int q = 0; q < NA; ++q) {
                if (!((live >> q) & 1u)) continue;
                const uint32_t arc = t + (uint32_t)q * kIncThreads;
                const uint32_t x = lds_ld(tour + arc);
                const uint32_t s = x & 0xFFFFu;
                if (s == E) {
                    live &= ~(1u << q);
                    continue;
                }
                const uint32_t y = lds_ld(tour + s);
                const uint32_t nx = (y & 0xFFFFu) | (((x >> 16) + (y >> 16)) << 16);
                lds_st(tour + arc, nx);
                if ((y & 0xFFFFu) == E) live &= ~(1u << q);
            }
        }
    }
    INC_TS(8);
    __syncthreads();
    // ---- every item's place among the new items; its root's anchor by a max-scan.  The result
    // stays in LDS for the splice: os[place] = slot, oa[place] = the old rank it follows ----
    uint32_t* os = reinterpret_cast<uint32_t*>(keys);  // (the keys are dead since the ranking)
    uint32_t* oa = os + kIncMax;
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t x = t + (uint32_t)q * kIncThreads;
        if (x >= m) continue;
        if (FG) {
            // the place of x (no left child), of x's parent (x its last left child)
            if (!(fl[q] & 1u)) {
                const uint32_t px = m - (tour[2u * x] >> 16);
                os[px] = n0 + 1u + x;
                oa[px] = 0u;
            }
            if (fl[q] & 2u) {
                const uint32_t px = m - (tour[2u * x + 1u] >> 16);
                os[px] = n0 + 1u + lp[x];
                oa[px] = 0u;
            }
        } else {
            const uint32_t h = hd[x];
            const uint32_t px = m - (tour[2u * h] >> 16) + (x - h);
            os[px] = n0 + 1u + x;
            oa[px] = 0u;
        }
    }
    __syncthreads();
    // a root's anchor at the first place of its subtree (its own place in RGA order; in Fugue
    // order its leftmost descendant's); the max-scan carries it over the subtree
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t x = t + (uint32_t)q * kIncThreads;
        if (x < m && lp[x] == V) oa[m - (tour[2u * x] >> 16)] = A[x];
    }
    __syncthreads();
    {
        // inclusive max-scan over places (roots come in anchor order, each before its subtree)
        const uint32_t lo = min(m, t * Q), hi = min(m, lo + Q);
        uint32_t mx = 0;
        for (uint32_t i = lo; i < hi; ++i) mx = max(mx, oa[i]);
        uint32_t inc = mx;
        const uint32_t lane = t & 63u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= (uint32_t)o) inc = max(inc, y);
        }
        if (lane == 63u) red[t >> 6] = inc;
        __syncthreads();
        uint32_t run = 0;
        for (uint32_t w = 0; w < (t >> 6); ++w) run = max(run, red[w]);
        const uint32_t prev = (uint32_t)__shfl_up((int)inc, 1);
        run = max(run, lane ? prev : 0u);
        for (uint32_t i = lo; i < hi; ++i) {
            run = max(run, oa[i]);
            oa[i] = run;
        }
    }
    INC_TS(9);
    // the largest key now held, for the next call's check (tile 0; the slot this call writes is
    // not the one any workgroup of it reads)
    if (blockIdx.x == a.nsearch) {
        uint64_t km = max(kmax, maxkey0);
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(km >> 32), o) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)km, o);
            km = max(km, y);
        }
        if ((t & 63u) == 0)
            atomicMax(reinterpret_cast<unsigned long long*>(&a.ctl[I_MAXKEY + (a.call & 1u)]),
                      (unsigned long long)km);
    }
    __syncthreads();
    INC_TS(10);
}
#undef INC_TS

// Number of new items anchored before old rank k (la is non-decreasing).
__device__ __forceinline__ uint32_t anchored_before(const uint32_t* la, uint32_t m, uint32_t k) {
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (la[mid] < k) lo = mid + 1u;
        else hi = mid;
    }
    return lo;
}

// ---- splice: the new order of one tile; rank rewritten; the tile's text totals ----------------
// Tile b takes old ranks [k0, k1) and the new items anchored in [k0, k1) (os / la: the new items
// by place, in LDS): its outputs are the places [k0 + c(k0), k1 + c(k1)), c(k) = new items
// anchored before k.  Returns {bytes, codepoints} of its outputs; range = its output places.
__device__ __forceinline__ uint2 inc_splice_tile(const IncArgs& a, uint32_t b, uint32_t* rsum,
                                                 uint32_t* cb, const uint32_t* os,
                                                 const uint32_t* la, uint32_t* cwl,
                                                 const uint32_t (&sl)[kSpliceRanks],
                                                 const uint32_t (&cwq)[kSpliceRanks], uint2& range) {
    const uint32_t N0 = a.n0 + 1u, m = a.m;
    const uint32_t k0 = b * kSpliceTile, k1 = min(N0, k0 + kSpliceTile);
    // the tile's first output place (every thread finds it: the words go to LDS at place - o0)
    const uint32_t o0 = k0 + (m ? anchored_before(la, m, k0) : 0u);
    if (threadIdx.x < 2u) cb[threadIdx.x] = m ? anchored_before(la, m, threadIdx.x ? k1 : k0) : 0u;
    const uint32_t kb = k0 + threadIdx.x * kSpliceRanks;
    uint32_t bytes = 0, cps = 0;
    // c(k) for the thread's first rank by binary search; the next ranks search again only past
    // an anchor (a whole subtree of new items shares one anchor, so no linear walk over them)
    uint32_t c = (m && kb < k1) ? anchored_before(la, m, kb) : 0u;
#pragma unroll
    for (int q = 0; q < (int)kSpliceRanks; ++q) {
        const uint32_t k = kb + q;
        if (k >= k1) break;
        if (q && c < m && la[c] < k) c = anchored_before(la, m, k);
        const uint32_t np = k + c;
        a.seq2[np] = sl[q];
        cwl[np - o0] = cwq[q];
        a.rank2[sl[q]] = np;
        const uint32_t w = word_bytes(cwq[q]);
        bytes += w;
        cps += w ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t c0 = cb[0], c1 = cb[1];
    for (uint32_t j = c0 + threadIdx.x; j < c1; j += kIncThreads) {
        const uint32_t sj = os[j], np = la[j] + 1u + j;
        const uint32_t cwj = slot_word(a.cp, sj);
        a.seq2[np] = sj;
        cwl[np - o0] = cwj;
        a.rank2[sj] = np;
        const uint32_t w = word_bytes(cwj);
        bytes += w;
        cps += w ? 1u : 0u;
    }
    // the tile's totals (one barrier; rsum is used for nothing else, so no trailing barrier)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    bytes = wave_incl_scan(bytes);
    cps = wave_incl_scan(cps);
    if (lane == 63u) {
        rsum[wv] = bytes;
        rsum[kIncThreads / 64 + wv] = cps;
    }
    __syncthreads();
    uint32_t tb = 0, tc = 0;
#pragma unroll
    for (int i = 0; i < (int)(kIncThreads / 64); ++i) {
        tb += rsum[i];
        tc += rsum[kIncThreads / 64 + i];
    }
    range = make_uint2(k0 + c0, k1 + c1);
    return make_uint2(tb, tc);
}

// ---- decoupled look-back over the tiles: the bytes / codepoints of the tiles before tile b ------
// Per tile a status word (call epoch << 2 | 1: aggregate published, | 2: inclusive prefix
// published) and two values; a workgroup publishes its aggregate, then its first wave reads up to
// 64 predecessors at once (nearest first) until it meets an inclusive prefix, spinning on those
// not yet published.  Workgroups are dispatched in index order, so every predecessor runs.
__device__ __forceinline__ uint32_t lb_state(const uint32_t* f, uint32_t epoch) {
    const uint32_t v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    return (v >> 2) == epoch ? (v & 3u) : 0u;
}
__device__ __forceinline__ void lb_publish(const IncArgs& a, uint32_t b, uint64_t v, uint32_t st,
                                           uint32_t epoch) {
    (st == 2u ? a.lb_inc : a.lb_agg)[b] = v;
    __hip_atomic_store(&a.lb_flag[b], (epoch << 2) | st, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t inc_lookback(const IncArgs& a, uint32_t b, uint64_t agg,
                                                 uint64_t* excl_lds) {
    const uint32_t epoch = (uint32_t)(a.call & 0x3FFFFFFFu);
    if (threadIdx.x == 0) lb_publish(a, b, agg, b == 0 ? 2u : 1u, epoch);
    if (b == 0) return 0;
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        uint64_t excl = 0;
        int64_t j0 = (int64_t)b - 1;
        for (;;) {
            const int64_t j = j0 - (int64_t)lane;
            uint32_t st = j >= 0 ? lb_state(a.lb_flag + j, epoch) : 2u;
            const uint64_t inc2 = __ballot(st == 2u);
            // lanes up to (and including) the nearest inclusive prefix must all be published
            const uint32_t p = inc2 ? (uint32_t)__builtin_ctzll(inc2) : 64u;
            const uint64_t need = p >= 63u ? ~0ull : ((2ull << p) - 1ull);
            if (__ballot(st == 0u) & need) {
                __builtin_amdgcn_s_sleep(1);
                continue;  // (re-read the window)
            }
            uint64_t v = 0;
            if (lane <= p && j >= 0) v = (lane == p) ? a.lb_inc[j] : a.lb_agg[j];
            // (64-bit sum over the wave: bytes in the low half, codepoints in the high half)
#pragma unroll
            for (int o = 32; o; o >>= 1) {
                const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), o) << 32) |
                                   (uint32_t)__shfl_xor((int)(uint32_t)v, o);
                v += y;
            }
            excl += v;
            if (p < 64u) break;
            j0 -= 64;
        }
        if (lane == 0) {
            lb_publish(a, b, excl + agg, 2u, epoch);
            *excl_lds = excl;
        }
    }
    __syncthreads();
    return *excl_lds;
}

// ---- text: the UTF-8 of one tile's output places at byte offset `base` --------------------------
// (the places were written by this workgroup's splice: no other workgroup's writes are read)
__device__ __forceinline__ void inc_text_tile(const IncArgs& a, uint2 range, uint64_t base,
                                              const uint32_t* cwl, uint32_t* red) {
    for (uint32_t o0 = range.x; o0 < range.y; o0 += kSpliceTile) {
        const uint32_t ob = o0 + threadIdx.x * kSpliceRanks;
        uint32_t cw[kSpliceRanks], L[kSpliceRanks];
        // (the codepoint words the splice staged in LDS by place)
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q)
            cw[q] = ob + q < range.y ? cwl[ob + q - range.x] : kDelBitI;
        uint32_t tot = 0;
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) {
            L[q] = word_bytes(cw[q]);
            tot += L[q];
        }
        uint32_t all;
        const uint32_t off = block_excl_scan<kIncThreads / 64>(tot, red, all);
        uint8_t* o = a.text + base + off;
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) {
            const uint32_t c = cw[q] & kCpMaskI, n = L[q];
            if (n) {
                const uint32_t s0 = 6u * (n - 1u);
                o[0] = (uint8_t)(n == 1u ? c : (((0xFF00u >> n) & 0xFFu) | (c >> s0)));
                if (n > 1u) o[1] = (uint8_t)(0x80u | ((c >> (s0 - 6u)) & 63u));
                if (n > 2u) o[2] = (uint8_t)(0x80u | ((c >> (s0 - 12u)) & 63u));
                if (n > 3u) o[3] = (uint8_t)(0x80u | (c & 63u));
            }
            o += n;
        }
        base += all;
    }
}

// ---- the places of the roots that may sort below an old sibling (concurrent inserts), by the
// first a.nsearch workgroups of k_inc.  In the RGA pre-order a root x of key k under old parent p
// follows p's old children that sort above it, with their subtrees, so it goes before the first
// rank after p that holds an old child of p with a key <= k (x's id is greater than every old one:
// equal keys put x first) or that leaves p's subtree (an item whose parent ranks before p); its
// anchor is the rank before that.  Search workgroup b takes the roots b, b + nsearch, ... in item
// order, kSearchRound ranks per round, and publishes each anchor stamped with the call (a search
// that ran kIncScan ranks without an answer publishes 0xFFFFFFFF: the call merges in full).  The
// tile workgroups wait for the stamps only when they hold such roots; the searchers come first in
// the grid and wait for nothing, so they are dispatched before any tile that waits on them.
constexpr uint32_t kSearchThreads = kIncThreads;
constexpr uint32_t kSearchPer = kIncMax / kSearchThreads;       // items (and ranks) per thread
constexpr uint32_t kSearchRound = kSearchThreads * kSearchPer;  // ranks per round
static_assert(kIncScan % kSearchRound == 0, "search rounds");
__device__ __forceinline__ void inc_search(const IncArgs& a, uint32_t sb, uint32_t* red,
                                           uint32_t& target, uint32_t& found) {
    const uint32_t t = threadIdx.x, m = a.m, n0 = a.n0;
    const uint64_t maxkey0 = a.ctl[I_MAXKEY + ((a.call & 1u) ^ 1u)];
    uint32_t hard = 0;
#pragma unroll
    for (int q = 0; q < (int)kSearchPer; ++q) {
        const uint32_t i = t * kSearchPer + (uint32_t)q;
        if (i < m && a.parent[n0 + 1u + i] <= n0 && a.key[n0 + 1u + i] <= maxkey0) hard |= 1u << q;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan<kSearchThreads / 64>((uint32_t)__popc(hard), red, tot);
    if (tot > kIncHard) return;  // (block-uniform: the tiles merge in full without waiting)
    for (uint32_t b = sb; b < tot; b += a.nsearch) {
        if (b >= ex && b < ex + (uint32_t)__popc(hard)) {  // (the (b - ex)-th set bit: one thread)
            uint32_t h = hard;
            for (uint32_t k = b - ex; k; --k) h &= h - 1u;
            target = t * kSearchPer + (uint32_t)__ffs(h) - 1u;
            found = 0xFFFFFFFFu;
        }
        __syncthreads();
        const uint32_t i = target;
        const uint32_t p = a.parent[n0 + 1u + i], r0 = a.rank[p];
        const uint64_t k = a.key[n0 + 1u + i];
        uint32_t f = 0xFFFFFFFFu;
        for (uint32_t c = 0; c < kIncScan; c += kSearchRound) {
            uint32_t best = 0xFFFFFFFFu;
#pragma unroll
            for (int q = 0; q < (int)kSearchPer; ++q) {
                const uint32_t r = r0 + 1u + c + (uint32_t)q * kSearchThreads + t;
                bool stop = r > n0;  // (the document's end)
                if (!stop) {
                    const uint32_t sl = a.seq[r], pr = a.parent[sl];
                    stop = pr == p ? a.key[sl] <= k : a.rank[pr] < r0;
                }
                if (stop) best = min(best, r);
            }
            if (best != 0xFFFFFFFFu) atomicMin(&found, best);
            __syncthreads();
            f = found;
            __syncthreads();  // (every thread has read it before the next round's atomics)
            if (f != 0xFFFFFFFFu) break;  // (block-uniform)
        }
        if (t == 0)
            __hip_atomic_store(&a.hanc[i], ((uint64_t)(uint32_t)a.call << 32) | (f != 0xFFFFFFFFu ? f - 1u : 0xFFFFFFFFu),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- the whole incremental merge in one launch: one workgroup per tile of old ranks ------------
// Every workgroup orders the new items itself (the forest is small: the same result in each, no
// grid-wide barrier), splices its tile, takes its byte offset by look-back and writes its text.
// The last tile's workgroup reports the totals to the host-mapped result block.
__global__ __launch_bounds__(kIncThreads) void k_inc(IncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t red[kIncThreads / 64];
    __shared__ uint32_t rsum[2 * (kIncThreads / 64)];
    __shared__ uint32_t cb[2];
    __shared__ uint32_t flag, nhard;
    __shared__ uint64_t excl_lds;
    if (blockIdx.x < a.nsearch) {  // (block-uniform: a search workgroup)
        inc_search(a, blockIdx.x, red, flag, nhard);
        return;
    }
    const uint32_t b = blockIdx.x - a.nsearch;  // the tile
    // the tile's old order, loaded before the forest so that the round trip overlaps it
    uint32_t sl[kSpliceRanks];
    {
        const uint32_t k0 = b * kSpliceTile, k1 = min(a.n0 + 1u, k0 + kSpliceTile);
        const uint32_t kb = k0 + threadIdx.x * kSpliceRanks;
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) sl[q] = kb + q < k1 ? a.seq[kb + q] : 0u;
    }
    uint32_t cwq[kSpliceRanks];
    if (a.m && a.hasl) {  // (Fugue)
        if (a.m <= kIncThreads)
            inc_forest<1, true>(a, lds, red, flag, nhard, sl, cwq);
        else if (a.m <= 2u * kIncThreads)
            inc_forest<2, true>(a, lds, red, flag, nhard, sl, cwq);
        else
            inc_forest<kIncMax / kIncThreads, true>(a, lds, red, flag, nhard, sl, cwq);
    } else if (a.m) {
        if (a.m <= kIncThreads)
            inc_forest<1, false>(a, lds, red, flag, nhard, sl, cwq);
        else if (a.m <= 2u * kIncThreads)
            inc_forest<2, false>(a, lds, red, flag, nhard, sl, cwq);
        else
            inc_forest<kIncMax / kIncThreads, false>(a, lds, red, flag, nhard, sl, cwq);
    } else {
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) cwq[q] = slot_word(a.cp, sl[q]);
    }
    if (!a.m && threadIdx.x == 0) {
        flag = 0;
        if (b == 0) {  // (carry the largest key over to this call's slot)
            const uint64_t km = a.ctl[I_MAXKEY + ((a.call & 1u) ^ 1u)];
            atomicMax(reinterpret_cast<unsigned long long*>(&a.ctl[I_MAXKEY + (a.call & 1u)]),
                      (unsigned long long)km);
        }
    }
    __syncthreads();
    const uint32_t f = flag;
    uint64_t tot = 0;
    if (f == 0) {
        const uint32_t* os = reinterpret_cast<const uint32_t*>(lds);
        const uint32_t* la = os + kIncMax;
        // the tile's codepoint words by place, in the forest's tour region (dead by now)
        uint32_t* cwl = reinterpret_cast<uint32_t*>(lds + 12u * kIncMax + 4u * (kIncMax + 2u));
        uint2 range;
        const uint2 agg = inc_splice_tile(a, b, rsum, cb, os, la, cwl, sl, cwq, range);
        const uint64_t agg64 = ((uint64_t)agg.y << 32) | agg.x;
        const uint64_t excl = inc_lookback(a, b, agg64, &excl_lds);
        const uint64_t base = (uint32_t)excl;
        if (base + agg.x <= a.text_cap) inc_text_tile(a, range, base, cwl, red);
        tot = excl + agg64;
    }
    if (b + 1u == a.nblk && threadIdx.x == 0) {
        const uint64_t bytes = (uint32_t)tot, cps = tot >> 32;
        a.hres[0] = f ? f : (bytes > a.text_cap ? F_TEXT : 0u);
        a.hres[1] = bytes;
        a.hres[2] = cps;
        __threadfence_system();
        a.hres[3] = a.call;
    }
}

// (Fugue) The left-child bits of the parents of the left children among slots [lo, hi].
__global__ __launch_bounds__(256) void k_inc_hasl(const uint32_t* parent, const uint8_t* cp,
                                                  uint32_t lo, uint32_t hi, uint32_t* hasl) {
    for (uint64_t s = lo + blockIdx.x * 256ull + threadIdx.x; s <= hi; s += 256ull * gridDim.x)
        if (cp_word(cp, (uint32_t)s) & kLeftBitI) {
            const uint32_t p = parent[s];
            atomicOr(&hasl[p >> 5], 1u << (p & 31u));
        }
}

// The largest sibling key of items 1..n (state rebuild) into ctl[slot].
__global__ __launch_bounds__(256) void k_inc_maxkey(const uint64_t* key, uint32_t n, uint64_t* dst) {
    uint64_t mx = 0;
    for (uint64_t s = 1 + blockIdx.x * 256ull + threadIdx.x; s <= n; s += 256ull * gridDim.x)
        mx = max(mx, key[s] & ~kLeftKeyI);  // (without the Fugue side bit)
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(mx >> 32), o) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)mx, o);
        mx = max(mx, y);
    }
    if ((threadIdx.x & 63u) == 0 && mx)
        atomicMax(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)mx);
}

int ifail(Engine& E, const char* what, hipError_t e) {
    E.err = std::string(what) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();
    return CRDT_HIP_EDEVICE;
}
#define ICHK(expr, what)                                 \
    do {                                                 \
        hipError_t _e = (expr);                          \
        if (_e != hipSuccess) return ifail(E, what, _e); \
    } while (0)

hipError_t inc_setup() {
    static const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_inc),
                                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)inc_forest_lds(kIncMax));
    return e;
}

template <class T>
hipError_t igrow(T** p, uint64_t& cap, uint64_t need) {
    if (need <= cap) return hipSuccess;
    dfree(*p);
    cap = 0;
    hipError_t e = dalloc(p, need);
    if (e == hipSuccess) cap = need;
    return e;
}

// Room for an order of `items` items and a text of `bytes` bytes.
int inc_reserve(Engine& E, IncState& s, uint64_t items, uint64_t bytes) {
    const uint64_t need = items + 1 + kIncMax;  // (room for the next call's new items)
    if (need > s.cap) {
        // grown with the contents kept: the current order and the ranks are copied over
        const uint64_t cap = std::max<uint64_t>({need, 2 * s.cap, 4096});
        uint32_t *q0 = nullptr, *q1 = nullptr, *r0 = nullptr, *r1 = nullptr;
        hipError_t e = dalloc(&q0, cap);
        if (e == hipSuccess) e = dalloc(&q1, cap);
        if (e == hipSuccess) e = dalloc(&r0, cap);
        if (e == hipSuccess) e = dalloc(&r1, cap);
        if (e == hipSuccess && s.cap) {
            e = hipMemcpyAsync(q0, s.seq[s.cur], s.cap * 4, hipMemcpyDeviceToDevice, E.stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(r0, s.rank[s.cur], s.cap * 4, hipMemcpyDeviceToDevice, E.stream);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(E.stream);
        if (e != hipSuccess) {
            dfree(q0);
            dfree(q1);
            dfree(r0);
            dfree(r1);
            s.valid = false;
            return ifail(E, "incremental order arrays", e);
        }
        // (Fugue) the left-child bits, kept too
        uint32_t* h0 = nullptr;
        const uint64_t hw = cap / 32 + 1, hw_old = s.cap ? s.cap / 32 + 1 : 0;
        e = dalloc(&h0, hw);
        if (e == hipSuccess) e = hipMemsetAsync(h0, 0, hw * 4, E.stream);
        if (e == hipSuccess && hw_old)
            e = hipMemcpyAsync(h0, s.hasl, hw_old * 4, hipMemcpyDeviceToDevice, E.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(E.stream);
        if (e != hipSuccess) {
            dfree(q0);
            dfree(q1);
            dfree(r0);
            dfree(r1);
            dfree(h0);
            s.valid = false;
            return ifail(E, "incremental left-child bits", e);
        }
        dfree(s.seq[0]);
        dfree(s.seq[1]);
        dfree(s.rank[0]);
        dfree(s.rank[1]);
        dfree(s.hasl);
        s.seq[0] = q0;
        s.seq[1] = q1;
        s.rank[0] = r0;
        s.rank[1] = r1;
        s.hasl = h0;
        s.cur = 0;
        s.cap = cap;
    }
    const uint64_t ntiles = (s.cap + kSpliceTile - 1) / kSpliceTile + 1;
    if (ntiles > s.lb_cap) {
        dfree(s.lb_flag);
        dfree(s.lb_agg);
        dfree(s.lb_inc);
        s.lb_cap = 0;
        ICHK(dalloc(&s.lb_flag, ntiles), "hipMalloc look-back");
        ICHK(dalloc(&s.lb_agg, ntiles), "hipMalloc look-back");
        ICHK(dalloc(&s.lb_inc, ntiles), "hipMalloc look-back");
        ICHK(hipMemsetAsync(s.lb_flag, 0, ntiles * 4, E.stream), "clear look-back");
        s.lb_cap = ntiles;
    }
    const uint64_t tcap = bytes + 64;
    if (tcap > s.text_cap)
        ICHK(igrow(&s.text, s.text_cap, std::max<uint64_t>(tcap, 2 * s.text_cap)), "hipMalloc text");
    if (!s.hanc) {  // (stamps of call 0: no call reads them)
        ICHK(dalloc(&s.hanc, (uint64_t)kIncMax), "hipMalloc search anchors");
        ICHK(hipMemset(s.hanc, 0, kIncMax * 8ull), "clear search anchors");
    }
    if (!s.ctl) {
        ICHK(dalloc(&s.ctl, (uint64_t)I_N), "hipMalloc counters");
        ICHK(hipMemset(s.ctl, 0, I_N * 8), "clear counters");
    }
    if (!s.hres) {
        ICHK(hipHostMalloc(reinterpret_cast<void**>(&s.hres), 64,
                           hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc result");
        std::memset(s.hres, 0, 64);
        ICHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.dres), s.hres, 0),
             "mapped result pointer");
    }
    return CRDT_HIP_OK;
}

IncArgs make_args(Replica& r, IncState& s, uint32_t n0, uint32_t m) {
    IncArgs a{};
    a.n0 = n0;
    a.m = m;
    a.parent = r.logs.parent;
    a.key = r.logs.key;
    a.cp = r.logs.cp;
    a.rank = s.rank[s.cur];
    a.rank2 = s.rank[s.cur ^ 1];
    a.seq = s.seq[s.cur];
    a.seq2 = s.seq[s.cur ^ 1];
    a.lb_flag = s.lb_flag;
    a.lb_agg = s.lb_agg;
    a.lb_inc = s.lb_inc;
    a.nblk = (uint32_t)((n0 + 1ull + kSpliceTile - 1) / kSpliceTile);
    a.text = s.text;
    a.text_cap = s.text_cap;
    a.ctl = s.ctl;
    a.hres = s.dres;
    a.call = ++s.calls;
    a.hasl = r.logs.fugue ? s.hasl : nullptr;  // (selects the Fugue forest)
    a.hanc = s.hanc;
    return a;
}

// (Fugue) set the left-child bits of the parents of the left children among slots [lo, hi].
int inc_hasl(Engine& E, Replica& r, IncState& s, uint32_t lo, uint32_t hi) {
    if (!r.logs.fugue || hi < lo) return CRDT_HIP_OK;
    k_inc_hasl<<<std::max<uint32_t>(1, std::min<uint32_t>(grid_for(hi - lo + 1u, 256), 1024)), 256, 0,
                 E.stream>>>(r.logs.parent, r.logs.cp, lo, hi, s.hasl);
    ICHK(hipGetLastError(), "left-child bits");
    return CRDT_HIP_OK;
}

// CRDT_INC_PROFILE=1: per call, the kernel's device time (events), the forest's phases and the
// host times, to stderr
bool inc_profile() {
    static const bool on = [] {
        const char* e = std::getenv("CRDT_INC_PROFILE");
        return e && *e && *e != '0';
    }();
    return on;
}

// One launch, then a wait for the result block (sync: for the whole stream).
int inc_run(Engine& E, IncState& s, IncArgs& a, bool sync) {
    hipStream_t st = E.stream;
    ICHK(inc_setup(), "incremental merge setup");
    const bool prof = inc_profile();
    hipEvent_t* ev = s.pev;  // (per state: a state lives on one context and device)
    if (prof && !ev[0]) {
        for (int k = 0; k < 2; ++k) ICHK(hipEventCreate(&ev[k]), "event");
        ICHK(dalloc(&s.tsp, 16), "timestamps");
    }
    uint64_t* tsp = s.tsp;
    a.tsp = prof ? tsp : nullptr;
    const auto h0 = std::chrono::steady_clock::now();
    if (prof) ICHK(hipEventRecord(ev[0], st), "event");
    // (RGA: leading search workgroups for the roots an old sibling may precede)
    a.nsearch = a.m && !a.hasl ? std::min(a.m, kIncSearchers) : 0u;
    k_inc<<<a.nsearch + a.nblk, kIncThreads, inc_forest_lds(kIncMax), st>>>(a);
    ICHK(hipGetLastError(), "incremental merge launch");
    if (prof) ICHK(hipEventRecord(ev[1], st), "event");
    const auto h1 = std::chrono::steady_clock::now();
    // The result block is written last, after a system-scope fence, so the host can take it as
    // soon as it lands instead of waiting for the stream to report completion (a blocking wait
    // costs ~10 us of wake-up on top of the kernel).  Later work on the stream is ordered behind
    // the kernel anyway; a caller that copies the text waits for the stream (sync = true).  A
    // result that does not arrive within a bound falls back to the stream wait, which reports
    // any device error.
    bool landed = false;
    if (!sync && !prof) {
        const auto t0 = std::chrono::steady_clock::now();
        volatile const uint64_t* stamp = s.hres + 3;
        for (uint32_t spin = 0;; ++spin) {
            if (*stamp == a.call) {
                landed = true;
                break;
            }
            if ((spin & 1023u) == 1023u &&
                std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50))
                break;
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (!landed) ICHK(hipStreamSynchronize(st), "incremental merge sync");
    if (prof) {
        const auto h2 = std::chrono::steady_clock::now();
        float t = 0;
        (void)hipEventElapsedTime(&t, ev[0], ev[1]);
        uint64_t ts[11] = {};
        if (a.m) ICHK(hipMemcpy(ts, tsp, sizeof(ts), hipMemcpyDeviceToHost), "timestamps");
        std::fprintf(stderr, "[inc] m %u n0 %u tiles %u | kernel %.1f us | forest", a.m, a.n0,
                     a.nblk, 1e3 * t);
        for (int k = 1; k < 11; ++k) std::fprintf(stderr, " %.1f", (ts[k] - ts[k - 1]) / 100.0);
        std::fprintf(stderr, " | host enqueue %.1f wait %.1f us\n",
                     std::chrono::duration<double, std::micro>(h1 - h0).count(),
                     std::chrono::duration<double, std::micro>(h2 - h1).count());
    }
    if (s.hres[3] != a.call) {
        E.err = "incremental merge: no result from the device";
        return CRDT_HIP_EDEVICE;
    }
    return CRDT_HIP_OK;
}

// Full merge (engine ORDER mode) and a state built from it.
int inc_rebuild(Engine& E, Replica& r, IncState& s) {
    s.valid = false;
    int rc = replica_reserve(E, r, r.n);
    if (rc) return rc;
    std::vector<DocInfo> docs{DocInfo{r.n, r.vis_bytes}};
    rc = E.plan(r.logs, docs);
    if (rc) return rc;
    std::vector<uint8_t> raw;
    rc = E.merge(r.logs, Engine::ORDER, nullptr, nullptr, nullptr, &raw, nullptr);
    if (rc) return rc;
    if (raw.size() != (size_t)r.n * 4) {
        E.err = "order output size mismatch";
        return CRDT_HIP_EBADLOG;
    }
    rc = inc_reserve(E, s, r.n, r.vis_bytes);
    if (rc) return rc;
    hipStream_t st = E.stream;
    s.hseq.resize((size_t)r.n + 1);
    s.hseq[0] = 0;
    if (r.n) std::memcpy(s.hseq.data() + 1, raw.data(), raw.size());
    ICHK(hipMemcpyAsync(s.seq[s.cur], s.hseq.data(), (r.n + 1ull) * 4, hipMemcpyHostToDevice, st),
         "upload order");
    // the largest key, into the slot the next call reads (that call copies it forward)
    ICHK(hipMemsetAsync(s.ctl, 0, I_N * 8, st), "clear counters");
    const uint64_t next = s.calls + 1;
    k_inc_maxkey<<<std::max<uint32_t>(1, std::min<uint32_t>(grid_for(r.n, 256), 1024)), 256, 0, st>>>(
        r.logs.key, r.n, s.ctl + I_MAXKEY + ((next & 1u) ^ 1u));
    if (r.logs.fugue) {  // the left-child bits of the whole log
        ICHK(hipMemsetAsync(s.hasl, 0, (s.cap / 32 + 1) * 4, st), "clear left-child bits");
        if ((rc = inc_hasl(E, r, s, 1u, r.n))) return rc;
    }
    IncArgs a = make_args(r, s, r.n, 0);  // m = 0: the splice copies the order and sets the ranks
    rc = inc_run(E, s, a, true);
    if (rc) return rc;
    if (s.hres[0] || s.hres[1] != r.vis_bytes || s.hres[2] != r.vis_cp) {
        E.err = "incremental merge state: rebuilt text disagrees with the replica's counters";
        return CRDT_HIP_EBADLOG;
    }
    s.cur ^= 1;
    s.n = r.n;
    s.valid = true;
    return CRDT_HIP_OK;
}

}  // namespace

IncState::~IncState() {
    dfree(seq[0]);
    dfree(seq[1]);
    dfree(rank[0]);
    dfree(rank[1]);
    dfree(tsp);
    for (hipEvent_t e : pev)
        if (e) (void)hipEventDestroy(e);
    dfree(hasl);
    dfree(hanc);
    dfree(lb_flag);
    dfree(lb_agg);
    dfree(lb_inc);
    dfree(text);
    dfree(ctl);
    if (hres) (void)hipHostFree(hres);
}

int replica_merge_inc(Engine& E, Replica& r, std::vector<uint8_t>* text, uint64_t* bytes,
                      uint64_t* cps, uint32_t* path) {
    int rc = replica_settle(E, r);
    if (rc) return rc;
    IncState& s = r.inc;
    if (path) *path = 0;
    ICHK(hipSetDevice(E.device), "hipSetDevice");
    // (the look-back packs {bytes, codepoints} as two u32 halves: a text of 4 GiB or more merges
    // in full)
    bool fast = s.valid && r.n >= s.n && r.n - s.n <= kIncMax && r.vis_bytes < (1ull << 32);
    if (fast) {
        rc = inc_reserve(E, s, r.n, r.vis_bytes);  // (grows keeping the order)
        if (rc) return rc;
        fast = s.valid && r.n + 1ull <= s.cap;
    }
    if (fast) {
        IncArgs a = make_args(r, s, s.n, r.n - s.n);
        rc = inc_run(E, s, a, text != nullptr);
        if (rc) return rc;
        if (s.hres[0] == 0) {
            if (s.hres[1] != r.vis_bytes || s.hres[2] != r.vis_cp) {
                E.err = "incremental merge disagrees with the replica's counters";
                s.valid = false;
                return CRDT_HIP_EBADLOG;
            }
            // (Fugue) the new left children's parents have one now
            if ((rc = inc_hasl(E, r, s, a.n0 + 1u, a.n0 + a.m))) return rc;
            s.cur ^= 1;
            s.n = r.n;
            if (path) *path = 1;
        } else {
            fast = false;  // a concurrent update, a huge sibling group, ...: merge in full
        }
    }
    if (!fast) {
        rc = inc_rebuild(E, r, s);
        if (rc) return rc;
    }
    if (bytes) *bytes = s.hres[1];
    if (cps) *cps = s.hres[2];
    if (text) {
        text->resize(s.hres[1]);
        if (!text->empty())
            ICHK(hipMemcpy(text->data(), s.text, text->size(), hipMemcpyDeviceToHost), "copy text");
    }
    return CRDT_HIP_OK;
}

}  // namespace crdt
