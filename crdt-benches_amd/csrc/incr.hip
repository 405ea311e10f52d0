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
//   race an older one.  The new forest (at most kIncMax items) is ordered in one workgroup
//   (k_inc_forest): children grouped by parent and ranked among their siblings (roots by
//   (anchor rank asc, key desc), other groups by key desc), then an Euler tour of the forest
//   ranked by pointer jumping in LDS gives every new item its place.  k_inc_splice merges the old
//   order with the new items (an old rank k moves to k + #new items anchored before it) and
//   rewrites `rank`; k_inc_text writes the text of the new order.  Deletes change no order: the
//   tombstone bits the decode set make those items weigh nothing in k_inc_text.
//
// Anything else — a root whose key is not above every old key (a concurrent update), more than
// kIncMax new items, a Fugue replica — falls back to a full merge (engine ORDER mode), which also
// rebuilds the state.  Every fast-path merge is checked against the decode's counters (bytes and
// codepoints of the visible text) by the host.
#include <hip/hip_cooperative_groups.h>

#include <algorithm>
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

constexpr uint32_t kIncThreads = 1024;
constexpr uint32_t kSpliceRanks = 4;                                // old ranks per thread
constexpr uint32_t kSpliceTile = kIncThreads * kSpliceRanks;        // old ranks per tile
constexpr uint32_t kIncGroupMax = 1024;  // largest sibling group ranked in k_inc_forest
constexpr uint32_t kIncThinGroup = 32;   // more roots than this: ranked one wave per root
constexpr uint32_t kCpMaskI = 0x001FFFFFu;
constexpr uint32_t kDelBitI = 0x00800000u;

// device counters (u64)
enum ICtl { I_FLAG = 0, I_MAXKEY, I_BYTES, I_CPS, I_N };
// I_FLAG bits: the fast path does not apply (the host merges in full)
constexpr uint64_t F_KEY = 1, F_ORDER = 2, F_GROUP = 4, F_TEXT = 8;

struct IncArgs {
    uint32_t n0, m;             // items the order covers, items appended since
    const uint32_t* parent;     // replica slot arrays (slot = id)
    const uint64_t* key;
    const uint8_t* cp;
    uint32_t* rank;             // slot -> rank
    const uint32_t* seq;        // rank -> slot (n0 + 1 entries)
    uint32_t* seq2;             // the new order (n0 + 1 + m entries)
    uint32_t* ins_s;            // the new items in their order: slot
    uint32_t* ins_a;            //   and the old rank they follow (non-decreasing)
    uint4* bsum;                // per splice block: {bytes, codepoints, first output, end}
    uint32_t nblk;
    uint8_t* text;
    uint64_t text_cap;
    uint64_t* ctl;
    uint64_t* hres;             // host-mapped result {flag, bytes, codepoints, call number}
    uint64_t* tsp;              // (CRDT_INC_PROFILE) phase timestamps of the forest, or null
    uint64_t call;              // this call's number (a stale result block is detected)
};

typedef __attribute__((address_space(3))) uint32_t lds_u32i_t;
__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) { return *(volatile lds_u32i_t*)p; }
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) { *(volatile lds_u32i_t*)p = v; }

__device__ __forceinline__ uint32_t cp_word(const uint8_t* cp, uint32_t s) {
    return (uint32_t)cp[3ull * s] | ((uint32_t)cp[3ull * s + 1] << 8) |
           ((uint32_t)cp[3ull * s + 2] << 16);
}
// UTF-8 bytes of slot s in the text (0: the document start or a tombstone)
__device__ __forceinline__ uint32_t slot_bytes(const uint8_t* cp, uint32_t s) {
    if (s == 0) return 0;
    const uint32_t c = cp_word(cp, s);
    return (c & kDelBitI) ? 0u : utf8_len(c & kCpMaskI);
}

__device__ __forceinline__ uint32_t block_max_u32(uint32_t x, uint32_t* lds) {
#pragma unroll
    for (int o = 32; o; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    if ((threadIdx.x & 63u) == 0) lds[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t t = 0;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) t = max(t, lds[i]);
    __syncthreads();
    return t;
}

// ---- k_inc_forest: the order of the appended items (one workgroup) -----------------------------
// Items i = 0..m-1 are slots n0 + 1 + i.  Local node m is a virtual root V whose children are
// the items with an old parent.  LDS (dynamic): see the carve-up below.
__host__ __device__ constexpr uint32_t inc_forest_lds(uint32_t mmax) {
    return 2u * (mmax + 2u)          // lp: local parent (u16)
           + 4u * (mmax + 2u)        // start: child count -> segment start (u32)
           + 2u * (mmax + 2u)        // ch: children by segment, then sorted (u16)
           + 8u * mmax               // keys (u64), later the output pairs
           + 4u * mmax               // A: anchor rank of a root (u32)
           + 4u * (2u * mmax + 4u)   // tour successor (u16) and suffix sum (u16), packed u32
           + 2u * mmax               // vrk: ranks among many roots (u16)
           + 64u;
}

#define INC_TS(i) \
    if (a.tsp && threadIdx.x == 0) a.tsp[i] = wall_clock64()
__device__ __forceinline__ void inc_forest(const IncArgs& a, uint8_t* lds, uint32_t* red,
                                           uint32_t& flag) {
    constexpr uint32_t Q = kIncMax / kIncThreads;  // items per thread
    const uint32_t t = threadIdx.x, m = a.m, n0 = a.n0;
    uint64_t* keys = reinterpret_cast<uint64_t*>(lds);
    uint32_t* A = reinterpret_cast<uint32_t*>(keys + kIncMax);
    uint32_t* start = A + kIncMax;                          // kIncMax + 2
    uint32_t* tour = start + (kIncMax + 2u);                // 2 kIncMax + 4: succ | sum << 16
    uint16_t* lp = reinterpret_cast<uint16_t*>(tour + (2u * kIncMax + 4u));  // kIncMax + 2
    uint16_t* ch = lp + (kIncMax + 2u);                     // kIncMax + 2
    uint16_t* vrk = ch + (kIncMax + 2u);                    // kIncMax: ranks among the roots
    if (t == 0) flag = 0;
    INC_TS(0);
    const uint64_t maxkey0 = a.ctl[I_MAXKEY];
    // ---- load: parents, keys, anchors; counts cleared ----
    uint32_t plc[Q];
    uint64_t kmax = 0;
    for (uint32_t x = t; x <= m + 1u; x += kIncThreads) start[x] = 0;
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
        for (int q = 0; q < (int)Q; ++q) {
            const uint32_t i = t + (uint32_t)q * kIncThreads;
            if (i >= m) continue;
            keys[i] = kk[q];
            kmax = max(kmax, kk[q]);
            if (pp[q] <= n0) {  // a root: after its old parent, ahead of the parent's old children
                lp[i] = (uint16_t)m;
                A[i] = a.rank[pp[q]];
                if (kk[q] <= maxkey0) bad |= (uint32_t)F_KEY;
            } else {
                const uint32_t l = pp[q] - (n0 + 1u);
                if (l >= i) bad |= (uint32_t)F_ORDER;  // (parents precede their children)
                lp[i] = (uint16_t)(l < i ? l : m);
                A[i] = 0;
            }
        }
        if (bad) atomicOr(&flag, bad);
    }
    INC_TS(1);
    __syncthreads();
    // ---- child counts; each child keeps its place among its parent's children ----
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t i = t + (uint32_t)q * kIncThreads;
        plc[q] = i < m ? atomicAdd(&start[lp[i]], 1u) : 0u;
    }
    INC_TS(2);
    __syncthreads();
    // ---- segment starts: exclusive scan over nodes 0..m (m + 1 <= kIncMax + 1 counts) ----
    {
        constexpr uint32_t P = (kIncMax + 1u + kIncThreads - 1u) / kIncThreads + 1u;
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
            const uint32_t ai = A[i];
            const uint64_t ki = keys[i];
            uint32_t r = 0;
            for (uint32_t s = lane; s < nv; s += 64) {
                const uint32_t j = ch[v0 + s];
                const uint32_t aj = A[j];
                const uint64_t kj = keys[j];
                r += (aj < ai || (aj == ai && (kj > ki || (kj == ki && j > i)))) ? 1u : 0u;
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
        const uint32_t ai = A[i];
        const uint64_t ki = keys[i];
        uint32_t r = 0;
        for (uint32_t s = g0; s < g1; ++s) {
            const uint32_t j = ch[s];
            const uint32_t aj = A[j];
            const uint64_t kj = keys[j];
            r += (aj < ai || (aj == ai && (kj > ki || (kj == ki && j > i)))) ? 1u : 0u;
        }
        rk[q] = r;
    }
    INC_TS(5);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t i = t + (uint32_t)q * kIncThreads;
        if (i < m) ch[start[lp[i]] + rk[q]] = (uint16_t)i;
    }
    INC_TS(6);
    __syncthreads();
    if (flag) {  // (block-uniform after the barrier)
        if (t == 0) a.ctl[I_FLAG] = flag;
        return;
    }
    if (t == 0) a.ctl[I_FLAG] = 0;
    // ---- Euler tour of the forest: down(x) = 2x, up(x) = 2x + 1 (x = 0..m, V = m), end E ----
    // succ in the low 16 bits, the arc's weight (1 for an item's down arc) in the high 16
    const uint32_t E = 2u * m + 2u, V = m;
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t x = t + (uint32_t)q * kIncThreads;
        if (x >= m) continue;
        const uint32_t c0 = start[x], c1 = start[x + 1u];
        const uint32_t sd = c1 > c0 ? 2u * ch[c0] : 2u * x + 1u;
        const uint32_t p = lp[x], pos = start[p] + rk[q];
        const uint32_t su = pos + 1u < start[p + 1u] ? 2u * ch[pos + 1u] : 2u * p + 1u;
        tour[2u * x] = sd | (1u << 16);
        tour[2u * x + 1u] = su;
    }
    if (t == 0) {
        const uint32_t c0 = start[V], c1 = start[V + 1u];
        tour[2u * V] = c1 > c0 ? 2u * ch[c0] : 2u * V + 1u;
        tour[2u * V + 1u] = E;
        tour[E] = E;
    }
    INC_TS(7);
    __syncthreads();
    // ---- pointer jumping without barriers: a record (succ | weight of [arc, succ) << 16) is a
    // valid stretch of the tour at all times, so joining it with an old or a new record of its
    // successor is equally right; each thread jumps its own arcs until they reach the end (every
    // pass at least doubles... or extends a record by one arc: E passes bound it) ----
    {
        constexpr int NA = (int)((2u * kIncMax + 4u + kIncThreads - 1u) / kIncThreads);
        uint32_t live = 0;
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            const uint32_t arc = t + (uint32_t)q * kIncThreads;
            live |= (arc < E ? 1u : 0u) << q;
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
    // ---- every item's place among the new items; its root's anchor by a max-scan ----
    uint32_t* os = reinterpret_cast<uint32_t*>(keys);  // (keys are dead) slot by place
    uint32_t* oa = os + kIncMax;                       // a root's anchor by place, else 0
    uint32_t pa[Q], px[Q];
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t x = t + (uint32_t)q * kIncThreads;
        px[q] = x < m ? m - (tour[2u * x] >> 16) : 0u;
        pa[q] = (x < m && lp[x] == V) ? A[x] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (int)Q; ++q) {
        const uint32_t x = t + (uint32_t)q * kIncThreads;
        if (x < m) {
            os[px[q]] = n0 + 1u + x;
            oa[px[q]] = pa[q];
        }
    }
    __syncthreads();
    {
        // inclusive max-scan over places (roots come in anchor order, each before its subtree)
        const uint32_t lo = min(m, t * Q), hi = min(m, lo + Q);
        uint32_t mx = 0;
        for (uint32_t i = lo; i < hi; ++i) mx = max(mx, oa[i]);
        // exclusive max over the threads before this one
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
            a.ins_s[i] = os[i];
            a.ins_a[i] = run;
        }
    }
    // the largest key now held (the next merge's check)
    __syncthreads();  // (red is reused)
    INC_TS(9);
    {
        const uint32_t hi32 = block_max_u32((uint32_t)(kmax >> 32), red);
        const uint32_t lo32 = block_max_u32((uint32_t)(kmax >> 32) == hi32 ? (uint32_t)kmax : 0u, red);
        if (t == 0) {
            const uint64_t km = ((uint64_t)hi32 << 32) | lo32;
            if (km > maxkey0) a.ctl[I_MAXKEY] = km;
        }
    }
    INC_TS(10);
}
#undef INC_TS

// Number of new items anchored before old rank k (ins_a is non-decreasing).
__device__ __forceinline__ uint32_t anchored_before(const uint32_t* ins_a, uint32_t m, uint32_t k) {
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ins_a[mid] < k) lo = mid + 1u;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t ld_flag(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- splice: the new order of one tile; rank rewritten; the tile's text sums -------------------
// Tile b takes old ranks [k0, k1) and the new items anchored in [k0, k1): its outputs are the
// places [k0 + c(k0), k1 + c(k1)), c(k) = new items anchored before k.
// la: the anchors (ins_a) copied to LDS by inc_load_anchors (searched there, not in HBM: ins_a
// was written by one workgroup, and a dependent chain of loads from another XCD's L2 is slow).
__device__ __forceinline__ void inc_load_anchors(const IncArgs& a, uint32_t* la) {
    for (uint32_t j = threadIdx.x; j < a.m; j += kIncThreads) la[j] = a.ins_a[j];
    __syncthreads();
}
__device__ __forceinline__ void inc_splice_tile(const IncArgs& a, uint32_t b, uint32_t* red,
                                                uint32_t* cb, const uint32_t* la) {
    const uint32_t N0 = a.n0 + 1u, m = a.m;
    const uint32_t k0 = b * kSpliceTile, k1 = min(N0, k0 + kSpliceTile);
    if (threadIdx.x < 2u) cb[threadIdx.x] = m ? anchored_before(la, m, threadIdx.x ? k1 : k0) : 0u;
    const uint32_t kb = k0 + threadIdx.x * kSpliceRanks;
    uint32_t sl[kSpliceRanks];
#pragma unroll
    for (int q = 0; q < (int)kSpliceRanks; ++q) sl[q] = kb + q < k1 ? a.seq[kb + q] : 0u;
    uint32_t bytes = 0, cps = 0;
#pragma unroll
    for (int q = 0; q < (int)kSpliceRanks; ++q) {
        const uint32_t k = kb + q;
        if (k >= k1) break;
        // (a search per rank: a whole subtree of new items shares one anchor)
        const uint32_t c = m ? anchored_before(la, m, k) : 0u;
        const uint32_t np = k + c;
        a.seq2[np] = sl[q];
        a.rank[sl[q]] = np;
        const uint32_t w = slot_bytes(a.cp, sl[q]);
        bytes += w;
        cps += w ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t c0 = cb[0], c1 = cb[1];
    for (uint32_t j = c0 + threadIdx.x; j < c1; j += kIncThreads) {
        const uint32_t s = a.ins_s[j], np = la[j] + 1u + j;
        a.seq2[np] = s;
        a.rank[s] = np;
        const uint32_t w = slot_bytes(a.cp, s);
        bytes += w;
        cps += w ? 1u : 0u;
    }
    uint32_t tb, tc;
    (void)block_excl_scan<kIncThreads / 64>(bytes, red, tb);
    (void)block_excl_scan<kIncThreads / 64>(cps, red, tc);
    if (threadIdx.x == 0) a.bsum[b] = make_uint4(tb, tc, k0 + c0, k1 + c1);
}

// ---- text: the UTF-8 of one tile's outputs, at the bytes of the tiles before it ----------------
__device__ __forceinline__ void inc_text_tile(const IncArgs& a, uint32_t b, uint32_t* red) {
    // the tile's range and the bytes of the tiles before it, and the first chunk's items and
    // codepoint words, all loaded before the first wait
    const uint4 me = a.bsum[b];
    uint32_t p = 0;
    for (uint32_t i = threadIdx.x; i < b; i += kIncThreads) p += a.bsum[i].x;
    uint32_t cw[kSpliceRanks];
    auto load = [&](uint32_t o0) {
        const uint32_t ob = o0 + threadIdx.x * kSpliceRanks;
        uint32_t sl[kSpliceRanks];
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) sl[q] = ob + q < me.w ? a.seq2[ob + q] : 0u;
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) cw[q] = sl[q] ? cp_word(a.cp, sl[q]) : kDelBitI;
    };
    load(me.z);
    uint32_t ptot;
    (void)block_excl_scan<kIncThreads / 64>(p, red, ptot);
    uint64_t base = ptot;
    if (base + me.x > a.text_cap) return;  // (flagged from the totals)
    for (uint32_t o0 = me.z; o0 < me.w; o0 += kSpliceTile) {
        if (o0 != me.z) load(o0);
        uint32_t L[kSpliceRanks];
        uint32_t tot = 0;
#pragma unroll
        for (int q = 0; q < (int)kSpliceRanks; ++q) {
            L[q] = (cw[q] & kDelBitI) ? 0u : utf8_len(cw[q] & kCpMaskI);
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

// The totals (one workgroup): the flag, bytes and codepoints of every tile, to the host-mapped
// result block, stamped with the call number.
__device__ __forceinline__ void inc_totals(const IncArgs& a, uint32_t ntiles, uint32_t* red) {
    uint32_t b = 0, c = 0;
    for (uint32_t i = threadIdx.x; i < ntiles; i += kIncThreads) {
        const uint4 v = a.bsum[i];
        b += v.x;
        c += v.y;
    }
    uint32_t tb, tc;
    (void)block_excl_scan<kIncThreads / 64>(b, red, tb);
    (void)block_excl_scan<kIncThreads / 64>(c, red, tc);
    if (threadIdx.x == 0) {
        const uint64_t f = ld_flag(&a.ctl[I_FLAG]) | (tb > a.text_cap ? F_TEXT : 0u);
        a.ctl[I_BYTES] = tb;
        a.ctl[I_CPS] = tc;
        a.hres[0] = f;
        a.hres[1] = tb;
        a.hres[2] = tc;
        __threadfence_system();
        a.hres[3] = a.call;
    }
}

// ---- the three phases as kernels (stream order between them) ------------------------------------
__global__ __launch_bounds__(kIncThreads) void k_inc_forest(IncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t red[kIncThreads / 64];
    __shared__ uint32_t flag;
    if (a.m) inc_forest(a, lds, red, flag);
    else if (threadIdx.x == 0) a.ctl[I_FLAG] = 0;
}
__global__ __launch_bounds__(kIncThreads) void k_inc_splice(IncArgs a) {
    __shared__ uint32_t red[kIncThreads / 64];
    __shared__ uint32_t cb[2];
    __shared__ uint32_t la[kIncMax];
    if (ld_flag(&a.ctl[I_FLAG])) return;
    inc_load_anchors(a, la);
    inc_splice_tile(a, blockIdx.x, red, cb, la);
}
__global__ __launch_bounds__(kIncThreads) void k_inc_text(IncArgs a) {
    __shared__ uint32_t red[kIncThreads / 64];
    if (blockIdx.x == gridDim.x - 1u) {  // (the last workgroup also reports)
        inc_totals(a, gridDim.x - 1u, red);
        return;
    }
    if (ld_flag(&a.ctl[I_FLAG])) return;
    inc_text_tile(a, blockIdx.x, red);
}

// ---- all three in one cooperative launch (grid-wide barriers between the phases) -----------------
__global__ __launch_bounds__(kIncThreads) void k_inc_all(IncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t red[kIncThreads / 64];
    __shared__ uint32_t cb[2];
    __shared__ uint32_t flag;
    namespace cg = cooperative_groups;
    cg::grid_group grid = cg::this_grid();
    if (blockIdx.x == 0) {
        if (a.m) inc_forest(a, lds, red, flag);
        else if (threadIdx.x == 0) a.ctl[I_FLAG] = 0;
    }
    grid.sync();
    const bool go = ld_flag(&a.ctl[I_FLAG]) == 0;
    if (go && blockIdx.x < a.nblk) {
        uint32_t* la = reinterpret_cast<uint32_t*>(lds);
        inc_load_anchors(a, la);
        for (uint32_t b = blockIdx.x; b < a.nblk; b += gridDim.x) {
            inc_splice_tile(a, b, red, cb, la);
            __syncthreads();
        }
    }
    grid.sync();
    if (go)
        for (uint32_t b = blockIdx.x; b < a.nblk; b += gridDim.x) {
            inc_text_tile(a, b, red);
            __syncthreads();
        }
    if (blockIdx.x == gridDim.x - 1u) inc_totals(a, go ? a.nblk : 0u, red);
}

// The largest sibling key of items 1..n (state rebuild).
__global__ __launch_bounds__(256) void k_inc_maxkey(const uint64_t* key, uint32_t n, uint64_t* ctl) {
    uint64_t mx = 0;
    for (uint64_t s = 1 + blockIdx.x * 256ull + threadIdx.x; s <= n; s += 256ull * gridDim.x)
        mx = max(mx, key[s]);
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(mx >> 32), o) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)mx, o);
        mx = max(mx, y);
    }
    if ((threadIdx.x & 63u) == 0 && mx)
        atomicMax(reinterpret_cast<unsigned long long*>(&ctl[I_MAXKEY]), (unsigned long long)mx);
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

// Dynamic LDS of the forest kernels, and the cooperative grid (workgroups that fit at once).
struct IncLaunch {
    hipError_t err = hipSuccess;
    uint32_t coop_grid = 0;
};
const IncLaunch& inc_launch_info(int device) {
    static IncLaunch info = [device] {
        IncLaunch li;
        const int lds = (int)inc_forest_lds(kIncMax);
        li.err = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_inc_forest),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (li.err == hipSuccess)
            li.err = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_inc_all),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        int per_cu = 0, cus = 0, coop = 0;
        if (li.err == hipSuccess)
            li.err = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, reinterpret_cast<const void*>(&k_inc_all), kIncThreads, lds);
        if (li.err == hipSuccess)
            li.err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        if (li.err == hipSuccess)
            li.err = hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device);
        if (li.err == hipSuccess && coop) li.coop_grid = (uint32_t)std::max(0, per_cu * cus);
        return li;
    }();
    return info;
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

// Room for an order of `items` items and a text of `bytes` bytes.  Growing the order arrays
// drops the state (the next merge rebuilds it).
int inc_reserve(Engine& E, IncState& s, uint64_t items, uint64_t bytes) {
    const uint64_t need = items + 1 + kIncMax;  // (room for the next call's new items)
    if (need > s.cap) {
        // grown with the contents kept: the current order and the ranks are copied over
        const uint64_t cap = std::max<uint64_t>({need, 2 * s.cap, 4096});
        uint32_t *q0 = nullptr, *q1 = nullptr, *rk = nullptr;
        hipError_t e = dalloc(&q0, cap);
        if (e == hipSuccess) e = dalloc(&q1, cap);
        if (e == hipSuccess) e = dalloc(&rk, cap);
        if (e == hipSuccess && s.cap) {
            e = hipMemcpyAsync(q0, s.seq[s.cur], s.cap * 4, hipMemcpyDeviceToDevice, E.stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(rk, s.rank, s.cap * 4, hipMemcpyDeviceToDevice, E.stream);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(E.stream);
        if (e != hipSuccess) {
            dfree(q0);
            dfree(q1);
            dfree(rk);
            s.valid = false;
            return ifail(E, "incremental order arrays", e);
        }
        dfree(s.seq[0]);
        dfree(s.seq[1]);
        dfree(s.rank);
        s.seq[0] = q0;
        s.seq[1] = q1;
        s.rank = rk;
        s.cur = 0;
        s.cap = cap;
    }
    const uint64_t nblk = (s.cap + kSpliceTile - 1) / kSpliceTile + 1;
    ICHK(igrow(&s.bsum, s.bsum_cap, nblk), "hipMalloc tile sums");
    ICHK(igrow(&s.ins, s.ins_cap, 2ull * kIncMax), "hipMalloc new-item order");
    const uint64_t tcap = bytes + 64;
    if (tcap > s.text_cap)
        ICHK(igrow(&s.text, s.text_cap, std::max<uint64_t>(tcap, 2 * s.text_cap)), "hipMalloc text");
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
    a.rank = s.rank;
    a.seq = s.seq[s.cur];
    a.seq2 = s.seq[s.cur ^ 1];
    a.ins_s = s.ins;
    a.ins_a = s.ins + kIncMax;
    a.bsum = s.bsum;
    a.nblk = (uint32_t)((n0 + 1ull + kSpliceTile - 1) / kSpliceTile);
    a.text = s.text;
    a.text_cap = s.text_cap;
    a.ctl = s.ctl;
    a.hres = s.dres;
    a.call = ++s.calls;
    return a;
}

// CRDT_INC_PROFILE=1: per call, device times of the phases (events) and host times, to stderr
bool inc_profile() {
    static const bool on = [] {
        const char* e = std::getenv("CRDT_INC_PROFILE");
        return e && *e && *e != '0';
    }();
    return on;
}

// The three phases (one cooperative launch, or three launches), then a wait for the result.
int inc_run(Engine& E, IncState& s, IncArgs& a) {
    hipStream_t st = E.stream;
    const IncLaunch& li = inc_launch_info(E.device);
    ICHK(li.err, "incremental merge setup");
    const uint32_t lds = inc_forest_lds(kIncMax);
    const bool prof = inc_profile();
    static hipEvent_t ev[4] = {};
    static uint64_t* tsp = nullptr;
    if (prof && !ev[0]) {
        for (auto& e : ev) ICHK(hipEventCreate(&e), "event");
        ICHK(dalloc(&tsp, 16), "timestamps");
    }
    a.tsp = prof ? tsp : nullptr;
    const auto h0 = std::chrono::steady_clock::now();
    if (prof) ICHK(hipEventRecord(ev[0], st), "event");
    if (E.inc_coop && li.coop_grid) {
        const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(li.coop_grid, a.nblk));
        void* args[] = {&a};
        ICHK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_inc_all), dim3(grid),
                                        dim3(kIncThreads), args, lds, st),
             "k_inc_all launch");
        if (prof)
            for (int k = 1; k < 4; ++k) ICHK(hipEventRecord(ev[k], st), "event");
    } else {
        k_inc_forest<<<1, kIncThreads, a.m ? lds : 0, st>>>(a);
        if (prof) ICHK(hipEventRecord(ev[1], st), "event");
        k_inc_splice<<<a.nblk, kIncThreads, 0, st>>>(a);
        if (prof) ICHK(hipEventRecord(ev[2], st), "event");
        k_inc_text<<<a.nblk + 1u, kIncThreads, 0, st>>>(a);
        if (prof) ICHK(hipEventRecord(ev[3], st), "event");
        ICHK(hipGetLastError(), "incremental merge launch");
    }
    const auto h1 = std::chrono::steady_clock::now();
    ICHK(hipStreamSynchronize(st), "incremental merge sync");
    if (prof && a.tsp && a.m) {
        uint64_t ts[11] = {};
        ICHK(hipMemcpy(ts, a.tsp, sizeof(ts), hipMemcpyDeviceToHost), "timestamps");
        std::fprintf(stderr, "[inc-forest] us:");
        for (int k = 1; k < 11; ++k) std::fprintf(stderr, " %.1f", (ts[k] - ts[k - 1]) / 100.0);
        std::fprintf(stderr, " | total %.1f\n", (ts[10] - ts[0]) / 100.0);
    }
    if (prof) {
        const auto h2 = std::chrono::steady_clock::now();
        float t[3] = {};
        for (int k = 0; k < 3; ++k) (void)hipEventElapsedTime(&t[k], ev[k], ev[k + 1]);
        std::fprintf(stderr, "[inc] m %u n0 %u coop %d | device forest %.1f splice %.1f text %.1f us"
                     " | host enqueue %.1f wait %.1f us\n", a.m, a.n0, (int)(E.inc_coop && li.coop_grid),
                     1e3 * t[0], 1e3 * t[1], 1e3 * t[2],
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
    ICHK(hipMemsetAsync(s.ctl, 0, I_N * 8, st), "clear counters");
    k_inc_maxkey<<<std::max<uint32_t>(1, std::min<uint32_t>(grid_for(r.n, 256), 1024)), 256, 0, st>>>(
        r.logs.key, r.n, s.ctl);
    IncArgs a = make_args(r, s, r.n, 0);  // m = 0: the splice copies the order and sets the ranks
    rc = inc_run(E, s, a);
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
    dfree(rank);
    dfree(ins);
    dfree(bsum);
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
    if (r.logs.fugue) {  // (the fast path covers RGA order only)
        std::vector<uint8_t> t;
        uint64_t len = 0, dig = 0, c = 0;
        rc = replica_merge(E, r, text ? &t : nullptr, &len, &dig, nullptr, &c);
        if (rc) return rc;
        if (text) *text = std::move(t);
        if (bytes) *bytes = len;
        if (cps) *cps = c;
        return CRDT_HIP_OK;
    }
    ICHK(hipSetDevice(E.device), "hipSetDevice");
    bool fast = s.valid && r.n >= s.n && r.n - s.n <= kIncMax;
    if (fast) {
        rc = inc_reserve(E, s, r.n, r.vis_bytes);  // (grows keeping the order)
        if (rc) return rc;
        fast = s.valid && r.n + 1ull <= s.cap;
    }
    if (fast) {
        IncArgs a = make_args(r, s, s.n, r.n - s.n);
        rc = inc_run(E, s, a);
        if (rc) return rc;
        if (s.hres[0] == 0) {
            if (s.hres[1] != r.vis_bytes || s.hres[2] != r.vis_cp) {
                E.err = "incremental merge disagrees with the replica's counters";
                s.valid = false;
                return CRDT_HIP_EBADLOG;
            }
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
