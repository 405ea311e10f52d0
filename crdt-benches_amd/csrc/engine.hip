// engine.hip — gfx950 kernels of the merge path and their host orchestration.
//
// Replaces diamond-types' OpLog::checkout_tip (/root/reference/src/rope.rs:134-136): anchor
// op log -> merged document.  Document order is the RGA order: pre-order of the tree
// item -> children (children = items whose origin_left is the item), siblings by (lamport,
// agent) descending.  Pipeline per wave:
//   count   k_count      child count per parent                      (atomics, L2-local)
//   scan    k_scan_*     exclusive scan of counts -> segment starts    (DPP wave scans)
//   place   k_place      children scattered into parent segments
//   link    k_link       sibling order (inline for <= 2 children), first-child / next-sibling
//           k_sortmid    wave-per-segment rank sort (3..64 children, ds_permute/shuffles)
//           k_sortbig    workgroup bitonic sort (> 64 children; LDS <= 4096, else global)
//   walk1   k_walk1      Euler-tour sublist sums from every splitter (node id % M == 0)
//   rank    k_pred/k_winit/k_wstep  prefix ranks of the splitter lists (pointer jumping)
//   walk2   k_doctotals + k_walk2   re-walk; every visible item's UTF-8 lands at its offset
//   digest  k_leafhash + k_docdigest  xxh64 tree digest per document
// The Euler tour is never materialised: succ(down v) = down(first_child v) or up v;
// succ(up v) = down(next_sibling v) or up(parent v).  Weighted list ranking (down arc of a
// visible item = its UTF-8 length, every other arc 0) yields each item's byte offset directly,
// which fuses the tombstone scan and compaction into the ranking.
#include "engine.hpp"

#include <algorithm>
#include <cstring>

#include "util.hpp"

namespace crdt {

namespace {

constexpr uint32_t kNil = 0xFFFFFFFFu;
constexpr uint32_t kVis = 0x80000000u;   // meta: visible item
constexpr uint32_t kItem = 0x40000000u;  // meta: real item (not the document-start node)
constexpr uint32_t kCpMask = 0x001FFFFFu;
constexpr int kBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;
constexpr uint32_t kLeaf = 4096;
constexpr int kMidGrid = 2048;
constexpr int kBigGrid = 256;
constexpr int kBigThreads = 1024;
constexpr int kBigLds = 4096;

enum Stage { S_COUNT, S_SCAN, S_PLACE, S_LINK, S_WALK1, S_RANK, S_WALK2, S_DIGEST, S_N };

struct WaveArgs {
    uint32_t nslots, log2m, ndocs, S;
    uint32_t step_limit;
    const uint32_t* chunk_doc;
    const uint2* docs;  // {wave-relative base slot, n}
    const uint32_t* in_parent;
    const uint32_t* in_lamport;
    const uint16_t* in_agent;
    const uint8_t* in_deleted;
    const uint32_t* in_cp;
    uint32_t* deg;
    uint32_t* cstart;
    uint32_t* child;
    uint2* dn;  // {first_child, meta}
    uint2* up;  // {next_sibling, parent}
    uint32_t* defer;
    uint32_t* bigl;
    uint32_t* ctl;  // [0] deferred segments, [1] big segments, [2] error bits
    uint32_t* sw;
    uint32_t* snext;
    uint32_t* tlen;
    uint32_t* icnt;  // items reached by walk2, per document (reachability check)
    uint64_t* toff;
    uint32_t* loff;
    uint64_t* leafh;
    uint64_t* dig;
    uint8_t* text;
    uint64_t text_cap;
};

// ---------------------------------------------------------------------------------------------
// wave / block primitives
// ---------------------------------------------------------------------------------------------
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xf, false);
}
// Inclusive wave64 prefix sum with DPP: row_shr 1,2,4,8 inside 16-lane rows, then
// row_bcast:15 and row_bcast:31 carry across rows (GFX9 DPP, valid on gfx950).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x = dpp_add<0x111, 0xf>(x);
    x = dpp_add<0x112, 0xf>(x);
    x = dpp_add<0x114, 0xf>(x);
    x = dpp_add<0x118, 0xf>(x);
    x = dpp_add<0x142, 0xa>(x);
    x = dpp_add<0x143, 0xc>(x);
    return x;
}

// Exclusive scan over the block's threads (NW waves); returns the block total in `total`.
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* lds, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(x);
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        uint32_t t = lds[i];
        off += (i < (int)w) ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return off + inc - x;
}

__device__ __forceinline__ uint32_t utf8_len(uint32_t c) {
    return c < 0x80u ? 1u : c < 0x800u ? 2u : c < 0x10000u ? 3u : 4u;
}

__device__ __forceinline__ uint64_t sib_key(const WaveArgs& a, uint32_t c) {
    return ((uint64_t)a.in_lamport[c] << 16) | (uint64_t)a.in_agent[c];
}

__device__ __forceinline__ uint2 doc_of(const WaveArgs& a, uint32_t g) {
    return a.docs[a.chunk_doc[g >> a.log2m]];
}

// ---------------------------------------------------------------------------------------------
// count / scan / place
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_count(WaveArgs a) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.nslots) return;
    const uint2 doc = doc_of(a, g);
    const uint32_t local = g - doc.x;
    if (local - 1u >= doc.y) return;  // document-start node or padding
    uint32_t p = a.in_parent[g];
    if (p > doc.y || p == local) { atomicOr(&a.ctl[2], 1u); p = 0; }
    atomicAdd(&a.deg[doc.x + p], 1u);
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

__global__ __launch_bounds__(kBlock) void k_place(WaveArgs a) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.nslots) return;
    const uint2 doc = doc_of(a, g);
    const uint32_t local = g - doc.x;
    if (local - 1u >= doc.y) return;
    uint32_t p = a.in_parent[g];
    if (p > doc.y || p == local) p = 0;  // flagged by k_count
    const uint32_t gp = doc.x + p;
    // decrementing restores deg[] to all-zero for the next wave (no memset needed)
    const uint32_t r = atomicSub(&a.deg[gp], 1u) - 1u;
    a.child[a.cstart[gp] + r] = g;
}

// ---------------------------------------------------------------------------------------------
// link: sibling order -> first_child / next_sibling
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_link(WaveArgs a) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= a.nslots) return;
    const uint2 doc = doc_of(a, g);
    const uint32_t local = g - doc.x;
    if (local > doc.y) return;  // padding
    uint32_t meta = 0;
    if (local != 0) {
        meta = (a.in_cp[g] & kCpMask) | kItem | (a.in_deleted[g] ? 0u : kVis);
    } else {
        a.up[g] = make_uint2(kNil, kNil);  // document start: no sibling, no parent
    }
    const uint32_t s0 = a.cstart[g], cnt = a.cstart[g + 1] - s0;
    uint32_t fc = kNil;
    if (cnt == 1) {
        const uint32_t c0 = a.child[s0];
        fc = c0;
        a.up[c0] = make_uint2(kNil, g);
    } else if (cnt == 2) {
        uint32_t c0 = a.child[s0], c1 = a.child[s0 + 1];
        if (sib_key(a, c0) < sib_key(a, c1)) { uint32_t t = c0; c0 = c1; c1 = t; }
        fc = c0;
        a.up[c0] = make_uint2(c1, g);
        a.up[c1] = make_uint2(kNil, g);
    } else if (cnt > 2) {
        a.defer[atomicAdd(&a.ctl[0], 1u)] = g;  // first_child written by the sort kernels
    }
    a.dn[g] = make_uint2(fc, meta);
}

// One wave per deferred segment of 3..64 children: rank = #siblings with a greater key, then
// ds_permute scatters ids into rank order and shuffles hand each lane its successor.
__global__ __launch_bounds__(kBlock) void k_sortmid(WaveArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * kBlock) >> 6;
    const uint32_t nd = a.ctl[0];
    for (uint32_t i = (blockIdx.x * kBlock + threadIdx.x) >> 6; i < nd; i += nw) {
        const uint32_t p = a.defer[i];
        const uint32_t s0 = a.cstart[p], cnt = a.cstart[p + 1] - s0;
        if (cnt > 64) {
            if (lane == 0) a.bigl[atomicAdd(&a.ctl[1], 1u)] = p;
            continue;
        }
        const bool on = lane < cnt;
        const uint32_t c = on ? a.child[s0 + lane] : 0u;
        const uint64_t k = on ? sib_key(a, c) : 0ull;
        const uint32_t khi = (uint32_t)(k >> 32), klo = (uint32_t)k;
        uint32_t rank = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t hj = (uint32_t)__shfl((int)khi, (int)j);
            const uint32_t lj = (uint32_t)__shfl((int)klo, (int)j);
            rank += (hj > khi) || (hj == khi && lj > klo);
        }
        // lane r <- id of rank r
        const uint32_t sorted =
            (uint32_t)__builtin_amdgcn_ds_permute((int)((on ? rank : lane) << 2), (int)c);
        const uint32_t succ = (uint32_t)__shfl((int)sorted, (int)((lane + 1) & 63));
        const uint32_t ns_of_rank = (lane + 1 < cnt) ? succ : kNil;
        const uint32_t ns = (uint32_t)__shfl((int)ns_of_rank, (int)(on ? rank : 0));
        if (on) {
            a.up[c] = make_uint2(ns, p);
            if (rank == 0) a.dn[p].x = c;
        }
    }
}

// Bitonic sort (descending by key) of one sibling segment with the "flip" formulation: every
// compare-exchange has the same direction, so the virtual -inf padding up to a power of two
// never has to be stored.
__global__ __launch_bounds__(kBigThreads) void k_sortbig(WaveArgs a) {
    __shared__ uint64_t skey[kBigLds];
    __shared__ uint32_t sid[kBigLds];
    const uint32_t nb = a.ctl[1];
    for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
        const uint32_t p = a.bigl[bi];
        const uint32_t s0 = a.cstart[p], cnt = a.cstart[p + 1] - s0;
        uint32_t P = 1;
        while (P < cnt) P <<= 1;
        uint32_t* seg = a.child + s0;
        if (P <= (uint32_t)kBigLds) {
            for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) {
                sid[i] = seg[i];
                skey[i] = sib_key(a, seg[i]);
            }
            __syncthreads();
            for (uint32_t k = 2; k <= P; k <<= 1) {
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t t = threadIdx.x; t < P / 2; t += kBigThreads) {
                        const uint32_t i = (t / j) * 2 * j + (t % j);
                        const uint32_t l = (j == (k >> 1)) ? (i ^ (k - 1)) : (i ^ j);
                        if (l < cnt && skey[i] < skey[l]) {
                            uint64_t tk = skey[i]; skey[i] = skey[l]; skey[l] = tk;
                            uint32_t ti = sid[i]; sid[i] = sid[l]; sid[l] = ti;
                        }
                    }
                    __syncthreads();
                }
            }
            for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) seg[i] = sid[i];
            __syncthreads();
        } else {
            for (uint32_t k = 2; k <= P; k <<= 1) {
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t t = threadIdx.x; t < P / 2; t += kBigThreads) {
                        const uint32_t i = (t / j) * 2 * j + (t % j);
                        const uint32_t l = (j == (k >> 1)) ? (i ^ (k - 1)) : (i ^ j);
                        if (l < cnt) {
                            const uint32_t ci = seg[i], cl = seg[l];
                            if (sib_key(a, ci) < sib_key(a, cl)) { seg[i] = cl; seg[l] = ci; }
                        }
                    }
                    __syncthreads();
                }
            }
        }
        for (uint32_t i = threadIdx.x; i < cnt; i += kBigThreads) {
            const uint32_t c = seg[i];
            a.up[c] = make_uint2(i + 1 < cnt ? seg[i + 1] : kNil, p);
        }
        if (threadIdx.x == 0) a.dn[p].x = seg[0];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Euler-tour walks (sublist list ranking).  Splitters: both arcs of every node whose wave slot
// is a multiple of M (every document-start node is one).  Splitter s <-> node (s>>1)<<log2m,
// arc (s&1) (0 = down, 1 = up).
// ---------------------------------------------------------------------------------------------
template <bool ORDER>
__device__ __forceinline__ uint32_t arc_weight(uint32_t meta) {
    if (ORDER) return (meta >> 30) & 1u;
    return (meta & kVis) ? utf8_len(meta & kCpMask) : 0u;
}

template <bool ORDER>
__global__ __launch_bounds__(kBlock) void k_walk1(WaveArgs a) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= a.S) return;
    const uint32_t m = a.log2m, mask = (1u << m) - 1u;
    uint32_t v = (s >> 1) << m;
    bool up = s & 1u;
    uint32_t sum = 0, steps = 0, nxt = kNil;
    for (;;) {
        uint32_t nv;
        bool nup;
        if (!up) {
            const uint2 r = a.dn[v];
            sum += arc_weight<ORDER>(r.y);
            if (r.x != kNil) { nv = r.x; nup = false; } else { nv = v; nup = true; }
        } else {
            const uint2 r = a.up[v];
            if (r.x != kNil) { nv = r.x; nup = false; }
            else if (r.y != kNil) { nv = r.y; nup = true; }
            else break;  // up arc of the document start: end of this document's tour
        }
        if ((nv & mask) == 0) { nxt = ((nv >> m) << 1) | (nup ? 1u : 0u); break; }
        v = nv;
        up = nup;
        if (++steps > a.step_limit) { atomicOr(&a.ctl[2], 2u); break; }
    }
    a.sw[s] = sum;
    a.snext[s] = nxt;
}

// pred[] <- reverse links of the splitter lists (pred pre-filled with kNil).
__global__ __launch_bounds__(kBlock) void k_pred(const uint32_t* __restrict__ snext, uint32_t S,
                                                  uint32_t* __restrict__ pred) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    const uint32_t nx = snext[s];
    if (nx != kNil) pred[nx] = s;
}
__global__ __launch_bounds__(kBlock) void k_winit(const uint32_t* __restrict__ sw,
                                                   const uint32_t* __restrict__ pred, uint32_t S,
                                                   uint32_t* __restrict__ val,
                                                   uint32_t* __restrict__ ptr) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    const uint32_t p = pred[s];
    val[s] = p != kNil ? sw[p] : 0u;
    ptr[s] = p;
}
// One pointer-jumping round: val = exclusive prefix over the splitter list so far.
__global__ __launch_bounds__(kBlock) void k_wstep(const uint32_t* __restrict__ vin,
                                                   const uint32_t* __restrict__ pin, uint32_t S,
                                                   uint32_t* __restrict__ vout,
                                                   uint32_t* __restrict__ pout) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= S) return;
    const uint32_t p = pin[s];
    uint32_t v = vin[s], q = kNil;
    if (p != kNil) {
        v += vin[p];
        q = pin[p];
    }
    vout[s] = v;
    pout[s] = q;
}

// Single workgroup: per-document length, 16-aligned text offsets, leaf offsets.
template <bool ORDER>
__global__ __launch_bounds__(1024) void k_doctotals(WaveArgs a, const uint32_t* __restrict__ spref) {
    __shared__ uint64_t st[1024];
    __shared__ uint32_t sl[1024];
    uint64_t carry_t = 0;
    uint32_t carry_l = 0;
    for (uint32_t d0 = 0; d0 < a.ndocs; d0 += 1024) {
        const uint32_t d = d0 + threadIdx.x;
        uint32_t tl = 0;
        if (d < a.ndocs) {
            const uint2 doc = a.docs[d];
            tl = ORDER ? doc.y : spref[((doc.x >> a.log2m) << 1) | 1u];
            a.tlen[d] = tl;
        }
        const uint64_t sz = ORDER ? (uint64_t)tl : (((uint64_t)tl + 15u) & ~15ull);
        const uint32_t nl = ORDER ? 0u : (tl + kLeaf - 1u) / kLeaf;
        st[threadIdx.x] = sz;
        sl[threadIdx.x] = nl;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scans
            const uint64_t xt = threadIdx.x >= o ? st[threadIdx.x - o] : 0ull;
            const uint32_t xl = threadIdx.x >= o ? sl[threadIdx.x - o] : 0u;
            __syncthreads();
            st[threadIdx.x] += xt;
            sl[threadIdx.x] += xl;
            __syncthreads();
        }
        if (d < a.ndocs) {
            a.toff[d] = carry_t + st[threadIdx.x] - sz;
            a.loff[d] = carry_l + sl[threadIdx.x] - nl;
        }
        carry_t += st[1023];
        carry_l += sl[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        a.toff[a.ndocs] = carry_t;
        a.loff[a.ndocs] = carry_l;
        if (carry_t > a.text_cap) atomicOr(&a.ctl[2], 4u);
    }
}

template <bool ORDER>
__global__ __launch_bounds__(kBlock) void k_walk2(WaveArgs a, const uint32_t* __restrict__ spref) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= a.S) return;
    if (a.ctl[2] & 4u) return;  // text capacity exceeded: never write out of bounds
    const uint32_t m = a.log2m, mask = (1u << m) - 1u;
    uint32_t v = (s >> 1) << m;
    bool up = s & 1u;
    const uint32_t d = a.chunk_doc[v >> m];
    const uint64_t obase = a.toff[d];
    const uint64_t lim = a.toff[d + 1] - obase;  // this document's own output range
    const uint32_t docbase = a.docs[d].x;
    uint32_t off = spref[s];
    uint32_t steps = 0, items = 0;
    uint8_t* __restrict__ text = a.text;
    uint32_t* __restrict__ order = reinterpret_cast<uint32_t*>(a.text);
    for (;;) {
        uint32_t nv;
        bool nup;
        if (!up) {
            const uint2 r = a.dn[v];
            const uint32_t meta = r.y;
            items += (meta >> 30) & 1u;
            if (ORDER) {
                if (meta & kItem) {
                    if (off >= lim) { atomicOr(&a.ctl[2], 8u); break; }
                    order[obase + off++] = v - docbase;
                }
            } else if (meta & kVis) {
                const uint32_t c = meta & kCpMask;
                if (off + (uint64_t)utf8_len(c) > lim) {
                    atomicOr(&a.ctl[2], 8u);
                    break;
                }
                uint8_t* o = text + obase + off;
                if (c < 0x80u) {
                    o[0] = (uint8_t)c;
                    off += 1;
                } else if (c < 0x800u) {
                    o[0] = (uint8_t)(0xC0u | (c >> 6));
                    o[1] = (uint8_t)(0x80u | (c & 63u));
                    off += 2;
                } else if (c < 0x10000u) {
                    o[0] = (uint8_t)(0xE0u | (c >> 12));
                    o[1] = (uint8_t)(0x80u | ((c >> 6) & 63u));
                    o[2] = (uint8_t)(0x80u | (c & 63u));
                    off += 3;
                } else {
                    o[0] = (uint8_t)(0xF0u | (c >> 18));
                    o[1] = (uint8_t)(0x80u | ((c >> 12) & 63u));
                    o[2] = (uint8_t)(0x80u | ((c >> 6) & 63u));
                    o[3] = (uint8_t)(0x80u | (c & 63u));
                    off += 4;
                }
            }
            if (r.x != kNil) { nv = r.x; nup = false; } else { nv = v; nup = true; }
        } else {
            const uint2 r = a.up[v];
            if (r.x != kNil) { nv = r.x; nup = false; }
            else if (r.y != kNil) { nv = r.y; nup = true; }
            else break;
        }
        if ((nv & mask) == 0) break;
        v = nv;
        up = nup;
        if (++steps > a.step_limit) { atomicOr(&a.ctl[2], 2u); break; }
    }
    if (items) atomicAdd(&a.icnt[d], items);
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

__global__ __launch_bounds__(kBlock) void k_leafhash(WaveArgs a, uint32_t leaf_cap) {
    const uint32_t L = blockIdx.x * kBlock + threadIdx.x;
    if (L >= leaf_cap || L >= a.loff[a.ndocs]) return;
    uint32_t lo = 0, hi = a.ndocs;  // last d with loff[d] <= L
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.loff[mid] <= L) lo = mid; else hi = mid;
    }
    const uint32_t d = lo, j = L - a.loff[d];
    const uint32_t tl = a.tlen[d];
    const uint32_t len = min(kLeaf, tl - j * kLeaf);
    a.leafh[L] = xxh64_aligned(a.text + a.toff[d] + (uint64_t)j * kLeaf, len, 0);
}

__global__ __launch_bounds__(kBlock) void k_docdigest(WaveArgs a, bool hash) {
    const uint32_t d = blockIdx.x * kBlock + threadIdx.x;
    if (d >= a.ndocs) return;
    if (a.icnt[d] != a.docs[d].y) atomicOr(&a.ctl[2], 16u);  // unreachable items: a cycle
    if (!hash) return;
    const uint32_t l0 = a.loff[d], l1 = a.loff[d + 1];
    a.dig[d] = xxh64_aligned(reinterpret_cast<const uint8_t*>(a.leafh + l0), (l1 - l0) * 8u,
                             a.tlen[d]);
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

__global__ __launch_bounds__(kBlock) void k_replicate(
    const uint32_t* __restrict__ bp, const uint32_t* __restrict__ bl,
    const uint16_t* __restrict__ ba, const uint8_t* __restrict__ bd,
    const uint32_t* __restrict__ bc, uint64_t src, uint32_t* __restrict__ rp,
    uint32_t* __restrict__ rl, uint16_t* __restrict__ ra, uint8_t* __restrict__ rd,
    uint32_t* __restrict__ rc, uint64_t dst, Perm P) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x + 1;
    if (k > P.n) return;
    const uint64_t o = dst + perm_apply(P, k);
    rp[o] = perm_apply(P, bp[src + k]);
    rl[o] = bl[src + k];
    ra[o] = ba[src + k];
    rd[o] = bd[src + k];
    rc[o] = bc[src + k];
}

template <class T>
hipError_t dalloc(T** p, uint64_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}
template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}
inline uint32_t grid_for(uint64_t n, uint32_t block = kBlock) {
    return (uint32_t)((n + block - 1) / block);
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
    dfree(parent); dfree(lamport); dfree(agent); dfree(deleted); dfree(cp);
    dfree(docs_rel); dfree(chunk_doc);
    cap_slots = cap_docs = cap_chunks = 0;
}

Engine::~Engine() {
    if (stream) (void)hipStreamSynchronize(stream);
    dfree(deg_); dfree(cstart_); dfree(child_); dfree(defer_); dfree(bigl_); dfree(scan_sums_);
    dfree(ctl_); dfree(dn_); dfree(up_); dfree(sw_); dfree(snext_); dfree(pred_); dfree(v0_);
    dfree(v1_); dfree(p0_); dfree(p1_); dfree(tlen_); dfree(icnt_); dfree(loff_); dfree(toff_); dfree(dig_);
    dfree(leafh_); dfree(text_);
    if (host_ctl_) (void)hipHostFree(host_ctl_);
    if (host_dig_) (void)hipHostFree(host_dig_);
    if (host_len_) (void)hipHostFree(host_len_);
    for (hipEvent_t e : ev_) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
}

int Engine::fail(const char* what, hipError_t e) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();
    return CRDT_HIP_EDEVICE;
}

#define HIPCHK(expr, what)                         \
    do {                                           \
        hipError_t _e = (expr);                    \
        if (_e != hipSuccess) return fail(what, _e); \
    } while (0)

std::string Engine::init(int dev) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return std::string("no HIP device: ") + hipGetErrorString(e);
    if (dev < 0 || dev >= n) return "device index out of range";
    device = dev;
    if ((e = hipSetDevice(dev)) != hipSuccess) return hipGetErrorString(e);
    if ((e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)) != hipSuccess)
        return hipGetErrorString(e);
    ev_.resize(2 * S_N + 2);
    for (hipEvent_t& x : ev_)
        if ((e = hipEventCreate(&x)) != hipSuccess) return hipGetErrorString(e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&host_ctl_), 64)) != hipSuccess)
        return hipGetErrorString(e);
    return "";
}

int Engine::plan(DeviceLogs& L, const std::vector<DocInfo>& docs) {
    const uint64_t M = 1ull << log2m;
    L.log2m = log2m;
    L.docs = docs;
    L.doc_slot.resize(docs.size());
    L.waves.clear();
    L.items = 0;
    uint64_t slot = 0;
    const uint64_t hard_max = (1ull << 31) - M;
    for (uint32_t d = 0; d < docs.size(); ++d) {
        const uint64_t ds = (docs[d].n + 1 + M - 1) / M * M;
        if (ds > hard_max) { err = "document too large for one wave"; return CRDT_HIP_ERANGE; }
        if (L.waves.empty() || (uint64_t)L.waves.back().nslots + ds > max_wave_slots) {
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
        w.text_cap += (docs[d].text_cap + 15) & ~15ull;
        w.leaf_cap += (docs[d].text_cap + kLeaf - 1) / kLeaf;
        w.order_cap += docs[d].n;
        L.items += docs[d].n;
        slot += ds;
    }
    L.total_slots = slot;
    const uint64_t nchunks = slot / M;
    if (slot > L.cap_slots) {
        dfree(L.parent); dfree(L.lamport); dfree(L.agent); dfree(L.deleted); dfree(L.cp);
        HIPCHK(dalloc(&L.parent, slot), "hipMalloc logs.parent");
        HIPCHK(dalloc(&L.lamport, slot), "hipMalloc logs.lamport");
        HIPCHK(dalloc(&L.agent, slot), "hipMalloc logs.agent");
        HIPCHK(dalloc(&L.deleted, slot), "hipMalloc logs.deleted");
        HIPCHK(dalloc(&L.cp, slot), "hipMalloc logs.cp");
        L.cap_slots = slot;
    }
    if (docs.size() > L.cap_docs) {
        dfree(L.docs_rel);
        HIPCHK(dalloc(&L.docs_rel, docs.size()), "hipMalloc logs.docs");
        L.cap_docs = docs.size();
    }
    if (nchunks > L.cap_chunks) {
        dfree(L.chunk_doc);
        HIPCHK(dalloc(&L.chunk_doc, nchunks), "hipMalloc logs.chunk_doc");
        L.cap_chunks = nchunks;
    }
    return upload_tables(L);
}

int Engine::upload_tables(DeviceLogs& L) {
    const uint32_t nd = (uint32_t)L.docs.size();
    if (nd == 0) return CRDT_HIP_OK;
    std::vector<uint2> rel(nd);
    std::vector<uint32_t> local(nd);
    for (const Wave& w : L.waves)
        for (uint32_t k = 0; k < w.ndocs; ++k) {
            const uint32_t d = w.first_doc + k;
            rel[d] = make_uint2((uint32_t)(L.doc_slot[d] - w.slot0), L.docs[d].n);
            local[d] = k;
        }
    HIPCHK(hipMemcpyAsync(L.docs_rel, rel.data(), nd * sizeof(uint2), hipMemcpyHostToDevice, stream),
           "upload docs");
    uint64_t* dslot = nullptr;
    uint32_t* dlocal = nullptr;
    HIPCHK(dalloc(&dslot, nd), "hipMalloc doc_slot");
    HIPCHK(dalloc(&dlocal, nd), "hipMalloc doc_local");
    hipError_t e = hipMemcpyAsync(dslot, L.doc_slot.data(), nd * 8, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(dlocal, local.data(), nd * 4, hipMemcpyHostToDevice, stream);
    const uint64_t nchunks = L.total_slots >> L.log2m;
    if (e == hipSuccess) {
        k_chunk_doc<<<grid_for(nchunks), kBlock, 0, stream>>>(dslot, dlocal, nd, nchunks, L.log2m,
                                                              L.chunk_doc);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    dfree(dslot);
    dfree(dlocal);
    if (e != hipSuccess) return fail("chunk table", e);
    return CRDT_HIP_OK;
}

int Engine::upload(DeviceLogs& L, const crdt_hip_oplog_view* views, uint32_t n) {
    const uint64_t S = L.total_slots;
    std::vector<uint32_t> par(S, 0), lam(S, 0), c(S, 0);
    std::vector<uint16_t> ag(S, 0);
    std::vector<uint8_t> del(S, 1);
    for (uint32_t d = 0; d < n; ++d) {
        const crdt_hip_oplog_view& v = views[d];
        const uint64_t b = L.doc_slot[d] + 1;
        if (v.n == 0) continue;
        std::memcpy(&par[b], v.parent, v.n * 4ull);
        std::memcpy(&lam[b], v.lamport, v.n * 4ull);
        std::memcpy(&ag[b], v.agent, v.n * 2ull);
        std::memcpy(&del[b], v.deleted, v.n);
        std::memcpy(&c[b], v.cp, v.n * 4ull);
    }
    HIPCHK(hipMemcpy(L.parent, par.data(), S * 4, hipMemcpyHostToDevice), "upload parent");
    HIPCHK(hipMemcpy(L.lamport, lam.data(), S * 4, hipMemcpyHostToDevice), "upload lamport");
    HIPCHK(hipMemcpy(L.agent, ag.data(), S * 2, hipMemcpyHostToDevice), "upload agent");
    HIPCHK(hipMemcpy(L.deleted, del.data(), S, hipMemcpyHostToDevice), "upload deleted");
    HIPCHK(hipMemcpy(L.cp, c.data(), S * 4, hipMemcpyHostToDevice), "upload cp");
    return CRDT_HIP_OK;
}

int Engine::ensure_scratch(const Wave& w, uint32_t ndocs_total) {
    const uint64_t slots = w.nslots;
    if (slots > cap_slots_) {
        dfree(deg_); dfree(cstart_); dfree(child_); dfree(defer_); dfree(bigl_);
        dfree(scan_sums_); dfree(dn_); dfree(up_);
        HIPCHK(dalloc(&deg_, slots + 16), "hipMalloc deg");
        HIPCHK(hipMemset(deg_, 0, (slots + 16) * 4), "memset deg");
        HIPCHK(dalloc(&cstart_, slots + 16), "hipMalloc cstart");
        HIPCHK(dalloc(&child_, slots), "hipMalloc child");
        HIPCHK(dalloc(&defer_, slots / 3 + 64), "hipMalloc defer");
        HIPCHK(dalloc(&bigl_, slots / 65 + 64), "hipMalloc bigl");
        HIPCHK(dalloc(&scan_sums_, slots / kScanTile + 2), "hipMalloc scan sums");
        HIPCHK(dalloc(&dn_, slots), "hipMalloc dn");
        HIPCHK(dalloc(&up_, slots), "hipMalloc up");
        cap_slots_ = slots;
    }
    if (!ctl_) HIPCHK(dalloc(&ctl_, 16), "hipMalloc ctl");
    const uint64_t S = 2 * (slots >> log2m);
    if (S > cap_splitters_) {
        dfree(sw_); dfree(snext_); dfree(pred_); dfree(v0_); dfree(v1_); dfree(p0_); dfree(p1_);
        HIPCHK(dalloc(&sw_, S), "hipMalloc sw");
        HIPCHK(dalloc(&snext_, S), "hipMalloc snext");
        HIPCHK(dalloc(&pred_, S), "hipMalloc pred");
        HIPCHK(dalloc(&v0_, S), "hipMalloc v0");
        HIPCHK(dalloc(&v1_, S), "hipMalloc v1");
        HIPCHK(dalloc(&p0_, S), "hipMalloc p0");
        HIPCHK(dalloc(&p1_, S), "hipMalloc p1");
        cap_splitters_ = S;
    }
    if (w.ndocs + 1 > cap_docs_) {
        dfree(tlen_); dfree(icnt_); dfree(loff_); dfree(toff_); dfree(dig_);
        HIPCHK(dalloc(&tlen_, w.ndocs + 1), "hipMalloc tlen");
        HIPCHK(dalloc(&icnt_, w.ndocs + 1), "hipMalloc icnt");
        HIPCHK(dalloc(&loff_, w.ndocs + 1), "hipMalloc loff");
        HIPCHK(dalloc(&toff_, w.ndocs + 1), "hipMalloc toff");
        HIPCHK(dalloc(&dig_, w.ndocs + 1), "hipMalloc dig");
        cap_docs_ = w.ndocs + 1;
    }
    const uint64_t tb = std::max<uint64_t>(w.text_cap, w.order_cap * 4) + 64;
    if (tb > cap_text_) {
        dfree(text_);
        HIPCHK(dalloc(&text_, tb), "hipMalloc text");
        cap_text_ = tb;
    }
    if (w.leaf_cap + 1 > cap_leaves_) {
        dfree(leafh_);
        HIPCHK(dalloc(&leafh_, w.leaf_cap + 1), "hipMalloc leaf hashes");
        cap_leaves_ = w.leaf_cap + 1;
    }
    if (ndocs_total > cap_host_docs_) {
        if (host_dig_) (void)hipHostFree(host_dig_);
        if (host_len_) (void)hipHostFree(host_len_);
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&host_dig_), ndocs_total * 8ull), "pinned dig");
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&host_len_), ndocs_total * 4ull), "pinned len");
        cap_host_docs_ = ndocs_total;
    }
    return CRDT_HIP_OK;
}

int Engine::run_wave(DeviceLogs& L, const Wave& w, Mode mode, std::vector<float>& stage_ms,
                     std::vector<uint32_t>& stage_launches) {
    WaveArgs a{};
    a.nslots = w.nslots;
    a.log2m = log2m;
    a.ndocs = w.ndocs;
    a.S = 2 * (w.nslots >> log2m);
    a.step_limit = 2u * w.nslots + 4u;
    a.chunk_doc = L.chunk_doc + (w.slot0 >> log2m);
    a.docs = L.docs_rel + w.first_doc;
    a.in_parent = L.parent + w.slot0;
    a.in_lamport = L.lamport + w.slot0;
    a.in_agent = L.agent + w.slot0;
    a.in_deleted = L.deleted + w.slot0;
    a.in_cp = L.cp + w.slot0;
    a.deg = deg_; a.cstart = cstart_; a.child = child_; a.dn = dn_; a.up = up_;
    a.defer = defer_; a.bigl = bigl_; a.ctl = ctl_; a.sw = sw_; a.snext = snext_;
    a.tlen = tlen_; a.icnt = icnt_; a.toff = toff_; a.loff = loff_; a.leafh = leafh_; a.dig = dig_;
    a.text = text_;
    a.text_cap = mode == ORDER ? w.order_cap : cap_text_ - 64;
    const bool ord = mode == ORDER;
    const uint32_t gs = grid_for(w.nslots), gS = grid_for(a.S);
    const uint32_t nb = (uint32_t)((w.nslots + kScanTile - 1) / kScanTile);
    hipStream_t s = stream;

#define REC(i) HIPCHK(hipEventRecord(ev_[i], s), "event record")
    HIPCHK(hipMemsetAsync(ctl_, 0, 64, s), "memset ctl");
    HIPCHK(hipMemsetAsync(icnt_, 0, w.ndocs * 4ull, s), "memset icnt");
    REC(0);
    k_count<<<gs, kBlock, 0, s>>>(a);
    REC(1);
    k_scan_reduce<<<nb, kBlock, 0, s>>>(deg_, w.nslots, scan_sums_);
    k_scan_top<<<1, 1024, 0, s>>>(scan_sums_, nb, cstart_, w.nslots);
    k_scan_apply<<<nb, kBlock, 0, s>>>(deg_, w.nslots, scan_sums_, cstart_);
    REC(2);
    k_place<<<gs, kBlock, 0, s>>>(a);
    REC(3);
    k_link<<<gs, kBlock, 0, s>>>(a);
    k_sortmid<<<kMidGrid, kBlock, 0, s>>>(a);
    k_sortbig<<<kBigGrid, kBigThreads, 0, s>>>(a);
    REC(4);
    if (ord) k_walk1<true><<<gS, kBlock, 0, s>>>(a);
    else k_walk1<false><<<gS, kBlock, 0, s>>>(a);
    REC(5);
    HIPCHK(hipMemsetAsync(pred_, 0xFF, a.S * 4ull, s), "memset pred");
    k_pred<<<gS, kBlock, 0, s>>>(snext_, a.S, pred_);
    k_winit<<<gS, kBlock, 0, s>>>(sw_, pred_, a.S, v0_, p0_);
    const uint32_t rounds = ceil_log2(std::max<uint32_t>(w.max_splitters_per_doc, 2));
    uint32_t *vi = v0_, *pi = p0_, *vo = v1_, *po = p1_;
    for (uint32_t r = 0; r < rounds; ++r) {
        k_wstep<<<gS, kBlock, 0, s>>>(vi, pi, a.S, vo, po);
        std::swap(vi, vo);
        std::swap(pi, po);
    }
    const uint32_t* spref = vi;
    REC(6);
    if (ord) {
        k_doctotals<true><<<1, 1024, 0, s>>>(a, spref);
        k_walk2<true><<<gS, kBlock, 0, s>>>(a, spref);
    } else {
        k_doctotals<false><<<1, 1024, 0, s>>>(a, spref);
        k_walk2<false><<<gS, kBlock, 0, s>>>(a, spref);
    }
    REC(7);
    if (!ord) k_leafhash<<<grid_for(w.leaf_cap + 1), kBlock, 0, s>>>(a, (uint32_t)(w.leaf_cap + 1));
    k_docdigest<<<grid_for(w.ndocs), kBlock, 0, s>>>(a, !ord);
    REC(8);
#undef REC
    HIPCHK(hipGetLastError(), "kernel launch");
    HIPCHK(hipMemcpyAsync(host_len_ + w.first_doc, tlen_, w.ndocs * 4ull, hipMemcpyDeviceToHost, s),
           "copy lens");
    if (!ord)
        HIPCHK(hipMemcpyAsync(host_dig_ + w.first_doc, dig_, w.ndocs * 8ull, hipMemcpyDeviceToHost, s),
               "copy digests");
    HIPCHK(hipMemcpyAsync(host_ctl_, ctl_, 16, hipMemcpyDeviceToHost, s), "copy ctl");
    HIPCHK(hipStreamSynchronize(s), "merge wave");
    static const int stage_of_interval[8] = {S_COUNT, S_SCAN, S_PLACE, S_LINK,
                                             S_WALK1, S_RANK, S_WALK2, S_DIGEST};
    static const uint32_t launches[8] = {1, 3, 1, 3, 1, 0, 2, 2};
    for (int i = 0; i < 8; ++i) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ev_[i], ev_[i + 1]), "event time");
        stage_ms[stage_of_interval[i]] += ms;
        stage_launches[stage_of_interval[i]] += launches[i];
    }
    stage_launches[S_RANK] += 2 + rounds;
    if (host_ctl_[2]) {
        (void)hipMemset(deg_, 0, (cap_slots_ + 16) * 4);  // restore the all-zero invariant
        err = "malformed op log detected on device (flags " + std::to_string(host_ctl_[2]) + ")";
        return CRDT_HIP_EBADLOG;
    }
    return CRDT_HIP_OK;
}

int Engine::merge(DeviceLogs& L, Mode mode, uint64_t* digests, uint64_t* lens, crdt_hip_stats* st,
                  std::vector<uint8_t>* text_out, std::vector<uint64_t>* text_offsets) {
    HIPCHK(hipSetDevice(device), "hipSetDevice");
    if ((text_out || text_offsets) && L.waves.size() > 1) {
        err = "text output needs a single-wave merge";
        return CRDT_HIP_EINVAL;
    }
    std::vector<float> stage_ms(S_N, 0.f);
    std::vector<uint32_t> stage_launches(S_N, 0);
    const uint32_t ndocs = (uint32_t)L.docs.size();
    HIPCHK(hipEventRecord(ev_[2 * S_N], stream), "event record");
    for (const Wave& w : L.waves) {
        int rc = ensure_scratch(w, ndocs);
        if (rc) return rc;
        rc = run_wave(L, w, mode, stage_ms, stage_launches);
        if (rc) return rc;
        if (text_out) {
            uint64_t total = 0;
            std::vector<uint64_t> offs(w.ndocs + 1);
            HIPCHK(hipMemcpy(offs.data(), toff_, (w.ndocs + 1) * 8ull, hipMemcpyDeviceToHost),
                   "copy offsets");
            total = offs[w.ndocs] * (mode == ORDER ? 4 : 1);
            text_out->resize(total);
            if (total)
                HIPCHK(hipMemcpy(text_out->data(), text_, total, hipMemcpyDeviceToHost), "copy text");
            if (text_offsets) *text_offsets = offs;
        }
    }
    HIPCHK(hipEventRecord(ev_[2 * S_N + 1], stream), "event record");
    HIPCHK(hipEventSynchronize(ev_[2 * S_N + 1]), "event sync");
    uint64_t text_bytes = 0;
    for (uint32_t d = 0; d < ndocs; ++d) {
        if (lens) lens[d] = host_len_[d];
        if (digests) digests[d] = host_dig_[d];
        text_bytes += host_len_[d];
    }
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->items = L.items;
        st->docs = ndocs;
        st->text_bytes = text_bytes;
        st->waves = (uint32_t)L.waves.size();
        st->nstages = S_N;
        for (int i = 0; i < S_N; ++i) {
            st->stage_ns[i] = (uint64_t)((double)stage_ms[i] * 1e6);
            st->stage_launches[i] = stage_launches[i];
        }
        float tot = 0;
        HIPCHK(hipEventElapsedTime(&tot, ev_[2 * S_N], ev_[2 * S_N + 1]), "event time");
        st->total_ns = (uint64_t)((double)tot * 1e6);
    }
    return CRDT_HIP_OK;
}

int Engine::replicate(DeviceLogs& B, DeviceLogs& R, uint32_t replicas, uint32_t relabel,
                      uint64_t seed) {
    const uint32_t nb = (uint32_t)B.docs.size();
    if (nb == 0) { err = "no base logs"; return CRDT_HIP_EINVAL; }
    std::vector<DocInfo> docs;
    const uint64_t total = (uint64_t)nb * replicas;
    if (total > 0xFFFFFFFFull) { err = "too many documents"; return CRDT_HIP_ERANGE; }
    docs.reserve(total);
    for (uint64_t r = 0; r < total; ++r) docs.push_back(B.docs[r % nb]);
    int rc = plan(R, docs);
    if (rc) return rc;
    for (uint64_t r = 0; r < total; ++r) {
        const uint32_t b = (uint32_t)(r % nb);
        const uint32_t n = B.docs[b].n;
        if (n == 0) continue;
        Perm P{};
        P.kind = relabel;
        P.n = n;
        P.bits = std::max<uint32_t>(2, ceil_log2(n));
        const uint64_t h = mix64(seed, r);
        P.shift = (uint32_t)(h % n);
        for (int k = 0; k < 3; ++k) {
            P.mul[k] = (uint32_t)mix64(h, 2 * k) | 1u;
            P.add[k] = (uint32_t)mix64(h, 2 * k + 1);
        }
        k_replicate<<<grid_for(n), kBlock, 0, stream>>>(
            B.parent, B.lamport, B.agent, B.deleted, B.cp, B.doc_slot[b], R.parent, R.lamport,
            R.agent, R.deleted, R.cp, R.doc_slot[r], P);
    }
    HIPCHK(hipGetLastError(), "replicate launch");
    HIPCHK(hipStreamSynchronize(stream), "replicate");
    return CRDT_HIP_OK;
}

}  // namespace crdt
