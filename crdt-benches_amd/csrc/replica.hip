// replica.hip — device-side decode of Downstream updates into a resident replica (replica.hpp).
//
// Replaces diamond-types' decode_and_add (/root/reference/src/rope.rs:222-224) with the
// semantics of OpLog::apply_update (oplog.cpp), for a whole batch of updates per call:
//   k_upd_parse  one thread per update: header checks -> {first id, items, deletes, data
//                word offset}; per-256-update aggregates (items, deletes, largest last id)
//   k_upd_top    one workgroup: exclusive scan of the aggregates, seeded with the replica's
//                size (ids known before the batch)
//   k_upd_scan   per update: item and delete offsets in the flattened batch, ids known before
//                and after it (prefix max of last ids), causal readiness (first <= known + 1)
//   k_upd_items  per flattened item, 4 per thread: parent check; in the write pass the item's
//                fields go to slot id.  Ids known before the update are skipped, so the first
//                update carrying an id wins, exactly as in the sequential decoder
//   k_upd_dels   per flattened delete: target check; in the write pass the tombstone bit of
//                the target's codepoint word is set by atomicOr, so a target deleted twice is
//                counted once
// The check passes run before the write passes on the same stream and the write passes do
// nothing once any check failed: a rejected batch leaves the replica unchanged, and the host
// waits once per batch.  Visible codepoints / bytes are kept incrementally from the items
// written and the tombstones newly set.
#include "replica.hpp"

#include <algorithm>
#include <cstring>

#include "oplog.hpp"
#include "util.hpp"
#include "wave.hpp"

namespace crdt {
namespace {

constexpr int kUB = 256;            // threads per block (updates per block in parse / scan)
constexpr int kItemsPerThread = 1;
constexpr uint32_t kCpMaskR = 0x001FFFFFu;
constexpr uint32_t kMaxGrid = 1024;  // write passes: one counter atomic per block

// device counters (u64)
enum UCtl { U_ERR = 0, U_ITEMS, U_DELS, U_MAXID, U_ADD_CP, U_ADD_B, U_DEL_CP, U_DEL_B,
            U_PLAN,  // replay: the decode's sizes differ from the ones the merge was planned with
            U_N };
// U_ERR bits
constexpr uint64_t E_HEADER = 1, E_NOT_READY = 2, E_PARENT = 4, E_DELETE = 8, E_BOUNDS = 16,
                   E_FUGUE = 32;

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int o = 32; o; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= (uint32_t)o) x = max(x, y);
    }
    return x;
}
// Exclusive max-scan over the block (identity 0); `total` = block max.
template <int NW>
__device__ __forceinline__ uint32_t block_excl_max(uint32_t x, uint32_t* lds, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_max(x);
    if (lane == 63u) lds[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const uint32_t t = lds[i];
        off = (i < (int)w) ? max(off, t) : off;
        tot = max(tot, t);
    }
    __syncthreads();
    total = tot;
    const uint32_t prev = (uint32_t)__shfl_up((int)inc, 1);
    return max(off, lane ? prev : 0u);
}

// Sum of x over the block, valid in thread 0 (a device-wide counter then takes one atomic per
// block: thousands of same-address atomics, one per wave, serialise at the L2 and cost more
// than the decode itself).
__device__ __forceinline__ uint32_t block_sum_t0(uint32_t x, uint32_t* lds) {
    x = wave_sum(x);
    if ((threadIdx.x & 63u) == 0) lds[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t t = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kUB / 64; ++i) t += lds[i];
    __syncthreads();
    return t;
}

struct UpdArgs {
    const uint32_t* buf;  // the batch, as words (every update starts 4-aligned)
    const uint64_t* off;  // n + 1 byte offsets
    uint32_t n;
    uint64_t len;
    uint4* hdr;
    uint4* scan;
    uint4* blk;
    uint32_t nblk;
    uint32_t known0;  // items of the replica before the batch
    uint64_t* ctl;
    // replica slot arrays (slot = id)
    uint32_t* parent;
    uint64_t* key;  // lamport << 16 | agent
    uint8_t* cp;    // 3 bytes per slot: codepoint | kDelBit (cp3_put / cp3_get)
    uint64_t cap_slots;
    uint32_t* imap;  // per flattened item / delete: its update (found by the check pass, reused
    uint32_t* dmap;  //   by the write pass instead of a second binary search)
    uint32_t fugue;  // Fugue replica: version-2 updates, cp bit 31 = left child (oplog.hpp)
};

__global__ __launch_bounds__(kUB) void k_upd_parse(UpdArgs a) {
    __shared__ uint32_t l0[kUB / 64], l1[kUB / 64], l2[kUB / 64];
    const uint32_t u = blockIdx.x * kUB + threadIdx.x;
    uint32_t first = 1, nit = 0, m = 0, wo = 0;
    if (u < a.n) {
        const uint64_t o0 = a.off[u], o1 = a.off[u + 1];
        bool bad = o0 > o1 || o1 > a.len || (o0 & 3u) || o1 - o0 < 24;
        if (!bad) {
            const uint32_t* h = a.buf + (o0 >> 2);
            const uint32_t h0 = h[0], h1 = h[1], f = h[2], ni = h[3], mm = h[5];
            const uint64_t need =
                24ull + 16ull * ni + ((2ull * ni + 3ull) / 4ull) * 4ull + 4ull * mm;
            bad = h0 != kUpdateMagic ||
                  (h1 != kUpdateVersion && !(h1 == kUpdateVersionFugue && a.fugue)) ||
                  need > o1 - o0;
            if (!bad) {
                first = f;
                nit = ni;
                m = mm;
                wo = (uint32_t)(o0 >> 2) + 6u;
            }
        }
        if (bad) atomicOr((unsigned long long*)&a.ctl[U_ERR], (unsigned long long)E_HEADER);
        a.hdr[u] = make_uint4(first, nit, m, wo);
    }
    // per-block aggregates: items, deletes, largest last id (first + items - 1)
    const uint32_t last = nit ? first + nit - 1u : 0u;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t s0 = wave_sum(nit), s1 = wave_sum(m), s2 = wave_max(last);
    if (lane == 0) {
        l0[w] = s0;
        l1[w] = s1;
        l2[w] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t0 = 0, t1 = 0, t2 = 0;
        for (int i = 0; i < kUB / 64; ++i) {
            t0 += l0[i];
            t1 += l1[i];
            t2 = max(t2, l2[i]);
        }
        a.blk[blockIdx.x] = make_uint4(t0, t1, t2, 0u);
    }
}

// One workgroup: block aggregates -> exclusive prefixes (max seeded with known0), totals.
__global__ __launch_bounds__(1024) void k_upd_top(UpdArgs a) {
    __shared__ uint32_t l0[16], l1[16], l2[16];
    uint32_t c0 = 0, c1 = 0, c2 = a.known0;
    for (uint32_t base = 0; base < a.nblk; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint4 v = i < a.nblk ? a.blk[i] : make_uint4(0, 0, 0, 0);
        uint32_t t0, t1, t2;
        const uint32_t e0 = block_excl_scan<16>(v.x, l0, t0);
        const uint32_t e1 = block_excl_scan<16>(v.y, l1, t1);
        const uint32_t e2 = block_excl_max<16>(v.z, l2, t2);
        if (i < a.nblk) a.blk[i] = make_uint4(c0 + e0, c1 + e1, max(c2, e2), 0u);
        c0 += t0;
        c1 += t1;
        c2 = max(c2, t2);
    }
    if (threadIdx.x == 0) {
        a.ctl[U_ITEMS] = c0;
        a.ctl[U_DELS] = c1;
        a.ctl[U_MAXID] = c2;
    }
}

__global__ __launch_bounds__(kUB) void k_upd_scan(UpdArgs a) {
    __shared__ uint32_t l0[kUB / 64], l1[kUB / 64], l2[kUB / 64];
    const uint32_t u = blockIdx.x * kUB + threadIdx.x;
    const uint4 h = u < a.n ? a.hdr[u] : make_uint4(1, 0, 0, 0);
    const uint32_t last = h.y ? h.x + h.y - 1u : 0u;
    uint32_t t;
    const uint32_t e0 = block_excl_scan<kUB / 64>(h.y, l0, t);
    const uint32_t e1 = block_excl_scan<kUB / 64>(h.z, l1, t);
    const uint32_t e2 = block_excl_max<kUB / 64>(last, l2, t);
    if (u >= a.n) return;
    const uint4 b = a.blk[blockIdx.x];
    const uint32_t kb = max(b.z, e2);  // ids known before update u
    const uint32_t ka = max(kb, last);
    if (h.x == 0 || (uint64_t)h.x > (uint64_t)kb + 1u)
        atomicOr((unsigned long long*)&a.ctl[U_ERR], (unsigned long long)E_NOT_READY);
    a.scan[u] = make_uint4(b.x + e0, b.y + e1, kb, ka);
}

// last update u with scan[u].<field> <= j (scan[0].<field> == 0 <= j)
template <int F>
__device__ __forceinline__ uint32_t find_update(const uint4* __restrict__ scan, uint32_t n,
                                                uint32_t j) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint4 s = scan[mid];
        if ((F == 0 ? s.x : s.y) <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}

template <bool WRITE>
__global__ __launch_bounds__(kUB) void k_upd_items(UpdArgs a) {
    if (WRITE && a.ctl[U_ERR]) return;
    const uint32_t T = (uint32_t)a.ctl[U_ITEMS];
    uint32_t add_cp = 0, add_b = 0;
    uint64_t err = 0;
    const uint32_t stride = gridDim.x * kUB * kItemsPerThread;
    for (uint32_t j0 = (blockIdx.x * kUB + threadIdx.x) * kItemsPerThread; j0 < T; j0 += stride) {
        uint32_t u = WRITE ? a.imap[j0] : find_update<0>(a.scan, a.n, j0);
        uint4 h = a.hdr[u], s = a.scan[u];
#pragma unroll
        for (int q = 0; q < kItemsPerThread; ++q) {
            const uint32_t j = j0 + (uint32_t)q;
            if (j >= T) break;
            while (j >= s.x + h.y) {  // next update holding items
                ++u;
                h = a.hdr[u];
                s = a.scan[u];
            }
            if (!WRITE) a.imap[j] = u;
            const uint32_t k = j - s.x, id = h.x + k;
            if (id <= s.z) continue;  // already known (decode_and_add is idempotent)
            const uint32_t par = a.buf[h.w + k];
            if (par != 0u && par >= id) {
                err |= E_PARENT;
                continue;
            }
            const uint32_t c = a.buf[h.w + 3u * h.y + k], lam = a.buf[h.w + 2u * h.y + k];
            const bool left = a.fugue && (c & kUpdateSideBit);
            if (a.fugue && ((left && par == 0u) || lam == 0xFFFFFFFFu)) {
                err |= E_FUGUE;  // a left child of the document start, or the content-row key
                continue;
            }
            if (WRITE) {
                if ((uint64_t)id >= a.cap_slots) {
                    err |= E_BOUNDS;
                    continue;
                }
                a.parent[id] = par;
                a.key[id] = ((uint64_t)lam << 16) | (left ? kLeftKey : 0ull) |
                            reinterpret_cast<const uint16_t*>(a.buf + h.w + 4u * h.y)[k];
                // live; a left child never carries the previous-slot flag
                cp3_put(a.cp, id, (c & kCpMaskR) | (left ? kLeftBit : (par == id - 1u ? kSeqBit : 0u)));
                add_cp += 1u;
                add_b += utf8_len(c & kCpMaskR);
            }
        }
    }
    if (err) atomicOr((unsigned long long*)&a.ctl[U_ERR], (unsigned long long)err);
    if (WRITE) {
        __shared__ uint32_t red[kUB / 64];
        const uint32_t s0 = block_sum_t0(add_cp, red), s1 = block_sum_t0(add_b, red);
        if (threadIdx.x == 0 && s0) {
            atomicAdd((unsigned long long*)&a.ctl[U_ADD_CP], (unsigned long long)s0);
            atomicAdd((unsigned long long*)&a.ctl[U_ADD_B], (unsigned long long)s1);
        }
    }
}

template <bool WRITE>
__global__ __launch_bounds__(kUB) void k_upd_dels(UpdArgs a) {
    if (WRITE && a.ctl[U_ERR]) return;
    const uint32_t Dm = (uint32_t)a.ctl[U_DELS];
    uint32_t del_cp = 0, del_b = 0;
    uint64_t err = 0;
    for (uint32_t j = blockIdx.x * kUB + threadIdx.x; j < Dm; j += gridDim.x * kUB) {
        const uint32_t u = WRITE ? a.dmap[j] : find_update<1>(a.scan, a.n, j);
        if (!WRITE) a.dmap[j] = u;
        const uint4 h = a.hdr[u], s = a.scan[u];
        const uint32_t dw = h.w + 4u * h.y + (2u * h.y + 3u) / 4u;
        const uint32_t id = a.buf[dw + (j - s.y)];
        if (id == 0u || id > s.w) {  // unknown item (s.w = ids known after update u)
            err |= E_DELETE;
            continue;
        }
        if (WRITE) {
            // the tombstone bit is bit 7 of the slot's third byte: one atomic on its dword
            const uint64_t b = 3ull * id + 2u;
            const uint32_t sh = 8u * (uint32_t)(b & 3u) + 7u;
            const uint32_t old = atomicOr(reinterpret_cast<uint32_t*>(a.cp + (b & ~3ull)), 1u << sh);
            if (!((old >> sh) & 1u)) {  // newly tombstoned
                del_cp += 1u;
                del_b += utf8_len(cp3_get(a.cp, id) & kCpMaskR);
            }
        }
    }
    if (err) atomicOr((unsigned long long*)&a.ctl[U_ERR], (unsigned long long)err);
    if (WRITE) {
        __shared__ uint32_t red[kUB / 64];
        const uint32_t s0 = block_sum_t0(del_cp, red), s1 = block_sum_t0(del_b, red);
        if (threadIdx.x == 0 && s0) {
            atomicAdd((unsigned long long*)&a.ctl[U_DEL_CP], (unsigned long long)s0);
            atomicAdd((unsigned long long*)&a.ctl[U_DEL_B], (unsigned long long)s1);
        }
    }
}

// padding / unused slots: a tombstoned child of the document start with key 0 (never visible,
// pruned by the merge)
__global__ __launch_bounds__(kUB) void k_rep_pad(uint32_t* parent, uint64_t* key, uint8_t* cp,
                                                 uint64_t s0, uint64_t s1) {
    const uint64_t g = s0 + (uint64_t)blockIdx.x * kUB + threadIdx.x;
    if (g >= s1) return;
    parent[g] = 0;
    key[g] = 0;
    cp3_put(cp, g, kDelBit);
}

// Replica clone: the three slot arrays in one launch (main.rs:64); the codepoint column as the
// dwords of its padded byte size.
__global__ __launch_bounds__(kUB) void k_rep_copy(const uint32_t* __restrict__ sp,
                                                  const uint64_t* __restrict__ sk,
                                                  const uint8_t* __restrict__ sc,
                                                  uint32_t* __restrict__ dp, uint64_t* __restrict__ dk,
                                                  uint8_t* __restrict__ dc, uint64_t n) {
    // (the codepoint column's dwords number about 3/4 of the slots, or more for tiny replicas:
    // the loop runs over both)
    const uint64_t nw = cp3_bytes(n) / 4, m = nw > n ? nw : n;
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sc);
    uint32_t* dw = reinterpret_cast<uint32_t*>(dc);
    for (uint64_t g = (uint64_t)blockIdx.x * kUB + threadIdx.x; g < m; g += (uint64_t)gridDim.x * kUB) {
        if (g < n) {
            dp[g] = sp[g];
            dk[g] = sk[g];
        }
        if (g < nw) dw[g] = sw[g];
    }
}

// Replay: the sizes the enqueued merge was planned with (n items, visible bytes) against the
// ones the decode produced.
__global__ void k_replay_check(uint64_t* ctl, uint32_t n0, uint64_t bytes0, uint32_t n_plan,
                               uint64_t bytes_plan) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t n = ctl[U_MAXID] > n0 ? ctl[U_MAXID] : n0;
    const uint64_t bytes = bytes0 + ctl[U_ADD_B] - ctl[U_DEL_B];
    ctl[U_PLAN] = (n != n_plan || bytes != bytes_plan || ctl[U_ERR]) ? 1u : 0u;
}

thread_local uint64_t grow_gen = 0;  // counts grow() reallocations (replica generations)

int hip_fail(Engine& E, const char* what, hipError_t e) {
    E.err = std::string(what) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();
    return CRDT_HIP_EDEVICE;
}

#define RCHK(expr, what)                                \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(E, what, _e); \
    } while (0)

template <class T>
hipError_t grow(T** p, uint64_t& cap, uint64_t need) {
    if (need <= cap) return hipSuccess;
    ++grow_gen;
    dfree(*p);
    cap = 0;
    hipError_t e = dalloc(p, need);
    if (e == hipSuccess) cap = need;
    return e;
}

}  // namespace

Replica::~Replica() {
    for (void* p : graveyard) pool_free(p);
    dfree(ubuf);
    dfree(uoff);
    dfree(uhdr);
    dfree(uscan);
    dfree(ublk);
    dfree(imap);
    dfree(dmap);
    dfree(uctl);
    pool_free(hctl, true);
}

int replica_reserve(Engine& E, Replica& r, uint64_t items) {
    DeviceLogs& L = r.logs;
    const uint64_t need = (items + 1 + 63) / 64 * 64;
    if (need > (1ull << 31) - 64) {
        E.err = "replica too large (ids are u32 slots of one wave)";
        return CRDT_HIP_ERANGE;
    }
    if (need <= L.cap_slots) return CRDT_HIP_OK;
    const uint64_t cap = std::min<uint64_t>((1ull << 31) - 64,
                                            std::max<uint64_t>({need, 2 * L.cap_slots, 4096}));
    uint32_t* par = nullptr;
    uint8_t* c = nullptr;
    uint64_t* key = nullptr;
    hipError_t e = dalloc(&par, cap);
    if (e == hipSuccess) e = dalloc(&key, cap);
    if (e == hipSuccess) e = dalloc(&c, cp3_bytes(cap));
    const uint64_t old = L.cap_slots;
    hipStream_t s = E.stream;
    if (e == hipSuccess && old) {
        e = hipMemcpyAsync(par, L.parent, old * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(key, L.key, old * 8, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(c, L.cp, old * 3, hipMemcpyDeviceToDevice, s);
    }
    if (e == hipSuccess) {
        k_rep_pad<<<grid_for(cap - old, kUB), kUB, 0, s>>>(par, key, c, old, cap);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(s);
        dfree(par); dfree(key); dfree(c);
        return hip_fail(E, "replica reserve", e);
    }
    // the old arrays may still be read by queued work: freed at the replica's next wait
    for (void* p : {(void*)L.parent, (void*)L.key, (void*)L.cp})
        if (p) r.graveyard.push_back(p);
    L.parent = par;
    L.key = key;
    L.cp = c;
    L.cap_slots = cap;
    r.gen++;
    return CRDT_HIP_OK;
}

int replica_upload(Engine& E, Replica& r, const crdt_hip_oplog_view* v) {
    RCHK(hipSetDevice(E.device), "hipSetDevice");
    const uint32_t n = v ? v->n : 0u;
    int rc = replica_reserve(E, r, n);
    if (rc) return rc;
    r.inc.valid = false;
    r.n = n;
    r.vis_cp = r.vis_bytes = 0;
    r.version++;
    r.logs.fugue = v && v->side;  // a Fugue replica (its merges run the Fugue rows)
    if (!n) return CRDT_HIP_OK;
    DeviceLogs& L = r.logs;
    // on the engine stream, after the padding kernel replica_reserve may have queued there (a
    // null-stream copy does not wait for a non-blocking stream and could be overwritten by it)
    hipStream_t s = E.stream;
    RCHK(hipMemcpyAsync(L.parent + 1, v->parent, n * 4ull, hipMemcpyHostToDevice, s), "upload parent");
    std::vector<uint8_t> c(3ull * n);
    std::vector<uint64_t> key(n);
    for (uint32_t i = 0; i < n; ++i) {
        const bool left = v->side && v->side[i];
        if (v->side && (v->lamport[i] == 0xFFFFFFFFu || (left && v->parent[i] == 0))) {
            E.err = "invalid Fugue log (lamport 0xFFFFFFFF or a left child of the document start)";
            return CRDT_HIP_EBADLOG;
        }
        key[i] = ((uint64_t)v->lamport[i] << 16) | v->agent[i] | (left ? kLeftKey : 0ull);
        cp3_put(c.data(), i, (v->cp[i] & kCpMaskR) | (v->deleted[i] ? kDelBit : 0u) |
                                 (left ? kLeftBit : (v->parent[i] == i ? kSeqBit : 0u)));
        if (!v->deleted[i]) {
            r.vis_cp += 1;
            r.vis_bytes += utf8_len_cp(v->cp[i] & kCpMaskR);
        }
    }
    RCHK(hipMemcpyAsync(L.key + 1, key.data(), n * 8ull, hipMemcpyHostToDevice, s), "upload key");
    RCHK(hipMemcpyAsync(L.cp + 3, c.data(), c.size(), hipMemcpyHostToDevice, s), "upload cp");
    RCHK(hipStreamSynchronize(s), "upload sync");  // (key, c and the caller's view are released)
    return CRDT_HIP_OK;
}

int replica_copy(Engine& E, const Replica& src, Replica& dst) {
    RCHK(hipSetDevice(E.device), "hipSetDevice");
    dst.inc.valid = false;
    if (src.pending) {
        E.err = "replica has an unsettled decode";
        return CRDT_HIP_EINVAL;
    }
    const uint64_t cap = src.logs.cap_slots;
    int rc = replica_reserve(E, dst, cap ? cap - 1 : 0);
    if (rc) return rc;
    const DeviceLogs& S = src.logs;
    DeviceLogs& D = dst.logs;
    hipStream_t s = E.stream;
    if (cap) {
        // (no wait: every later use of the copy, decode and merge, is on the same stream)
        k_rep_copy<<<(uint32_t)std::min<uint64_t>(grid_for(cap, kUB), 4096), kUB, 0, s>>>(
            S.parent, S.key, S.cp, D.parent, D.key, D.cp, cap);
        RCHK(hipGetLastError(), "replica copy");
    }
    dst.n = src.n;
    D.fugue = S.fugue;
    dst.vis_cp = src.vis_cp;
    dst.vis_bytes = src.vis_bytes;
    dst.version++;
    return CRDT_HIP_OK;
}

int updates_upload(Engine& E, UpdateBatch& ub, const uint8_t* buf, uint64_t len,
                   const uint64_t* offsets, uint32_t n) {
    if (n && (!buf || !offsets)) {
        E.err = "null update buffer or offsets";
        return CRDT_HIP_EINVAL;
    }
    if (len >= (1ull << 32) - 16) {
        E.err = "update batch of 4 GiB or more";
        return CRDT_HIP_ERANGE;
    }
    RCHK(hipSetDevice(E.device), "hipSetDevice");
    RCHK(dalloc(&ub.buf, (len + 4) & ~3ull), "hipMalloc update buffer");
    RCHK(dalloc(&ub.off, n + 1ull), "hipMalloc update offsets");
    // on the engine's stream (the decode kernels run there; a null-stream copy would not be
    // ordered with them), waited for before the caller's buffers may go
    if (len) RCHK(hipMemcpyAsync(ub.buf, buf, len, hipMemcpyHostToDevice, E.stream), "upload updates");
    if (n)
        RCHK(hipMemcpyAsync(ub.off, offsets, (n + 1ull) * 8, hipMemcpyHostToDevice, E.stream),
             "upload offsets");
    RCHK(hipStreamSynchronize(E.stream), "upload updates");
    ub.len = len;
    ub.n = n;
    // the largest id the batch carries, from its headers (first id, items at words 2, 3); a
    // malformed header leaves it unknown (the device decoder rejects such a batch anyway)
    ub.max_id = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t o0 = offsets[i], o1 = offsets[i + 1];
        if (o0 > o1 || o1 > len || o1 - o0 < 24) {
            ub.max_id = 0;
            break;
        }
        uint32_t first, items;
        std::memcpy(&first, buf + o0 + 8, 4);
        std::memcpy(&items, buf + o0 + 12, 4);
        if (items) ub.max_id = std::max<uint32_t>(ub.max_id, first + items - 1);
    }
    return CRDT_HIP_OK;
}

UpdateBatch::~UpdateBatch() {
    dfree(buf);
    dfree(off);
}

int replica_apply(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                  const uint64_t* offsets, uint32_t n) {
    return replica_decode(E, r, buf, len, offsets, n, false);
}

int replica_apply_resident(Engine& E, Replica& r, const UpdateBatch& ub) {
    int rc = replica_settle(E, r);
    if (rc) return rc;
    rc = replica_decode_enqueue(E, r, ub.buf, ub.len, ub.off, ub.n, true, ub.max_id, true);
    if (rc) return rc;
    return replica_settle(E, r);
}

int replica_decode(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                   const uint64_t* offsets, uint32_t n, bool resident) {
    int rc = replica_settle(E, r);
    if (rc) return rc;
    rc = replica_decode_enqueue(E, r, buf, len, offsets, n, resident, 0, true);
    if (rc) return rc;
    return replica_settle(E, r);
}

// Everything a decode may allocate (or wait for), before its launches.
int decode_prepare(Engine& E, Replica& r, uint64_t len, uint32_t n, bool resident,
                   uint32_t max_id) {
    if (len >= (1ull << 32) - 16) {
        E.err = "update batch of 4 GiB or more";
        return CRDT_HIP_ERANGE;
    }
    RCHK(hipSetDevice(E.device), "hipSetDevice");
    // ids a batch can add: up to its largest id if known, else every item takes at least 16
    // bytes of it
    int rc = replica_reserve(E, r, max_id ? std::max<uint64_t>(r.n, max_id)
                                          : (uint64_t)r.n + len / 16 + 1);
    if (rc) return rc;
    const uint64_t g0 = grow_gen;
    const uint32_t nblk = (n + kUB - 1) / kUB;
    if (!resident) RCHK(grow(&r.ubuf, r.ubuf_cap, (len + 4) & ~3ull), "hipMalloc update buffer");
    if (n + 1ull > r.ucap) {
        dfree(r.uoff); dfree(r.uhdr); dfree(r.uscan);
        r.ucap = 0;
        const uint64_t c = std::max<uint64_t>(n + 1ull, 1024);
        RCHK(dalloc(&r.uoff, c), "hipMalloc update offsets");
        RCHK(dalloc(&r.uhdr, c), "hipMalloc update headers");
        RCHK(dalloc(&r.uscan, c), "hipMalloc update scan");
        r.ucap = c;
        r.gen++;
    }
    RCHK(grow(&r.ublk, r.ublk_cap, (uint64_t)nblk), "hipMalloc update blocks");
    // every item takes at least 16 bytes of the batch, every delete 4
    RCHK(grow(&r.imap, r.imap_cap, len / 16 + 1), "hipMalloc item map");
    RCHK(grow(&r.dmap, r.dmap_cap, len / 4 + 1), "hipMalloc delete map");
    if (!r.uctl) {
        RCHK(dalloc(&r.uctl, (uint64_t)U_N), "hipMalloc update counters");
        r.gen++;
    }
    if (!r.hctl) {
        RCHK(pool_alloc(reinterpret_cast<void**>(&r.hctl), U_N * 8, true), "hipHostMalloc");
        r.gen++;
    }
    if (grow_gen != g0) r.gen++;
    return CRDT_HIP_OK;
}

// The decode's launches (capturable: no allocation, no wait).
int decode_launch(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                  const uint64_t* offsets, uint32_t n, bool resident, bool copy_counters);

int replica_decode_enqueue(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                           const uint64_t* offsets, uint32_t n, bool resident, uint32_t max_id,
                           bool copy_counters) {
    if (n == 0) return CRDT_HIP_OK;
    if (!buf || !offsets) {
        E.err = "null update buffer or offsets";
        return CRDT_HIP_EINVAL;
    }
    int rc = decode_prepare(E, r, len, n, resident, max_id);
    if (rc) return rc;
    return decode_launch(E, r, buf, len, offsets, n, resident, copy_counters);
}

int decode_launch(Engine& E, Replica& r, const uint8_t* buf, uint64_t len,
                  const uint64_t* offsets, uint32_t n, bool resident, bool copy_counters) {
    if (n == 0) return CRDT_HIP_OK;
    hipStream_t s = E.stream;
    const uint32_t nblk = (n + kUB - 1) / kUB;
    if (!resident) {
        RCHK(hipMemcpyAsync(r.ubuf, buf, len, hipMemcpyHostToDevice, s), "upload updates");
        RCHK(hipMemcpyAsync(r.uoff, offsets, (n + 1ull) * 8, hipMemcpyHostToDevice, s),
             "upload update offsets");
    }
    RCHK(hipMemsetAsync(r.uctl, 0, U_N * 8, s), "memset update counters");
    DeviceLogs& L = r.logs;
    UpdArgs a{};
    a.buf = reinterpret_cast<const uint32_t*>(resident ? buf : r.ubuf);
    a.off = resident ? offsets : r.uoff;
    a.n = n;
    a.len = len;
    a.hdr = r.uhdr;
    a.scan = r.uscan;
    a.blk = r.ublk;
    a.nblk = nblk;
    a.known0 = r.n;
    a.ctl = r.uctl;
    a.parent = L.parent;
    a.key = L.key;
    a.cp = L.cp;
    a.cap_slots = L.cap_slots;
    a.imap = r.imap;
    a.dmap = r.dmap;
    a.fugue = L.fugue ? 1u : 0u;
    const uint32_t gi = std::min<uint64_t>(kMaxGrid, grid_for(len / 16 / kItemsPerThread + 1, kUB));
    const uint32_t gd = std::min<uint64_t>(kMaxGrid, grid_for(len / 4 + 1, kUB));
    k_upd_parse<<<nblk, kUB, 0, s>>>(a);
    k_upd_top<<<1, 1024, 0, s>>>(a);
    k_upd_scan<<<nblk, kUB, 0, s>>>(a);
    k_upd_items<false><<<gi, kUB, 0, s>>>(a);
    k_upd_dels<false><<<gd, kUB, 0, s>>>(a);
    k_upd_items<true><<<gi, kUB, 0, s>>>(a);
    k_upd_dels<true><<<gd, kUB, 0, s>>>(a);
    RCHK(hipGetLastError(), "update kernels");
    if (copy_counters)
        RCHK(hipMemcpyAsync(r.hctl, r.uctl, U_N * 8, hipMemcpyDeviceToHost, s), "copy update counters");
    r.pending = true;
    return CRDT_HIP_OK;
}

int replica_settle(Engine& E, Replica& r) {
    if (!r.pending && r.graveyard.empty()) return CRDT_HIP_OK;
    RCHK(hipStreamSynchronize(E.stream), "update sync");
    for (void* p : r.graveyard) pool_free(p, false, true);
    r.graveyard.clear();
    if (!r.pending) return CRDT_HIP_OK;
    r.pending = false;
    r.version++;
    const uint64_t* c = r.hctl;
    if (c[U_ERR]) {
        const uint64_t e = c[U_ERR];
        E.err = e & E_HEADER      ? "not an update, unsupported version or truncated update"
                : e & E_NOT_READY ? "update is not causally ready (missing items)"
                : e & E_PARENT    ? "update item references an unknown parent"
                : e & E_DELETE    ? "update deletes an unknown item"
                : e & E_FUGUE     ? "Fugue update item: a left child of the document start or lamport 0xFFFFFFFF"
                                  : "update writes outside the replica";
        return CRDT_HIP_EBADLOG;
    }
    r.n = (uint32_t)std::max<uint64_t>(r.n, c[U_MAXID]);
    r.vis_cp = r.vis_cp + c[U_ADD_CP] - c[U_DEL_CP];
    r.vis_bytes = r.vis_bytes + c[U_ADD_B] - c[U_DEL_B];
    return CRDT_HIP_OK;
}

int replica_merge(Engine& E, Replica& r, std::vector<uint8_t>* text, uint64_t* len,
                  uint64_t* digest, crdt_hip_stats* st, uint64_t* cps) {
    int rc = replica_settle(E, r);
    if (rc) return rc;
    rc = replica_reserve(E, r, r.n);
    if (rc) return rc;
    std::vector<DocInfo> docs{DocInfo{r.n, r.vis_bytes}};
    rc = E.plan(r.logs, docs);
    if (rc) return rc;
    // the compact list of the non-seq items, rebuilt for the decoded contents (as a resident
    // batch's input encoding builds it once)
    if ((rc = E.nsq_reserve(r.logs)) || (rc = E.nsq_launch(r.logs))) return rc;
    return E.merge(r.logs, Engine::TEXT, digest, len, st, text, nullptr, cps);
}

ReplayState::~ReplayState() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
}

namespace {
void drop_graph(ReplayState& st) {
    if (st.exec) (void)hipGraphExecDestroy(st.exec);
    if (st.graph) (void)hipGraphDestroy(st.graph);
    st.exec = nullptr;
    st.graph = nullptr;
    st.key.clear();
}
}  // namespace

int replica_replay(Engine& E, const Replica& init, const UpdateBatch& ub, ReplayState& st,
                   uint64_t* cps, uint64_t* bytes, uint64_t* digest) {
    if (st.init != &init || st.ub != &ub || st.init_version != init.version) {
        st.init = &init;
        st.ub = &ub;
        st.init_version = init.version;
        st.known = false;
        drop_graph(st);
    }
    Replica& w = st.work;
    int rc = replica_settle(E, w);
    if (rc) return rc;
    if (init.pending) {
        E.err = "replica has an unsettled decode";
        return CRDT_HIP_EINVAL;
    }
    if (st.known && E.plan_cache && ub.n && ub.buf && ub.off) {
        // ---- the sizes are known: one graph for the closure ---------------------------------
        // prepare (everything that may allocate, upload or wait), then the launches
        const uint64_t cap = init.logs.cap_slots;
        rc = replica_reserve(E, w, cap ? cap - 1 : 0);
        if (rc) return rc;
        w.n = init.n;  // the copy below
        w.inc.valid = false;
        rc = decode_prepare(E, w, ub.len, ub.n, true, ub.max_id);
        if (rc) return rc;
        // (test hook: with plan_shrink the planned sizes are off by one, forcing the fallback)
        const uint64_t b_plan = st.bytes_after + (E.plan_shrink ? 1u : 0u);
        std::vector<DocInfo> docs{DocInfo{st.n_after, b_plan}};
        rc = E.plan(w.logs, docs);
        if (rc) return rc;
        rc = E.nsq_reserve(w.logs);
        if (rc) return rc;
        if (!E.plans_known(w.logs)) {
            st.known = false;  // the shape's plan was forgotten: learn it again below
        } else {
            Engine::AsyncMerge m;
            rc = E.merge_async_prepare(w.logs, m, false);
            if (rc) return rc;
            const std::vector<uint64_t> key = {
                E.generation(), w.gen, init.gen, (uint64_t)(uintptr_t)&init, init.n, init.vis_bytes,
                cap, (uint64_t)(uintptr_t)&ub, ub.len, ub.n, st.n_after, b_plan,
                // (knobs that change what is captured: a closure captured under other settings
                // is not replayed)
                (uint64_t)E.nsq_list, (uint64_t)E.contraction, (uint64_t)E.runs_slots,
                (uint64_t)E.stile_text, (uint64_t)E.xcd_order, (uint64_t)E.text_scatter,
                (uint64_t)E.fuse_text, (uint64_t)E.lanes};
            hipStream_t s = E.stream;
            if (key != st.key || !st.exec) {
                drop_graph(st);
                RCHK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), "begin capture");
                rc = CRDT_HIP_OK;
                if (cap) {
                    const DeviceLogs& S = init.logs;
                    DeviceLogs& D = w.logs;
                    k_rep_copy<<<(uint32_t)std::min<uint64_t>(grid_for(cap, kUB), 4096), kUB, 0, s>>>(
                        S.parent, S.key, S.cp, D.parent, D.key, D.cp, cap);
                }
                if (!rc) rc = decode_launch(E, w, ub.buf, ub.len, ub.off, ub.n, true, false);
                if (!rc) {
                    k_replay_check<<<1, 64, 0, s>>>(w.uctl, init.n, init.vis_bytes, st.n_after,
                                                    b_plan);
                    if (hipMemcpyAsync(w.hctl, w.uctl, U_N * 8, hipMemcpyDeviceToHost, s) !=
                        hipSuccess)
                        rc = hip_fail(E, "copy update counters", hipGetLastError());
                }
                if (!rc) rc = E.nsq_launch(w.logs);  // (the decoded contents' nsq list)
                if (!rc) rc = E.merge_async_enqueue(w.logs, m);
                hipGraph_t g = nullptr;
                const hipError_t ce = hipStreamEndCapture(s, &g);
                if (rc) {
                    if (g) (void)hipGraphDestroy(g);
                    w.pending = false;
                    return rc;
                }
                if (ce != hipSuccess) return hip_fail(E, "end capture", ce);
                st.graph = g;
                RCHK(hipGraphInstantiate(&st.exec, g, nullptr, nullptr, 0), "graph instantiate");
                st.key = key;
            }
            w.pending = true;  // the graph holds the decode
            RCHK(hipGraphLaunch(st.exec, s), "graph launch");
            RCHK(hipStreamSynchronize(s), "replay sync");
            w.vis_cp = init.vis_cp;
            w.vis_bytes = init.vis_bytes;
            uint64_t c1 = 0, b1 = 0, d1 = 0;
            const int mrc = E.merge_async_finish(w.logs, m, &d1, &b1, &c1, nullptr);
            if (w.hctl[U_PLAN] == 0 && mrc == CRDT_HIP_OK) {
                rc = replica_settle(E, w);  // no wait left: applies the counters
                if (rc) return rc;
                if (cps) *cps = c1;
                if (bytes) *bytes = b1;
                if (digest) *digest = d1;
                return CRDT_HIP_OK;
            }
            // the sizes changed (or the batch was rejected): merge again from the decode's counts
            rc = replica_settle(E, w);
            if (rc) return rc;
            rc = replica_merge(E, w, nullptr, bytes, digest, nullptr, cps);
            if (rc) return rc;
            st.n_after = w.n;
            st.bytes_after = w.vis_bytes;
            return CRDT_HIP_OK;
        }
    }
    // ---- first replay (or sizes unknown): clone, decode, wait, merge -----------------------
    rc = replica_copy(E, init, w);  // main.rs:64
    if (rc) return rc;
    rc = replica_decode_enqueue(E, w, ub.buf, ub.len, ub.off, ub.n, true, ub.max_id, true);
    if (rc) return rc;
    rc = replica_settle(E, w);  // main.rs:65-67 (a rejected batch changes nothing)
    if (rc) return rc;
    rc = replica_merge(E, w, nullptr, bytes, digest, nullptr, cps);  // main.rs:68
    if (rc) return rc;
    st.known = true;
    st.n_after = w.n;
    st.bytes_after = w.vis_bytes;
    return CRDT_HIP_OK;
}

}  // namespace crdt
