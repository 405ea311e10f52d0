// util.cpp — host xxh64 (published XXH64 algorithm) and the document tree digest.
#include "util.hpp"

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace crdt {

namespace {
constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL,
                   P3 = 0x165667B19E3779F9ULL, P4 = 0x85EBCA77C2B2AE63ULL,
                   P5 = 0x27D4EB2F165667C5ULL;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t load64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
inline uint32_t load32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t round1(uint64_t acc, uint64_t x) { return rotl(acc + x * P2, 31) * P1; }
inline uint64_t merge1(uint64_t acc, uint64_t v) { return (acc ^ round1(0, v)) * P1 + P4; }
}  // namespace

uint64_t xxh64(const void* data, size_t len, uint64_t seed) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    const uint8_t* const end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
        for (; end - p >= 32; p += 32)
            for (int k = 0; k < 4; ++k) v[k] = round1(v[k], load64(p + 8 * k));
        h = rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18);
        for (int k = 0; k < 4; ++k) h = merge1(h, v[k]);
    } else {
        h = seed + P5;
    }
    h += len;
    for (; end - p >= 8; p += 8) h = rotl(h ^ round1(0, load64(p)), 27) * P1 + P4;
    if (end - p >= 4) { h = rotl(h ^ (load32(p) * P1), 23) * P2 + P3; p += 4; }
    for (; p < end; ++p) h = rotl(h ^ (*p * P5), 11) * P1;
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}

uint64_t tree_digest(const uint8_t* text, size_t len) {
    const size_t leaf = 4096;
    std::vector<uint64_t> hs((len + leaf - 1) / leaf);
    for (size_t i = 0; i < hs.size(); ++i) {
        const size_t n = std::min(leaf, len - i * leaf);
        hs[i] = xxh64(text + i * leaf, n, 0);
    }
    const size_t group = 4096;  // > 16 MiB: leaf digests hashed in groups of 4096 (seed = index)
    if (hs.size() > group) {
        std::vector<uint64_t> gs((hs.size() + group - 1) / group);
        for (size_t k = 0; k < gs.size(); ++k)
            gs[k] = xxh64(hs.data() + k * group, std::min(group, hs.size() - k * group) * 8, k);
        hs.swap(gs);
    }
    return xxh64(hs.data(), hs.size() * 8, (uint64_t)len);
}

namespace {
constexpr size_t kPoolMaxBlock = 256ull << 20;  // larger blocks go straight to HIP
constexpr size_t kPoolMaxCached = 4ull << 30;   // bytes kept per pool

struct Pool {
    std::mutex mu;
    std::unordered_map<void*, uint64_t> live;                 // pooled block -> key
    std::unordered_map<uint64_t, std::vector<void*>> cached;  // key -> free blocks
    size_t cached_bytes = 0;
};

Pool& pool(bool host) {
    static Pool dev, hst;
    return host ? hst : dev;
}

size_t size_class(size_t bytes) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    return c;
}

hipError_t raw_alloc(void** p, size_t bytes, bool host) {
    return host ? hipHostMalloc(p, bytes) : hipMalloc(p, bytes);
}
void raw_free(void* p, bool host) { (void)(host ? hipHostFree(p) : hipFree(p)); }

// Return every cached block to HIP (on an allocation failure).
void drain(Pool& P, bool host) {
    std::vector<void*> blocks;
    {
        std::lock_guard<std::mutex> g(P.mu);
        for (auto& kv : P.cached)
            for (void* b : kv.second) blocks.push_back(b);
        P.cached.clear();
        P.cached_bytes = 0;
    }
    for (void* b : blocks) raw_free(b, host);
}
}  // namespace

hipError_t pool_alloc(void** p, size_t bytes, bool host) {
    *p = nullptr;
    if (bytes > kPoolMaxBlock) return raw_alloc(p, bytes, host);
    int dev = 0;
    if (!host) (void)hipGetDevice(&dev);
    const size_t c = size_class(bytes);
    const uint64_t key = ((uint64_t)dev << 48) | c;
    Pool& P = pool(host);
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.cached.find(key);
        if (it != P.cached.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            P.cached_bytes -= c;
            P.live[*p] = key;
            return hipSuccess;
        }
    }
    hipError_t e = raw_alloc(p, c, host);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        drain(P, host);
        e = raw_alloc(p, c, host);
    }
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    std::lock_guard<std::mutex> g(P.mu);
    P.live[*p] = key;
    return hipSuccess;
}

void pool_free(void* p, bool host, bool synced) {
    if (!p) return;
    Pool& P = pool(host);
    uint64_t key = 0;
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.live.find(p);
        if (it != P.live.end()) {
            key = it->second;
            P.live.erase(it);
        }
    }
    if (!key) {  // not pooled (a large block)
        raw_free(p, host);
        return;
    }
    if (!synced) (void)hipDeviceSynchronize();  // what hipFree would wait for
    const size_t c = (size_t)(key & ((1ull << 48) - 1));
    {
        std::lock_guard<std::mutex> g(P.mu);
        if (P.cached_bytes + c <= kPoolMaxCached) {
            P.cached[key].push_back(p);
            P.cached_bytes += c;
            return;
        }
    }
    raw_free(p, host);
}

}  // namespace crdt
