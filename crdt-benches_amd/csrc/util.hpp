// util.hpp — small host helpers shared by the engine's host code: UTF-8, xxh64, splitmix64.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>

namespace crdt {

constexpr uint32_t NIL = 0xFFFFFFFFu;

// Caching allocator (util.cpp) for device blocks and pinned host blocks up to 256 MiB: freed
// blocks are kept per device and power-of-two size class and handed out again, so objects made
// and dropped every step (the downstream loop clones a replica, applies a batch, merges and
// drops it) do not pay hipMalloc / hipFree each time.  pool_free synchronises the device before
// caching a block, as hipFree would, so a cached block is never still in use by queued work.
hipError_t pool_alloc(void** p, size_t bytes, bool host = false);
// synced: the caller has already waited for every use of the block (no device wait here)
void pool_free(void* p, bool host = false, bool synced = false);

inline size_t utf8_len_cp(uint32_t c) { return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4; }

inline size_t utf8_put(uint32_t c, char* o) {
    if (c < 0x80) { o[0] = (char)c; return 1; }
    if (c < 0x800) { o[0] = (char)(0xC0 | (c >> 6)); o[1] = (char)(0x80 | (c & 63)); return 2; }
    if (c < 0x10000) {
        o[0] = (char)(0xE0 | (c >> 12)); o[1] = (char)(0x80 | ((c >> 6) & 63));
        o[2] = (char)(0x80 | (c & 63));
        return 3;
    }
    o[0] = (char)(0xF0 | (c >> 18)); o[1] = (char)(0x80 | ((c >> 12) & 63));
    o[2] = (char)(0x80 | ((c >> 6) & 63)); o[3] = (char)(0x80 | (c & 63));
    return 4;
}

// Decode UTF-8 into codepoints (appends).  Returns false on malformed input.
template <class Vec>
bool utf8_decode(const char* s, size_t n, Vec& out) {
    const unsigned char* p = (const unsigned char*)s;
    size_t i = 0;
    while (i < n) {
        uint32_t c = p[i];
        size_t k;
        if (c < 0x80) k = 1;
        else if ((c >> 5) == 6) { k = 2; c &= 0x1F; }
        else if ((c >> 4) == 14) { k = 3; c &= 0x0F; }
        else if ((c >> 3) == 30) { k = 4; c &= 0x07; }
        else return false;
        if (i + k > n) return false;
        for (size_t j = 1; j < k; ++j) {
            if ((p[i + j] & 0xC0) != 0x80) return false;
            c = (c << 6) | (p[i + j] & 63);
        }
        out.push_back(c);
        i += k;
    }
    return true;
}

inline size_t utf8_count(const char* s, size_t n) {
    size_t c = 0;
    for (size_t i = 0; i < n; ++i) c += ((unsigned char)s[i] & 0xC0) != 0x80;
    return c;
}

__host__ __device__ inline uint64_t splitmix64(uint64_t& state) {
    uint64_t z = (state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// Counter-based variant (identical on host and device): hash of (seed, i).
__host__ __device__ inline uint64_t mix64(uint64_t seed, uint64_t i) {
    uint64_t s = seed ^ (i * 0xD1B54A32D192ED03ULL);
    return splitmix64(s);
}

uint64_t xxh64(const void* data, size_t len, uint64_t seed);
uint64_t tree_digest(const uint8_t* text, size_t len);

}  // namespace crdt
