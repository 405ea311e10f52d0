// wave.hpp — wave64 / workgroup primitives shared by the gfx950 kernels (engine.hip,
// replica.hip).  Header-only, internal linkage.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "util.hpp"

namespace crdt {
namespace {

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
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63);
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

// ---- device memory (host side) ----
template <class T>
hipError_t dalloc(T** p, uint64_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    return pool_alloc(reinterpret_cast<void**>(p), count * sizeof(T));
}
template <class T>
void dfree(T*& p) {
    pool_free(p);
    p = nullptr;
}
inline uint32_t grid_for(uint64_t n, uint32_t block = 256) {
    return (uint32_t)((n + block - 1) / block);
}

}  // namespace
}  // namespace crdt
