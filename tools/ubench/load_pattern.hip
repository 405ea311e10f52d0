// Microbenchmark: per-lane contiguous 64 B (4 x dwordx4 at lane stride 64 B) vs lane-interleaved
// dwordx4 (lane stride 16 B) streaming reads, 2 GiB of u32, one u32 written per thread.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_contig(const uint32_t* __restrict__ in, uint32_t* out, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t * 16 >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(in + t * 16);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { uint4 v = p[q]; s += v.x ^ v.y ^ v.z ^ v.w; }
    out[t] = s;
}
__global__ __launch_bounds__(256) void k_inter(const uint32_t* __restrict__ in, uint32_t* out, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t wbase = (t >> 6) * 1024, lane = t & 63;
    if (wbase >= n) return;
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = *reinterpret_cast<const uint4*>(in + wbase + q * 256 + lane * 4);
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[t] = s;
}
// contiguous per lane, staged through LDS (coalesced global loads, transposed in LDS)
__global__ __launch_bounds__(256) void k_lds(const uint32_t* __restrict__ in, uint32_t* out, uint64_t n) {
    __shared__ uint32_t sm[4][1024 + 64];
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t wbase = (t >> 6) * 1024;
    if (wbase >= n) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = *reinterpret_cast<const uint4*>(in + wbase + q * 256 + lane * 4);
        const uint32_t i = q * 256 + lane * 4;
        const uint32_t pi = i + (i >> 4);  // pad 1 dword per 16
        sm[w][pi] = v.x; sm[w][pi + 1] = v.y; sm[w][pi + 2] = v.z; sm[w][pi + 3] = v.w;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += sm[w][lane * 17 + k] ^ k;
    out[t] = s;
}
// scattered atomicOr on a bit array (5% of slots), sequential reads
__global__ __launch_bounds__(256) void k_atom(const uint32_t* __restrict__ in, uint32_t* bits, uint64_t n, uint32_t span) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t wbase = (t >> 6) * 1024, lane = t & 63;
    if (wbase >= n) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = *reinterpret_cast<const uint4*>(in + wbase + q * 256 + lane * 4);
        uint32_t a[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4; ++j) {
            if ((a[j] & 31) == 0) {
                uint64_t tgt = (wbase & ~(uint64_t)(span - 1)) + (a[j] >> 5) % span;
                atomicOr(&bits[tgt >> 5], 1u << (tgt & 31));
            }
        }
    }
}

// two u32 arrays + one u8 array, classify-like: per-lane contiguous 16 slots
__global__ __launch_bounds__(256) void k_contig3(const uint32_t* __restrict__ in, const uint32_t* __restrict__ in2,
                                                 const uint8_t* __restrict__ in3, uint32_t* out, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t * 16 >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(in + t * 16);
    const uint4* p2 = reinterpret_cast<const uint4*>(in2 + t * 16);
    const uint4 d = *reinterpret_cast<const uint4*>(in3 + t * 16);
    uint32_t s = d.x ^ d.y ^ d.z ^ d.w;
#pragma unroll
    for (int q = 0; q < 4; ++q) { uint4 v = p[q]; uint4 w = p2[q]; s += v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.y ^ w.z ^ w.w; }
    out[t] = s;
}
// same, lane-interleaved u32 loads
__global__ __launch_bounds__(256) void k_inter3(const uint32_t* __restrict__ in, const uint32_t* __restrict__ in2,
                                                const uint8_t* __restrict__ in3, uint32_t* out, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t wbase = (t >> 6) * 1024, lane = t & 63;
    if (wbase >= n) return;
    const uint4 d = *reinterpret_cast<const uint4*>(in3 + t * 16);
    uint32_t s = d.x ^ d.y ^ d.z ^ d.w;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = *reinterpret_cast<const uint4*>(in + wbase + q * 256 + lane * 4);
        uint4 w = *reinterpret_cast<const uint4*>(in2 + wbase + q * 256 + lane * 4);
        s += v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.y ^ w.z ^ w.w;
    }
    out[t] = s;
}

int main() {
    const uint64_t n = 512ull << 20;  // 512 Mi u32 = 2 GiB
    uint32_t *in, *out, *bits, *in2;
    uint8_t* in3;
    hipMalloc(&in, n * 4); hipMalloc(&out, n / 16 * 4); hipMalloc(&bits, n / 8 + 64);
    hipMalloc(&in2, n * 4); hipMalloc(&in3, n);
    hipMemset(in2, 1, n * 4); hipMemset(in3, 0, n);
    // fill with pseudo-random words
    {
        uint32_t* h = (uint32_t*)malloc(64 << 20);
        uint64_t x = 88172645463325252ull;
        for (uint64_t i = 0; i < (16u << 20); ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint32_t)x; }
        for (uint64_t o = 0; o < n; o += 16u << 20) hipMemcpy(in + o, h, 64 << 20, hipMemcpyHostToDevice);
        free(h);
    }
    hipMemset(bits, 0, n / 8 + 64);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const uint32_t grid = (uint32_t)(n / 16 / 256);
    const char* names[] = {"contig64B", "interleaved16B", "lds_transpose", "atomicOr_5pct_span256K",
                           "contig3 (9 B/slot)", "inter3 (9 B/slot)"};
    const double bytes[] = {4, 4, 4, 4, 9, 9};
    for (int k = 0; k < 6; ++k) {
        float best = 1e9;
        for (int it = 0; it < 6; ++it) {
            hipEventRecord(e0);
            if (k == 0) k_contig<<<grid, 256>>>(in, out, n);
            if (k == 1) k_inter<<<grid, 256>>>(in, out, n);
            if (k == 2) k_lds<<<grid, 256>>>(in, out, n);
            if (k == 3) k_atom<<<grid, 256>>>(in, bits, n, 1u << 18);
            if (k == 4) k_contig3<<<grid, 256>>>(in, in2, in3, out, n);
            if (k == 5) k_inter3<<<grid, 256>>>(in, in2, in3, out, n);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (it) best = ms < best ? ms : best;
        }
        printf("%-24s %8.3f ms  %7.1f GB/s\n", names[k], best, n * bytes[k] / best / 1e6);
    }
    return 0;
}
