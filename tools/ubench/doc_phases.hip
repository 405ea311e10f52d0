// Microbenchmark of the latencies that shape k_doctree (one 1024-thread workgroup per CU, 256
// workgroups, s_memtime cycles measured by thread 0 of each workgroup, median over workgroups):
//   barrier      cycles per __syncthreads with 16 waves (loop of 64)
//   chain        cycles per step of a dependent LDS pointer chase (x = lds[x]), every lane of
//                every wave chasing its own random cycle
//   chain_alu    the same with ~24 dependent VALU ops per step (a walk step's arithmetic)
//   chain_wave1  one wave chasing alone (the others waiting at the barrier)
//   phase12      one "offsets-like" phase: 12 independent LDS reads + 12 dependent ones + ALU per
//                thread, then a barrier (cycles per phase, loop of 32)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int T = 1024;
constexpr int N = 16384;  // u32 LDS cells (64 KiB)

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

__global__ __launch_bounds__(T) void k_bench(const uint32_t* __restrict__ perm, uint64_t* out,
                                            int steps) {
    __shared__ uint32_t L[N];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < N; i += T) L[i] = perm[i];
    __syncthreads();
    const uint64_t c_start = clk(), w_start = wall_clock64();
    uint64_t r[5];
    // barrier
    uint64_t t0 = clk();
    for (int i = 0; i < 64; ++i) __syncthreads();
    uint64_t t1 = clk();
    r[0] = (t1 - t0) / 64;
    // dependent chain, every lane
    uint32_t x = (t * 7919u) % N;
    __syncthreads();
    t0 = clk();
    for (int i = 0; i < steps; ++i) x = L[x];
    __syncthreads();
    t1 = clk();
    r[1] = (t1 - t0) / steps;
    // chain + dependent ALU (24 ops)
    uint32_t y = x % N, acc = t;
    __syncthreads();
    t0 = clk();
    for (int i = 0; i < steps; ++i) {
        uint32_t v = L[y];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc = (acc ^ v) + 0x9E3779B1u;
            acc = (acc >> 3) | (acc << 29);
            v = v * 5u + 1u;
        }
        y = (v ^ (acc & 0)) % N;
    }
    __syncthreads();
    t1 = clk();
    r[2] = (t1 - t0) / steps;
    // one wave alone
    uint32_t z = x % N;
    __syncthreads();
    t0 = clk();
    if (t < 64)
        for (int i = 0; i < steps; ++i) z = L[z];
    __syncthreads();
    t1 = clk();
    r[3] = (t1 - t0) / steps;
    // offsets-like phase
    uint32_t s = 0;
    __syncthreads();
    t0 = clk();
    for (int rep = 0; rep < 32; ++rep) {
        uint32_t a[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) a[j] = L[(t + j * T + rep) % N];
#pragma unroll
        for (int j = 0; j < 12; ++j) s += L[a[j] % N] + (a[j] & 0x3FFFFu);
        __syncthreads();
    }
    t1 = clk();
    r[4] = (t1 - t0) / 32;
    // pure VALU: one dependent chain per lane, all 16 waves (cycles per op)
    uint32_t q = t;
    __syncthreads();
    t0 = clk();
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %0, %0, %1" : "+v"(q) : "v"(t));
    }
    __syncthreads();
    t1 = clk();
    const uint64_t dep16 = (t1 - t0) / (64 * 32);
    // the same chain on 4 waves only (one per SIMD)
    uint32_t q4 = t;
    __syncthreads();
    t0 = clk();
    if ((t >> 6) < 4) {
#pragma unroll 1
        for (int i = 0; i < 64; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %0, %0, %1" : "+v"(q4) : "v"(t));
        }
    }
    __syncthreads();
    t1 = clk();
    const uint64_t dep4 = (t1 - t0) / (64 * 32);
    // four independent chains per lane, 16 waves
    uint32_t a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3;
    __syncthreads();
    t0 = clk();
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t"
                         "v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %4\n\tv_xor_b32 %2, %2, %4\n\tv_xor_b32 %3, %3, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(t));
    }
    __syncthreads();
    t1 = clk();
    const uint64_t ind16 = (t1 - t0) / (64 * 32);
    // a chain through v_cmp / v_cndmask (VALU writing and reading an SGPR mask), 16 waves
    uint32_t c = t;
    __syncthreads();
    t0 = clk();
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(c) : "v"(t) : "vcc");
    }
    __syncthreads();
    t1 = clk();
    const uint64_t sel16 = (t1 - t0) / (64 * 16);
    if (t == 0) {
        out[2048 + blockIdx.x * 4 + 0] = dep16;
        out[2048 + blockIdx.x * 4 + 1] = dep4;
        out[2048 + blockIdx.x * 4 + 2] = ind16;
        out[2048 + blockIdx.x * 4 + 3] = sel16;
        out[blockIdx.x * 8 + 7] ^= q + q4 + a0 + a1 + a2 + a3 + c;
    }
    if (t == 0) {
        for (int k = 0; k < 5; ++k) out[blockIdx.x * 8 + k] = r[k];
        out[blockIdx.x * 8 + 7] = x + y + z + s + acc;
        out[blockIdx.x * 8 + 5] = clk() - c_start;
        out[blockIdx.x * 8 + 6] = wall_clock64() - w_start;
    }
}

int main() {
    std::vector<uint32_t> perm(N);
    // one random cycle over all cells (Sattolo)
    for (int i = 0; i < N; ++i) perm[i] = i;
    uint64_t st = 12345;
    for (int i = N - 1; i > 0; --i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        int j = (int)((st >> 33) % (uint64_t)i);
        std::swap(perm[i], perm[j]);
    }
    uint32_t* dp;
    uint64_t* dout;
    hipMalloc(&dp, N * 4);
    hipMalloc(&dout, (256 * 8 + 256 * 4) * 8);
    hipMemcpy(dp, perm.data(), N * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_bench, dim3(256), dim3(T), 0, 0, dp, dout, 200);
        hipDeviceSynchronize();
    }
    std::vector<uint64_t> out(256 * 8 + 256 * 4);
    hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
    const char* names[5] = {"barrier", "chain", "chain_alu", "chain_wave1", "phase12"};
    for (int k = 0; k < 5; ++k) {
        std::vector<uint64_t> v(256);
        for (int b = 0; b < 256; ++b) v[b] = out[b * 8 + k];
        std::sort(v.begin(), v.end());
        std::printf("%-12s median %llu cycles (min %llu max %llu)\n", names[k],
                    (unsigned long long)v[128], (unsigned long long)v[0], (unsigned long long)v[255]);
    }
    const char* n2[4] = {"dep_op_16w", "dep_op_4w", "indep_op_16w", "select_step_16w"};
    for (int k = 0; k < 4; ++k) {
        std::vector<uint64_t> v(256);
        for (int b = 0; b < 256; ++b) v[b] = out[2048 + b * 4 + k];
        std::sort(v.begin(), v.end());
        std::printf("%-16s median %llu cycles per op (wave-op time on its SIMD)\n", n2[k],
                    (unsigned long long)v[128]);
    }
    std::printf("clock: %.2f GHz (block 0: %llu cycles in %llu x 10 ns)\n",
                (double)out[5] / (double)out[6] / 10.0, (unsigned long long)out[5],
                (unsigned long long)out[6]);
    return 0;
}
