// ilp_bench.hip -- register-only compression throughput of one vs two independent messages per lane (the
// instruction-level parallelism a hashing wave offers its SIMD), at a fixed occupancy.  No memory traffic in the
// loop: message words come from the lane id and the block counter.  Every wave also reads the shader clock
// (clock64) and the 100 MHz constant clock (wall_clock64) around its loop, so each line reports the clock the
// SIMDs ran at and, from the event time, a SIMD's cycles per 64 lane-blocks (one wave-block).  The
// k_dep lines time one wave per SIMD running dependent / independent chains of single instructions: the issue
// cycles of one wave64 instruction and the latency a dependent one waits.
//   hipcc -O3 --offload-arch=gfx950 -I dispersy_amd/csrc tools/ilp_bench.hip -o tools/ilp_bench && tools/ilp_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dsy_hash.h"

using namespace dsy;

template <class H, int CH, int WAVES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
k_ilp(uint32_t nblocks, uint32_t* out, unsigned long long* clk) {
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    H st[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) st[c].init();
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t base[CH][16];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) base[c][i] = lane * 0x9e3779b9u + (2u * i + 1u) * 0x85ebca6bu + c;
    for (uint32_t b = 0; b < nblocks; ++b) {
        uint32_t w[CH][16];
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int i = 0; i < 16; ++i) w[c][i] = base[c][i] ^ b;  // one full-rate op per word
        if constexpr (CH == 1) {
            st[0].compress(w[0]);
        } else {
            st[0].compress(w[0]);
            st[1].compress(w[1]);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) x ^= st[c].h[0] ^ st[c].h[1];
    if (x == 0x12345678u) out[lane] = x;
    const unsigned long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = w1 - w0;
    }
}

// One wave per SIMD: CHAINS independent chains of one instruction, 64 deep each per iteration.
template <int OP, int CHAINS>
__global__ void __launch_bounds__(256) k_dep(uint32_t iters, uint32_t* out, unsigned long long* clk) {
    uint32_t a[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = threadIdx.x * 0x9e3779b9u + c;
    const uint32_t y = threadIdx.x ^ 0x5bd1e995u, z = 7;
    const unsigned long long c0 = clock64();
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 64 / CHAINS; ++u)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) {
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(y));
                else if (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(y), "v"(z));
                else if (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[c]) : "v"(y), "v"(z));
                else asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(y), "v"(z));
            }
    }
    const unsigned long long c1 = clock64();
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x ^= a[c];
    if (x == 0x12345678u) out[threadIdx.x] = x;
    if (threadIdx.x == 0) clk[blockIdx.x] = c1 - c0;
}

template <int OP, int CHAINS>
static void run_dep(const char* name) {
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    unsigned long long* clk;
    hipMalloc(&out, 256 * 4);
    hipMalloc(&clk, (size_t)cus * 8);
    const uint32_t iters = 2048;
    k_dep<OP, CHAINS><<<cus, 256>>>(8, out, clk);
    k_dep<OP, CHAINS><<<cus, 256>>>(iters, out, clk);
    hipDeviceSynchronize();
    unsigned long long h[1024];
    hipMemcpy(h, clk, (size_t)cus * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < cus; ++i) s += (double)h[i];
    printf("dep      %-14s chains/wave %d, 1 wave/SIMD: %.2f shader cycles per wave64 instruction\n", name, CHAINS,
           s / cus / (64.0 * iters));
    hipFree(out);
    hipFree(clk);
}

template <class H, int CH, int WAVES>
static void run(const char* name, uint32_t ops_per_block) {
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t blocks = cus * WAVES;  // WAVES workgroups of 4 waves per CU = WAVES waves per SIMD
    const uint32_t nb = 4096 / CH;
    uint32_t* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&clk, (size_t)blocks * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_ilp<H, CH, WAVES><<<blocks, 256>>>(8, out, clk);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k_ilp<H, CH, WAVES><<<blocks, 256>>>(nb, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double blk = 5.0 * blocks * 256 * (double)nb * CH;
    unsigned long long h[2 * 256 * 8];
    hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost);
    double cyc = 0, wall = 0;
    for (uint32_t i = 0; i < blocks; ++i) cyc += (double)h[2 * i], wall += (double)h[2 * i + 1];
    const double ghz = cyc / wall * 0.1;  // wall_clock64 ticks at 100 MHz
    // a SIMD's cycles per 64 lane-blocks from the event time at the measured clock (grid-wide, so it does not assume
    // that every workgroup of the grid is resident at once)
    const double simd_cycles = ghz * 1e9 * 4.0 * cus / (blk / (ms * 1e-3) / 64.0);
    printf("%-8s chains/lane %d waves/SIMD %d: %.1f Gblk/s = %.1f T canonical ops/s (%.3f of 78.64); %.2f GHz, "
           "%.0f SIMD cycles per 64 lane-blocks\n", name, CH, WAVES, blk / (ms * 1e-3) / 1e9,
           blk * ops_per_block / (ms * 1e-3) / 1e12, blk * ops_per_block / (ms * 1e-3) / 1e12 / 78.64, ghz,
           simd_cycles);
    hipFree(out);
    hipFree(clk);
}

int main() {
    run_dep<0, 1>("v_add_u32");
    run_dep<0, 8>("v_add_u32");
    run_dep<2, 1>("v_bitop3_b32");
    run_dep<2, 8>("v_bitop3_b32");
    run_dep<1, 1>("v_alignbit_b32");
    run_dep<1, 8>("v_alignbit_b32");
    run_dep<3, 1>("v_add3_u32");
    run_dep<3, 8>("v_add3_u32");
    run<Md5, 1, 1>("md5", 500);
    run<Md5, 1, 2>("md5", 500);
    run<Md5, 1, 3>("md5", 500);
    run<Md5, 2, 1>("md5", 500);
    run<Md5, 1, 4>("md5", 500);
    run<Md5, 2, 4>("md5", 500);
    run<Md5, 1, 8>("md5", 500);
    run<Md5, 2, 2>("md5", 500);
    run<Sha1, 1, 4>("sha1", 961);
    run<Sha1, 2, 4>("sha1", 961);
    run<Sha1, 1, 8>("sha1", 961);
    run<Sha1, 2, 2>("sha1", 961);
    return 0;
}
