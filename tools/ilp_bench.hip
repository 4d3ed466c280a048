// ilp_bench.hip -- register-only compression throughput of one vs two independent messages per lane (the
// instruction-level parallelism a hashing wave offers its SIMD), at a fixed occupancy.  No memory traffic in the
// loop: message words come from the lane id and the block counter.
//   hipcc -O3 --offload-arch=gfx950 -I dispersy_amd/csrc tools/ilp_bench.hip -o tools/ilp_bench && tools/ilp_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dsy_hash.h"

using namespace dsy;

template <class H, int CH, int WAVES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
k_ilp(uint32_t nblocks, uint32_t* out) {
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
}

template <class H, int CH, int WAVES>
static void run(const char* name, uint32_t ops_per_block) {
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t blocks = cus * WAVES;  // WAVES workgroups of 4 waves per CU = WAVES waves per SIMD
    const uint32_t nb = 4096 / CH;
    uint32_t* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_ilp<H, CH, WAVES><<<blocks, 256>>>(8, out);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k_ilp<H, CH, WAVES><<<blocks, 256>>>(nb, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double blk = 5.0 * blocks * 256 * (double)nb * CH;
    printf("%-8s chains/lane %d waves/SIMD %d: %.1f Gblk/s = %.1f T canonical ops/s (%.3f of 78.64)\n", name, CH, WAVES,
           blk / (ms * 1e-3) / 1e9, blk * ops_per_block / (ms * 1e-3) / 1e12,
           blk * ops_per_block / (ms * 1e-3) / 1e12 / 78.64);
    hipFree(out);
}

int main() {
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
