// Probe (not part of the product): does ds_read_b128 at a 4-byte-aligned LDS address return the 16 bytes at that
// address on gfx950 (HSA's unaligned mode)?  Prints OK or the first mismatch.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) lds[i] = 0x01000000u * (i & 255) + i;
    __syncthreads();
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)lds + 4 * (threadIdx.x * 13 + 1);
    uint4 v;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
    out[4 * threadIdx.x] = v.x; out[4 * threadIdx.x + 1] = v.y; out[4 * threadIdx.x + 2] = v.z; out[4 * threadIdx.x + 3] = v.w;
}
int main() {
    uint32_t* d;
    hipMalloc(&d, 4 * 4 * 64);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    std::vector<uint32_t> h(256);
    hipMemcpy(h.data(), d, 1024, hipMemcpyDeviceToHost);
    for (int t = 0; t < 64; ++t)
        for (int j = 0; j < 4; ++j) {
            const int i = t * 13 + 1 + j;
            const uint32_t want = 0x01000000u * (i & 255) + i;
            if (h[4 * t + j] != want) { printf("MISMATCH lane %d word %d got %08x want %08x\n", t, j, h[4 * t + j], want); return 1; }
        }
    printf("OK\n");
    return 0;
}
