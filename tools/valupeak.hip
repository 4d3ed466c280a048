// valupeak.hip -- measured peak of 32-bit integer VALU issue on the whole chip (the INT32 roofline denominator).
//
// Every lane runs 8 independent dependency chains of one VALU instruction (inline asm, so the compiler can neither
// fold nor reorder them); 256 threads per workgroup, 2 or 8 workgroups per CU.  Reported: lane-ops/s and the
// implied lane-ops per CU per clock at the nominal 2.4 GHz.  Not part of the product; built and run by hand:
//   hipcc -O3 --offload-arch=gfx950 tools/valupeak.hip -o tools/valupeak && tools/valupeak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));       \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

enum Op { kAdd = 0, kXor, kAlign, kAdd3, kBfi, kBitop3, kXad, kMix, kAlignConst, kRotConst, kAddLit, kAdd3S, kPerm, kLshlOr, kLshl64, kLshlAdd64, kMov64, kCndmask, kNOps };
static const char* kNames[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_add3_u32", "v_bfi_b32",
                               "v_bitop3_b32", "v_xad_u32", "mix(add3,align,bfi,xor)", "v_alignbit x,y,5",
                               "v_alignbit x,x,5 (rotate)", "v_add_u32 literal", "v_add3_u32 x,y,sgpr", "v_perm_b32",
                               "v_lshl_or_b32", "v_lshlrev_b64", "v_lshl_add_u64", "v_mov_b64", "v_cndmask_b32 (sgpr mask)"};

#define STEP3(OPSTR, X, Y, Z) asm volatile(OPSTR : "+v"(X) : "v"(Y), "v"(Z))
#define STEP2(OPSTR, X, Y) asm volatile(OPSTR : "+v"(X) : "v"(Y))

template <int OP>
__device__ __forceinline__ void step8(uint32_t* a, uint32_t y, uint32_t z) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (OP == kAdd) STEP2("v_add_u32 %0, %0, %1", a[c], y);
        else if (OP == kXor) STEP2("v_xor_b32 %0, %0, %1", a[c], y);
        else if (OP == kAlign) STEP3("v_alignbit_b32 %0, %0, %1, %2", a[c], y, z);
        else if (OP == kAdd3) STEP3("v_add3_u32 %0, %0, %1, %2", a[c], y, z);
        else if (OP == kBfi) STEP3("v_bfi_b32 %0, %0, %1, %2", a[c], y, z);
        else if (OP == kBitop3) STEP3("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", a[c], y, z);
        else if (OP == kXad) STEP3("v_xad_u32 %0, %0, %1, %2", a[c], y, z);
        else if (OP == kAlignConst) asm volatile("v_alignbit_b32 %0, %0, %1, 5" : "+v"(a[c]) : "v"(y));
        else if (OP == kRotConst) asm volatile("v_alignbit_b32 %0, %0, %0, 5" : "+v"(a[c]));
        else if (OP == kAddLit) asm volatile("v_add_u32 %0, 0x5a827999, %0" : "+v"(a[c]));
        else if (OP == kAdd3S) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(y), "s"(z));
        else if (OP == kPerm) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(y), "v"(z));
        else if (OP == kLshlOr) asm volatile("v_lshl_or_b32 %0, %0, 5, %1" : "+v"(a[c]) : "v"(y));
        else if (OP == kLshl64 || OP == kLshlAdd64 || OP == kMov64) {
            // 64-bit operands: the chain's register and the next one as a pair (c even), counted as one lane-op
            if ((c & 1) == 0) {
                uint64_t v = ((uint64_t)a[c + 1] << 32) | a[c];
                const uint64_t w = ((uint64_t)y << 32) | z;
                if (OP == kLshl64) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(v));
                else if (OP == kLshlAdd64) asm volatile("v_lshl_add_u64 %0, %0, 7, %1" : "+v"(v) : "v"(w));
                else asm volatile("v_mov_b64 %0, %1" : "+v"(v) : "v"(w));
                a[c] = (uint32_t)v;
                a[c + 1] = (uint32_t)(v >> 32);
            }
        } else if (OP == kCndmask) {
            const uint64_t m = 0x5555555555555555ull ^ z;
            asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(y), "s"(m));
        }
        else {
            if ((c & 3) == 0) STEP3("v_add3_u32 %0, %0, %1, %2", a[c], y, z);
            else if ((c & 3) == 1) STEP3("v_alignbit_b32 %0, %0, %1, %2", a[c], y, z);
            else if ((c & 3) == 2) STEP3("v_bfi_b32 %0, %0, %1, %2", a[c], y, z);
            else STEP2("v_xor_b32 %0, %0, %1", a[c], y);
        }
    }
}

template <int OP>
__global__ void __launch_bounds__(256) k_peak(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) a[c] = seed * (threadIdx.x + 1) + c * 0x9e3779b9u;
    const uint32_t y = seed ^ threadIdx.x, z = 7 + (seed & 15);
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) step8<OP>(a, y, z);
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) x ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int OP>
static double run(uint32_t* d_out, int cus, uint32_t iters, int wg_per_cu) {
    const uint32_t grid = cus * wg_per_cu;
    hipLaunchKernelGGL(k_peak<OP>, dim3(grid), dim3(256), 0, 0, d_out, iters, 3u);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_peak<OP>, dim3(grid), dim3(256), 0, 0, d_out, iters, 3u + r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double lane_ops = (double)grid * 256 * iters * 64 * reps;  // 8 unrolled x 8 chains per iteration
    return lane_ops / (ms / 1e3);
}

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? atoi(argv[1]) : 4096;
    int cus = 0, clk_khz = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    uint32_t* d_out;
    CK(hipMalloc(&d_out, (size_t)cus * 16 * 256 * 4));
    printf("CUs=%d  reported max clock=%.0f MHz  iters=%u\n", cus, clk_khz / 1e3, iters);
    for (int wg : {2, 8}) {
        double r[kNOps];
        r[0] = run<kAdd>(d_out, cus, iters, wg);
        r[1] = run<kXor>(d_out, cus, iters, wg);
        r[2] = run<kAlign>(d_out, cus, iters, wg);
        r[3] = run<kAdd3>(d_out, cus, iters, wg);
        r[4] = run<kBfi>(d_out, cus, iters, wg);
        r[5] = run<kBitop3>(d_out, cus, iters, wg);
        r[6] = run<kXad>(d_out, cus, iters, wg);
        r[7] = run<kMix>(d_out, cus, iters, wg);
        r[8] = run<kAlignConst>(d_out, cus, iters, wg);
        r[9] = run<kRotConst>(d_out, cus, iters, wg);
        r[10] = run<kAddLit>(d_out, cus, iters, wg);
        r[11] = run<kAdd3S>(d_out, cus, iters, wg);
        r[12] = run<kPerm>(d_out, cus, iters, wg);
        r[13] = run<kLshlOr>(d_out, cus, iters, wg);
        r[14] = run<kLshl64>(d_out, cus, iters, wg);
        r[15] = run<kLshlAdd64>(d_out, cus, iters, wg);
        r[16] = run<kMov64>(d_out, cus, iters, wg);
        r[17] = run<kCndmask>(d_out, cus, iters, wg);
        for (int i = 0; i < kNOps; ++i) {
            // the 64-bit rows issue 4 instructions per 8 chains: report instructions x lanes
            const double f = (i == kLshl64 || i == kLshlAdd64 || i == kMov64) ? 0.5 : 1.0;
            r[i] *= f;
            printf("wg/CU=%d %-26s %7.2f T lane-ops/s  = %6.1f lane-ops/CU/clk @2.4GHz\n", wg, kNames[i], r[i] / 1e12,
                   r[i] / cus / 2.4e9);
        }
    }
    return 0;
}
