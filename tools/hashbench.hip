// hashbench.hip -- A/B microbenchmark of per-lane message loading strategies for the digest kernels.
// Not part of the product; built and run by hand (see tools/README.md).  Each variant hashes the same packets
// (one packet per lane, MD5 or SHA-1 of prefix || packet) and XORs the digest into an output word so nothing is
// dead-code eliminated.  Variants interleave in one process (guide §5.4 rule 24).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "../dispersy_amd/csrc/dsy_message.h"

using namespace dsy;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

static uint64_t g_checksum;
enum Variant { kDirect = 0, kAlignedFake = 1, kNoLoad = 2, kAlignedFunnel = 3, kPrefetch = 4, kCoop = 5, kPure = 6, kDma = 7, kFast = 8 };

// aligned 80-byte window + register funnel shift: correct for middle blocks
__device__ __forceinline__ void load_block_funnel(const uint8_t* src, uint32_t* w) {
    const uintptr_t a = (uintptr_t)src;
    const uint4* base = (const uint4*)(a & ~(uintptr_t)15);
    const uint32_t sh = (uint32_t)(a & 15);
    uint32_t d[20];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        uint4 v = base[q];
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
    const uint32_t dw = sh >> 2, by = (sh & 3) * 8;
    uint32_t e[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) e[i] = (dw & 2) ? d[i + 2] : d[i];
    uint32_t f[17];
#pragma unroll
    for (int i = 0; i < 17; ++i) f[i] = (dw & 1) ? e[i + 1] : e[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = by ? __builtin_amdgcn_alignbyte(f[i + 1], f[i], sh & 3) : f[i];
}

template <class H, int V>
__device__ __forceinline__ void block_variant(const KeyView& kv, uint32_t b, uint32_t nb, uint32_t* w) {
    constexpr int BLK = H::block_bytes;
    const uint32_t total = kv.plen + kv.len;
    const uint32_t o0 = b * BLK;
    const bool middle = o0 >= kv.plen && o0 + BLK <= total;
    if (V == kDirect || !middle) {
        message_block<H>(kv, b, nb, w);
        return;
    }
    const uint8_t* src = kv.key + (o0 - kv.plen);
    if (V == kAlignedFake) {
        const uint4* p = (const uint4*)((uintptr_t)src & ~(uintptr_t)15);
#pragma unroll
        for (int q = 0; q < BLK / 16; ++q) {
            uint4 v = p[q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
    } else if (V == kNoLoad) {
#pragma unroll
        for (int i = 0; i < H::words; ++i) w[i] = (uint32_t)(uintptr_t)src * (i + 1);
    } else {
        load_block_funnel(src, w);
    }
    if (H::big_endian) {
#pragma unroll
        for (int i = 0; i < H::words; ++i) w[i] = bswap32(w[i]);
    }
}

template <class H>
__device__ __forceinline__ bool is_middle(const KeyView& kv, uint32_t b) {
    const uint32_t o0 = b * H::block_bytes;
    return o0 >= kv.plen && o0 + H::block_bytes <= kv.plen + kv.len;
}

// software-pipelined: the raw words of block b+1 are loaded before block b is compressed
template <class H>
__device__ __forceinline__ void hash_key_prefetch(const KeyView& kv, H& st) {
    st.init();
    const uint32_t nb = n_blocks(kv.plen + kv.len, H::block_bytes, H::len_bytes);
    uint32_t nxt[H::words];
    auto raw_load = [&](uint32_t b, uint32_t* w) {
        const uint8_t* src = kv.key + (b * H::block_bytes - kv.plen);
#pragma unroll
        for (int q = 0; q < H::block_bytes / 16; ++q) {
            uint4 v = load_u128_unaligned(src + 16 * q);
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
    };
    if (nb > 0 && is_middle<H>(kv, 0)) raw_load(0, nxt);
    for (uint32_t b = 0; b < nb; ++b) {
        uint32_t w[H::words];
        const bool mid = is_middle<H>(kv, b);
#pragma unroll
        for (int i = 0; i < H::words; ++i) w[i] = nxt[i];
        if (b + 1 < nb && is_middle<H>(kv, b + 1)) raw_load(b + 1, nxt);
        if (mid) {
            if (H::big_endian) {
#pragma unroll
                for (int i = 0; i < H::words; ++i) w[i] = bswap32(w[i]);
            }
        } else {
            message_block<H>(kv, b, nb, w);
        }
        st.compress(w);
    }
}

// cooperative wave load of one 64-byte block per lane: lane l fetches 16 B of lane (16*i + l/4)'s block in
// instruction i, so 4 consecutive lanes read one packet's contiguous 64 bytes; staged through LDS (80-byte
// lane stride: conflict-free ds_read_b128).  Global loads for block b+1 are issued before block b is hashed.
template <class H>
__device__ __forceinline__ void hash_key_coop(const KeyView& kv, H& st, uint32_t* lds) {
    static_assert(H::block_bytes == 64, "coop path is for 64-byte blocks");
    const uint32_t lane = threadIdx.x & 63;
    st.init();
    const uint32_t nb = n_blocks(kv.plen + kv.len, 64, H::len_bytes);
    // wave-wide maximum block count (lanes are sorted by nb, so this is ~nb)
    uint32_t nbmax = nb;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, d, 64));
    uint4 pf[4];
    auto issue = [&](uint32_t b) {
        const bool mid = b < nb && is_middle<H>(kv, b);
        const uint64_t a = (uint64_t)(uintptr_t)(kv.key + (b * 64 - kv.plen));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 16 * i + (lane >> 2);
            const uint32_t alo = __shfl((int)(uint32_t)a, j, 64), ahi = __shfl((int)(uint32_t)(a >> 32), j, 64);
            const int mj = __shfl((int)mid, j, 64);
            const uint8_t* src = (const uint8_t*)(uintptr_t)(((uint64_t)ahi << 32) | alo) + 16 * (lane & 3);
            pf[i] = mj ? load_u128_unaligned(src) : make_uint4(0, 0, 0, 0);
        }
    };
    auto stage = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 16 * i + (lane >> 2);
            *(uint4*)&lds[j * 20 + 4 * (lane & 3)] = pf[i];
        }
    };
    issue(0);
    for (uint32_t b = 0; b < nbmax; ++b) {
        stage();
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint4 v = *(const uint4*)&lds[lane * 20 + 4 * q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        if (b + 1 < nbmax) issue(b + 1);
        if (b < nb) {
            if (is_middle<H>(kv, b)) {
                if (H::big_endian) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = bswap32(w[i]);
                }
            } else {
                message_block<H>(kv, b, nb, w);
            }
            st.compress(w);
        }
    }
}

// LDS-DMA staged: per stage, the wave copies the next 128 B of all 64 keys with 8 global_load_lds_dwordx4
// (each instruction = 8 keys x 128 contiguous bytes), double-buffered; lanes read their own 2 blocks with
// conflict-free ds_read_b128 (chunk slot (c - lane/2) & 7 within the key's 128-B row).
template <class H>
__device__ __forceinline__ void hb_hash_key_dma(const KeyView& kv, H& st, uint8_t* buf0) {
    static_assert(H::block_bytes == 64, "64-byte blocks");
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;  // <= 3
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    uint32_t nbmax = nb;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, d, 64));
    const uint32_t nst = (nbmax + 1) >> 1;
    uint32_t preword = 0;
    for (uint32_t j = 0; j < r; ++j) preword |= (uint32_t)kv.pre[j] << (8 * j);
    const uint64_t base = (uint64_t)(uintptr_t)kv.key - r;
    const uint32_t keyend = kv.len + r;  // bytes of window that hold prefix-slot + key
    auto issue = [&](uint32_t s, uint8_t* buf) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int p = 8 * i + (lane >> 3);
            const uint32_t blo = __shfl((int)(uint32_t)base, p, 64), bhi = __shfl((int)(uint32_t)(base >> 32), p, 64);
            const uint32_t kend = __shfl((int)keyend, p, 64);
            const uint32_t c = ((lane & 7) + (p >> 1)) & 7;
            const uint8_t* src = (const uint8_t*)(uintptr_t)(((uint64_t)bhi << 32) | blo) + s * 128 + 16 * c;
            if (s * 128 < kend)
                __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + i * 1024), 16, 0, 0);
        }
    };
    st.init();
    issue(0, buf0);
    for (uint32_t s = 0; s < nst; ++s) {
        uint8_t* cur = buf0 + (s & 1) * 8192;
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        __builtin_amdgcn_wave_barrier();
        if (s + 1 < nst) issue(s + 1, buf0 + ((s + 1) & 1) * 8192);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const uint32_t b = 2 * s + bb;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = 4 * bb + q;
                const uint32_t slot = (c - (lane >> 1)) & 7;
                const uint4 v = *(const uint4*)(cur + (lane >> 3) * 1024 + 16 * (8 * (lane & 7) + slot));
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
            if (b < nb) {
                const uint32_t o0 = b * 64;
                if (b == 0 && r) w[0] = (w[0] & ~((1u << (8 * r)) - 1u)) | preword;
                if (o0 + 64 > total) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int rel = (int)total - (int)o0 - 4 * i;
                        if (rel <= 0) w[i] = rel == 0 ? 0x80u : 0u;
                        else if (rel < 4) w[i] = (w[i] & ((1u << (8 * rel)) - 1u)) | (0x80u << (8 * rel));
                    }
                }
                if (H::big_endian) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = bswap32(w[i]);
                }
                if (b + 1 == nb) {
                    const uint64_t bits = (uint64_t)total * 8u;
                    if (H::big_endian) { w[14] = (uint32_t)(bits >> 32); w[15] = (uint32_t)bits; }
                    else { w[14] = (uint32_t)bits; w[15] = (uint32_t)(bits >> 32); }
                }
                st.compress(w);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): reads of `cur` done before it is re-filled
    }
}

__device__ __forceinline__ void wait_vm(int k) {
    // s_waitcnt vmcnt(k) for the few counts the DMA pipeline needs (immediates must be constants)
    switch (k) {
        case 0: __builtin_amdgcn_s_waitcnt(0x0f70); break;
        case 4: __builtin_amdgcn_s_waitcnt(0x0f74); break;
        case 8: __builtin_amdgcn_s_waitcnt(0x0f78); break;
        case 12: __builtin_amdgcn_s_waitcnt(0x0f7c); break;
        case 16: __builtin_amdgcn_s_waitcnt(0x4f70); break;
        case 24: __builtin_amdgcn_s_waitcnt(0x4f78); break;
        case 32: __builtin_amdgcn_s_waitcnt(0x8f70); break;
        default: __builtin_amdgcn_s_waitcnt(0x0f70); break;
    }
}

struct NullHash {
    static constexpr int kind = 0, block_bytes = 64, len_bytes = 8, digest_bytes = 16, words = 16;
    static constexpr bool big_endian = false;
    uint32_t h[4];
    __device__ __forceinline__ void init() { h[0] = h[1] = h[2] = h[3] = 0; }
    __device__ __forceinline__ void compress(const uint32_t* m) {
#pragma unroll
        for (int i = 0; i < 16; ++i) h[i & 3] ^= m[i];
    }
    __device__ __forceinline__ uint32_t be_word(int i) const { return h[i]; }
};

template <class H, int S, int NB>
__device__ __forceinline__ void hash_key_dma2(const KeyView& kv, H& st, uint8_t* buf0) {
    constexpr int CS = 4 * S;          // 16-byte chunks per key per stage
    constexpr int PPI = 64 / CS;       // keys per DMA instruction
    constexpr int NI = 4 * S;          // DMA instructions per stage (64 keys * S * 64 B / 1 KiB)
    constexpr int SH = S == 1 ? 2 : S == 2 ? 1 : 0;
    constexpr int STAGE = S * 64 * 64; // bytes per stage buffer
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    uint32_t nbmax = nb;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, d, 64));
    const uint32_t nst = (nbmax + S - 1) / S;
    uint32_t preword = 0;
    for (uint32_t j = 0; j < r; ++j) preword |= (uint32_t)kv.pre[j] << (8 * j);
    const uint64_t base = (uint64_t)(uintptr_t)kv.key - r;
    const uint32_t keyend = kv.len + r;
    auto issue = [&](uint32_t s) {
        uint8_t* buf = buf0 + (s % NB) * STAGE;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int p = PPI * i + lane / CS;
            const uint32_t blo = __shfl((int)(uint32_t)base, p, 64), bhi = __shfl((int)(uint32_t)(base >> 32), p, 64);
            const uint32_t kend = __shfl((int)keyend, p, 64);
            const uint32_t c = ((lane % CS) + (p >> SH)) % CS;
            const uint64_t b64 = ((uint64_t)bhi << 32) | blo;
            const uint64_t a = (s * (S * 64) < kend) ? b64 + s * (S * 64) + 16 * c : b64;  // always issue
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)a, (__attribute__((address_space(3))) void*)(buf + i * 1024), 16, 0, 0);
        }
    };
    st.init();
#pragma unroll
    for (int k = 0; k < NB - 1; ++k)
        if (k < (int)nst) issue(k);
    for (uint32_t s = 0; s < nst; ++s) {
        const int after = (int)min(nst - 1, s + NB - 2) - (int)s;
        wait_vm(after * NI);
        __builtin_amdgcn_wave_barrier();
        if (s + NB - 1 < nst) issue(s + NB - 1);
        const uint8_t* cur = buf0 + (s % NB) * STAGE;
#pragma unroll
        for (int bb = 0; bb < S; ++bb) {
            const uint32_t b = S * s + bb;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = 4 * bb + q;
                const uint32_t slot = (c - (lane >> SH)) % CS;
                const uint4 v = *(const uint4*)(cur + (lane / PPI) * 1024 + 16 * (CS * (lane % PPI) + slot));
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
            if (b < nb) {
                const uint32_t o0 = b * 64;
                if (b == 0 && r) w[0] = (w[0] & ~((1u << (8 * r)) - 1u)) | preword;
                if (o0 + 64 > total) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int rel = (int)total - (int)o0 - 4 * i;
                        if (rel <= 0) w[i] = rel == 0 ? 0x80u : 0u;
                        else if (rel < 4) w[i] = (w[i] & ((1u << (8 * rel)) - 1u)) | (0x80u << (8 * rel));
                    }
                }
                if (H::big_endian) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = bswap32(w[i]);
                }
                if (b + 1 == nb) {
                    const uint64_t bits = (uint64_t)total * 8u;
                    if (H::big_endian) { w[14] = (uint32_t)(bits >> 32); w[15] = (uint32_t)bits; }
                    else { w[14] = (uint32_t)bits; w[15] = (uint32_t)(bits >> 32); }
                }
                st.compress(w);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
}

template <class H, int S, int NB>
__global__ void __launch_bounds__(64) k_hash_dma(const uint8_t* blob, const uint64_t* off, const uint32_t* order,
                                                 uint32_t n, const uint8_t* pre, uint32_t plen, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const uint32_t key = order ? order[min(i, n - 1)] : min(i, n - 1);
    const uint64_t a = off[key], e = off[key + 1];
    KeyView kv{blob + a, (uint32_t)(e - a), pre, plen};
    H st;
    hash_key_dma2<H, S, NB>(kv, st, dyn);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < H::digest_bytes / 4; ++j) x ^= st.be_word(j);
    if (i < n) out[i] = x;
}

template <class H, int S, int NB>
float run_dma(const uint8_t* blob, const uint64_t* off, const uint32_t* order, uint32_t n, const uint8_t* pre,
              uint32_t plen, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + 63) / 64);
    const size_t dl = (size_t)NB * S * 4096;
    hipLaunchKernelGGL((k_hash_dma<H, S, NB>), grid, dim3(64), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_hash_dma<H, S, NB>), grid, dim3(64), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n), ord(n), byk(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    if (order) {
        CK(hipMemcpy(ord.data(), order, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) byk[ord[i]] = h[i];
    } else byk = h;
    uint64_t cs = 0;
    for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + byk[i];
    g_checksum = cs;
    return ms / reps;
}

template <class H, int V>
__global__ void __launch_bounds__(256) k_hash(const uint8_t* blob, const uint64_t* off, const uint32_t* order,
                                              uint32_t n, const uint8_t* pre, uint32_t plen, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t key = order ? order[i] : i;
    const uint64_t a = off[key], e = off[key + 1];
    KeyView kv{blob + a, (uint32_t)(e - a), pre, plen};
    H st;
    __shared__ uint32_t lds[4 * 64 * 20];
    if (V == kPrefetch) {
        hash_key_prefetch<H>(kv, st);
    } else if (V == kDma) {
        extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
        hb_hash_key_dma<H>(kv, st, dyn + (threadIdx.x >> 6) * 16384);
    } else if (V == kFast) {
        hash_key<H>(kv, st);
    } else if (V == kCoop) {
        hash_key_coop<H>(kv, st, lds + (threadIdx.x >> 6) * 64 * 20);
    } else if (V == kPure) {
        st.init();
        const uint32_t nb = n_blocks(kv.plen + kv.len, H::block_bytes, H::len_bytes);
        uint32_t w[H::words];
        for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
            for (int i = 0; i < H::words; ++i) w[i] = (uint32_t)a * (i + 1) + b;
            st.compress(w);
        }
    } else {
        st.init();
        const uint32_t nb = n_blocks(kv.plen + kv.len, H::block_bytes, H::len_bytes);
        uint32_t w[H::words];
        for (uint32_t b = 0; b < nb; ++b) {
            block_variant<H, V>(kv, b, nb, w);
            st.compress(w);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < H::digest_bytes / 4; ++j) x ^= st.be_word(j);
    out[i] = x;
}

template <class H, int V>
float run(const uint8_t* blob, const uint64_t* off, const uint32_t* order, uint32_t n, const uint8_t* pre,
          uint32_t plen, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + 255) / 256);
    const size_t dl = V == kDma ? 4 * 16384 : 0;
    hipLaunchKernelGGL((k_hash<H, V>), grid, dim3(256), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_hash<H, V>), grid, dim3(256), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    uint64_t cs = 0;
    for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + h[order ? i : i];
    // checksum over the digests in key order (invert the permutation) so variants are comparable
    if (order) {
        std::vector<uint32_t> ord(n);
        CK(hipMemcpy(ord.data(), order, n * 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> byk(n);
        for (uint32_t i = 0; i < n; ++i) byk[ord[i]] = h[i];
        cs = 0;
        for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + byk[i];
    }
    g_checksum = cs;
    return ms / reps;
}

// the product's hash_key_dma (dsy_message.h) in WG-thread workgroups, one 64-key wave-task per wave
// load-only probe: the DMA pattern of hash_key_dma_reg<S> with every stage's 64*S-byte piece aligned down to a
// 64*S boundary (pieces = whole cache lines); consumes the LDS bytes with a cheap XOR (not a digest)
template <int S, int WG, bool ALIGN>
__global__ void __launch_bounds__(WG) k_load_probe(const uint8_t* blob, const uint64_t* off, const uint32_t* order,
                                                   uint32_t n, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    using G = DmaGeometry<S, 1>;
    uint8_t* lds_wave = dyn + (threadIdx.x >> 6) * G::kWaveBytes;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * WG + threadIdx.x;
    const uint32_t key = order ? order[min(i, n - 1)] : min(i, n - 1);
    const uint64_t a = off[key], e = off[key + 1];
    const uint32_t len = i < n ? (uint32_t)(e - a) : 0u;
    const uint64_t start = (uint64_t)(uintptr_t)(blob + a) - 1;  // 1-byte prefix
    const uint64_t base = ALIGN ? start & ~(uint64_t)(S * 64 - 1) : start;
    const uint32_t total = (uint32_t)(start - base) + 1 + len + 9;
    uint32_t nst = (total + S * 64 - 1) / (S * 64);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nst = max(nst, (uint32_t)__shfl_xor((int)nst, d, 64));
    uint32_t acc = 0;
    for (uint32_t s = 0; s < nst; ++s) {
#pragma unroll
        for (int k = 0; k < G::kInsts; ++k) {
            const int p = G::kKeysPerInst * k + (int)(lane / G::kChunks);
            const uint32_t blo = __shfl((int)(uint32_t)base, p, 64), bhi = __shfl((int)(uint32_t)(base >> 32), p, 64);
            const uint32_t pend = __shfl((int)total, p, 64);
            const uint32_t c = lane % G::kChunks;
            const uint64_t b64 = ((uint64_t)bhi << 32) | blo;
            if (s * (S * 64) < pend)
                __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(b64 + s * (S * 64) + 16 * c),
                                                 (__attribute__((address_space(3))) void*)(lds_wave + k * 1024), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0x0f70);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4 * S; ++q) acc ^= *(const uint32_t*)(lds_wave + (lane / G::kKeysPerInst) * 1024 + 16 * (G::kChunks * (lane % G::kKeysPerInst) + q));
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    if (i < n) out[i] = acc;
}

template <int S, int WG, bool ALIGN>
float run_probe(const uint8_t* blob, const uint64_t* off, const uint32_t* order, uint32_t n, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + WG - 1) / WG);
    const size_t dl = (size_t)(WG / 64) * DmaGeometry<S, 1>::kWaveBytes;
    hipLaunchKernelGGL((k_load_probe<S, WG, ALIGN>), grid, dim3(WG), dl, 0, blob, off, order, n, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_load_probe<S, WG, ALIGN>), grid, dim3(WG), dl, 0, blob, off, order, n, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    g_checksum = 0;
    return ms / reps;
}

template <class H, int S, int WG>
__global__ void __launch_bounds__(WG) k_hash_dma_r(const uint8_t* blob, const uint64_t* off, const uint32_t* order,
                                                   uint32_t n, const uint8_t* pre, uint32_t plen, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const uint32_t i = blockIdx.x * WG + threadIdx.x;
    const uint32_t key = order ? order[min(i, n - 1)] : min(i, n - 1);
    const uint64_t a = off[key], e = off[key + 1];
    KeyView kv{blob + a, i < n ? (uint32_t)(e - a) : 0u, pre, plen};
    H st;
    hash_key_dma_reg<H, S>(kv, st, dyn + (threadIdx.x >> 6) * DmaGeometry<S, 1>::kWaveBytes);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < H::digest_bytes / 4; ++j) x ^= st.be_word(j);
    if (i < n) out[i] = x;
}

template <class H, int S, int WG>
float run_dma_r(const uint8_t* blob, const uint64_t* off, const uint32_t* order, uint32_t n, const uint8_t* pre,
                uint32_t plen, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + WG - 1) / WG);
    const size_t dl = (size_t)(WG / 64) * DmaGeometry<S, 1>::kWaveBytes;
    hipLaunchKernelGGL((k_hash_dma_r<H, S, WG>), grid, dim3(WG), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_hash_dma_r<H, S, WG>), grid, dim3(WG), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n), ord(n), byk(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    if (order) {
        CK(hipMemcpy(ord.data(), order, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) byk[ord[i]] = h[i];
    } else byk = h;
    uint64_t cs = 0;
    for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + byk[i];
    g_checksum = cs;
    return ms / reps;
}

// EXPERIMENT (not in the product; result in DESIGN.md): line-aligned variant (64-byte-block hashes): every DMA piece is one whole, aligned 128-byte line of the key's
// window [start & ~127, ...), so a key of L bytes costs ceil((mis + L + pad) / 128) lines instead of the ~2x that
// unaligned 128-byte pieces touch (tools/hashbench probes: 4.6 vs 3.4 TB/s loads-only, 10.2 vs 17.6 GB fetched
// for 8 GB of packets).  Two stage buffers form a per-key ring of 16 chunks; block b of the message sits at window
// byte mis + 64 b and is assembled from 5 aligned 16-byte chunks by a per-lane funnel shift.  In every iteration a
// lane compresses the (at most two) blocks that end inside the stages landed so far, from registers, while the
// next stage's DMA is in flight.  Dead lanes issue nothing; every wait is vmcnt(0).
template <class H, int S = 2>
__device__ __forceinline__ void hb_hash_key_dma_aligned(const KeyView& kv, H& st, uint8_t* lds_wave) {
    static_assert(H::block_bytes == 64, "LDS-DMA staging is for 64-byte blocks");
    using G = DmaGeometry<S, 1>;
    constexpr uint32_t kSt = 64 * S;  // stage bytes per key (aligned to kSt)
    constexpr int kD = 4 * (4 * S + 1);  // dwords of the chunks S blocks need
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    const uint64_t start = (uint64_t)(uintptr_t)kv.key - r;
    const uint64_t base = start & ~(uint64_t)(kSt - 1);
    const uint32_t mis = (uint32_t)(start - base);
    const uint32_t wend = mis + 64 * nb;  // window bytes the message's blocks occupy
    const uint32_t dend = mis + total;    // stages past the key's last byte hold only padding: not loaded
    uint32_t nst = (wend + kSt - 1) / kSt;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nst = max(nst, (uint32_t)__shfl_xor((int)nst, d, 64));
    uint32_t preword = 0;
    for (uint32_t j = 0; j < r; ++j) preword |= (uint32_t)kv.pre[j] << (8 * j);
    // the key's 16-byte chunk C of the window (stage C / kChunks) lives in buffer (stage & 1) at the slot
    // hash_key_dma_reg's layout gives chunk C % kChunks
    const uint32_t row = (lane / G::kKeysPerInst) * 1024 + 16 * G::kChunks * (lane % G::kKeysPerInst);
    auto chunk_addr = [&](uint32_t C) {
        const uint32_t c = C % G::kChunks;
        return lds_wave + ((C / G::kChunks) & 1) * G::kStageBytes + row +
               16 * ((c - (lane >> G::kShift)) % G::kChunks);
    };
    auto issue = [&](uint32_t s) {
        uint8_t* buf = lds_wave + (s & 1) * G::kStageBytes;
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const int p = G::kKeysPerInst * i + (int)(lane / G::kChunks);
            const uint32_t blo = __shfl((int)(uint32_t)base, p, 64), bhi = __shfl((int)(uint32_t)(base >> 32), p, 64);
            const uint32_t pend = __shfl((int)dend, p, 64);
            const uint32_t c = ((lane % G::kChunks) + ((uint32_t)p >> G::kShift)) % G::kChunks;
            const uint64_t b64 = ((uint64_t)bhi << 32) | blo;
            if (s * kSt < pend)
                __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(b64 + s * kSt + 16 * c),
                                                 (__attribute__((address_space(3))) void*)(buf + i * 1024), 16, 0, 0);
        }
    };
    st.init();
    // the funnel shift (dword part as two select masks, byte part), the same for every block of the key
    const uint32_t m2 = (mis & 8) ? ~0u : 0u, m1 = (mis & 4) ? ~0u : 0u, bs = mis & 3;
    uint32_t b = 0;  // this lane's next block
    if (nst) issue(0);
    for (uint32_t s = 0; s < nst; ++s) {
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): stage s has landed
        __builtin_amdgcn_wave_barrier();
        // the blocks b .. b+S-1 that end inside stages <= s (a block not done yet starts in stage s-1 or s)
        const uint32_t lim = kSt * (s + 1);
        const uint32_t C0 = (mis + 64 * b) >> 4;
        uint32_t d[kD];
#pragma unroll
        for (int q = 0; q < kD / 4; ++q) {
            const uint4 v = *(const uint4*)chunk_addr(C0 + q);
            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): buffer (s-1) & 1 may be refilled now
        __builtin_amdgcn_wave_barrier();
        if (s + 1 < nst) issue(s + 1);
#pragma unroll 1
        for (uint32_t u = 0, b0 = b; u < (uint32_t)S; ++u) {
            const uint32_t bb = b0 + u;
            if (bb < nb && mis + 64 * bb + 64 <= lim) {
                // f[j] = d[ds + j] by value selects (no indexed register array), then w[i] = bytes bs.. of f[i], f[i+1]
                uint32_t e[18], f[17];
#pragma unroll
                for (int i = 0; i < 18; ++i) e[i] = bop3<kCh>(m2, d[i + 2], d[i]);
#pragma unroll
                for (int i = 0; i < 17; ++i) f[i] = bop3<kCh>(m1, e[i + 1], e[i]);
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_alignbyte(f[i + 1], f[i], bs);
                const uint32_t o0 = bb * 64;
                if (bb == 0 && r) w[0] = (w[0] & ~low_bytes_mask(r)) | preword;
                if (o0 + 64 > total) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int rel = (int)total - (int)o0 - 4 * i;
                        if (rel <= 0) w[i] = rel == 0 ? 0x80u : 0u;
                        else if (rel < 4) w[i] = (w[i] & ((1u << (8 * rel)) - 1u)) | (0x80u << (8 * rel));
                    }
                }
                if (H::big_endian) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = bswap32(w[i]);
                }
                if (bb + 1 == nb) {
                    const uint64_t bits = (uint64_t)total * 8u;
                    if (H::big_endian) { w[14] = (uint32_t)(bits >> 32); w[15] = (uint32_t)bits; }
                    else { w[14] = (uint32_t)bits; w[15] = (uint32_t)(bits >> 32); }
                }
                st.compress(w);
                ++b;
            }
            if (S > 1) {
#pragma unroll
                for (int i = 0; i < kD - 16; ++i) d[i] = d[i + 16];  // the next block's chunks
            }
        }
    }
}

template <class H, int MODE, int WG>
__global__ void __launch_bounds__(WG) k_hash_pad(const uint8_t* blob, const uint64_t* poff, const uint32_t* lens,
                                                 const uint32_t* order, uint32_t n, const uint8_t* pre, uint32_t plen,
                                                 uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const uint32_t i = blockIdx.x * WG + threadIdx.x;
    const uint32_t key = order ? order[min(i, n - 1)] : min(i, n - 1);
    KeyView kv{blob + poff[key], i < n ? lens[key] : 0u, pre, plen};
    H st;
    uint8_t* lw = dyn + (threadIdx.x >> 6) * DmaGeometry<2, 1>::kWaveBytes;
    if (MODE == 0) hash_key_dma_reg<H, 2>(kv, st, lw);
    // timing only: the product's line copy puts packets kLineBias bytes into their lines; this tool's pad layout is
    // 128-byte aligned, so the digests differ from the product's (the loads and the work per block do not)
    else hash_key_dma_lines<H>(kv, st, lw, (uint32_t)pre[0], blob);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < H::digest_bytes / 4; ++j) x ^= st.be_word(j);
    if (i < n) out[i] = x;
}

template <class H, int MODE, int WG>
float run_pad(const uint8_t* blob, const uint64_t* poff, const uint32_t* lens, const uint32_t* order, uint32_t n,
              const uint8_t* pre, uint32_t plen, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + WG - 1) / WG);
    const size_t dl = (size_t)(WG / 64) * DmaGeometry<2, 1>::kWaveBytes;
    hipLaunchKernelGGL((k_hash_pad<H, MODE, WG>), grid, dim3(WG), dl, 0, blob, poff, lens, order, n, pre, plen, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_hash_pad<H, MODE, WG>), grid, dim3(WG), dl, 0, blob, poff, lens, order, n, pre, plen, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n), ord(n), byk(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    if (order) {
        CK(hipMemcpy(ord.data(), order, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) byk[ord[i]] = h[i];
    } else byk = h;
    uint64_t cs = 0;
    for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + byk[i];
    g_checksum = cs;
    return ms / reps;
}

template <class H, int S, int WG>
__global__ void __launch_bounds__(WG) k_hash_dma_a(const uint8_t* blob, const uint64_t* off, const uint32_t* order,
                                                   uint32_t n, const uint8_t* pre, uint32_t plen, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const uint32_t i = blockIdx.x * WG + threadIdx.x;
    const uint32_t key = order ? order[min(i, n - 1)] : min(i, n - 1);
    const uint64_t a = off[key], e = off[key + 1];
    KeyView kv{blob + a, i < n ? (uint32_t)(e - a) : 0u, pre, plen};
    H st;
    hb_hash_key_dma_aligned<H, S>(kv, st, dyn + (threadIdx.x >> 6) * DmaGeometry<S, 2>::kWaveBytes);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < H::digest_bytes / 4; ++j) x ^= st.be_word(j);
    if (i < n) out[i] = x;
}

template <class H, int S, int WG>
float run_dma_a(const uint8_t* blob, const uint64_t* off, const uint32_t* order, uint32_t n, const uint8_t* pre,
                uint32_t plen, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + WG - 1) / WG);
    const size_t dl = (size_t)(WG / 64) * DmaGeometry<S, 2>::kWaveBytes;
    hipLaunchKernelGGL((k_hash_dma_a<H, S, WG>), grid, dim3(WG), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_hash_dma_a<H, S, WG>), grid, dim3(WG), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n), ord(n), byk(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    if (order) {
        CK(hipMemcpy(ord.data(), order, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) byk[ord[i]] = h[i];
    } else byk = h;
    uint64_t cs = 0;
    for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + byk[i];
    g_checksum = cs;
    return ms / reps;
}

template <class H, int S, int NB, int WG, int FLAGS>
__global__ void __launch_bounds__(WG) k_hash_dma_p(const uint8_t* blob, const uint64_t* off, const uint32_t* order,
                                                   uint32_t n, const uint8_t* pre, uint32_t plen, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const uint32_t i = blockIdx.x * WG + threadIdx.x;
    const uint32_t key = order ? order[min(i, n - 1)] : min(i, n - 1);
    const uint64_t a = off[key], e = off[key + 1];
    KeyView kv{blob + a, i < n ? (uint32_t)(e - a) : 0u, pre, plen};
    H st;
    hash_key_dma<H, S, NB, FLAGS>(kv, st, dyn + (threadIdx.x >> 6) * DmaGeometry<S, NB>::kWaveBytes);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < H::digest_bytes / 4; ++j) x ^= st.be_word(j);
    if (i < n) out[i] = x;
}

template <class H, int S, int NB, int WG, int FLAGS>
float run_dma_p(const uint8_t* blob, const uint64_t* off, const uint32_t* order, uint32_t n, const uint8_t* pre,
                uint32_t plen, uint32_t* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid((n + WG - 1) / WG);
    const size_t dl = (size_t)(WG / 64) * DmaGeometry<S, NB>::kWaveBytes;
    hipLaunchKernelGGL((k_hash_dma_p<H, S, NB, WG, FLAGS>), grid, dim3(WG), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_hash_dma_p<H, S, NB, WG, FLAGS>), grid, dim3(WG), dl, 0, blob, off, order, n, pre, plen, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n), ord(n), byk(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    if (order) {
        CK(hipMemcpy(ord.data(), order, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) byk[ord[i]] = h[i];
    } else byk = h;
    uint64_t cs = 0;
    for (uint32_t i = 0; i < n; ++i) cs = cs * 1000003u + byk[i];
    g_checksum = cs;
    return ms / reps;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1000000;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int lo = argc > 3 ? atoi(argv[3]) : 100, hi = argc > 4 ? atoi(argv[4]) : 1500;
    std::mt19937_64 rng(42);
    std::vector<uint64_t> off(n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) off[i + 1] = off[i] + lo + rng() % (hi - lo + 1);
    const uint64_t bytes = off[n];
    std::vector<uint8_t> blob((bytes + 256 + 7) & ~7ull);
    for (size_t i = 0; i < blob.size(); i += 8) { uint64_t v = rng(); memcpy(&blob[i], &v, 8); }
    // orders: by block count (descending: the load-balancing permutation), a random permutation (packets of a
    // wave scattered over the whole blob, like modulo-style claims), and random-then-sorted
    std::vector<uint32_t> order(n), scat(n), scat_sorted(n);
    std::iota(order.begin(), order.end(), 0);
    auto nbk = [&](uint32_t x) { return (off[x + 1] - off[x] + 1 + 8) / 64; };
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return nbk(x) > nbk(y); });
    std::iota(scat.begin(), scat.end(), 0);
    std::shuffle(scat.begin(), scat.end(), rng);
    scat_sorted = scat;
    std::stable_sort(scat_sorted.begin(), scat_sorted.end(), [&](uint32_t x, uint32_t y) { return nbk(x) > nbk(y); });
    uint64_t blocks = 0;
    for (uint32_t i = 0; i < n; ++i) blocks += (off[i + 1] - off[i] + 1 + 8) / 64 + 1;
    uint8_t *d_blob, *d_pre;
    uint64_t* d_off;
    uint32_t *d_order, *d_out, *d_scat, *d_scat_sorted;
    CK(hipMalloc(&d_blob, blob.size() + 64));
    d_blob += 64;
    CK(hipMalloc(&d_off, (n + 1) * 8));
    CK(hipMalloc(&d_order, n * 4));
    CK(hipMalloc(&d_out, n * 4));
    CK(hipMalloc(&d_scat, n * 4));
    CK(hipMalloc(&d_scat_sorted, n * 4));
    CK(hipMemcpy(d_scat, scat.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_scat_sorted, scat_sorted.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_pre, 256));
    CK(hipMemcpy(d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_order, order.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_pre, 0x2a, 256));
    // the same packets, each starting on a 128-byte line
    std::vector<uint64_t> poff(n);
    std::vector<uint32_t> lens(n);
    uint64_t pat = 0;
    for (uint32_t i = 0; i < n; ++i) {
        poff[i] = pat;
        lens[i] = (uint32_t)(off[i + 1] - off[i]);
        pat = (pat + lens[i] + 127) & ~127ull;
    }
    std::vector<uint8_t> pblob(pat + 256, 0);
    for (uint32_t i = 0; i < n; ++i) memcpy(&pblob[poff[i]], &blob[off[i]], lens[i]);
    uint8_t* d_pblob;
    uint64_t* d_poff;
    uint32_t* d_lens;
    CK(hipMalloc(&d_pblob, pblob.size() + 256));
    d_pblob += 128;  // the prefix byte before the first packet is read (and patched) by the unaligned path
    CK(hipMalloc(&d_poff, n * 8));
    CK(hipMalloc(&d_lens, n * 4));
    CK(hipMemcpy(d_pblob, pblob.data(), pblob.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_poff, poff.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lens, lens.data(), n * 4, hipMemcpyHostToDevice));
    printf("n=%u bytes=%.1f MB blocks(md5)=%llu padded=%.1f MB\n", n, bytes / 1e6, (unsigned long long)blocks, pat / 1e6);
    for (int round = 0; round < 2; ++round) {
        struct R { const char* name; float ms; uint64_t cs = 0; };
        std::vector<R> rs;
#define V(NAME, CALL) { float ms_ = CALL; rs.push_back({NAME, ms_, g_checksum}); }
        V("md5 dmareg(2) wg256", (run_dma_r<Md5, 2, 256>(d_blob, d_off, d_order, n, d_pre, 1, d_out, reps)));
        V("md5 dmareg(2) padded", (run_pad<Md5, 0, 256>(d_pblob, d_poff, d_lens, d_order, n, d_pre, 1, d_out, reps)));
        V("md5 pa padded", (run_pad<Md5, 1, 256>(d_pblob, d_poff, d_lens, d_order, n, d_pre, 1, d_out, reps)));
        V("md5 dmareg(2) plen0", (run_dma_r<Md5, 2, 256>(d_blob, d_off, d_order, n, d_pre, 0, d_out, reps)));
        V("md5 pa plen0", (run_pad<Md5, 1, 256>(d_pblob, d_poff, d_lens, d_order, n, d_pre, 0, d_out, reps)));
        V("md5 dmareg(2) plen3", (run_dma_r<Md5, 2, 256>(d_blob, d_off, d_order, n, d_pre, 3, d_out, reps)));
        V("md5 pa plen3", (run_pad<Md5, 1, 256>(d_pblob, d_poff, d_lens, d_order, n, d_pre, 3, d_out, reps)));
        V("md5 dmareg(2) plen4", (run_dma_r<Md5, 2, 256>(d_blob, d_off, d_order, n, d_pre, 4, d_out, reps)));
        V("md5 pa plen4", (run_pad<Md5, 1, 256>(d_pblob, d_poff, d_lens, d_order, n, d_pre, 4, d_out, reps)));
        V("sha1 dmareg(2) wg256", (run_dma_r<Sha1, 2, 256>(d_blob, d_off, d_order, n, d_pre, 1, d_out, reps)));
        V("sha1 pa padded", (run_pad<Sha1, 1, 256>(d_pblob, d_poff, d_lens, d_order, n, d_pre, 1, d_out, reps)));
        V("md5 dmareg(2) scat", (run_dma_r<Md5, 2, 256>(d_blob, d_off, d_scat_sorted, n, d_pre, 1, d_out, reps)));
        V("md5 pa scat", (run_pad<Md5, 1, 256>(d_pblob, d_poff, d_lens, d_scat_sorted, n, d_pre, 1, d_out, reps)));
        V("probe S=2 aligned", (run_probe<2, 256, true>(d_blob, d_off, d_order, n, d_out, reps)));
#undef V
        for (auto& r : rs) (void)0;
        for (auto& r : rs)
            printf("round %d  %-26s %8.3f ms  %7.1f GB/s  %6.2f Gblk/s  cs=%016llx\n", round, r.name, r.ms,
                   bytes / r.ms / 1e6, blocks / r.ms / 1e6, (unsigned long long)r.cs);
    }
    return 0;
}
