// dsy_hash.h -- per-lane Merkle-Damgard compression functions for gfx950 (one message per lane).
//
// The reference digests `prefix || key` with hashlib's MD5 / SHA-1 / SHA-2 (bloomfilter.py:25, :147-161,
// :168-170).  These are the RFC 1321 / FIPS 180-4 compression functions written for a 64-lane wavefront:
// every lane owns one message, all state lives in VGPRs, the 16 (or 32) message words of the current block are
// passed in registers, and every rotate maps to a single v_alignbit_b32.  Bitwise selects are written so the
// compiler emits v_bfi_b32 and 3-input adds fold into v_add3_u32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsy {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, uint32_t s) { return __builtin_amdgcn_alignbit(x, x, 32u - s); }
__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t s) { return __builtin_amdgcn_alignbit(x, x, s); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t rotr64(uint64_t x, uint32_t s) { return (x >> s) | (x << (64u - s)); }
// bitwise select: (m & a) | (~m & b)  -> v_bfi_b32
__device__ __forceinline__ uint32_t sel32(uint32_t m, uint32_t a, uint32_t b) { return b ^ (m & (a ^ b)); }
__device__ __forceinline__ uint64_t sel64(uint64_t m, uint64_t a, uint64_t b) { return b ^ (m & (a ^ b)); }

// CDNA4's v_bitop3_b32: any boolean function of three operands in ONE full-rate instruction (tools/valupeak:
// v_bitop3_b32 issues at the v_xor_b32 rate, while the three-operand v_bfi_b32 / v_add3_u32 / v_alignbit_b32
// issue at half of it).  The truth table is indexed the usual way: operand 0 <-> 0xF0, 1 <-> 0xCC, 2 <-> 0xAA.
template <uint32_t LUT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
    return (uint32_t)__builtin_amdgcn_bitop3_b32((int)a, (int)b, (int)c, LUT);
}
template <uint32_t LUT>
__device__ __forceinline__ uint64_t bop3_64(uint64_t a, uint64_t b, uint64_t c) {
    return ((uint64_t)bop3<LUT>((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
           bop3<LUT>((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
constexpr uint32_t kXor3 = 0xF0 ^ 0xCC ^ 0xAA;                   // a ^ b ^ c
constexpr uint32_t kCh = (0xF0 & 0xCC) | (~0xF0 & 0xAA & 0xFF);    // a ? b : c   (MD5 F, SHA Ch)
constexpr uint32_t kMaj = (0xF0 & 0xCC) | (0xF0 & 0xAA) | (0xCC & 0xAA);
constexpr uint32_t kMd5G = (0xF0 & 0xAA) | (0xCC & ~0xAA & 0xFF);  // (b & d) | (c & ~d)
constexpr uint32_t kMd5I = (0xCC ^ (0xF0 | (~0xAA & 0xFF))) & 0xFF; // c ^ (b | ~d)

// x + K with K a 32-bit literal in the instruction (LIT) or left to the compiler
template <bool LIT>
__device__ __forceinline__ uint32_t addk(uint32_t x, uint32_t k) {
    if constexpr (LIT) {
        uint32_t r;
        asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "i"(k), "v"(x));
        return r;
    } else {
        return x + k;
    }
}

// --------------------------------------------------------------------------------------------------- MD5
struct Md5 {
    static constexpr int kind = 0;
    static constexpr int block_bytes = 64;
    static constexpr int len_bytes = 8;
    static constexpr int digest_bytes = 16;
    static constexpr bool big_endian = false;
    static constexpr int words = 16;
    uint32_t h[4];

    __device__ __forceinline__ void init() {
        h[0] = 0x67452301u; h[1] = 0xefcdab89u; h[2] = 0x98badcfeu; h[3] = 0x10325476u;
    }

    // LIT: every round constant is a literal operand of one v_add_u32 (x + K) instead of an SGPR the compiler keeps
    // for all 64 of them (and an add3 that reads it) -- the responder's wave-task loop (k_pair_test) needs those
    // SGPRs for its task state, which otherwise spills into VGPR lanes (v_writelane / v_readlane, VALU work on every
    // wave-task).  Same instruction count per step.
    template <bool LIT = false>
    __device__ __forceinline__ void compress(const uint32_t* m) {
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#define DSY_MD5_STEP(f, a, b, c, d, x, k, s) a = b + rotl32(a + (f) + addk<LIT>((x), (k)), s)
        // round 1: F = (b & c) | (~b & d)
        DSY_MD5_STEP(bop3<kCh>(b, c, d), a, b, c, d, m[0], 0xd76aa478u, 7);
        DSY_MD5_STEP(bop3<kCh>(a, b, c), d, a, b, c, m[1], 0xe8c7b756u, 12);
        DSY_MD5_STEP(bop3<kCh>(d, a, b), c, d, a, b, m[2], 0x242070dbu, 17);
        DSY_MD5_STEP(bop3<kCh>(c, d, a), b, c, d, a, m[3], 0xc1bdceeeu, 22);
        DSY_MD5_STEP(bop3<kCh>(b, c, d), a, b, c, d, m[4], 0xf57c0fafu, 7);
        DSY_MD5_STEP(bop3<kCh>(a, b, c), d, a, b, c, m[5], 0x4787c62au, 12);
        DSY_MD5_STEP(bop3<kCh>(d, a, b), c, d, a, b, m[6], 0xa8304613u, 17);
        DSY_MD5_STEP(bop3<kCh>(c, d, a), b, c, d, a, m[7], 0xfd469501u, 22);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        DSY_MD5_STEP(bop3<kCh>(b, c, d), a, b, c, d, m[8], 0x698098d8u, 7);
        DSY_MD5_STEP(bop3<kCh>(a, b, c), d, a, b, c, m[9], 0x8b44f7afu, 12);
        DSY_MD5_STEP(bop3<kCh>(d, a, b), c, d, a, b, m[10], 0xffff5bb1u, 17);
        DSY_MD5_STEP(bop3<kCh>(c, d, a), b, c, d, a, m[11], 0x895cd7beu, 22);
        DSY_MD5_STEP(bop3<kCh>(b, c, d), a, b, c, d, m[12], 0x6b901122u, 7);
        DSY_MD5_STEP(bop3<kCh>(a, b, c), d, a, b, c, m[13], 0xfd987193u, 12);
        DSY_MD5_STEP(bop3<kCh>(d, a, b), c, d, a, b, m[14], 0xa679438eu, 17);
        DSY_MD5_STEP(bop3<kCh>(c, d, a), b, c, d, a, m[15], 0x49b40821u, 22);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        // round 2: G = (b & d) | (c & ~d)
        DSY_MD5_STEP(bop3<kMd5G>(b, c, d), a, b, c, d, m[1], 0xf61e2562u, 5);
        DSY_MD5_STEP(bop3<kMd5G>(a, b, c), d, a, b, c, m[6], 0xc040b340u, 9);
        DSY_MD5_STEP(bop3<kMd5G>(d, a, b), c, d, a, b, m[11], 0x265e5a51u, 14);
        DSY_MD5_STEP(bop3<kMd5G>(c, d, a), b, c, d, a, m[0], 0xe9b6c7aau, 20);
        DSY_MD5_STEP(bop3<kMd5G>(b, c, d), a, b, c, d, m[5], 0xd62f105du, 5);
        DSY_MD5_STEP(bop3<kMd5G>(a, b, c), d, a, b, c, m[10], 0x02441453u, 9);
        DSY_MD5_STEP(bop3<kMd5G>(d, a, b), c, d, a, b, m[15], 0xd8a1e681u, 14);
        DSY_MD5_STEP(bop3<kMd5G>(c, d, a), b, c, d, a, m[4], 0xe7d3fbc8u, 20);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        DSY_MD5_STEP(bop3<kMd5G>(b, c, d), a, b, c, d, m[9], 0x21e1cde6u, 5);
        DSY_MD5_STEP(bop3<kMd5G>(a, b, c), d, a, b, c, m[14], 0xc33707d6u, 9);
        DSY_MD5_STEP(bop3<kMd5G>(d, a, b), c, d, a, b, m[3], 0xf4d50d87u, 14);
        DSY_MD5_STEP(bop3<kMd5G>(c, d, a), b, c, d, a, m[8], 0x455a14edu, 20);
        DSY_MD5_STEP(bop3<kMd5G>(b, c, d), a, b, c, d, m[13], 0xa9e3e905u, 5);
        DSY_MD5_STEP(bop3<kMd5G>(a, b, c), d, a, b, c, m[2], 0xfcefa3f8u, 9);
        DSY_MD5_STEP(bop3<kMd5G>(d, a, b), c, d, a, b, m[7], 0x676f02d9u, 14);
        DSY_MD5_STEP(bop3<kMd5G>(c, d, a), b, c, d, a, m[12], 0x8d2a4c8au, 20);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        // round 3: H = b ^ c ^ d
        DSY_MD5_STEP(bop3<kXor3>(b, c, d), a, b, c, d, m[5], 0xfffa3942u, 4);
        DSY_MD5_STEP(bop3<kXor3>(a, b, c), d, a, b, c, m[8], 0x8771f681u, 11);
        DSY_MD5_STEP(bop3<kXor3>(d, a, b), c, d, a, b, m[11], 0x6d9d6122u, 16);
        DSY_MD5_STEP(bop3<kXor3>(c, d, a), b, c, d, a, m[14], 0xfde5380cu, 23);
        DSY_MD5_STEP(bop3<kXor3>(b, c, d), a, b, c, d, m[1], 0xa4beea44u, 4);
        DSY_MD5_STEP(bop3<kXor3>(a, b, c), d, a, b, c, m[4], 0x4bdecfa9u, 11);
        DSY_MD5_STEP(bop3<kXor3>(d, a, b), c, d, a, b, m[7], 0xf6bb4b60u, 16);
        DSY_MD5_STEP(bop3<kXor3>(c, d, a), b, c, d, a, m[10], 0xbebfbc70u, 23);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        DSY_MD5_STEP(bop3<kXor3>(b, c, d), a, b, c, d, m[13], 0x289b7ec6u, 4);
        DSY_MD5_STEP(bop3<kXor3>(a, b, c), d, a, b, c, m[0], 0xeaa127fau, 11);
        DSY_MD5_STEP(bop3<kXor3>(d, a, b), c, d, a, b, m[3], 0xd4ef3085u, 16);
        DSY_MD5_STEP(bop3<kXor3>(c, d, a), b, c, d, a, m[6], 0x04881d05u, 23);
        DSY_MD5_STEP(bop3<kXor3>(b, c, d), a, b, c, d, m[9], 0xd9d4d039u, 4);
        DSY_MD5_STEP(bop3<kXor3>(a, b, c), d, a, b, c, m[12], 0xe6db99e5u, 11);
        DSY_MD5_STEP(bop3<kXor3>(d, a, b), c, d, a, b, m[15], 0x1fa27cf8u, 16);
        DSY_MD5_STEP(bop3<kXor3>(c, d, a), b, c, d, a, m[2], 0xc4ac5665u, 23);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        // round 4: I = c ^ (b | ~d)
        DSY_MD5_STEP(bop3<kMd5I>(b, c, d), a, b, c, d, m[0], 0xf4292244u, 6);
        DSY_MD5_STEP(bop3<kMd5I>(a, b, c), d, a, b, c, m[7], 0x432aff97u, 10);
        DSY_MD5_STEP(bop3<kMd5I>(d, a, b), c, d, a, b, m[14], 0xab9423a7u, 15);
        DSY_MD5_STEP(bop3<kMd5I>(c, d, a), b, c, d, a, m[5], 0xfc93a039u, 21);
        DSY_MD5_STEP(bop3<kMd5I>(b, c, d), a, b, c, d, m[12], 0x655b59c3u, 6);
        DSY_MD5_STEP(bop3<kMd5I>(a, b, c), d, a, b, c, m[3], 0x8f0ccc92u, 10);
        DSY_MD5_STEP(bop3<kMd5I>(d, a, b), c, d, a, b, m[10], 0xffeff47du, 15);
        DSY_MD5_STEP(bop3<kMd5I>(c, d, a), b, c, d, a, m[1], 0x85845dd1u, 21);
        if constexpr (LIT) __builtin_amdgcn_sched_barrier(0);  // (no hoisting of the next x + K adds)
        DSY_MD5_STEP(bop3<kMd5I>(b, c, d), a, b, c, d, m[8], 0x6fa87e4fu, 6);
        DSY_MD5_STEP(bop3<kMd5I>(a, b, c), d, a, b, c, m[15], 0xfe2ce6e0u, 10);
        DSY_MD5_STEP(bop3<kMd5I>(d, a, b), c, d, a, b, m[6], 0xa3014314u, 15);
        DSY_MD5_STEP(bop3<kMd5I>(c, d, a), b, c, d, a, m[13], 0x4e0811a1u, 21);
        DSY_MD5_STEP(bop3<kMd5I>(b, c, d), a, b, c, d, m[4], 0xf7537e82u, 6);
        DSY_MD5_STEP(bop3<kMd5I>(a, b, c), d, a, b, c, m[11], 0xbd3af235u, 10);
        DSY_MD5_STEP(bop3<kMd5I>(d, a, b), c, d, a, b, m[2], 0x2ad7d2bbu, 15);
        DSY_MD5_STEP(bop3<kMd5I>(c, d, a), b, c, d, a, m[9], 0xeb86d391u, 21);
#undef DSY_MD5_STEP
        h[0] += a; h[1] += b; h[2] += c; h[3] += d;
    }

    // digest as big-endian 32-bit words (MD5 emits its state little-endian)
    __device__ __forceinline__ uint32_t be_word(int i) const { return bswap32(h[i]); }
};

// ------------------------------------------------------------------------------------------------- SHA-1
struct Sha1 {
    static constexpr int kind = 1;
    static constexpr int block_bytes = 64;
    static constexpr int len_bytes = 8;
    static constexpr int digest_bytes = 20;
    static constexpr bool big_endian = true;
    static constexpr int words = 16;
    uint32_t h[5];

    __device__ __forceinline__ void init() {
        h[0] = 0x67452301u; h[1] = 0xefcdab89u; h[2] = 0x98badcfeu; h[3] = 0x10325476u; h[4] = 0xc3d2e1f0u;
    }

    template <bool LIT = false>
    __device__ __forceinline__ void compress(const uint32_t* m) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = m[i];
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
        for (int t = 0; t < 80; ++t) {
            uint32_t x;
            if (t < 16) {
                x = w[t];
            } else {
                x = rotl32(bop3<kXor3>(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
                w[t & 15] = x;
            }
            uint32_t f, k;
            if (t < 20) { f = bop3<kCh>(b, c, d); k = 0x5a827999u; }
            else if (t < 40) { f = bop3<kXor3>(b, c, d); k = 0x6ed9eba1u; }
            else if (t < 60) { f = bop3<kMaj>(b, c, d); k = 0x8f1bbcdcu; }
            else { f = bop3<kXor3>(b, c, d); k = 0xca62c1d6u; }
            uint32_t tmp = rotl32(a, 5) + f + e + k + x;
            e = d; d = c; c = rotl32(b, 30); b = a; a = tmp;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    }

    __device__ __forceinline__ uint32_t be_word(int i) const { return h[i]; }
};

// ----------------------------------------------------------------------------------------------- SHA-256
__device__ __constant__ static const uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

struct Sha256 {
    static constexpr int kind = 2;
    static constexpr int block_bytes = 64;
    static constexpr int len_bytes = 8;
    static constexpr int digest_bytes = 32;
    static constexpr bool big_endian = true;
    static constexpr int words = 16;
    uint32_t h[8];

    __device__ __forceinline__ void init() {
        h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
        h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
    }

    template <bool LIT = false>
    __device__ __forceinline__ void compress(const uint32_t* m) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = m[i];
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            uint32_t x;
            if (t < 16) {
                x = w[t];
            } else {
                uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                uint32_t s0 = bop3<kXor3>(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
                uint32_t s1 = bop3<kXor3>(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
                x = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
                w[t & 15] = x;
            }
            uint32_t S1 = bop3<kXor3>(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
            uint32_t t1 = hh + S1 + bop3<kCh>(e, f, g) + kSha256K[t] + x;
            uint32_t S0 = bop3<kXor3>(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
            uint32_t t2 = S0 + bop3<kMaj>(a, b, c);
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }

    __device__ __forceinline__ uint32_t be_word(int i) const { return h[i]; }
};

// ------------------------------------------------------------------------------------- SHA-512 / SHA-384
__device__ __constant__ static const uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

template <bool k384>
struct Sha512T {
    static constexpr int kind = k384 ? 3 : 4;
    static constexpr int block_bytes = 128;
    static constexpr int len_bytes = 16;
    static constexpr int digest_bytes = k384 ? 48 : 64;
    static constexpr bool big_endian = true;
    static constexpr int words = 32;  // 32-bit words per block
    uint64_t h[8];

    __device__ __forceinline__ void init() {
        if (k384) {
            h[0] = 0xcbbb9d5dc1059ed8ull; h[1] = 0x629a292a367cd507ull; h[2] = 0x9159015a3070dd17ull;
            h[3] = 0x152fecd8f70e5939ull; h[4] = 0x67332667ffc00b31ull; h[5] = 0x8eb44a8768581511ull;
            h[6] = 0xdb0c2e0d64f98fa7ull; h[7] = 0x47b5481dbefa4fa4ull;
        } else {
            h[0] = 0x6a09e667f3bcc908ull; h[1] = 0xbb67ae8584caa73bull; h[2] = 0x3c6ef372fe94f82bull;
            h[3] = 0xa54ff53a5f1d36f1ull; h[4] = 0x510e527fade682d1ull; h[5] = 0x9b05688c2b3e6c1full;
            h[6] = 0x1f83d9abfb41bd6bull; h[7] = 0x5be0cd19137e2179ull;
        }
    }

    // m: 32 big-endian-decoded 32-bit words (word 2i is the high half of 64-bit word i)
    template <bool LIT = false>  // (no literal form: the 64-bit constants are kept by the compiler)
    __device__ __forceinline__ void compress(const uint32_t* m) {
        uint64_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = ((uint64_t)m[2 * i] << 32) | m[2 * i + 1];
        uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
        for (int t = 0; t < 80; ++t) {
            uint64_t x;
            if (t < 16) {
                x = w[t];
            } else {
                uint64_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                uint64_t s0 = bop3_64<kXor3>(rotr64(w15, 1), rotr64(w15, 8), w15 >> 7);
                uint64_t s1 = bop3_64<kXor3>(rotr64(w2, 19), rotr64(w2, 61), w2 >> 6);
                x = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
                w[t & 15] = x;
            }
            uint64_t S1 = bop3_64<kXor3>(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
            uint64_t t1 = hh + S1 + bop3_64<kCh>(e, f, g) + kSha512K[t] + x;
            uint64_t S0 = bop3_64<kXor3>(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
            uint64_t t2 = S0 + bop3_64<kMaj>(a, b, c);
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }

    __device__ __forceinline__ uint32_t be_word(int i) const {
        return (i & 1) ? (uint32_t)h[i >> 1] : (uint32_t)(h[i >> 1] >> 32);
    }
};
using Sha384 = Sha512T<true>;
using Sha512 = Sha512T<false>;

}  // namespace dsy
