// dsy_message.h -- building Merkle-Damgard blocks of `prefix || key` per lane, and slicing digests into
// Bloom-filter bit positions exactly like bloomfilter.py:158-171.
#pragma once
#include "dsy_hash.h"

namespace dsy {

// Everything a lane needs to hash one key under one filter's salt.
struct KeyView {
    const uint8_t* key;  // device pointer to the key bytes
    uint32_t len;        // key length in bytes
    const uint8_t* pre;  // device (or kernarg) pointer to the prefix bytes
    uint32_t plen;       // prefix length (0..255)
};

__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);  // gfx950 HSA runs with unaligned access mode: one global_load_dword
    return v;
}

__device__ __forceinline__ uint4 load_u128_unaligned(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // one global_load_dwordx4
    return v;
}

// Little-endian 32-bit word of the padded message at byte offset o, without reading outside the key or the
// prefix: message = pre[0:plen] || key[0:len] || 0x80 || 0x00...  (length words are patched separately).
__device__ __forceinline__ uint32_t message_word_slow(const KeyView& kv, uint32_t o) {
    const uint32_t total = kv.plen + kv.len;
    if (o >= kv.plen && o + 4 <= total) return load_u32_unaligned(kv.key + (o - kv.plen));
    uint32_t w = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t off = o + j;
        uint32_t byte;
        if (off < kv.plen) byte = kv.pre[off];
        else if (off < total) byte = kv.key[off - kv.plen];
        else byte = (off == total) ? 0x80u : 0u;
        w |= byte << (8 * j);
    }
    return w;
}

__device__ __forceinline__ uint32_t n_blocks(uint32_t total, int block_bytes, int len_bytes) {
    return (total + len_bytes) / block_bytes + 1;
}

// Block b of the padded message into w[] (H::words 32-bit words, already in the hash's byte order).
template <class H>
__device__ __forceinline__ void message_block(const KeyView& kv, uint32_t b, uint32_t nb, uint32_t* w) {
    constexpr int BLK = H::block_bytes;
    const uint32_t total = kv.plen + kv.len;
    const uint32_t o0 = b * BLK;
    if (o0 >= kv.plen && o0 + BLK <= total) {
        const uint8_t* src = kv.key + (o0 - kv.plen);
#pragma unroll
        for (int q = 0; q < BLK / 16; ++q) {
            uint4 v = load_u128_unaligned(src + 16 * q);
            w[4 * q + 0] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < H::words; ++i) w[i] = message_word_slow(kv, o0 + 4 * i);
    }
    if (H::big_endian) {
#pragma unroll
        for (int i = 0; i < H::words; ++i) w[i] = bswap32(w[i]);
    }
    if (b + 1 == nb) {  // final block: message length in bits
        const uint64_t bits = (uint64_t)total * 8u;
        if (H::big_endian) {
            w[H::words - 2] = (uint32_t)(bits >> 32);
            w[H::words - 1] = (uint32_t)bits;
            if (H::words == 32) { w[28] = 0; w[29] = 0; }
        } else {
            w[14] = (uint32_t)bits;
            w[15] = (uint32_t)(bits >> 32);
        }
    }
}

template <class H>
__device__ __forceinline__ void hash_key(const KeyView& kv, H& st) {
    st.init();
    const uint32_t nb = n_blocks(kv.plen + kv.len, H::block_bytes, H::len_bytes);
    uint32_t w[H::words];
    for (uint32_t b = 0; b < nb; ++b) {
        message_block<H>(kv, b, nb, w);
        st.compress(w);
    }
}

// The i-th big-endian chunk of the digest (struct '>H' / '>L' / '>Q' codes, bloomfilter.py:135-140, :158-160).
template <class H, int CHUNK>
__device__ __forceinline__ uint64_t digest_chunk(const H& st, int i) {
    if (CHUNK == 2) {
        const uint32_t w = st.be_word(i >> 1);
        return (i & 1) ? (w & 0xffffu) : (w >> 16);
    } else if (CHUNK == 4) {
        return st.be_word(i);
    } else {
        return ((uint64_t)st.be_word(2 * i) << 32) | st.be_word(2 * i + 1);
    }
}

template <class H, int CHUNK>
struct ChunkLimit {
    static constexpr int kmax = H::digest_bytes / CHUNK;
};

// pos = chunk % m  (bloomfilter.py:171).  'H'/'L' chunks are < 2^32 and their filters have m < 2^31.
template <int CHUNK>
__device__ __forceinline__ uint64_t bit_position(uint64_t chunk, uint64_t m) {
    if (CHUNK == 8) return chunk % m;
    return (uint32_t)chunk % (uint32_t)m;
}

}  // namespace dsy
