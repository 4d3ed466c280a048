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

// Generic path: any prefix length (0..255); boundary blocks are assembled word by word.
template <class H>
__device__ __forceinline__ void hash_key_generic(const KeyView& kv, H& st) {
    st.init();
    const uint32_t nb = n_blocks(kv.plen + kv.len, H::block_bytes, H::len_bytes);
    uint32_t w[H::words];
    for (uint32_t b = 0; b < nb; ++b) {
        message_block<H>(kv, b, nb, w);
        st.template compress<true>(w);
    }
}

// Bytes 0..r-1 of a little-endian word (r = 0..4).
__device__ __forceinline__ uint32_t low_bytes_mask(uint32_t r) { return r >= 4 ? 0xffffffffu : (1u << (8 * r)) - 1u; }

// Fast path for prefixes of 0..4 bytes (the wire carries exactly one, conversion.py:725,769; BASELINE config 1
// uses four): every block is
// four (eight) unaligned 16-byte loads of the key; block 0 is shifted right by the prefix length with
// v_alignbyte and the prefix OR-ed in; the final block(s) are masked in registers (0x80 terminator, zeros,
// bit length).  Loads of block b+1 are issued before block b is compressed (one block of software prefetch).
// Reads may run up to block_bytes-1 bytes past the key: the blob carries DSY_BLOB_GUARD readable bytes.
template <class H>
__device__ __forceinline__ void hash_key_short_prefix(const KeyView& kv, H& st) {
    constexpr int BLK = H::block_bytes, NW = H::words;
    const uint32_t r = kv.plen;
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, BLK, H::len_bytes);
    uint32_t preword = 0;
    for (uint32_t j = 0; j < r; ++j) preword |= (uint32_t)kv.pre[j] << (8 * j);
    auto load = [&](uint32_t b, uint32_t* w) {
        const bool has = b == 0 ? kv.len > 0 : b * BLK - r < kv.len;
        const uint8_t* src = b == 0 ? kv.key : kv.key + (b * BLK - r);
        if (has) {
#pragma unroll
            for (int q = 0; q < BLK / 16; ++q) {
                const uint4 v = load_u128_unaligned(src + 16 * q);
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NW; ++i) w[i] = 0;
        }
    };
    st.init();
    uint32_t nxt[NW];
    load(0, nxt);
    for (uint32_t b = 0; b < nb; ++b) {
        uint32_t w[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) w[i] = nxt[i];
        if (b + 1 < nb) load(b + 1, nxt);
        const uint32_t o0 = b * BLK;
        if (b == 0 && r) {
#pragma unroll
            for (int i = NW - 1; i >= 1; --i) w[i] = __builtin_amdgcn_alignbyte(w[i], w[i - 1], 4 - r);
            w[0] = (r == 4 ? 0u : (w[0] << (8 * r))) | preword;
        }
        if (o0 + BLK > total) {
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int rel = (int)total - (int)o0 - 4 * i;
                if (rel <= 0) w[i] = rel == 0 ? 0x80u : 0u;
                else if (rel < 4) w[i] = (w[i] & ((1u << (8 * rel)) - 1u)) | (0x80u << (8 * rel));
            }
        }
        if (H::big_endian) {
#pragma unroll
            for (int i = 0; i < NW; ++i) w[i] = bswap32(w[i]);
        }
        if (b + 1 == nb) {
            const uint64_t bits = (uint64_t)total * 8u;
            if (H::big_endian) {
                w[NW - 2] = (uint32_t)(bits >> 32);
                w[NW - 1] = (uint32_t)bits;
                if constexpr (NW == 32) { w[28] = 0; w[29] = 0; }
            } else {
                w[14] = (uint32_t)bits;
                w[15] = (uint32_t)(bits >> 32);
            }
        }
        st.template compress<true>(w);
    }
}

// ---------------------------------------------------------------------------------------------------------
// LDS-DMA staged hashing for 64-byte-block hashes (MD5 / SHA-1 / SHA-256), one key per lane, called by ALL 64
// lanes of a wave together (wave-uniform control flow; idle lanes pass a zero-length key at a readable address).
//
// Each stage copies the next S*64 bytes of all 64 keys into LDS with 4*S `global_load_lds_dwordx4` wave
// instructions; every instruction moves 64/(4S) keys x S*64 contiguous bytes, so the memory system sees whole
// 128-byte pieces instead of 64 scattered 16-byte ones.  Within a key's LDS row the 16-byte chunks are rotated by
// (key >> SH) so the lanes' ds_read_b128 of "chunk c of my key" hit 16 distinct 4-bank groups.  NB buffers keep
// NB-1 stages in flight (counted vmcnt).  Requires every lane's prefix to be <= 4 bytes and DSY_BLOB_GUARD
// readable bytes before the first and after the last key (block 0 is fetched from key - plen).
__device__ __forceinline__ void wait_vmcnt(int k) {
    // s_waitcnt vmcnt(k), lgkm/exp counters untouched (immediates must be compile-time constants)
    switch (k) {
        case 0: __builtin_amdgcn_s_waitcnt(0x0f70); break;
        case 8: __builtin_amdgcn_s_waitcnt(0x0f78); break;
        case 16: __builtin_amdgcn_s_waitcnt(0x4f70); break;
        default: __builtin_amdgcn_s_waitcnt(0x0f70); break;
    }
}

template <int S, int NB>
struct DmaGeometry {
    static constexpr int kChunks = 4 * S;          // 16-byte chunks per key per stage
    static constexpr int kKeysPerInst = 64 / kChunks;
    static constexpr int kInsts = 4 * S;           // wave instructions per stage (64 keys * S*64 B / 1 KiB)
    static constexpr int kShift = S == 1 ? 2 : S == 2 ? 1 : 0;
    static constexpr int kStageBytes = S * 64 * 64;
    static constexpr int kWaveBytes = NB * kStageBytes;
};

// The DMA pieces one lane moves for its wave's 64 keys.  In wave instruction i of a stage the lane copies 16 bytes
// of key p_i = kKeysPerInst * i + lane / kChunks (chunk c_i of that key's stage window, rotated as above).  The
// keys' addresses and lengths are fixed for the whole hash, so each lane gathers its kInsts (address, live stages)
// pairs once per key -- kInsts x 3 shuffles -- instead of once per stage: per stage an instruction is then a
// compare, a 64-bit add and the load, with no LDS round trip (ds_bpermute) and no register pressure from hoisted
// per-stage address math between the loads (the per-stage form spilled to scratch in k_pair_test, and every
// scratch reload waited on vmcnt(0) -- on the stage's own DMA -- in the middle of issuing it).
template <int S>
struct DmaLanes {
    using G = DmaGeometry<S, 1>;
    uint64_t addr[G::kInsts];  // key p_i's stage-0 piece address
    uint32_t live[G::kInsts];  // stages of key p_i that hold message bytes
    // base: the lane's stage-0 window start (stage s covers [base + s*S*64, +S*64)); bytes: message bytes from base
    __device__ __forceinline__ void init(uint64_t base, uint32_t bytes) {
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t nst = (bytes + S * 64 - 1) / (S * 64);
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const int p = G::kKeysPerInst * i + (int)(lane / G::kChunks);
            const uint32_t blo = __shfl((int)(uint32_t)base, p, 64), bhi = __shfl((int)(uint32_t)(base >> 32), p, 64);
            live[i] = (uint32_t)__shfl((int)nst, p, 64);
            const uint32_t c = ((lane % G::kChunks) + ((uint32_t)p >> G::kShift)) % G::kChunks;
            addr[i] = (((uint64_t)bhi << 32) | blo) + 16 * c;
        }
    }
    // stage s of every key into the wave's LDS buffer (skip: no loads -- the DIAG compute-ceiling builds)
    template <bool SKIP = false>
    __device__ __forceinline__ void issue(uint32_t s, uint8_t* lds_wave) const {
        if constexpr (SKIP) return;
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i)
            if (s < live[i])
                __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(addr[i] + (uint64_t)s * (S * 64)),
                                                 (__attribute__((address_space(3))) void*)(lds_wave + i * 1024), 16, 0, 0);
    }
};

// A wave's LDS buffer (a generic pointer into __shared__ memory) as a local address the wave holds in an SGPR.
__device__ __forceinline__ uint32_t lds_local(uint8_t* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)p);
}

// The store's line copy puts every packet kLineBias bytes into a 128-byte line.  With one byte of slack in front of
// every packet, the message prefix || packet of a 1-byte prefix (every claim the reference builds, community.py:773,
// :911) starts exactly on the line, and the responder's blocks need no byte shift.
static constexpr uint64_t kLineBias = 1;

// Bytes of line copy a packet of `len` bytes takes: its 1-byte-prefixed message padded to whole 64-byte blocks
// (MD5 / SHA-1 / SHA-256: 0x80, zeros, the 8-byte bit length), in whole lines.  The copy holds the 0x80 after every
// packet and zeros up to the end of the final block (k_store_lines), so a 1-byte-prefixed message's blocks come out of
// the line copy already padded and the hashing kernel only writes the bit length (hash_key_dma_lines).
__host__ __device__ __forceinline__ uint64_t line_bytes_for(uint64_t len) {
    const uint64_t padded = 64 * ((len + kLineBias + 8) / 64 + 1);
    return (padded + 127) & ~127ull;
}

// DmaLanes for line-aligned keys (hash_key_dma_lines).  Piece i of a lane is 16-byte chunk c_i of key p_i = 8 i +
// lane / 8 with an XOR swizzle, c_i = (lane % 8) ^ (p_i / 2 % 8): key k's chunk q then sits at (its LDS row) + 16 (q ^
// (k / 2 % 8)), one XOR per read, and the 16 lanes of each ds_read_b128 bank group still hit 16 distinct 16-byte
// bank groups.  A piece is kept as what its issue needs: idx_i = 8 x (key p_i's first line) + c_i, its stage-0
// address in 16-byte units from the wave-uniform base (stage s: + 8 s), and how many bytes from there it has to load
// (two per register; stage s is live while 128 s < lim) -- per stage and piece an add, a 64-bit shift-add and a
// compare.  12 VGPRs per
// lane; needs the line copy under 64 GiB (idx < 2^32; pair_test_family checks).
struct DmaLinePieces {
    using G = DmaGeometry<2, 1>;
    uint32_t idx[G::kInsts];
    uint32_t lim2[G::kInsts / 2];  // bytes of pieces 2j (low half) / 2j+1 (high half) from their stage-0 start to load
    // key = base + line * 128 + kLineBias; a piece is live when it holds a byte of [line start, line start + end)
    // (end < 65536: the packet's bytes, or its padded message's up to the bit length).  Every lane's (line, end) goes
    // through the wave's LDS buffer, free until the first stage's DMA: one ds_write_b64 and eight broadcast
    // ds_read_b64 instead of sixteen ds_bpermute.
    __device__ __forceinline__ void init(const uint8_t* base, const uint8_t* key, uint32_t end, uint8_t* lds_wave) {
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t my_line = (uint32_t)((uint64_t)(key - base) >> 7);
        uint2* xs = (uint2*)lds_wave;
        xs[lane] = make_uint2(my_line, end);
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const uint32_t p = G::kKeysPerInst * i + lane / G::kChunks;
            const uint32_t c = (lane % G::kChunks) ^ ((p >> 1) & 7);
            const uint2 v = xs[p];
            idx[i] = (v.x << 3) + c;
            const uint32_t lim = max(v.y, 16 * c) - 16 * c;  // live while 128 s < lim
            if (i & 1) lim2[i / 2] |= lim << 16;
            else lim2[i / 2] = lim;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the reads are done before the first stage's DMA lands
        __builtin_amdgcn_wave_barrier();
    }
    // a 16-byte piece is loaded only when it holds bytes to hash: the last line of a packet moves only the chunks
    // its bytes reach (the rest of that line is padding)
    // lds: the wave's LDS buffer as a wave-uniform local address (lds_local), so each instruction's M0 is a scalar add
    template <bool SKIP = false>
    __device__ __forceinline__ void issue(uint32_t s, const uint8_t* base, uint32_t lds) const {
        if constexpr (SKIP) return;
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const uint32_t lim = (i & 1) ? lim2[i / 2] >> 16 : lim2[i / 2] & 0xffffu;
            if (s * 128 < lim)
                __builtin_amdgcn_global_load_lds((const void*)(base + ((uint64_t)(idx[i] + (s << 3)) << 4)),
                                                 (__attribute__((address_space(3))) void*)(uintptr_t)(lds + i * 1024),
                                                 16, 0, 0);
        }
    }
    // key k's (this lane's) chunk q of the staged line: its LDS row, then one XOR per chunk
    __device__ __forceinline__ static uint32_t row_of(uint32_t k) {
        return (k >> 3) * 1024 + 128 * (k & 7) + 16 * ((k >> 1) & 7);
    }
};

// Flags: kDmaSkipDead -- (NB == 2 only, where every wait is vmcnt(0)) lanes whose key has ended issue no load;
// kDmaPrio -- raise the wave's issue priority while it issues a stage's loads.
enum { kDmaSkipDead = 1, kDmaPrio = 2 };

// Message words of block b as loaded (little-endian, x[16]) -> the hash's input: the bytes past the message
// zeroed, the 0x80 terminator placed, byte-swapped for the big-endian hashes, the bit length in the final block.
// `full` (wave-uniform) says every lane's block lies wholly inside its message -- the common case with
// length-sorted lanes --, which leaves only the byte swap: no per-word compares or exec-mask branches.  The
// partial path is branch-free too (selects), so lanes of one wave with different lengths do not diverge.
template <class H>
__device__ __forceinline__ void finish_block(uint32_t* x, uint32_t o0, uint32_t total, bool last, bool full) {
    if (!full) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int rel = (int)total - (int)o0 - 4 * i;  // message bytes left at word i
            const uint32_t sh = (uint32_t)(rel & 3) * 8u;
            const uint32_t part = (x[i] & ((1u << sh) - 1u)) | (0x80u << sh);
            x[i] = rel >= 4 ? x[i] : (rel < 0 ? 0u : part);
        }
    }
    if (H::big_endian) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = bswap32(x[i]);
    }
    if (!full) {
        const uint64_t bits = (uint64_t)total * 8u;
        if (H::big_endian) {
            x[14] = last ? (uint32_t)(bits >> 32) : x[14];
            x[15] = last ? (uint32_t)bits : x[15];
        } else {
            x[14] = last ? (uint32_t)bits : x[14];
            x[15] = last ? (uint32_t)(bits >> 32) : x[15];
        }
    }
}

// finish_block for a block read from the line copy's padded message (line_bytes_for): the terminator and the zeros are
// in place already; only the byte swap and, in the final block, the bit length remain.
template <class H>
__device__ __forceinline__ void finish_block_padded(uint32_t* x, uint32_t total, bool last) {
    if (H::big_endian) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = bswap32(x[i]);
    }
    const uint64_t bits = (uint64_t)total * 8u;
    if (H::big_endian) {
        x[14] = last ? (uint32_t)(bits >> 32) : x[14];
        x[15] = last ? (uint32_t)bits : x[15];
    } else {
        x[14] = last ? (uint32_t)bits : x[14];
        x[15] = last ? (uint32_t)(bits >> 32) : x[15];
    }
}

// Wave-wide max / min of a lane value, wave-uniform (SGPR): DPP within each row of 16 lanes, then the four rows'
// results by readlane -- four VALU and four readlanes instead of six ds_bpermute round trips.  Every lane active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_max_uniform(uint32_t v) {
    v = max(v, dpp_u32<0xB1>(v));   // quad_perm [1, 0, 3, 2]
    v = max(v, dpp_u32<0x4E>(v));   // quad_perm [2, 3, 0, 1]
    v = max(v, dpp_u32<0x141>(v));  // row_half_mirror
    v = max(v, dpp_u32<0x140>(v));  // row_mirror
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return max(max(a, b), max(c, d));
}
__device__ __forceinline__ uint32_t wave_min_uniform(uint32_t v) {
    v = min(v, dpp_u32<0xB1>(v));
    v = min(v, dpp_u32<0x4E>(v));
    v = min(v, dpp_u32<0x141>(v));
    v = min(v, dpp_u32<0x140>(v));
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return min(min(a, b), min(c, d));
}

// wave minimum of a lane value
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

template <class H, int S = 2, int NB = 2, int FLAGS = 0>
__device__ __forceinline__ void hash_key_dma(const KeyView& kv, H& st, uint8_t* lds_wave) {
    static_assert(H::block_bytes == 64, "LDS-DMA staging is for 64-byte blocks");
    using G = DmaGeometry<S, NB>;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    uint32_t nbmax = nb;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, d, 64));
    const uint32_t nst = (nbmax + S - 1) / S;
    const uint32_t tmin = wave_min_u32(total);
    uint32_t preword = 0;
    for (uint32_t j = 0; j < r; ++j) preword |= (uint32_t)kv.pre[j] << (8 * j);
    const uint64_t base = (uint64_t)(uintptr_t)kv.key - r;  // window of block b starts at base + 64 b
    auto issue = [&](uint32_t s) {
        uint8_t* buf = lds_wave + (s % NB) * G::kStageBytes;
        if (FLAGS & kDmaPrio) __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const int p = G::kKeysPerInst * i + (int)(lane / G::kChunks);
            const uint32_t blo = __shfl((int)(uint32_t)base, p, 64), bhi = __shfl((int)(uint32_t)(base >> 32), p, 64);
            const uint32_t pend = __shfl((int)total, p, 64);
            const uint32_t c = ((lane % G::kChunks) + ((uint32_t)p >> G::kShift)) % G::kChunks;
            const uint64_t b64 = ((uint64_t)bhi << 32) | blo;
            const bool live = s * (S * 64) < pend;
            if ((FLAGS & kDmaSkipDead) && NB == 2) {
                if (live)
                    __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(b64 + s * (S * 64) + 16 * c),
                                                     (__attribute__((address_space(3))) void*)(buf + i * 1024), 16, 0, 0);
            } else {
                // always issue (the vmcnt accounting counts instructions); stages past the key re-read its start
                const uint64_t a = live ? b64 + s * (S * 64) + 16 * c : b64;
                __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)a,
                                                 (__attribute__((address_space(3))) void*)(buf + i * 1024), 16, 0, 0);
            }
        }
        if (FLAGS & kDmaPrio) __builtin_amdgcn_s_setprio(0);
    };
    st.init();
#pragma unroll
    for (int k = 0; k < NB - 1; ++k)
        if (k < (int)nst) issue(k);
    for (uint32_t s = 0; s < nst; ++s) {
        wait_vmcnt(((int)min(nst - 1, s + NB - 2) - (int)s) * G::kInsts);
        __builtin_amdgcn_wave_barrier();
        if (s + NB - 1 < nst) issue(s + NB - 1);
        const uint8_t* cur = lds_wave + (s % NB) * G::kStageBytes;
#pragma unroll
        for (int bb = 0; bb < S; ++bb) {
            const uint32_t b = S * s + bb;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = 4 * bb + q;
                const uint32_t slot = (c - (lane >> G::kShift)) % G::kChunks;
                const uint4 v = *(const uint4*)(cur + (lane / G::kKeysPerInst) * 1024 +
                                                16 * (G::kChunks * (lane % G::kKeysPerInst) + slot));
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
            if (b < nb) {
                const uint32_t o0 = b * 64;
                if (b == 0 && r) w[0] = (w[0] & ~low_bytes_mask(r)) | preword;
                finish_block<H>(w, o0, total, b + 1 == nb, o0 + 64 <= tmin);
                st.template compress<true>(w);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this stage's reads retire before its buffer refills
        __builtin_amdgcn_wave_barrier();
    }
}

// Single-buffer variant of hash_key_dma: one S*64-byte stage per key in LDS (S*4 KiB per wave); the stage is
// copied to registers as soon as it lands, and the next stage's DMA into the same buffer is issued before the
// blocks are compressed from the registers.  Half the LDS of the double-buffered form for the same amount in
// flight, so twice the waves fit a CU.  Dead lanes (key already ended) issue nothing; every wait is vmcnt(0).
// MODE (k_bloom DIAG diagnostics only): 0 = the product path, 1 = no packet loads (compress whatever the LDS buffer holds),
// 2 = loads only (no compress)
template <class H, int S = 1, int MODE = 0>
__device__ __forceinline__ void hash_key_dma_reg(const KeyView& kv, H& st, uint8_t* lds_wave) {
    static_assert(H::block_bytes == 64, "LDS-DMA staging is for 64-byte blocks");
    using G = DmaGeometry<S, 1>;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    uint32_t nbmax = nb;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, d, 64));
    const uint32_t nst = (nbmax + S - 1) / S;
    const uint32_t tmin = wave_min_u32(total);
    uint32_t preword = 0;
    for (uint32_t j = 0; j < r; ++j) preword |= (uint32_t)kv.pre[j] << (8 * j);
    DmaLanes<S> dl;
    dl.init((uint64_t)(uintptr_t)kv.key - r, total);
    st.init();
    if (nst) dl.template issue<MODE == 1>(0, lds_wave);
    for (uint32_t s = 0; s < nst; ++s) {
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): stage s has landed
        __builtin_amdgcn_wave_barrier();
        uint32_t w[S][16];
#pragma unroll
        for (int bb = 0; bb < S; ++bb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = 4 * bb + q;
                const uint32_t slot = (c - (lane >> G::kShift)) % G::kChunks;
                const uint4 v = *(const uint4*)(lds_wave + (lane / G::kKeysPerInst) * 1024 +
                                                16 * (G::kChunks * (lane % G::kKeysPerInst) + slot));
                w[bb][4 * q] = v.x; w[bb][4 * q + 1] = v.y; w[bb][4 * q + 2] = v.z; w[bb][4 * q + 3] = v.w;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the buffer is free again
        __builtin_amdgcn_wave_barrier();
        if (s + 1 < nst) dl.template issue<MODE == 1>(s + 1, lds_wave);
#pragma unroll
        for (int bb = 0; bb < S; ++bb) {
            const uint32_t b = S * s + bb;
            if (b < nb) {
                uint32_t* x = w[bb];
                const uint32_t o0 = b * 64;
                if (b == 0 && r) x[0] = (x[0] & ~low_bytes_mask(r)) | preword;
                finish_block<H>(x, o0, total, b + 1 == nb, o0 + 64 <= tmin);
                if (MODE != 2) st.template compress<true>(x);
                else st.h[0] ^= x[0] ^ x[5] ^ x[10] ^ x[15];
            }
        }
    }
}

// Line-staged packets (the store's line copy, dsy_capi.hip store_build_lines): every packet starts kLineBias = 1 byte
// into a 128-byte line, so stage s of a key is exactly line s of it -- every DMA piece is one whole line, no line is
// fetched twice (tools/hashbench: 70 vs 57 Gblk/s MD5 over the same packets, 4.3 vs 3.5 TB/s) -- and the message
// prefix || packet of a 1-byte prefix starts on the line: its blocks are the line's words as loaded, with the slack
// byte in front of the packet replaced by the prefix byte.  A prefix of r bytes shifts the message by r - 1 bytes
// (wave-uniform: one claim per wave): a uniform alignbyte funnel with a one-dword carry from the previous stage.
// Single 8 KiB buffer per wave, like hash_key_dma_reg<H, 2>.  Requires 1 <= r <= 4 (the responder routes other
// prefixes to the byte-wise path), kv.key = lines + 128 * line + kLineBias, at most 2^32 lines past `lines` (the
// copy's base, wave-uniform); line bytes past the packet are not loaded (their words are masked by finish_block) --
// except with PADDED (every lane's prefix is 1 byte, the message is line-aligned): the line copy holds the padded
// message (line_bytes_for), its pieces are loaded up to the bit length and the blocks need no masking.
// preword: the r prefix bytes, little-endian (wave-uniform: read once per claim).  nbmax: the wave's most blocks
// (wave-uniform; the caller has it).  MODE as in hash_key_dma_reg (k_pair_test DIAG diagnostics only).
template <class H, int MODE = 0, bool PADDED = false>
__device__ __forceinline__ void hash_key_dma_lines(const KeyView& kv, H& st, uint8_t* lds_wave, uint32_t preword,
                                                   const uint8_t* lines, uint32_t nbmax) {
    static_assert(H::block_bytes == 64, "LDS-DMA staging is for 64-byte blocks");
    static_assert(kLineBias == 1, "the shift below assumes one byte of slack before every packet");
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;  // wave-uniform, 1..4
    const uint32_t len = kv.len;
    const uint32_t total = r + len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    const uint32_t nst = (nbmax + 1) / 2;
    const uint32_t tmin = PADDED ? 0u : wave_min_uniform(total);
    DmaLinePieces dl;
    dl.init(lines, kv.key, PADDED ? 64 * nb - 8 : len + (uint32_t)kLineBias, lds_wave);  // stage s: line s of the packet
    st.init();
    // message byte j is line byte j - rr (rr = r - 1): the carry is the dword before the stage's first one, its top
    // rr bytes the message bytes before the stage (at stage 0 the first rr prefix bytes); the slack byte, line byte 0
    // of stage 0, becomes the last prefix byte
    const uint32_t rr = PADDED ? 0u : r - 1;
    uint32_t carry = rr ? (preword & low_bytes_mask(rr)) << (8 * (4 - rr)) : 0u;
    const uint32_t slack = (preword >> (8 * rr)) & 0xffu;
    const uint32_t sh = (4 - rr) & 3;  // alignbyte shift for rr in 1..3
    const uint32_t lds = lds_local(lds_wave);
    if (nst) dl.template issue<MODE == 1>(0, lines, lds);
    for (uint32_t s = 0; s < nst; ++s) {
        __builtin_amdgcn_s_waitcnt(0x0f70);
        __builtin_amdgcn_wave_barrier();
        uint32_t d[33];
        d[0] = carry;
        const uint32_t row = DmaLinePieces::row_of(lane);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 v = *(const uint4*)(lds_wave + (row ^ (16u * q)));
            d[1 + 4 * q] = v.x; d[2 + 4 * q] = v.y; d[3 + 4 * q] = v.z; d[4 + 4 * q] = v.w;
        }
        if (s == 0) d[1] = (d[1] & ~0xffu) | slack;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        if (s + 1 < nst) dl.template issue<MODE == 1>(s + 1, lines, lds);
        carry = d[32];
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const uint32_t b = 2 * s + bb;
            if (b < nb) {
                uint32_t x[16];
                // message word i of block b = line bytes [64 bb + 4 i - rr, +4): d[1 + 16 bb + i] shifted by rr
                if (rr == 0) {  // the 1-byte prefix of every reference claim: the line's words as loaded
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] = d[1 + 16 * bb + i];
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(d[1 + 16 * bb + i], d[16 * bb + i], sh);
                }
                const uint32_t o0 = b * 64;
                if (PADDED) finish_block_padded<H>(x, total, b + 1 == nb);
                else finish_block<H>(x, o0, total, b + 1 == nb, o0 + 64 <= tmin);
                if (MODE != 2) st.template compress<true>(x);
                else st.h[0] ^= x[0] ^ x[5] ^ x[10] ^ x[15];
            }
            // keep block 1's message words from being formed while block 0 compresses (register pressure: the
            // responder kernel's occupancy is set by its VGPR count)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <class H>
__device__ __forceinline__ void hash_key(const KeyView& kv, H& st) {
    if (kv.plen <= 4) hash_key_short_prefix<H>(kv, st);
    else hash_key_generic<H>(kv, st);
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

// ceil(2^32 / m) for 2 <= m < 2^31, else 0: the multiplier bit_position uses instead of a division per probe (the
// claim records carry it, DevRequest::m_recip, so the responder does not divide at all).
__host__ __device__ inline uint32_t mod_recip(uint64_t m) {
    return (m >= 2 && m < (1ull << 31)) ? (uint32_t)(0xFFFFFFFFu / (uint32_t)m) + 1u : 0u;
}

// pos = chunk % m  (bloomfilter.py:171), by multiply-high with recip = mod_recip(m) (m < 2^31 for 'H'/'L' chunks,
// bloomfilter.py:135-140).  A generic 32-bit remainder costs two quarter-rate multiplies and two conditional
// subtractions per probe (k probes per key); these cost one multiply-high and two full-rate ops:
//   'H' (a < 2^16, 8 <= m < 2^15): q = mulhi(a, ceil(2^32/m)) is floor(a/m) exactly -- the excess a*e/2^32 < 2^-16
//        is below the 1/m gap to the next integer -- so r = a - q*m (a 24-bit multiply).  m >= 8: check_family
//        refuses sizes that are not positive multiples of eight.
//   'L' (a < 2^32, 2^15 <= m < 2^31): q is floor(a/m) or one more, so r = a - q*m is right or wrapped below zero
//        (>= 2^32 - m); min(r, r + m) picks the right one.
// tests/test_bitmod.py checks both against % (every 'H' pair exhaustively) and the device positions against hashlib.
template <int CHUNK>
__device__ __forceinline__ uint64_t bit_position(uint64_t chunk, uint64_t m, uint32_t recip) {
    if constexpr (CHUNK == 8) {
        return chunk % m;
    } else if constexpr (CHUNK == 2) {
        const uint32_t a = (uint32_t)chunk;
        return a - __umul24(__umulhi(a, recip), (uint32_t)m);
    } else {
        const uint32_t a = (uint32_t)chunk;
        const uint32_t r = a - __umulhi(a, recip) * (uint32_t)m;
        return min(r, r + (uint32_t)m);
    }
}

template <int CHUNK>
__device__ __forceinline__ uint64_t bit_position(uint64_t chunk, uint64_t m) {
    return bit_position<CHUNK>(chunk, m, CHUNK == 8 ? 0u : mod_recip(m));
}

// Membership of one key: 1 when all k probed bits are set (bloomfilter.py:185-197).  Every chunk the digest holds
// is looked up -- no branch per probe, so the k loads go out together behind one wait instead of one round trip
// each -- and the ones past k do not count (their positions are < m, so the reads stay inside the filter).
template <class H, int CHUNK, class W>
__device__ __forceinline__ uint32_t filter_has_all(W* fb, const H& st, uint32_t k, uint64_t m, uint32_t recip) {
    constexpr int kmax = ChunkLimit<H, CHUNK>::kmax;
    uint32_t w[kmax], sh[kmax];
#pragma unroll
    for (int j = 0; j < kmax; ++j) {
        const uint64_t pos = bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m, recip);
        w[j] = fb[pos >> 5];
        sh[j] = (uint32_t)pos & 31u;
    }
    // the words are needed here, in order: every load has been issued before the first wait (left to itself the
    // scheduler interleaves load, wait, test to save registers)
#pragma unroll
    for (int j = 0; j < kmax; ++j) asm volatile("" : "+v"(w[j])::"memory");
    uint32_t ok = 1;
#pragma unroll
    for (int j = 0; j < kmax; ++j) ok &= (w[j] >> sh[j]) | (uint32_t)(j >= (int)k);
    return ok & 1u;
}

template <class H, int CHUNK, class W>
__device__ __forceinline__ uint32_t filter_has_all(W* fb, const H& st, uint32_t k, uint64_t m) {
    return filter_has_all<H, CHUNK>(fb, st, k, m, CHUNK == 8 ? 0u : mod_recip(m));
}

// Filter build of one key per lane (bloomfilter.py:172-178: filter |= 1 << pos for its k positions).  Called by the
// whole wave (`active`: the lane holds a key), so the wave-level modes can ballot and shuffle.
//   OR_MODE 0  one atomic OR per lane per probe.
//   OR_MODE 1  the k words are read first (one batch, as filter_has_all); a probe's OR is issued only by the lanes
//              whose bit is still clear, and skipped by the wave when none is (a saturating filter -- 100 k keys
//              into a 10 Kbit MTU filter -- needs almost no atomics after its first few thousand keys).
//   OR_MODE 2  OR_MODE 1, and when at most kOrLeaders lanes still need a probe, the lanes that need the same word
//              are merged into one OR by a leader (wave-aggregated atomicOr: a wave OR-reduction per distinct word).
static constexpr int kOrLeaders = 4;
// wbase: the lane's filter starts wbase words past fb (lanes of one wave may fill different filters; fb is uniform)
template <class H, int CHUNK, int OR_MODE, class W>
__device__ __forceinline__ void filter_set_all(W* fb, const H& st, uint32_t k, uint64_t m, bool active,
                                               uint32_t wbase = 0) {
    constexpr int kmax = ChunkLimit<H, CHUNK>::kmax;
    const uint32_t recip = CHUNK == 8 ? 0u : mod_recip(m);
    if constexpr (OR_MODE == 0) {
#pragma unroll
        for (int j = 0; j < kmax; ++j) {
            if (active && j < (int)k) {
                const uint64_t pos = bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m, recip);
                atomicOr(&fb[wbase + (uint32_t)(pos >> 5)], 1u << (pos & 31));
            }
        }
        return;
    }
    uint32_t w[kmax], idx[kmax], bit[kmax];
#pragma unroll
    for (int j = 0; j < kmax; ++j) {
        const uint64_t pos = active ? bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m, recip) : 0;
        idx[j] = wbase + (uint32_t)(pos >> 5);
        bit[j] = 1u << (pos & 31);
        w[j] = fb[idx[j]];
    }
#pragma unroll
    for (int j = 0; j < kmax; ++j) asm volatile("" : "+v"(w[j])::"memory");
#pragma unroll
    for (int j = 0; j < kmax; ++j) {
        const bool need = active && j < (int)k && !(w[j] & bit[j]);
        if constexpr (OR_MODE == 2) {
            uint64_t pend = __ballot(need);
            if (!pend) continue;
            if (__popcll(pend) <= kOrLeaders) {
                const uint32_t lane = threadIdx.x & 63;
                while (pend) {
                    const int leader = __builtin_ctzll(pend);
                    const uint32_t wi = (uint32_t)__shfl((int)idx[j], leader, 64);
                    const bool same = need && idx[j] == wi;
                    uint32_t v = same ? bit[j] : 0u;
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) v |= (uint32_t)__shfl_xor((int)v, d, 64);
                    if (lane == (uint32_t)leader) atomicOr(&fb[wi], v);
                    pend &= ~__ballot(same);
                }
                continue;
            }
        }
        if (need) atomicOr(&fb[idx[j]], bit[j]);
    }
}

}  // namespace dsy
