// dsy_bloom_kernels.hip -- single-filter Bloom kernels for gfx950: build (add), membership test, index dump.
//
// Mapping: one key per lane (Merkle-Damgard is sequential per message), 256-thread workgroups, a grid-stride
// loop over 64-key wave-tasks.  Large batches are first put in length-bucketed order (k_len_* below: a counting
// sort of the keys by compression-block count, longest first) so the 64 lanes of a wave run the same number of
// blocks; the sort writes 16-byte task records (blob offset, length, key index) that the hashing kernel reads
// contiguously.  Small filters (the ~10 Kbit MTU filters of community.py:637-666) live in LDS for the whole
// workgroup: the build ORs bits with ds_or_b32 and merges the LDS filter into HBM once per workgroup; the test
// stages the filter into LDS once and probes it there.  Large filters (m = 2^20..2^24 bits, BASELINE config 4)
// are probed/ORed in place in L2/HBM with global atomics.  MD5 and SHA-1 stage packet bytes through LDS with
// LDS-DMA when the filter is small (dsy_message.h hash_key_dma_reg); SHA-2 loads directly.
#include "dsy_kernels.h"

namespace dsy {

// ---------------------------------------------------------------------------------------------------------
// Line-aligned staging of PACKED keys (k_bloom: config 1's add_keys / __contains__ over a caller's blob, and claim
// filters over the store's line copy).  hash_key_dma_reg stages each key's message as windows [base + 128 s, +128)
// with base = key - prefix at any byte alignment: a window straddles two 128-byte lines, and the line it shares with
// the next window is requested again one stage later -- ~8 us later under load, past the XCD L2's turnover
// (4 MiB at ~0.7 TB/s), so it is fetched twice (config 1 moved 1.5-1.6x its bytes).  Here stage s moves
// whole LINES: line s + shift of the key (shift 0 or 1, below), 8 x 16-byte pieces, each line of the message once.
// A block of the message then starts anywhere in a line, so each key's LDS row is [carry 64 B][line 128 B]: the carry
// is the previous line's last 64 bytes (copied there, LDS to LDS, after a stage's reads), and the two blocks of a stage
// are the 128 bytes at row offset e0 (1..64, per key) -- 33 dword reads at a per-lane address and one alignbyte per
// word.
//   a = base & 127 (where the message starts in its first line)
//   a == 0       lag 0, shift 0: e0 = 64, stage s hashes blocks 2s, 2s + 1
//   1 <= a <= 64 lag 1, shift 0: e0 = a, stage s hashes blocks 2s - 1, 2s (stage 0's first slot is empty)
//   a > 64       lag 0, shift 1: e0 = a - 64; stage 0 stages line 1 and, as its carry, line 0's last 64 bytes (the
//                message starts there), so stage s hashes blocks 2s, 2s + 1
// A key takes line_stages(nb, a) = ceil((nb + lag) / 2) stages; the length sort (k_len_*, LenSort::line_mode) orders
// keys by that count, so a wave's lanes run the same number of stages.
struct LineStaging {
    static constexpr int kRowBytes = 192;                      // [carry 64 B][line 128 B] per key
    static constexpr int kInsts = 64 * kRowBytes / 1024;       // 12 DMA wave-instructions cover the wave's rows
    static constexpr int kWaveBytes = 64 * kRowBytes;          // 12 KiB per wave
};

__host__ __device__ __forceinline__ uint32_t line_lag(uint32_t a) { return (a >= 1u && a <= 64u) ? 1u : 0u; }
__host__ __device__ __forceinline__ uint32_t line_stages(uint32_t nb, uint32_t a) { return (nb + line_lag(a) + 1u) / 2u; }

// The pieces one lane moves for its wave's 64 keys.  DMA wave-instruction i writes LDS bytes [1024 i, +1024) of the
// wave's buffer, lane t the 16 bytes at 1024 i + 16 t: 16-byte slot g = 64 i + t is piece g % 12 of key g / 12's row
// (pieces 0-3 the carry, 4-11 the line).  Per piece: idx = its stage-0 address in 16-byte units from the wave-uniform
// base (stage s: + 8 s); lim: stage s >= 1 is live while 128 s < lim; m0: bit i = piece i is live at stage 0 (the
// first line's pieces before the message, and the carry pieces of keys with shift 1).  25 VGPRs.
struct DmaPackedPieces {
    using G = LineStaging;
    uint32_t idx[G::kInsts];
    uint32_t lim[G::kInsts];
    uint32_t m0;
    // line: the key's first line (from the wave base, < 2^28); lo / hi: the bytes to load, [lo, hi) from that line's
    // start (the prefix bytes are merged in registers, not loaded)
    __device__ __forceinline__ void init(uint32_t line, uint32_t shift, uint32_t lo, uint32_t hi, uint8_t* lds_wave) {
        const uint32_t lane = threadIdx.x & 63;
        uint4* xs = (uint4*)lds_wave;
        xs[lane] = make_uint4(line, shift, lo, hi);
        m0 = 0;
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const uint32_t g = 64u * i + lane;
            const uint32_t p = g / 12u, k = g % 12u;
            const uint4 v = xs[p];
            uint32_t start0, live0;  // the piece's stage-0 byte range [start0, +16) from the key's first line
            if (k < 4) {             // carry piece: line 0's bytes 64 + 16 k, staged only at stage 0 (shift 1)
                start0 = 64u + 16u * k;
                idx[i] = 8u * v.x + 4u + k;
                lim[i] = 0u;
                live0 = v.y;
            } else {
                const uint32_t c = k - 4u;
                start0 = 128u * v.y + 16u * c;
                idx[i] = 8u * (v.x + v.y) + c;
                lim[i] = v.w > start0 ? v.w - start0 : 0u;
                live0 = 1u;
            }
            live0 &= (start0 < v.w) & (start0 + 16u > v.z);
            m0 |= live0 << i;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the reads are done before the first stage's DMA lands
        __builtin_amdgcn_wave_barrier();
    }
    template <bool SKIP = false>
    __device__ __forceinline__ void issue(uint32_t s, const uint8_t* base, uint32_t lds) const {
        if constexpr (SKIP) return;
#pragma unroll
        for (int i = 0; i < G::kInsts; ++i) {
            const bool live = s ? 128u * s < lim[i] : ((m0 >> i) & 1u) != 0u;
            if (live)
                __builtin_amdgcn_global_load_lds((const void*)(base + ((uint64_t)(idx[i] + (s << 3)) << 4)),
                                                 (__attribute__((address_space(3))) void*)(uintptr_t)(lds + i * 1024),
                                                 16, 0, 0);
        }
    }
};

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d, 64);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

// prefix || key of every lane (prefix <= 4 bytes) through line-aligned LDS stages (above); called by ALL 64 lanes of a
// wave together (idle lanes: a zero-length key at any address).  Falls back to direct loads for a wave whose keys
// span 32 GiB or more (the pieces' 32-bit 16-byte offsets).  MODE as in hash_key_dma_reg (DIAG builds only).
template <class H, int MODE = 0>
__device__ __forceinline__ void hash_key_dma_packed(const KeyView& kv, H& st, uint8_t* lds_wave, uint32_t preword) {
    static_assert(H::block_bytes == 64, "LDS-DMA staging is for 64-byte blocks");
    using G = LineStaging;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = kv.plen;
    const uint32_t total = r + kv.len;
    const uint32_t nb = n_blocks(total, 64, H::len_bytes);
    const uint64_t base = (uint64_t)(uintptr_t)kv.key - r;
    const uint64_t wline = wave_min_u64(base >> 7);  // the wave's lowest line: piece offsets are 32-bit from there
    const uint64_t span = (base >> 7) - wline;
    if (__builtin_amdgcn_readfirstlane((uint32_t)(__ballot(span >= (1ull << 28)) != 0))) {
        hash_key<H>(kv, st);
        return;
    }
    const uint8_t* wbase = (const uint8_t*)(uintptr_t)(wline << 7);
    const uint32_t a = (uint32_t)base & 127u;
    const uint32_t lag = line_lag(a), shift = a > 64u ? 1u : 0u;
    const uint32_t e0 = a + 64u - 64u * lag - 128u * shift;  // 1..64
    const uint32_t nst = wave_max_uniform(line_stages(nb, a));
    const uint32_t tmin = wave_min_uniform(total);
    const uint32_t lag_min = wave_min_uniform(lag);  // the slot's highest block is 2 s + bb - lag_min
    DmaPackedPieces dl;
    dl.init((uint32_t)span, shift, a + r, a + total, lds_wave);
    st.init();
    const uint32_t lds = lds_local(lds_wave);
    const uint8_t* row = lds_wave + lane * G::kRowBytes;
    const uint32_t* win = (const uint32_t*)(row + (e0 & ~3u));
    const uint32_t sh = e0 & 3u;
    if (nst) dl.template issue<MODE == 1>(0, wbase, lds);
    for (uint32_t s = 0; s < nst; ++s) {
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): stage s has landed
        __builtin_amdgcn_wave_barrier();
        uint32_t d[33];
#pragma unroll
        for (int i = 0; i < 33; ++i) d[i] = win[i];
        // the line's last 64 bytes: the next stage's carry (four named registers: an array of them was kept in
        // scratch by the compiler)
        const uint4 t0 = *(const uint4*)(row + 128), t1 = *(const uint4*)(row + 144);
        const uint4 t2 = *(const uint4*)(row + 160), t3 = *(const uint4*)(row + 176);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the line slots are free again
        __builtin_amdgcn_wave_barrier();
        *(uint4*)(row) = t0;  // (the DMA below writes only the line slots)
        *(uint4*)(row + 16) = t1;
        *(uint4*)(row + 32) = t2;
        *(uint4*)(row + 48) = t3;
        if (s + 1 < nst) dl.template issue<MODE == 1>(s + 1, wbase, lds);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int b = (int)(2 * s + bb) - (int)lag;
            if (b >= 0 && b < (int)nb) {
                uint32_t x[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(d[16 * bb + i + 1], d[16 * bb + i], sh);
                if (b == 0 && r) x[0] = (x[0] & ~low_bytes_mask(r)) | preword;
                // (wave-uniform: every lane's block lies inside its message when the slot's highest one does)
                finish_block<H>(x, 64u * (uint32_t)b, total, b + 1 == (int)nb, 64u * (2 * s + bb + 1 - lag_min) <= tmin);
                if (MODE != 2) st.template compress<true>(x);
                else st.h[0] ^= x[0] ^ x[5] ^ x[10] ^ x[15];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

static constexpr uint32_t kLenBins = kLenSortBins;
static constexpr int kDmaS = 2;
static constexpr size_t kDmaWaveBytes = DmaGeometry<kDmaS, 1>::kWaveBytes;
static constexpr size_t kLineWaveBytes = LineStaging::kWaveBytes;

// bin of a key in the length sort, longest first: by compression blocks, or (line_mode: the line-staged hashing,
// hash_key_dma_packed) by block slots and lag -- a lane of lag 1 fills block slots 1 .. nb, one of lag 0 slots
// 0 .. nb - 1, so keys of equal nb + lag and equal lag run the same slots: a slot no lane of the wave needs (the empty
// first one of a lag-1 wave, the last one of an odd count) is skipped as a whole instead of hashed for a few lanes
__device__ __forceinline__ uint32_t len_bin(uint64_t off, uint64_t len, const LenSort& s) {
    uint32_t units = n_blocks(s.plen + (uint32_t)len, s.blk, s.lenb);
    if (s.line_mode) {
        const uint32_t lag = line_lag((s.base_lo + (uint32_t)off - s.plen) & 127u);
        units = 2u * (units + lag) + lag;
    }
    return kLenBins - 1u - min(units, kLenBins - 1u);
}

__device__ __forceinline__ void key_span(const uint64_t* __restrict__ offsets, const uint64_t* __restrict__ rows,
                                         const RowRec* __restrict__ rec, uint64_t i, uint64_t* off, uint32_t* len) {
    const uint64_t row = rows ? rows[i] : i;
    if (rec) {  // store rows: the packet's place in the store's line copy
        const RowRec r = rec[row];
        *off = r.off;
        *len = r.len;
        return;
    }
    const uint64_t a = offsets[row], e = offsets[row + 1];
    *off = a;
    *len = (uint32_t)(e - a);
}

// ---------------------------------------------------------------------------- length-bucketed task order
// pass 1: global histogram of bins (LDS-aggregated)
__global__ void __launch_bounds__(256) k_len_hist(LenSort s, const uint64_t* __restrict__ offsets,
                                                  const uint64_t* __restrict__ rows, const RowRec* __restrict__ rec, uint64_t n,
                                                  uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kLenBins];
    for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t off;
        uint32_t len;
        key_span(offsets, rows, rec, i, &off, &len);
        atomicAdd(&h[len_bin(off, len, s)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// pass 2: exclusive scan of the bins (one workgroup of kLenBins threads)
__global__ void __launch_bounds__(kLenBins) k_len_scan(uint32_t* __restrict__ hist) {
    __shared__ uint32_t part[kLenBins];
    const uint32_t t = threadIdx.x;
    const uint32_t v = hist[t];
    part[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kLenBins; d <<= 1) {
        const uint32_t add = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    hist[t] = part[t] - v;
}

// pass 3: scatter task records; each workgroup reserves its bins' ranges with one global atomic per bin
static constexpr uint32_t kScatterChunk = 4096;
__global__ void __launch_bounds__(256) k_len_scatter(LenSort s, const uint64_t* __restrict__ offsets,
                                                     const uint64_t* __restrict__ rows, const RowRec* __restrict__ rec, uint64_t n,
                                                     uint32_t* __restrict__ base, PairTask* __restrict__ tasks) {
    __shared__ uint32_t cnt[kLenBins];
    __shared__ uint32_t at[kLenBins];
    for (uint64_t c0 = (uint64_t)blockIdx.x * kScatterChunk; c0 < n; c0 += (uint64_t)gridDim.x * kScatterChunk) {
        const uint64_t c1 = min(n, c0 + kScatterChunk);
        for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x) cnt[i] = 0;
        __syncthreads();
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            uint64_t off;
            uint32_t len;
            key_span(offsets, rows, rec, i, &off, &len);
            atomicAdd(&cnt[len_bin(off, len, s)], 1u);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x) {
            at[i] = cnt[i] ? atomicAdd(&base[i], cnt[i]) : 0u;
            cnt[i] = 0;
        }
        __syncthreads();
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            PairTask tk;
            key_span(offsets, rows, rec, i, &tk.off, &tk.len);
            tk.slot = (uint32_t)i;
            const uint32_t b = len_bin(tk.off, tk.len, s);
            tasks[at[b] + atomicAdd(&cnt[b], 1u)] = tk;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------- hash + probe / set
// DIAG (DMA path, 2-byte chunks only): 0 = the product kernel; 1 = no packet loads (the stage is hashed as left in
// LDS: the compute ceiling); 2 = packet loads without the compression (the gather ceiling).  Diagnostics only, selected
// by the ctx's DSY_BLOOM_DIAG environment knob (tools/hash_sweep.py); results are meaningless for DIAG != 0.
// OP 0: add (filter_set_all, OR_MODE as there), OP 1: test (present[key] = all k bits set).
// DMA 0: direct loads (hash_key); 1: LDS-DMA windows at the key's own alignment (hash_key_dma_reg); 2: line-aligned
// LDS-DMA stages (hash_key_dma_packed: each line of a key moved once).
template <class H, int CHUNK, int OP, int DMA, int DIAG = 0, int OR_MODE = 0>
__global__ void __launch_bounds__(256, 3) k_bloom(const DevParams* __restrict__ prm, const uint8_t* __restrict__ blob,
                                               const uint64_t* __restrict__ offsets, const uint64_t* __restrict__ rows,
                                               const RowRec* __restrict__ rec, const PairTask* __restrict__ tasks, uint64_t n,
                                               uint32_t* __restrict__ filter, uint32_t nwords, int use_lds,
                                               uint8_t* __restrict__ present) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    constexpr size_t kWaveLds = DMA == 2 ? kLineWaveBytes : DMA == 1 ? kDmaWaveBytes : 0;
    uint8_t* my_dma = dyn_lds + (threadIdx.x >> 6) * kWaveLds;
    uint32_t* lds_filter = (uint32_t*)(dyn_lds + 4 * kWaveLds);
    const uint64_t m = prm->m_bits;
    const uint32_t k = prm->k;
    uint32_t preword = 0;  // the prefix's bytes, little-endian (DMA 2; <= 4 bytes)
    if constexpr (DMA == 2)
        for (uint32_t j = 0; j < min(prm->prefix_len, 4u); ++j) preword |= (uint32_t)prm->prefix[j] << (8 * j);
    if (use_lds) {
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) lds_filter[i] = OP == 0 ? 0u : filter[i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (n + 63) / 64;
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // (the wave index through readfirstlane: wave-uniform to the compiler, so the loop control is scalar)
    const uint64_t v0 = (uint64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t v = v0; v < waves; v += wstride) {
        const uint64_t i = v * 64 + lane;
        const bool active = i < n;
        // idle lanes hash an empty key; the LDS-DMA path still reads its stage from key - prefix_len, so the key
        // must sit past readable bytes: a packed blob has DSY_BLOB_GUARD of them before it, a store's line copy
        // (rec) keeps its guard inside the allocation
        KeyView kv{rec ? blob + DSY_BLOB_GUARD : blob, 0u, prm->prefix, prm->prefix_len};
        uint64_t slot = i;
        if (active) {
            if (tasks) {
                const PairTask tk = tasks[i];
                kv.key = blob + tk.off;
                kv.len = tk.len;
                slot = tk.slot;
            } else {
                uint64_t off;
                key_span(offsets, rows, rec, i, &off, &kv.len);
                kv.key = blob + off;
            }
        }
        H st;
        if constexpr (DMA == 2) hash_key_dma_packed<H, DIAG>(kv, st, my_dma, preword);
        else if constexpr (DMA == 1) hash_key_dma_reg<H, kDmaS, DIAG>(kv, st, my_dma);
        else hash_key<H>(kv, st);
        // two call sites, so each sees where its filter lives: ds_or / ds_read on the LDS copy, global atomics /
        // loads on the HBM one (one pointer picked at run time would be a flat pointer: every probe a flat atomic or
        // load behind its own vmcnt(0) wait -- 30 % of the SHA-1 add kernel)
        if constexpr (OP == 0) {
            if (use_lds) filter_set_all<H, CHUNK, OR_MODE>(lds_filter, st, k, m, active);
            else filter_set_all<H, CHUNK, OR_MODE>(filter, st, k, m, active);
        } else if (active) {
            const uint32_t ok = use_lds ? filter_has_all<H, CHUNK>(lds_filter, st, k, m)
                                        : filter_has_all<H, CHUNK>(filter, st, k, m);
            present[slot] = (uint8_t)ok;
        }
    }
    if (OP == 0 && use_lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) {
            const uint32_t val = lds_filter[i];
            if (val) atomicOr(&filter[i], val);
        }
    }
}

template <class H, int CHUNK>
__global__ void __launch_bounds__(256) k_bloom_indices(const DevParams* __restrict__ prm, const uint8_t* __restrict__ blob,
                                                       const uint64_t* __restrict__ offsets, uint64_t n,
                                                       uint64_t* __restrict__ out) {
    const uint64_t m = prm->m_bits;
    const uint32_t k = prm->k;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a = offsets[i], e = offsets[i + 1];
        KeyView kv{blob + a, (uint32_t)(e - a), prm->prefix, prm->prefix_len};
        H st;
        hash_key<H>(kv, st);
#pragma unroll
        for (int j = 0; j < ChunkLimit<H, CHUNK>::kmax; ++j)
            if (j < (int)k) out[i * k + j] = bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m);
    }
}

// ------------------------------------------------------------------------------ union of partial filters
__global__ void __launch_bounds__(256) k_or_reduce(const uint4* __restrict__ parts, uint32_t n_parts, uint64_t vecs,
                                                   uint64_t stride_vecs, uint4* __restrict__ out) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < vecs; i += step) {
        uint4 acc = parts[i];
        for (uint32_t g = 1; g < n_parts; ++g) {
            const uint4 v = parts[g * stride_vecs + i];
            acc.x |= v.x; acc.y |= v.y; acc.z |= v.z; acc.w |= v.w;
        }
        out[i] = acc;
    }
}

__global__ void __launch_bounds__(256) k_or_reduce_tail(const uint32_t* __restrict__ parts, uint32_t n_parts,
                                                        uint64_t first, uint64_t words, uint32_t* __restrict__ out) {
    const uint64_t w = first + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    uint32_t acc = 0;
    for (uint32_t g = 0; g < n_parts; ++g) acc |= parts[g * words + w];
    out[w] = acc;
}

hipError_t launch_or_reduce(const uint32_t* parts, uint32_t n_parts, uint64_t words, uint32_t* out, uint32_t max_grid,
                            hipStream_t stream) {
    // 16-byte vectors when every part starts 16-byte aligned (words % 4 == 0 and aligned base pointers)
    const bool vec = words % 4 == 0 && ((uintptr_t)parts % 16) == 0 && ((uintptr_t)out % 16) == 0;
    uint64_t done = 0;
    if (vec && words) {
        const uint64_t vecs = words / 4;
        const uint64_t want = (vecs + 255) / 256;
        const uint32_t grid = (uint32_t)(want < max_grid ? want : max_grid);
        hipLaunchKernelGGL(k_or_reduce, dim3(grid), dim3(256), 0, stream, (const uint4*)parts, n_parts, vecs, vecs,
                           (uint4*)out);
        done = words;
    }
    if (done < words) {
        const uint64_t rest = words - done;
        hipLaunchKernelGGL(k_or_reduce_tail, dim3((uint32_t)((rest + 255) / 256)), dim3(256), 0, stream, parts, n_parts,
                           done, words, out);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ dispatch
hipError_t launch_len_sort(const LenSort& s, const uint64_t* offsets, const uint64_t* rows, const RowRec* rec, uint64_t n,
                           uint32_t* d_bins, PairTask* d_tasks, uint32_t max_grid, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(d_bins, 0, kLenBins * 4, stream);
    if (e != hipSuccess) return e;
    const uint64_t want = (n + 255) / 256;
    const uint32_t grid = (uint32_t)(want < max_grid ? (want ? want : 1) : max_grid);
    hipLaunchKernelGGL(k_len_hist, dim3(grid), dim3(256), 0, stream, s, offsets, rows, rec, n, d_bins);
    hipLaunchKernelGGL(k_len_scan, dim3(1), dim3(kLenBins), 0, stream, d_bins);
    const uint64_t chunks = (n + kScatterChunk - 1) / kScatterChunk;
    const uint32_t sgrid = (uint32_t)(chunks < max_grid ? (chunks ? chunks : 1) : max_grid);
    hipLaunchKernelGGL(k_len_scatter, dim3(sgrid), dim3(256), 0, stream, s, offsets, rows, rec, n, d_bins, d_tasks);
    return hipGetLastError();
}

// Which staging k_bloom uses (bloom_staging): 2 = line-aligned (hash_key_dma_packed), 1 = windows at the key's own
// alignment (hash_key_dma_reg), 0 = direct loads.  LDS-DMA is for MD5 / SHA-1 (64-byte blocks; SHA-2 is
// compute-bound enough that direct loads match it) with prefixes of <= 4 bytes, when the LDS filter leaves room:
// line staging takes 12 KiB per wave, so three 4-wave workgroups per CU (the VGPR limit) fit beside filters of
// <= 5 KiB (the MTU filter is 1.3 KiB); window staging 8 KiB per wave.
int bloom_staging(const BloomLaunch& L) {
    if (!(L.kind == DSY_MD5 || L.kind == DSY_SHA1) || L.prm_prefix_len > 4) return 0;
    const uint64_t fbytes = L.use_lds ? (uint64_t)L.nwords * 4 : 0;
    if (((L.line_kinds >> L.kind) & 1u) && fbytes <= 5 * 1024) return 2;
    return fbytes <= 16 * 1024 ? 1 : 0;
}

template <class H, int CHUNK, int OP, int OR_MODE>
static hipError_t launch_op(const BloomLaunch& L, uint32_t grid) {
    const int dma = bloom_staging(L);
    const size_t lds = (dma == 2 ? 4 * kLineWaveBytes : dma == 1 ? 4 * kDmaWaveBytes : 0) +
                       (L.use_lds ? (size_t)L.nwords * 4 : 0);
    if constexpr (H::block_bytes == 64) {
        if (dma) {
            if constexpr (CHUNK == 2 && OR_MODE == 0) {
                if (L.diag == 1 || L.diag == 2) {
                    auto kern = dma == 2 ? (L.diag == 1 ? k_bloom<H, CHUNK, OP, 2, 1> : k_bloom<H, CHUNK, OP, 2, 2>)
                                         : (L.diag == 1 ? k_bloom<H, CHUNK, OP, 1, 1> : k_bloom<H, CHUNK, OP, 1, 2>);
                    launch_timed(kern, dim3(grid), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L.prm, L.blob,
                                 L.offsets, L.rows, L.rec, L.tasks, L.n, L.filter, L.nwords, L.use_lds, L.present);
                    return hipGetLastError();
                }
            }
            launch_timed(dma == 2 ? k_bloom<H, CHUNK, OP, 2, 0, OR_MODE> : k_bloom<H, CHUNK, OP, 1, 0, OR_MODE>,
                         dim3(grid), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L.prm, L.blob, L.offsets, L.rows,
                         L.rec, L.tasks, L.n, L.filter, L.nwords, L.use_lds, L.present);
            return hipGetLastError();
        }
    }
    launch_timed(k_bloom<H, CHUNK, OP, 0, 0, OR_MODE>, dim3(grid), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L.prm,
                 L.blob, L.offsets, L.rows, L.rec, L.tasks, L.n, L.filter, L.nwords, L.use_lds, L.present);
    return hipGetLastError();
}

template <class H, int CHUNK>
static hipError_t launch_family(const BloomLaunch& L) {
    const uint32_t block = 256;
    const uint64_t want = (L.n + block - 1) / block;
    const uint32_t grid = (uint32_t)(want < L.max_grid ? (want ? want : 1) : L.max_grid);
    switch (L.op) {
        case BloomOp::Add:
            switch (L.or_mode) {
                case 0: return launch_op<H, CHUNK, 0, 0>(L, grid);
                case 2: return launch_op<H, CHUNK, 0, 2>(L, grid);
                default: return launch_op<H, CHUNK, 0, 1>(L, grid);
            }
        case BloomOp::Test: return launch_op<H, CHUNK, 1, 0>(L, grid);
        case BloomOp::Indices:
            hipLaunchKernelGGL((k_bloom_indices<H, CHUNK>), dim3(grid), dim3(block), 0, L.stream, L.prm, L.blob,
                               L.offsets, L.n, L.indices);
            return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

template <class H>
static hipError_t launch_chunk(const BloomLaunch& L) {
    switch (L.chunk) {
        case 2: return launch_family<H, 2>(L);
        case 4: return launch_family<H, 4>(L);
        default: return launch_family<H, 8>(L);
    }
}

hipError_t launch_bloom(const BloomLaunch& L) {
    switch (L.kind) {
        case 0: return launch_chunk<Md5>(L);
        case 1: return L.chunk == 8 ? hipErrorInvalidValue : (L.chunk == 2 ? launch_family<Sha1, 2>(L) : launch_family<Sha1, 4>(L));
        case 2: return launch_chunk<Sha256>(L);
        case 3: return launch_chunk<Sha384>(L);
        default: return launch_chunk<Sha512>(L);
    }
}

}  // namespace dsy
